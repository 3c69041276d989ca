"""Debug: compiled (J o H)^n kernel vs the interpreter on the config-3 pattern; report bad columns."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from enf_pkg import load
from parity import make_flow, rand_params, colmajor_cuda, to_np
enf = load()
D = int(os.environ.get("D", "32"))
for N in [int(v) for v in os.environ.get("NS", "131072 131104 163840 200003").split()]:
    rng = np.random.default_rng(7 + D)
    layers = []
    for _ in range(4):
        layers += [(5, rand_params(rng, 5, D, np.float32)), (3, rand_params(rng, 3, D, np.float32))]
    X = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
    f = make_flow(enf, layers)
    Y, L = enf.with_logabsdet_jacobian(f, colmajor_cuda(X))
    Y, L = to_np(Y), to_np(L).reshape(-1)
    os.environ["ENF_NO_SPECIALIZE"] = "1"
    # interpreter reference: separate process state (static env read once) -> use a layer split trick:
    # apply the flow as two compositions (first 2 layers, then the rest) so the compiled path is not taken
    f1 = make_flow(enf, layers[:1]); f2 = make_flow(enf, layers[1:])
    Y1, L1 = enf.with_logabsdet_jacobian(f1, colmajor_cuda(X))
    Y2, L2 = enf.with_logabsdet_jacobian(f2, Y1)
    Yr, Lr = to_np(Y2), (to_np(L1) + to_np(L2)).reshape(-1)
    e = np.abs(Y - Yr).max(axis=0) / (np.abs(Yr).max(axis=0) + 1)
    el = np.abs(L - Lr) / (np.abs(Lr) + 1)
    bad = np.nonzero((e > 1e-4) | (el > 1e-4))[0]
    by = np.nonzero(e > 1e-4)[0]; bl = np.nonzero(el > 1e-4)[0]
    print(f"  Ybad {len(by)} Lbad {len(bl)}; bad tiles (32 cols):", np.unique(bad // 32)[:20], "n tiles", len(np.unique(bad // 32)))
    print(f"N={N}: max colerr {e.max():.3e} ladj {el.max():.3e} bad cols {len(bad)}", bad[:10], bad[-5:] if len(bad) else "")
    if len(bad):
        j = bad[0]
        print(" Y", Y[:6, j], "\n Yr", Yr[:6, j], "\n L", L[j], Lr[j])
