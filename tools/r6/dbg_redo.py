"""Debug probe (round 6): tests/test_gpu_parity.py::test_hj_program_exact_redo_edge_values' input through a
library build (argv[1]: 'product' or a path), printing where the NaN / Inf pattern differs from the oracle's."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
np.seterr(all="ignore")
from enf_pkg import load  # noqa: E402

enf = load()
if sys.argv[1] != "product":
    enf._lib.use_diagnostics_library(os.path.join(ROOT, sys.argv[1]))
import oracle  # noqa: E402
from parity import colmajor_cuda, make_flow, to_np  # noqa: E402
from test_gpu_parity import _hj_layers  # noqa: E402

D = int(sys.argv[2]) if len(sys.argv) > 2 else 32
rng = np.random.default_rng(11)
layers = _hj_layers(rng, D, 4)
N = 4096
X = rng.standard_normal((D, N)).astype(np.float32)
X[3, 7] = 3e30
X[0, 100] = -1e25
X[5, 101] = np.inf
X[D - 1, 2000] = np.nan
X[:, 4095] = 1e3
X = np.asfortranarray(X)
Yr, Lr = oracle.flow_apply(layers, X)
Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
Y, L = to_np(Y), to_np(L).reshape(-1)
for what, f in (("nan", np.isnan), ("inf", np.isinf)):
    bad = np.argwhere(f(Y) != f(Yr))
    cols = sorted(set(bad[:, 1].tolist()))
    print(what, "Y mismatches", len(bad), "columns", cols[:20])
    for c in cols[:6]:
        print(" col", c, "Y", Y[:6, c], "Yr", Yr[:6, c], "L", L[c], "Lr", Lr[c])
    badl = np.nonzero(f(L) != f(Lr))[0]
    print(what, "ladj mismatches", badl[:20], L[badl[:6]], Lr[badl[:6]])
