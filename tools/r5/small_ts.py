"""Phase clocks of the one-block whitening step (diagnostics library, ENF_SMALL_TS=1): the reference examples'
flows, 20 eager steps each; thread 0 of the kernel prints prologue / tiles / partials / update shader clocks.
--epoch: the 20 steps as one enf_whitening_epoch launch (one line per step) instead of 20 step launches."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
os.environ.setdefault("ENF_SMALL_TS", "1")

import torch  # noqa: E402

import bench_train  # noqa: E402
import oracle  # noqa: E402  (the examples' true flows only)
from enf_pkg import load  # noqa: E402

enf = load()
enf._lib.use_diagnostics_library()
dev = torch.device("cuda", 0)
epoch = "--epoch" in sys.argv
for ex in [a for a in sys.argv[1:] if not a.startswith("--")] or ["2d", "1d"]:
    D, true, init, nbatches, _ = bench_train.example_flows(ex)
    B = 100_000 // nbatches
    N = 20 * B
    rng = np.random.default_rng(1)
    X, _ = oracle.flow_apply(true, np.asfortranarray(rng.standard_normal((D, N))))
    mk = lambda layers: enf.compose(*[
        {0: lambda ps: enf.ScaleShiftTrafo(*ps), 1: lambda ps: enf.CenterStretch(*ps),
         2: lambda ps: enf.CenterContract(*ps), 3: lambda ps: enf.JohnsonTrafo(*ps),
         5: lambda ps: enf.HouseholderTrafo(ps[0])}[op](ps) for op, ps in reversed(layers)])
    Xd = torch.from_numpy(np.ascontiguousarray(np.asarray(X).T)).to(dev).t()
    print(f"== example {ex}: D={D} B={B} {'epoch kernel' if epoch else 'step launches'}", flush=True)
    enf.optimize_whitening(Xd, mk(init), enf.ADAGrad(), nbatches=20, nepochs=1, graph=False, _per_step=not epoch)
    torch.cuda.synchronize()
    sys.stdout.flush()
