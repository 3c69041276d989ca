"""One epoch of a reference example's training (bench_train.example_flows: its flow, data and batch size) through
optimize_whitening on one GPU -- a single enf_whitening_epoch launch -- for rocprofv3 PMC passes (tools/r5/run16.sh)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import torch  # noqa: E402

import bench_train  # noqa: E402
import oracle  # noqa: E402  (the example's true flow only, for the data)
from enf_pkg import load  # noqa: E402

enf = load()
ex = sys.argv[1] if len(sys.argv) > 1 else "2d"
D, true, init, nbatches, _ = bench_train.example_flows(ex)
rng = np.random.default_rng(1)
X, _ = oracle.flow_apply(true, np.asfortranarray(rng.standard_normal((D, 100_000))))
mk = lambda layers: enf.compose(*[
    {0: lambda ps: enf.ScaleShiftTrafo(*ps), 1: lambda ps: enf.CenterStretch(*ps),
     2: lambda ps: enf.CenterContract(*ps), 3: lambda ps: enf.JohnsonTrafo(*ps),
     5: lambda ps: enf.HouseholderTrafo(ps[0])}[op](ps) for op, ps in reversed(layers)])
Xd = torch.from_numpy(np.ascontiguousarray(np.asarray(X).T)).to("cuda:0").t()
r = enf.optimize_whitening(Xd, mk(init), enf.ADAGrad(), nbatches=nbatches, nepochs=1)
torch.cuda.synchronize()
print(ex, "steps", len(r.negll_history), "last negll", r.negll_history[-1])
