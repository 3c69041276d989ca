"""Run one chained-HouseholderTrafo flow (dense MFMA kernel) a few times, for rocprofv3 passes:
python tools/wy_one.py [D] [k] [f32|f64] [N] [reps]."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from enf_pkg import load  # noqa: E402

D, k = int(sys.argv[1]) if len(sys.argv) > 1 else 32, int(sys.argv[2]) if len(sys.argv) > 2 else 32
dt = np.float64 if (sys.argv[3] if len(sys.argv) > 3 else "f32") == "f64" else np.float32
N = int(sys.argv[4]) if len(sys.argv) > 4 else 10_000_000
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
enf = load()
f = enf.HouseholderTrafo(np.asfortranarray(np.random.default_rng(42).standard_normal((D, k)).astype(dt)))
X = torch.randn((N, D), device="cuda", dtype=torch.float64 if dt == np.float64 else torch.float32).t()
for _ in range(reps):
    Y, L = enf.with_logabsdet_jacobian(f, X)
torch.cuda.synchronize()
print("ok", D, k, np.dtype(dt).name, N, reps)
