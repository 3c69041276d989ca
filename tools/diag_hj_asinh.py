"""asinh accuracy of the compiled (J o H)^n program (enf_flow_hj.hip) in isolation, on the diagnostics
library (ENF_HJ_ASINH selects the form). One pair: H with v = e_1 (leaves rows 1.. unchanged), then J
with gamma = xi = 0, delta = lambda = 1, so rows 1.. of Y are asinh(x). Prints the max relative error
per |x| bin against float64 arcsinh of the fp32 inputs, and the worst elements."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from enf_pkg import load  # noqa: E402


def main():
    enf = load()
    enf._lib.use_diagnostics_library()
    D = 32
    rng = np.random.default_rng(1)
    v = np.concatenate([np.logspace(-30, 3, 200_000), rng.uniform(0, 0.4, 400_000)]).astype(np.float32)
    v = np.concatenate([v, -v])
    n = (v.size + D - 2) // (D - 1)
    X = np.zeros((D, n), np.float32)
    body = np.zeros((n, D - 1), np.float32)
    body.reshape(-1)[:v.size] = v
    X[1:] = body.T
    X = np.asfortranarray(X)
    e1 = np.zeros(D, np.float32)
    e1[0] = 1
    one, zero = np.ones(D, np.float32), np.zeros(D, np.float32)
    f = enf.compose(enf.JohnsonTrafo(zero, one, zero, one), enf.HouseholderTrafo(e1))
    Xd = torch.from_numpy(X.T.copy()).cuda().T  # column-major D x n view
    Y, _ = enf.with_logabsdet_jacobian(f, Xd)
    Y = Y.cpu().numpy()[1:]
    x = X[1:].astype(np.float64)
    ref = np.arcsinh(x)
    ok = ref != 0
    rel = np.zeros_like(ref)
    rel[ok] = np.abs(Y[ok] - ref[ok]) / np.abs(ref[ok])
    ax = np.abs(x)
    out = {"form": os.environ.get("ENF_HJ_ASINH", "2"), "max_rel": float(rel.max()), "bins": {}}
    edges = [0, 1e-20, 1e-5, 1e-3, 0.01, 0.03, 0.05, 0.08, 0.11, 0.14, 0.17, 0.2, 0.25, 0.3, 0.4, 1, 10, 1e3]
    for lo, hi in zip(edges[:-1], edges[1:]):
        m = (ax >= lo) & (ax < hi) & ok
        if m.any():
            out["bins"][f"{lo:g}-{hi:g}"] = float(rel[m].max())
    w = np.argsort(rel.reshape(-1))[-5:]
    out["worst"] = [(float(x.reshape(-1)[i]), float(Y.reshape(-1)[i]), float(ref.reshape(-1)[i]),
                     float(rel.reshape(-1)[i])) for i in w]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
