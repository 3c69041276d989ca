"""PCIe-inclusive throughput of the host-resident path (enf_flow_apply_host)
on the config-3 flow: X in host memory (pinned via torch, or pageable numpy), streamed through the
device ring, Y and ladj back in host memory. Prints one JSON line per variant."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import build_flow  # noqa: E402
from enf_pkg import load  # noqa: E402


def main():
    enf = load()
    D, N = 32, int(os.environ.get("INGEST_N", "20000000"))
    layers = build_flow(D, 4, np.float32)
    f = enf.compose(*[enf.HouseholderTrafo(ps[0]) if op == 5 else enf.JohnsonTrafo(*ps) for op, ps in reversed(layers)])
    torch.cuda.set_device(0)
    for kind in ("pinned", "pageable"):
        if kind == "pinned":
            Xt = torch.empty((N, D), dtype=torch.float32, pin_memory=True)
            Yt = torch.empty((N, D), dtype=torch.float32, pin_memory=True)
            X, Y = Xt.numpy().T, Yt.numpy().T  # column-major (D, N) views
        else:
            X = np.empty((D, N), dtype=np.float32, order="F")
            Y = np.empty((D, N), dtype=np.float32, order="F")
        X[...] = np.random.default_rng(0).standard_normal((N, D), dtype=np.float32).T
        for chunk in (1 << 20, 1 << 22):
            enf.stream_with_logabsdet_jacobian(f, X, chunk_cols=chunk, out=Y)  # warm-up
            reps = 3
            t0 = time.perf_counter()
            for _ in range(reps):
                enf.stream_with_logabsdet_jacobian(f, X, chunk_cols=chunk, out=Y)
            dt = (time.perf_counter() - t0) / reps
            print(json.dumps({"variant": f"host {kind}", "chunk_cols": chunk, "N": N, "D": D, "seconds": dt,
                              "samples_per_s": N / dt, "pcie_GBps_each_way": N * D * 4 / dt / 1e9}))


if __name__ == "__main__":
    main()
