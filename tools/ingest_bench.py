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


def raw_copy_ceiling(nbytes=1 << 30, reps=5):
    """PCIe ceilings on this box: pinned H2D alone, D2H alone, and both at once on two streams."""
    h_in = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d_b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    res = {}
    for name, up, down in (("h2d", True, False), ("d2h", False, True), ("both", True, True)):
        for it in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if up:
                with torch.cuda.stream(s1):
                    d_a.copy_(h_in, non_blocking=True)
            if down:
                with torch.cuda.stream(s2):
                    h_out.copy_(d_b, non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if it == 1:
                best = dt
            elif it > 1:
                best = min(best, dt)
        res[name + "_GBps_each_way"] = nbytes / best / 1e9
    print(json.dumps({"variant": "raw pinned copy ceiling", "bytes": nbytes, **res}))


def main():
    enf = load()
    raw_copy_ceiling()
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
