import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libenf.so on the device)")
    # diagnostics only: ENF_GUARD_ALLOC=1 | 2 puts every torch device allocation on guard
    # pages (tools/guard_alloc.cpp: data ending / starting at an unmapped page), so an out-of-range read or
    # write of any kernel faults in that kernel. Must be installed before the first device allocation.
    if os.environ.get("ENF_GUARD_ALLOC"):
        import torch

        so = os.path.join(ROOT, "tools", "libguard_alloc.so")
        alloc = torch.cuda.memory.CUDAPluggableAllocator(so, "enf_guard_malloc", "enf_guard_free")
        torch.cuda.memory.change_current_allocator(alloc)


@pytest.fixture(scope="session")
def oracle():
    import oracle as o  # test infrastructure: the checker

    o.build()
    return o


@pytest.fixture(scope="session")
def enf():
    from enf_pkg import load

    return load()


@pytest.fixture(scope="session")
def gpu(enf):
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch.cuda.is_available() is False")
    enf._lib.lib()
    return torch.device("cuda:0")


def load_golden_flow(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    layers = []
    for i, op in enumerate(z["ops"]):
        ps, q = [], 0
        while f"L{i}_p{q}" in z:
            ps.append(z[f"L{i}_p{q}"])
            q += 1
        layers.append((int(op), ps))
    return layers, z["X"], z["Y_exact"], z["ladj_exact"]
