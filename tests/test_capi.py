"""CPU: libenf.so loads and exports every entry point include/enf.h declares; argument validation
that needs no device (no compute calls without a GPU)."""
import ctypes
import os
import re

import numpy as np

from conftest import ROOT


def header_functions():
    src = open(os.path.join(ROOT, "include", "enf.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(enf_[a-z0-9_]+)\s*\(", src)))


def test_header_lists_all_exports(enf):
    names = header_functions()
    assert len(names) >= 19
    assert set(names) == set(enf._lib.EXPORTED)


def test_library_exports_every_symbol(enf):
    lib = ctypes.CDLL(enf._lib.LIB_PATH)
    for name in header_functions():
        assert hasattr(lib, name), name


def test_no_oracle_in_product(enf):
    """The product library links no part of the oracle (nm: no or_* symbols, no liboracle)."""
    import subprocess

    out = subprocess.run(["nm", "-D", enf._lib.LIB_PATH], capture_output=True, text=True).stdout
    assert not re.search(r"\bor_[a-z]", out)
    ldd = subprocess.run(["ldd", enf._lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in ldd


def test_shipping_library_reads_no_environment(enf):
    """The shipping libenf.so has no runtime tuning or diagnostic knobs: it
    imports no getenv/secure_getenv and contains none of the ENF_* knob names, which exist only in
    the ENF_DIAG=1 build (libenf_diag.so, tools/ only). The package binds libenf.so."""
    import subprocess

    path = os.path.join(os.path.dirname(enf._lib.DIAG_LIB_PATH), "libenf.so")
    assert enf._lib.LIB_PATH == path
    und = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True, text=True).stdout
    assert not re.search(r"\b(secure_)?getenv\b", und)
    blob = open(path, "rb").read()
    for knob in (b"ENF_DEBUG_MODE", b"ENF_HJ_R", b"ENF_FRAG_U", b"ENF_GRAD_REG", b"ENF_WY_MIN_K",
                 b"ENF_BLOCKS_PER_CU", b"ENF_NO_SPECIALIZE", b"ENF_LDS_GENERIC_KB"):
        assert knob not in blob, knob


def test_version_and_errors(enf):
    L = enf._lib.lib()
    assert L.enf_version().decode().startswith("0.1.0")
    arr = (enf._lib.Layer * 1)()
    arr[0].op = 3
    # invalid dtype, negative sizes, unknown op, NULL params, ld < D: all rejected before any GPU work
    assert L.enf_flow_apply(7, 2, 10, None, 2, None, 2, None, 0, arr, 1, None) == enf._lib.ENF_ERR_INVALID
    assert "dtype" in L.enf_last_error().decode()
    assert L.enf_flow_apply(0, -1, 10, None, 2, None, 2, None, 0, arr, 1, None) == enf._lib.ENF_ERR_INVALID
    assert L.enf_flow_apply(0, 4, 10, None, 2, None, 4, None, 0, arr, 1, None) == enf._lib.ENF_ERR_INVALID
    assert L.enf_flow_apply(0, 2, 10, None, 2, None, 2, None, 0, arr, 1, None) == enf._lib.ENF_ERR_INVALID
    assert "parameter 0 is NULL" in L.enf_last_error().decode()
    arr[0].op = 42
    assert L.enf_flow_apply(0, 2, 10, None, 2, None, 2, None, 0, arr, 1, None) == enf._lib.ENF_ERR_INVALID
    assert "unknown op" in L.enf_last_error().decode()
    arr[0].op = 5
    arr[0].k = 0
    assert L.enf_flow_apply(0, 2, 10, None, 2, None, 2, None, 0, arr, 1, None) == enf._lib.ENF_ERR_INVALID
    # N == 0 is a no-op that succeeds without touching memory
    arr[0].op, arr[0].k = 3, 0
    for q in range(4):
        arr[0].p[q] = 16
    assert L.enf_flow_apply(0, 2, 0, None, 2, None, 2, None, 0, arr, 1, None) == enf._lib.ENF_OK


def test_johnsonsu_argument_checks(enf):
    """enf_johnsonsu_eval / _sample reject bad arguments before any device work; n == 0 is a no-op."""
    L = enf._lib.lib()
    E = enf._lib.ENF_ERR_INVALID
    assert L.enf_johnsonsu_eval(5, 0, 4, 16, 16, 0.0, 1.0, 0.0, 1.0, None) == E
    assert L.enf_johnsonsu_eval(0, 7, 4, 16, 16, 0.0, 1.0, 0.0, 1.0, None) == E
    assert "unknown JohnsonSU function" in L.enf_last_error().decode()
    assert L.enf_johnsonsu_eval(0, 0, -1, 16, 16, 0.0, 1.0, 0.0, 1.0, None) == E
    assert L.enf_johnsonsu_eval(0, 0, 4, None, 16, 0.0, 1.0, 0.0, 1.0, None) == E
    assert L.enf_johnsonsu_eval(1, 6, 0, None, None, 0.0, 1.0, 0.0, 1.0, None) == enf._lib.ENF_OK
    assert L.enf_johnsonsu_sample(3, 4, 16, 0.0, 1.0, 0.0, 1.0, 1, 0, None) == E
    assert L.enf_johnsonsu_sample(0, 4, None, 0.0, 1.0, 0.0, 1.0, 1, 0, None) == E
    assert L.enf_johnsonsu_sample(0, 0, None, 0.0, 1.0, 0.0, 1.0, 1, 0, None) == enf._lib.ENF_OK


def test_johnsonsu_host_statistics(enf):
    """Host-side statistics of the JohnsonSU mirror (src/johnson_trafo.jl:21-26)."""
    import math

    d = enf.JohnsonSU(-15, 6.5, 0, 2.5)
    assert d.mean() == 0 - 2.5 * math.exp(6.5 ** -2 / 2) * math.sinh(-15 / 6.5)
    assert d.median() == 2.5 * math.sinh(15 / 6.5)
    assert d.location() == d.mean() and d.scale() == d.var()  # the reference's scale = var quirk
    assert d.minimum() == -math.inf and d.maximum() == math.inf and d.partype == np.float64


def test_param_count(enf):
    L = enf._lib.lib()
    arr = (enf._lib.Layer * 3)()
    for i, (op, k) in enumerate([(5, 3), (3, 0), (0, 0)]):
        arr[i].op, arr[i].k = op, k
        for q in range(4):
            arr[i].p[q] = 16
    n = ctypes.c_int64()
    assert L.enf_flow_param_count(32, arr, 3, ctypes.byref(n)) == 0
    assert n.value == 32 * 3 + 32 * 4 + 32 * 2


def test_comm_validation(enf):
    L = enf._lib.lib()
    comm = ctypes.c_void_p()
    assert L.enf_comm_init(ctypes.byref(comm), 0, b"\0" * 128, 0) == enf._lib.ENF_ERR_INVALID
    assert L.enf_allreduce_sum(None, None, 4, 0, None) == enf._lib.ENF_ERR_INVALID
    assert L.enf_adagrad_step(0, 4, None, None, None, 1.0, 0.1, 1e-7, None) == enf._lib.ENF_ERR_INVALID
    assert L.enf_adagrad_step(0, 0, None, None, None, 1.0, 0.1, 1e-7, None) == enf._lib.ENF_OK
