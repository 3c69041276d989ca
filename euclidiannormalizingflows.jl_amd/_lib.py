"""ctypes binding of libenf.so (include/enf.h) -- the only way the host package reaches the GPU.

The library is built in-tree by ``__graft_entry__.build()`` (csrc/Makefile) and lives next to this
file. There is no fallback: if the library or a GPU is missing, every compute call raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libenf.so")
# ENF_DIAG=1 build of the same sources (csrc/Makefile `diag`): tuning knobs and diagnostic kernel
# variants read from ENF_* environment variables. tools/ only; see use_diagnostics_library().
DIAG_LIB_PATH = os.path.join(_HERE, "libenf_diag.so")

ENF_OK, ENF_ERR_INVALID, ENF_ERR_HIP, ENF_ERR_UNSUPPORTED, ENF_ERR_RCCL = range(5)
ENF_F32, ENF_F64 = 0, 1
ENF_NEGLL_ZYGOTE = 0x100  # dtype flag of the training calls: report the loss the reference records (include/enf.h)
OP_SCALESHIFT, OP_CENTER_STRETCH, OP_CENTER_CONTRACT, OP_JOHNSON, OP_JOHNSON_INV, OP_HOUSEHOLDER = range(6)
UNIQUE_ID_BYTES = 128

# every symbol include/enf.h declares (checked by tests/test_capi.py)
EXPORTED = (
    "enf_version", "enf_last_error", "enf_device_count", "enf_set_device", "enf_get_device",
    "enf_malloc", "enf_free", "enf_memcpy", "enf_stream_synchronize", "enf_flow_apply", "enf_flow_apply_host",
    "enf_flow_param_count", "enf_flow_negll_grad_workspace", "enf_flow_negll_grad", "enf_flow_negll_workspace",
    "enf_flow_negll",
    "enf_adagrad_step", "enf_householder_normalize", "enf_householder_normalize_strided", "enf_comm_unique_id", "enf_comm_init",
    "enf_comm_destroy", "enf_allreduce_sum", "enf_johnsonsu_eval", "enf_johnsonsu_sample",
    "enf_whitening_step", "enf_whitening_apply", "enf_flow_vjp", "enf_flow_apply_cpu", "enf_whitening_step_dp",
    "enf_stream_copy", "enf_whitening_epoch",
)


class EnfError(RuntimeError):
    """A libenf call returned a non-OK enf_status."""

    def __init__(self, status: int, message: str):
        super().__init__(f"libenf error {status}: {message}")
        self.status = status


class Layer(ctypes.Structure):
    """enf_layer"""
    _fields_ = [("op", ctypes.c_int32), ("k", ctypes.c_int32), ("p", ctypes.c_void_p * 4)]


_lock = threading.Lock()
_lib = None

_vp, _i32, _i64, _sz, _dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_double
_SIGS = {
    "enf_version": (ctypes.c_char_p, []),
    "enf_last_error": (ctypes.c_char_p, []),
    "enf_device_count": (ctypes.c_int, [ctypes.POINTER(_i32)]),
    "enf_set_device": (ctypes.c_int, [_i32]),
    "enf_get_device": (ctypes.c_int, [ctypes.POINTER(_i32)]),
    "enf_malloc": (ctypes.c_int, [ctypes.POINTER(_vp), _sz]),
    "enf_free": (ctypes.c_int, [_vp]),
    "enf_memcpy": (ctypes.c_int, [_vp, _vp, _sz, _i32, _vp]),
    "enf_stream_synchronize": (ctypes.c_int, [_vp]),
    "enf_flow_apply": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _i32,
                                      ctypes.POINTER(Layer), _i32, _vp]),
    "enf_flow_apply_host": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _i32,
                                           ctypes.POINTER(Layer), _i32, _i64, _vp]),
    "enf_flow_param_count": (ctypes.c_int, [_i64, ctypes.POINTER(Layer), _i32, ctypes.POINTER(_i64)]),
    "enf_flow_negll_grad_workspace": (ctypes.c_int, [ctypes.c_int, _i64, _i64, ctypes.POINTER(Layer), _i32,
                                                     ctypes.POINTER(_sz)]),
    "enf_flow_negll_grad": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _vp, _i64, ctypes.POINTER(Layer), _i32,
                                           _vp, _vp, _sz, _vp]),
    "enf_flow_negll_workspace": (ctypes.c_int, [ctypes.c_int, _i64, _i64, ctypes.POINTER(_sz)]),
    "enf_flow_negll": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _vp, _i64, ctypes.POINTER(Layer), _i32, _vp, _vp, _sz,
                                      _vp]),
    "enf_flow_apply_cpu": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _i32,
                                          ctypes.POINTER(Layer), _i32, _i32]),
    "enf_flow_vjp": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _vp, _i64, _vp, _i64, _vp, ctypes.POINTER(Layer), _i32,
                                    _vp, _i64, _vp, _vp, _sz, _vp]),
    "enf_adagrad_step": (ctypes.c_int, [ctypes.c_int, _i64, _vp, _vp, _vp, _dbl, _dbl, _dbl, _vp]),
    "enf_householder_normalize": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _vp, _vp]),
    "enf_householder_normalize_strided": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _vp, _i64, _vp]),
    "enf_stream_copy": (ctypes.c_int, [_vp, _vp, _i64, _i32, _vp]),
    "enf_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "enf_comm_init": (ctypes.c_int, [ctypes.POINTER(_vp), _i32, ctypes.c_char_p, _i32]),
    "enf_comm_destroy": (ctypes.c_int, [_vp]),
    "enf_allreduce_sum": (ctypes.c_int, [_vp, _vp, _i64, ctypes.c_int, _vp]),
    "enf_whitening_step": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _vp, _i64, ctypes.POINTER(Layer), _i32, _vp, _vp,
                                          _vp, _i32, _vp, _i32, _dbl, _dbl, _vp, _vp, _sz, _vp]),
    "enf_whitening_epoch": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _vp, _i64, _i64, ctypes.POINTER(Layer), _i32, _vp,
                                           _vp, _vp, _i32, _vp, _i32, _dbl, _dbl, _vp, _vp, _sz, _vp]),
    "enf_whitening_apply": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _vp, _i64, _vp, _vp, _vp, _i32, _vp, _i32, _dbl,
                                           _dbl, _vp, _vp]),
    "enf_whitening_step_dp": (ctypes.c_int, [ctypes.c_int, _i64, _i64, _vp, _i64, ctypes.POINTER(Layer), _i32, _vp,
                                             _vp, _vp, _i32, _vp, _i32, _dbl, _dbl, _i64, _vp, _vp, _vp, _sz, _vp]),
    "enf_johnsonsu_eval": (ctypes.c_int, [ctypes.c_int, _i32, _i64, _vp, _vp, _dbl, _dbl, _dbl, _dbl, _vp]),
    "enf_johnsonsu_sample": (ctypes.c_int, [ctypes.c_int, _i64, _vp, _dbl, _dbl, _dbl, _dbl, ctypes.c_uint64,
                                            ctypes.c_uint64, _vp]),
}


def use_diagnostics_library(path: str | None = None) -> None:
    """Bind libenf_diag.so (or another build of the same ABI at `path`, e.g. an earlier round's library for
    an A/B) instead of libenf.so (tools under tools/ only; bench.py, the tests and the package never call
    this). Must run before the first lib() call."""
    global LIB_PATH
    if _lib is not None:
        raise RuntimeError("libenf is already loaded")
    LIB_PATH = path or DIAG_LIB_PATH


def loaded_path() -> str:
    """Path of the bound library (bench.py asserts it is the shipping libenf.so)."""
    lib()
    return LIB_PATH


def lib() -> ctypes.CDLL:
    """Load libenf.so once (raises if it was not built)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -c 'import "
                                       "__graft_entry__ as g; g.build()'` (hipcc, gfx950)")
                L = ctypes.CDLL(LIB_PATH)
                for name, (res, args) in _SIGS.items():
                    f = getattr(L, name)
                    f.restype, f.argtypes = res, args
                _lib = L
    return _lib


def check(status: int) -> None:
    if status != ENF_OK:
        raise EnfError(status, lib().enf_last_error().decode(errors="replace"))


def version() -> str:
    return lib().enf_version().decode()
