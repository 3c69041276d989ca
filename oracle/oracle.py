"""ctypes front end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this
module, and only as the checker or as the timed CPU baseline. The product path
(``libenf.so`` + the host package) never imports it.

The oracle restates bat/EuclidianNormalizingFlows.jl v0.1.0 (see enf_oracle.c for the
file:line of every function). Matrices are numpy arrays of shape (D, N) in Fortran
(column-major) order, i.e. sample j is the contiguous column X[:, j], exactly as in Julia.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")

OP_SCALESHIFT, OP_CENTER_STRETCH, OP_CENTER_CONTRACT, OP_JOHNSON, OP_JOHNSON_INV, OP_HOUSEHOLDER = range(6)
NPARAMS = {OP_SCALESHIFT: 2, OP_CENTER_STRETCH: 3, OP_CENTER_CONTRACT: 3, OP_JOHNSON: 4,
           OP_JOHNSON_INV: 4, OP_HOUSEHOLDER: 1}


class _Layer(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("k", ctypes.c_int32), ("p", ctypes.c_void_p * 4)]


def build() -> str:
    """Compile liboracle.so with gcc (oracle/Makefile) if it is missing or stale."""
    src = [os.path.join(_HERE, f) for f in ("enf_oracle.c", "enf_oracle_jsu.c", "enf_oracle_grad.c", "enf_oracle.h",
                                             "Makefile")]
    if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < max(os.path.getmtime(s) for s in src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        for S, T in (("f64", ctypes.c_double), ("f32", ctypes.c_float), ("f80", ctypes.c_longdouble)):
            for name in ("center_stretch", "center_contract", "center_contract_ladj"):
                f = getattr(_lib, f"or_{name}_{S}")
                f.restype, f.argtypes = T, [T] * 4
            for name in ("johnsontrafo", "johnsontrafo_inv", "deriv_johnsontrafo",
                         "deriv_johnsontrafo_inv", "johnsontrafo_ladj", "johnsontrafo_inv_ladj"):
                f = getattr(_lib, f"or_{name}_{S}")
                f.restype, f.argtypes = T, [T] * 5
            f = getattr(_lib, f"or_flow_apply_{S}")
            f.restype = ctypes.c_int
            f.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                          ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                          ctypes.POINTER(_Layer), ctypes.c_int32]
            f = getattr(_lib, f"or_flow_apply_mt_{S}")
            f.restype = ctypes.c_int
            f.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                          ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                          ctypes.POINTER(_Layer), ctypes.c_int32, ctypes.c_int]
            f = getattr(_lib, f"or_mvnormal_negll_{S}")
            f.restype = T
            f.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
        for S, T in (("f64", ctypes.c_double), ("f80", ctypes.c_longdouble)):
            f = getattr(_lib, f"or_param_count_{S}")
            f.restype, f.argtypes = ctypes.c_int64, [ctypes.c_int64, ctypes.POINTER(_Layer), ctypes.c_int32]
            f = getattr(_lib, f"or_negll_grad_{S}")
            f.restype = ctypes.c_int
            f.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(_Layer),
                          ctypes.c_int32, ctypes.c_void_p]
            f = getattr(_lib, f"or_optimize_whitening_{S}")
            f.restype = ctypes.c_int64
            f.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.POINTER(_Layer), ctypes.c_int32,
                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, T, T, ctypes.c_void_p,
                          ctypes.c_int32]
        f = _lib.or_norminvcdf_f64
        f.restype, f.argtypes = ctypes.c_double, [ctypes.c_double]
        f = _lib.or_jsu_eval_vec_f64
        f.restype = None
        f.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_double] * 4
        f = _lib.or_philox4x32_10
        f.restype = None
        f.argtypes = [ctypes.POINTER(ctypes.c_uint32 * 4), ctypes.POINTER(ctypes.c_uint32 * 2),
                      ctypes.POINTER(ctypes.c_uint32 * 4)]
        f = _lib.or_jsu_uniforms
        f.restype = None
        f.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
    return _lib


JSU_FNS = ("pdf", "logpdf", "cdf", "logcdf", "ccdf", "logccdf", "quantile")  # = enf_jsu_fn codes


def jsu_eval(fn: str, x, gamma, delta, xi, lam) -> np.ndarray:
    """JohnsonSU pdf/logpdf/cdf/logcdf/ccdf/logccdf/quantile (src/johnson_trafo.jl:120-129), in double."""
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    out = np.empty_like(x)
    lib().or_jsu_eval_vec_f64(JSU_FNS.index(fn), x.size, x.ctypes.data, out.ctypes.data,
                              float(gamma), float(delta), float(xi), float(lam))
    return out


def philox4x32_10(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().or_philox4x32_10(ctypes.byref(c), ctypes.byref(k), ctypes.byref(o))
    return tuple(o)


def jsu_uniforms(dtype, n: int, seed: int, offset: int = 0) -> np.ndarray:
    """The uniforms of enf_johnsonsu_sample (Philox4x32-10 stream, include/enf.h), as float64."""
    u = np.empty(n, dtype=np.float64)
    lib().or_jsu_uniforms(int(np.dtype(dtype) == np.float64), n, u.ctypes.data, seed, offset)
    return u


def _sfx(dtype) -> str:
    dt = np.dtype(dtype)
    if dt == np.float64:
        return "f64"
    if dt == np.float32:
        return "f32"
    if dt == np.longdouble and dt.itemsize > 8:
        return "f80"
    raise TypeError(f"oracle supports float32/float64, got {dt}")


def scalar(name: str, dtype, *args) -> float:
    """Evaluate one scalar reference function, e.g. scalar('johnsontrafo', np.float64, x, g, d, xi, l)."""
    return getattr(lib(), f"or_{name}_{_sfx(dtype)}")(*[float(np.dtype(dtype).type(a)) for a in args])


def _layers(layers, dtype, D):
    """layers: list of (op, params) with params a list of arrays; Householder params[0] is D x K."""
    keep = []
    arr = (_Layer * max(1, len(layers)))()
    for i, (op, params) in enumerate(layers):
        arr[i].op = op
        arr[i].k = 0
        for q, p in enumerate(params):
            a = np.asfortranarray(np.asarray(p, dtype=dtype))
            if op == OP_HOUSEHOLDER:
                a = a.reshape(D, -1, order="F")
                arr[i].k = a.shape[1]
            else:
                a = np.broadcast_to(a, (D,)).copy()
            keep.append(a)
            arr[i].p[q] = a.ctypes.data
    return arr, keep


def flow_apply(layers, X: np.ndarray, nthreads: int = 0):
    """Apply the composed flow (layers[0] innermost) to the column-major D x N matrix X.

    Returns (Y, ladj) with Y (D, N) Fortran-ordered and ladj (N,). nthreads > 0 selects the
    OpenMP column-block variant (same arithmetic per column)."""
    X = np.asfortranarray(X)
    D, N = X.shape
    Y = np.empty((D, N), dtype=X.dtype, order="F")
    ladj = np.empty(N, dtype=X.dtype)
    arr, keep = _layers(layers, X.dtype, D)
    S = _sfx(X.dtype)
    if nthreads > 0:
        rc = getattr(lib(), f"or_flow_apply_mt_{S}")(D, N, X.ctypes.data, D, Y.ctypes.data, D,
                                                     ladj.ctypes.data, arr, len(layers), nthreads)
    else:
        rc = getattr(lib(), f"or_flow_apply_{S}")(D, N, X.ctypes.data, D, Y.ctypes.data, D,
                                                  ladj.ctypes.data, arr, len(layers))
    if rc != 0:
        raise ValueError("oracle: unknown op in flow")
    del keep
    return Y, ladj


def flow_apply_hi(layers, X: np.ndarray, nthreads: int = 8):
    """The same flow evaluated in higher precision on the same (rounded) inputs and parameters:
    fp32 data in float64, fp64 data in x87 extended precision. Returned as float64; the stand-in
    for the exact values when measuring how accurate a T-precision evaluation is."""
    X = np.asfortranarray(X)
    hi = np.float64 if X.dtype == np.float32 else np.longdouble
    lay = [(op, [np.asarray(p).astype(hi) for p in ps]) for op, ps in layers]
    Y, L = flow_apply(lay, X.astype(hi), nthreads=nthreads)
    return np.asfortranarray(Y.astype(np.float64)), L.astype(np.float64)


def mvnormal_negll(Y: np.ndarray, ladj: np.ndarray) -> float:
    Y = np.asfortranarray(Y)
    D, N = Y.shape
    ladj = np.ascontiguousarray(ladj, dtype=Y.dtype)
    return getattr(lib(), f"or_mvnormal_negll_{_sfx(Y.dtype)}")(D, N, Y.ctypes.data, ladj.ctypes.data)


def _grad_dtype(dtype):
    if np.dtype(dtype) not in (np.dtype(np.float64), np.dtype(np.longdouble)):
        raise ValueError("oracle gradient: float64 or longdouble")
    return "f64" if np.dtype(dtype) == np.dtype(np.float64) else "f80"


def theta_of(layers, D, dtype=np.float64):
    """The flat parameter vector of a flow in the enf_flow_param_count layout (per layer, per field, length-D
    vectors; a Householder V as its D x k matrix, column-major)."""
    out = []
    for op, ps in layers:
        for p in ps:
            a = np.asarray(p, dtype=dtype)
            out.append(a.reshape(D, -1, order="F").reshape(-1, order="F") if op == OP_HOUSEHOLDER
                       else np.broadcast_to(a, (D,)).astype(dtype))
    return np.concatenate(out)


def _theta_layers(layers, theta, D):
    """ctypes layers whose parameter pointers point into theta (the layout of theta_of)."""
    arr = (_Layer * max(1, len(layers)))()
    o = 0
    esz = theta.dtype.itemsize
    for i, (op, ps) in enumerate(layers):
        arr[i].op = op
        arr[i].k = np.asarray(ps[0]).reshape(D, -1, order="F").shape[1] if op == OP_HOUSEHOLDER else 0
        for q in range(len(ps)):
            arr[i].p[q] = theta.ctypes.data + o * esz
            o += D * (arr[i].k if op == OP_HOUSEHOLDER else 1)
    return arr


def negll_grad(layers, X: np.ndarray):
    """mvnormal_negll_trafograd (src/optimize_whitening.jl:18-22) on the CPU: (negll, gradient) with the gradient
    flat in the enf_flow_param_count layout (theta_of). float64 or longdouble (x87) data."""
    X = np.asfortranarray(X)
    D, N = X.shape
    S = _grad_dtype(X.dtype)
    theta = theta_of(layers, D, X.dtype)
    arr = _theta_layers(layers, theta, D)
    out = np.zeros(1 + theta.size, dtype=X.dtype)
    if getattr(lib(), f"or_negll_grad_{S}")(D, N, X.ctypes.data, D, arr, len(layers), out.ctypes.data) != 0:
        raise ValueError("oracle: unknown op in flow")
    return float(out[0]), out[1:]


def scaleshift_ladj(layers) -> float:
    """sum log|a| over the flow's ScaleShiftTrafos (src/scale_shift_trafo.jl:22, over a's own length): what the
    reference's recorded negll carries extra under Zygote, where rrule(similar_fill) makes that ladj's primal zero
    (src/abstract_trafo.jl:30-33)."""
    return float(sum(np.sum(np.log(np.abs(np.asarray(ps[0], np.float64)))) for op, ps in layers if op == OP_SCALESHIFT))


def optimize_whitening(layers, X: np.ndarray, nbatches: int, nepochs: int, eta: float = 0.1, epsilon: float = 1e-8,
                       zygote: bool = False):
    """optimize_whitening (src/optimize_whitening.jl:25-45) with ADAGrad(eta, epsilon) on the CPU: returns
    (theta, acc, negll_history), theta in the theta_of layout. zygote=True records the loss as the reference does
    under Zygote (scaleshift_ladj of the step's parameters added to every entry); False the true negll. The
    minibatch size is round(N / nbatches) with ties to even, as Julia's round(Int, x) (optimize_whitening.jl:31)."""
    X = np.asfortranarray(X)
    D, N = X.shape
    S = _grad_dtype(X.dtype)
    theta = theta_of(layers, D, X.dtype)
    acc = np.full_like(theta, epsilon)
    arr = _theta_layers(layers, theta, D)
    bs = max(int(round(N / nbatches)), 1)
    hist = np.zeros(nepochs * (-(-N // bs)), dtype=X.dtype)
    n = getattr(lib(), f"or_optimize_whitening_{S}")(D, N, X.ctypes.data, arr, len(layers), theta.ctypes.data,
                                                     acc.ctypes.data, nbatches, nepochs, eta, epsilon, hist.ctypes.data,
                                                     1 if zygote else 0)
    if n < 0:
        raise ValueError("oracle: unknown op in flow")
    return theta, acc, hist[:n]


def inverse_layers(layers, dtype=np.float64):
    """InverseFunctions.inverse of a composition: reversed order, each layer inverted.

    ScaleShift: (1/a, -(1/a)*b) (src/scale_shift_trafo.jl:26-30); CenterStretch <-> CenterContract
    (src/center_stretch.jl:45,69); Johnson <-> JohnsonInv (src/johnson_trafo.jl:82,107);
    Householder: reversed columns (src/householder_trafo.jl:153-154)."""
    out = []
    for op, params in reversed(layers):
        if op == OP_SCALESHIFT:
            a = np.asarray(params[0], dtype=dtype)
            b = np.asarray(params[1], dtype=dtype)
            ainv = (dtype(1) / a).astype(dtype)
            out.append((op, [ainv, (-ainv * b).astype(dtype)]))
        elif op == OP_CENTER_STRETCH:
            out.append((OP_CENTER_CONTRACT, params))
        elif op == OP_CENTER_CONTRACT:
            out.append((OP_CENTER_STRETCH, params))
        elif op == OP_JOHNSON:
            out.append((OP_JOHNSON_INV, params))
        elif op == OP_JOHNSON_INV:
            out.append((OP_JOHNSON, params))
        elif op == OP_HOUSEHOLDER:
            V = np.asarray(params[0], dtype=dtype)
            V = V.reshape(V.shape[0], -1, order="F")
            out.append((op, [np.asfortranarray(V[:, ::-1])]))
        else:
            raise ValueError(op)
    return out
