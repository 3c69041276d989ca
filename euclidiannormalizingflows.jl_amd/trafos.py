"""Host mirror of the bat/EuclidianNormalizingFlows.jl transform API, backed by libenf.so.

Julia                                              here
-------------------------------------------------  ------------------------------------------------
ScaleShiftTrafo(a, b)  src/scale_shift_trafo.jl:4   ScaleShiftTrafo(a, b)
CenterStretch(a=0,b=1,c=0)  src/center_stretch.jl:25   CenterStretch(a=0.0, b=1.0, c=0.0)
CenterContract  src/center_stretch.jl:49            CenterContract(...)
JohnsonTrafo(gamma=10,delta=3.5,xi=10,lambda=1)     JohnsonTrafo(gamma=10.0, delta=3.5, xi=10.0, lambda_=1.0)
  src/johnson_trafo.jl:61
JohnsonTrafoInv  src/johnson_trafo.jl:86            JohnsonTrafoInv(...)
HouseholderTrafo(V)  src/householder_trafo.jl:127   HouseholderTrafo(V)  (vector or D x K matrix)
f ∘ g  (Base.ComposedFunction)                      f @ g  or  compose(f, g)
f(X)                                                f(X)
with_logabsdet_jacobian(f, X)                       with_logabsdet_jacobian(f, X) -> (Y, ladj)
InverseFunctions.inverse(f)                         inverse(f)

Batches are Julia's column-major D x N matrices: a torch tensor of shape (D, N) whose sample
columns are contiguous (stride (1, D)), e.g. ``Z.t()`` of a contiguous (N, D) tensor; other
strides are copied into that layout first. ``ladj`` is returned as a (1, N) row (Julia's
Adjoint row, src/abstract_trafo.jl:9); a single sample x of shape (D,) gives a 0-dim ladj.
Numeric types follow Julia's promotion (src/johnson_trafo.jl:30): Python ``int`` parameters do
not promote, Python ``float`` parameters are Float64, arrays/tensors carry their own dtype.
A composition runs as ONE fused enf_flow_apply launch per run of equal promoted type.

Where the data lives selects where it is computed, as in Julia (an Array runs the reference's CPU
methods): CUDA tensors run the HIP kernels (enf_flow_apply); host data -- numpy arrays, CPU tensors
and Python / numpy scalars -- runs libenf's host implementation (enf_flow_apply_cpu, SURVEY.md §8
config 1 "on CPU, no GPU"). Neither is a fallback for the other: a CUDA tensor without a usable GPU
fails, and host data never touches the GPU (stream_with_logabsdet_jacobian streams a host batch
through the GPU explicitly). A scalar x follows Julia's broadcasting (src/johnson_trafo.jl:74-76,
src/center_stretch.jl:37-39): with scalar parameters y and ladj are scalars; with vector parameters
y is the length-D vector of x broadcast against them and ladj their sum.
"""
from __future__ import annotations

import numbers
from typing import List, Sequence

import numpy as np
import torch

from . import _lib


class MethodError(TypeError):
    """Mirror of Julia's MethodError for call signatures the reference does not define."""


class DimensionMismatch(ValueError):
    """Mirror of Julia's DimensionMismatch for non-broadcastable parameter shapes."""


# ----------------------------------------------------------------------------- type helpers
_INT = "int"


def _kind(p):
    """Julia eltype class of a parameter: 'int', torch.float32 or torch.float64."""
    if isinstance(p, torch.Tensor):
        if p.dtype in (torch.float32, torch.float64):
            return p.dtype
        if p.dtype in (torch.float16, torch.bfloat16):
            return torch.float32
        return _INT
    if isinstance(p, np.ndarray) or isinstance(p, np.generic):
        dt = np.asarray(p).dtype
        if dt == np.float32 or dt == np.float16:
            return torch.float32
        if dt.kind == "f":
            return torch.float64
        return _INT
    if isinstance(p, (bool, numbers.Integral)):
        return _INT
    if isinstance(p, numbers.Real):
        return torch.float64
    if isinstance(p, (list, tuple)):
        ks = [_kind(q) for q in p]
        return _promote(*ks) if any(k != _INT for k in ks) else _INT
    raise TypeError(f"unsupported parameter type {type(p)}")


def _promote(*kinds):
    """float(promote_type(...)): any Float64 -> Float64; else any Float32 -> Float32; all ints -> Float64."""
    if torch.float64 in kinds:
        return torch.float64
    if torch.float32 in kinds:
        return torch.float32
    return torch.float64


def _as_cpu_array(p) -> np.ndarray:
    if isinstance(p, torch.Tensor):
        return p.detach().cpu().numpy()
    return np.asarray(p)


def _is_vector(p) -> bool:
    return _as_cpu_array(p).ndim >= 1


def _eq(a, b) -> bool:
    A, B = _as_cpu_array(a), _as_cpu_array(b)
    return A.shape == B.shape and bool(np.all(A == B))


def _isequal(a, b) -> bool:
    A, B = _as_cpu_array(a), _as_cpu_array(b)
    if A.shape != B.shape:
        return False
    if A.dtype.kind == "f" or B.dtype.kind == "f":
        return bool(np.all((A == B) | (np.isnan(A) & np.isnan(B))))
    return bool(np.all(A == B))


def _hashable(p):
    A = _as_cpu_array(p)
    return (A.shape, A.astype(np.float64).tobytes() if A.dtype.kind in "fiub" else A.tobytes())


# ----------------------------------------------------------------------------- base classes
class Trafo:
    """A leaf bijector. Subclasses set OP, FIELDS (parameter names, Julia field order)."""

    OP: int = -1
    FIELDS: Sequence[str] = ()

    def params(self) -> List:
        return [getattr(self, f) for f in self.FIELDS]

    def __call__(self, X):
        return _apply(self, X, want_ladj=False)[0]

    def __matmul__(self, other):
        return ComposedFunction(self, other)

    def __eq__(self, other):
        return type(self) is type(other) and all(_eq(a, b) for a, b in zip(self.params(), other.params()))

    def isequal(self, other) -> bool:
        return type(self) is type(other) and all(_isequal(a, b) for a, b in zip(self.params(), other.params()))

    def __hash__(self):
        return hash((type(self).__name__,) + tuple(_hashable(p) for p in self.params()))

    def __repr__(self):
        return f"{type(self).__name__}({', '.join(repr(p) for p in self.params())})"

    # -- device parameter cache: list of length-D (H: D x k, column-major) contiguous tensors. Julia's
    # transforms are immutable; these Python objects are not, so an entry is valid only for the
    # parameter values it was made from: reassigning a field drops the cache (__setattr__), and the
    # key carries a fingerprint of every parameter (value bytes of host arrays, the version counter
    # of tensors), so in-place changes are seen too.
    def __setattr__(self, name, value):
        if name in self.FIELDS:
            self.__dict__.pop("_dev_cache", None)
        object.__setattr__(self, name, value)

    def _cached(self, device, dtype, D: int, make):
        key = (str(device), dtype, D)
        fp = tuple(_fingerprint(p) for p in self.params())
        cache = self.__dict__.setdefault("_dev_cache", {})
        hit = cache.get(key)
        if hit is None or hit[0] != fp:
            hit = (fp, make())
            cache[key] = hit
        return hit[1]

    def _device_params(self, device, dtype, D: int):
        return self._cached(device, dtype, D, lambda: [_param_to_device(p, device, dtype, D, name) for p, name in
                                                       zip(self.params(), self.FIELDS)])

    def _k(self) -> int:
        return 0

    def _check_ladj_signature(self, is_vector_input: bool) -> None:
        """Raise MethodError where the reference defines no with_logabsdet_jacobian method."""


def _fingerprint(p):
    """Identity + content version of a parameter for the device cache key."""
    if isinstance(p, torch.Tensor):
        return ("t", id(p), p.data_ptr(), p._version, p.dtype, tuple(p.shape))
    if isinstance(p, np.ndarray):
        return ("a", p.dtype.str, p.shape, p.tobytes())
    if isinstance(p, (list, tuple)):
        return ("l", tuple(_fingerprint(q) for q in p))
    return ("s", type(p).__name__, p)


def _param_to_device(p, device, dtype, D, name):
    if isinstance(p, torch.Tensor):
        t = p.detach().to(device=device, dtype=dtype)
    else:
        t = torch.as_tensor(np.asarray(p, dtype=np.float64 if dtype == torch.float64 else np.float32),
                            device=device)
    if t.ndim == 0:
        t = t.reshape(1).expand(D)
    elif t.ndim == 1:
        if t.shape[0] == 1 and D != 1:
            t = t.expand(D)
        elif t.shape[0] != D:
            raise DimensionMismatch(f"parameter {name} has length {t.shape[0]}, data has {D} rows")
    else:
        raise DimensionMismatch(f"parameter {name} must be a scalar or a vector")
    return t.contiguous()


class ComposedFunction:
    """Base.ComposedFunction(outer, inner): (outer ∘ inner)(x) = outer(inner(x))."""

    def __init__(self, outer, inner):
        self.outer, self.inner = outer, inner

    def __call__(self, X):
        return _apply(self, X, want_ladj=False)[0]

    def __matmul__(self, other):
        return ComposedFunction(self, other)

    def __eq__(self, other):
        return isinstance(other, ComposedFunction) and self.outer == other.outer and self.inner == other.inner

    def __hash__(self):
        return hash(("ComposedFunction", hash(self.outer), hash(self.inner)))

    def __repr__(self):
        return f"({self.outer!r} ∘ {self.inner!r})"


def compose(*fs):
    """compose(f, g, h) == f ∘ g ∘ h (h applied first)."""
    if not fs:
        raise ValueError("compose needs at least one function")
    out = fs[-1]
    for f in reversed(fs[:-1]):
        out = ComposedFunction(f, out)
    return out


# ----------------------------------------------------------------------------- the transforms
class ScaleShiftTrafo(Trafo):
    """y = muladd(x, a, b); ladj = sum(log.(abs.(a))) (src/scale_shift_trafo.jl:4-30)."""
    OP = _lib.OP_SCALESHIFT
    FIELDS = ("a", "b")

    def __init__(self, a, b):
        self.a, self.b = a, b

    def inverse(self):
        a = _as_param_array(self.a)
        ainv = 1 / a
        return ScaleShiftTrafo(_restore_type(self.a, ainv), _restore_type(self.b, -ainv * _as_param_array(self.b)))

    def _k(self) -> int:
        # enf_layer.k = 1: `a` is a length-1 vector (expanded to the D rows on the device) whose ladj
        # constant sum(log.(abs.(a))) counts its single entry once (src/scale_shift_trafo.jl:22)
        return 1 if _is_vector(self.a) and np.size(_as_cpu_array(self.a)) == 1 else 0

    def _check_ladj_signature(self, is_vector_input):
        # with_logabsdet_jacobian is defined only for vector a and matrix x (scale_shift_trafo.jl:18-21)
        if not _is_vector(self.a) or is_vector_input:
            raise MethodError("with_logabsdet_jacobian(::ScaleShiftTrafo, x) is defined only for vector "
                              "parameters and a matrix x (src/scale_shift_trafo.jl:18-21)")


class CenterStretch(Trafo):
    """src/center_stretch.jl:25-45; ladj from the output: -sum(center_contract_ladj.(y))."""
    OP = _lib.OP_CENTER_STRETCH
    FIELDS = ("a", "b", "c")

    def __init__(self, a=0.0, b=1.0, c=0.0):
        self.a, self.b, self.c = a, b, c

    def inverse(self):
        return CenterContract(self.a, self.b, self.c)


class CenterContract(Trafo):
    """src/center_stretch.jl:49-69; ladj = sum(center_contract_ladj.(x))."""
    OP = _lib.OP_CENTER_CONTRACT
    FIELDS = ("a", "b", "c")

    def __init__(self, a=0.0, b=1.0, c=0.0):
        self.a, self.b, self.c = a, b, c

    def inverse(self):
        return CenterStretch(self.a, self.b, self.c)


class JohnsonTrafo(Trafo):
    """y = gamma + delta*asinh((x - xi)/lambda) (src/johnson_trafo.jl:29-32,61-82)."""
    OP = _lib.OP_JOHNSON
    FIELDS = ("gamma", "delta", "xi", "lambda_")

    def __init__(self, gamma=10.0, delta=3.5, xi=10.0, lambda_=1.0):
        self.gamma, self.delta, self.xi, self.lambda_ = gamma, delta, xi, lambda_

    def inverse(self):
        return JohnsonTrafoInv(self.gamma, self.delta, self.xi, self.lambda_)


class JohnsonTrafoInv(Trafo):
    """x = lambda*sinh((y - gamma)/delta) + xi; ladj from the output (src/johnson_trafo.jl:86-107)."""
    OP = _lib.OP_JOHNSON_INV
    FIELDS = ("gamma", "delta", "xi", "lambda_")

    def __init__(self, gamma=10.0, delta=3.5, xi=10.0, lambda_=1.0):
        self.gamma, self.delta, self.xi, self.lambda_ = gamma, delta, xi, lambda_

    def inverse(self):
        return JohnsonTrafo(self.gamma, self.delta, self.xi, self.lambda_)


class HouseholderTrafo(Trafo):
    """Chained reflections over the columns of V (src/householder_trafo.jl:127-160); ladj = 0."""
    OP = _lib.OP_HOUSEHOLDER
    FIELDS = ("V",)

    def __init__(self, V):
        if isinstance(V, (numbers.Real,)):
            raise MethodError("HouseholderTrafo needs a vector or a matrix V")
        self.V = V

    def _Vmat_shape(self):
        A = _as_cpu_array(self.V)
        return A.shape

    def _k(self) -> int:
        s = self._Vmat_shape()
        return 1 if len(s) == 1 else s[1]

    def inverse(self):
        # vector: itself (:153); matrix: reversed column order (:154)
        if len(self._Vmat_shape()) == 1:
            return self
        V = self.V
        if isinstance(V, torch.Tensor):
            return HouseholderTrafo(torch.flip(V, dims=(1,)))
        return HouseholderTrafo(np.ascontiguousarray(np.asarray(V)[:, ::-1]))

    def _device_params(self, device, dtype, D):
        def make():
            V = self.V
            t = V.detach().to(device=device, dtype=dtype) if isinstance(V, torch.Tensor) else \
                torch.as_tensor(np.asarray(V, dtype=np.float64 if dtype == torch.float64 else np.float32),
                                device=device)
            if t.ndim == 1:
                t = t.reshape(-1, 1)
            if t.ndim != 2 or t.shape[0] != D:
                raise DimensionMismatch(f"HouseholderTrafo V has {t.shape[0]} rows, data has {D}")
            return [t.t().contiguous()]  # column-major D x k == row-major k x D
        return self._cached(device, dtype, D, make)


def _as_param_array(p):
    if isinstance(p, torch.Tensor):
        return p
    if isinstance(p, (list, tuple)):
        return np.asarray(p, dtype=np.float64 if _kind(p) != torch.float32 else np.float32)
    if isinstance(p, numbers.Integral):
        return float(p)
    return p


def _restore_type(orig, val):
    if isinstance(orig, (list, tuple)):
        return np.asarray(val)
    return val


def inverse(f):
    """InverseFunctions.inverse: leaf algebra, and inverse(f ∘ g) = inverse(g) ∘ inverse(f)."""
    if isinstance(f, ComposedFunction):
        return ComposedFunction(inverse(f.inner), inverse(f.outer))
    if isinstance(f, Trafo):
        return f.inverse()
    raise MethodError(f"no inverse for {type(f)}")


def leaves(f) -> List[Trafo]:
    """The transforms of a composition in application order (innermost first)."""
    if isinstance(f, ComposedFunction):
        return leaves(f.inner) + leaves(f.outer)
    if isinstance(f, Trafo):
        return [f]
    raise MethodError(f"{type(f)} is not a transform of this package")


# ----------------------------------------------------------------------------- execution
def _to_matrix(X):
    """-> ((D, N) tensor where X lives -- CUDA or host --, restore info, is_vector)."""
    orig_np = isinstance(X, np.ndarray)
    if orig_np:
        Xt = torch.from_numpy(np.asarray(X))
    elif isinstance(X, torch.Tensor):
        Xt = X
    else:
        raise TypeError(f"unsupported input type {type(X)}")
    is_vec = Xt.ndim == 1
    if Xt.ndim not in (1, 2):
        raise DimensionMismatch("input must be a vector (D,) or a matrix (D, N)")
    M = Xt.reshape(-1, 1) if is_vec else Xt
    return M, (orig_np, Xt.is_cuda, X.device if isinstance(X, torch.Tensor) else None), is_vec


def _to_device_matrix(X):
    """-> (column-major (D, N) CUDA tensor, restore(Y, ladj) callable, is_vector). The training and VJP
    entry points run on the GPU only: host data is copied to the current GPU."""
    orig_np = isinstance(X, np.ndarray)
    if orig_np:
        Xt = torch.from_numpy(np.asarray(X))
    elif isinstance(X, torch.Tensor):
        Xt = X
    elif isinstance(X, numbers.Real):
        raise MethodError("scalar inputs are not supported by the batched path; use a length-1 vector")
    else:
        raise TypeError(f"unsupported input type {type(X)}")
    on_gpu = Xt.is_cuda
    is_vec = Xt.ndim == 1
    if Xt.ndim not in (1, 2):
        raise DimensionMismatch("input must be a vector (D,) or a matrix (D, N)")
    if not on_gpu:
        if not torch.cuda.is_available():
            raise RuntimeError("this entry point runs on a ROCm GPU only (torch.cuda.is_available() is False)")
        Xt = Xt.to("cuda")
    M = Xt.reshape(-1, 1) if is_vec else Xt
    return M, (orig_np, on_gpu, X.device if isinstance(X, torch.Tensor) else None), is_vec


def _colmajor(M: torch.Tensor, dtype) -> torch.Tensor:
    D, N = M.shape
    if M.dtype == dtype and (M.stride(0) == 1 or D == 1) and (M.stride(1) == D or N == 1):
        return M
    out = torch.empty((N, D), dtype=dtype, device=M.device).t()
    out.copy_(M)
    return out


def _new_colmajor(D, N, dtype, device):
    return torch.empty((N, D), dtype=dtype, device=device).t()


def _ld(M: torch.Tensor) -> int:
    D, N = M.shape
    return M.stride(1) if N > 1 else max(D, 1)


def _run_segment(trafos, M, dtype, ladj, accumulate):
    """One enf_flow_apply (device data) or enf_flow_apply_cpu (host data) over consecutive transforms
    of one promoted dtype."""
    D, N = M.shape
    dev = M.device
    Y = _new_colmajor(D, N, dtype, dev)
    if not M.is_cuda:
        keep = []
        arr = (_lib.Layer * max(1, len(trafos)))()
        for i, t in enumerate(trafos):
            ps = t._device_params(dev, dtype, D)
            keep.extend(ps)
            arr[i].op = t.OP
            arr[i].k = t._k()
            for q, p in enumerate(ps):
                arr[i].p[q] = p.data_ptr()
        _lib.check(_lib.lib().enf_flow_apply_cpu(
            _lib.ENF_F64 if dtype == torch.float64 else _lib.ENF_F32, D, N, M.data_ptr(), _ld(M), Y.data_ptr(),
            _ld(Y), ladj.data_ptr() if ladj is not None else None, 1 if accumulate else 0, arr, len(trafos), 0))
        del keep
        return Y
    keep = []
    arr = (_lib.Layer * max(1, len(trafos)))()
    for i, t in enumerate(trafos):
        ps = t._device_params(dev, dtype, D)
        keep.extend(ps)
        arr[i].op = t.OP
        arr[i].k = t._k()
        for q, p in enumerate(ps):
            arr[i].p[q] = p.data_ptr()
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(_lib.lib().enf_flow_apply(
            _lib.ENF_F64 if dtype == torch.float64 else _lib.ENF_F32, D, N, M.data_ptr(), _ld(M),
            Y.data_ptr(), _ld(Y), ladj.data_ptr() if ladj is not None else None, 1 if accumulate else 0,
            arr, len(trafos), stream))
    del keep
    return Y


def _apply_scalar(f, x, want_ladj: bool):
    """A scalar x (Julia's x::Real methods): a 1 x 1 batch when every parameter is a scalar, else x
    broadcast to the length-D vector of the parameters (D from the vector parameters)."""
    ts = leaves(f)
    for t in ts:
        if isinstance(t, HouseholderTrafo):
            raise MethodError("HouseholderTrafo is defined for vectors and matrices only (src/householder_trafo.jl:156-160)")
    lens = {np.size(_as_cpu_array(p)) for t in ts for p in t.params() if _is_vector(p)}
    lens.discard(1)
    if len(lens) > 1:
        raise DimensionMismatch(f"parameter vectors of lengths {sorted(lens)}")
    kx = _kind(x)
    dt = _promote(kx, *[_kind(p) for t in ts for p in t.params()])
    np_dt = np.float64 if dt == torch.float64 else np.float32
    if not lens and not any(_is_vector(p) for t in ts for p in t.params()):
        if want_ladj:
            for t in ts:
                t._check_ladj_signature(True)
        Y, L = _apply(f, np.full((1, 1), x, dtype=np_dt), want_ladj)
        y = np_dt(Y[0, 0]).item() if np_dt is np.float64 else np_dt(Y[0, 0])
        if not want_ladj:
            return y, None
        return y, (np_dt(L[0, 0]).item() if np_dt is np.float64 else np_dt(L[0, 0]))
    D = lens.pop() if lens else 1
    return _apply(f, np.full(D, x, dtype=np_dt), want_ladj)


def _apply_host_numpy(ts, X: np.ndarray, want_ladj: bool):
    """Host fast path (config 1: a numpy (D, N) batch): one enf_flow_apply_cpu call on numpy buffers, no
    torch tensors for X / Y / ladj. None when it does not apply (several promoted dtype runs, a vector
    input, an empty flow); the general path then handles the call with identical results."""
    if X.ndim != 2 or not ts or X.dtype not in (np.float32, np.float64):
        return None
    dt = _promote(_kind(X), *[_kind(p) for t in ts for p in t.params()])
    npdt = np.float64 if dt == torch.float64 else np.float32
    if X.dtype != npdt:
        return None  # a promotion run: the general path converts
    D, N = X.shape
    if want_ladj:
        for t in ts:
            t._check_ladj_signature(False)
    M = X if (X.flags.f_contiguous or N == 1 or D == 1) else np.asfortranarray(X)
    ldx = max(D, 1) if N <= 1 else M.strides[1] // M.itemsize
    if N > 1 and D > 1 and M.strides[0] != M.itemsize:
        M, ldx = np.asfortranarray(M), D
    Y = np.empty((D, N), dtype=npdt, order="F")
    L = np.empty((1, N), dtype=npdt) if want_ladj else None
    cpu = torch.device("cpu")
    arr = (_lib.Layer * len(ts))()
    keep = []
    for i, t in enumerate(ts):
        ps = t._device_params(cpu, dt, D)
        keep.extend(ps)
        arr[i].op = t.OP
        arr[i].k = t._k()
        for q, pt in enumerate(ps):
            arr[i].p[q] = pt.data_ptr()
    _lib.check(_lib.lib().enf_flow_apply_cpu(
        _lib.ENF_F64 if dt == torch.float64 else _lib.ENF_F32, D, N, M.ctypes.data, ldx, Y.ctypes.data, max(D, 1),
        L.ctypes.data if L is not None else None, 0, arr, len(ts), 0))
    del keep
    return Y, L


def _apply(f, X, want_ladj: bool):
    if isinstance(X, (numbers.Real, np.generic)) and not isinstance(X, bool) or \
            (isinstance(X, np.ndarray) and X.ndim == 0):
        return _apply_scalar(f, X.item() if isinstance(X, np.ndarray) else X, want_ladj)
    ts = leaves(f)
    if isinstance(X, np.ndarray):
        r = _apply_host_numpy(ts, X, want_ladj)
        if r is not None:
            return r
    M, restore, is_vec = _to_matrix(X)
    if want_ladj:
        for t in ts:
            t._check_ladj_signature(is_vec)
    D, N = M.shape
    # segments of equal running promoted type (Julia promotes layer by layer)
    segs = []
    cur = _kind(M)
    for t in ts:
        rd = _promote(cur, *[_kind(p) for p in t.params()])
        if segs and segs[-1][0] == rd:
            segs[-1][1].append(t)
        else:
            segs.append((rd, [t]))
        cur = rd
    if not segs:
        segs = [(_promote(cur), [])]
    ladj = None
    for i, (dt, group) in enumerate(segs):
        M = _colmajor(M, dt)
        seg_ladj = None
        if want_ladj:
            if ladj is None or ladj.dtype != dt:
                seg_ladj = torch.empty(N, dtype=dt, device=M.device)
                acc = False
            else:
                seg_ladj, acc = ladj, True
        else:
            acc = False
        M = _run_segment(group, M, dt, seg_ladj, acc)
        if want_ladj:
            ladj = seg_ladj if (ladj is None or seg_ladj is ladj) else ladj.to(dt) + seg_ladj
    Y = M
    orig_np, on_gpu, odev = restore
    if is_vec:
        Y = Y.reshape(-1)
        L = ladj.reshape(()) if ladj is not None else None
    else:
        L = ladj.reshape(1, N) if ladj is not None else None
    if not on_gpu:
        Y = Y.cpu()
        L = L.cpu() if L is not None else None
        if orig_np:
            Y = Y.numpy()
            L = L.numpy() if L is not None else None
    return Y, L


def with_logabsdet_jacobian(f, X):
    """ChangesOfVariables.with_logabsdet_jacobian(f, X) -> (Y, ladj), one fused launch per dtype run."""
    return _apply(f, X, want_ladj=True)


def stream_with_logabsdet_jacobian(f, X: np.ndarray, chunk_cols: int = 0, out=None, want_ladj: bool = True,
                                   device=None):
    """with_logabsdet_jacobian for a HOST-resident batch larger than (or not wanted in) device memory
    (SURVEY.md §8(f) item 2): X is a column-major (D, N) numpy array (np.asfortranarray; sample j =
    the contiguous column X[:, j], Julia's flatview layout); column chunks stream through the device
    (enf_flow_apply_host: copy-in, fused flow and copy-out overlap). Returns (Y, ladj) as numpy
    arrays (ladj shape (1, N)); ``out`` may be X itself for an in-place transform. The flow's
    parameters must share X's dtype (no mixed-precision promotion on this path)."""
    X = np.asarray(X)
    if X.ndim != 2 or not X.flags.f_contiguous:
        raise DimensionMismatch("stream_with_logabsdet_jacobian needs a column-major (D, N) array")
    dt = torch.float64 if X.dtype == np.float64 else torch.float32 if X.dtype == np.float32 else None
    if dt is None:
        raise MethodError("X must be float32 or float64")
    ts = leaves(f)
    if want_ladj:
        for t in ts:
            t._check_ladj_signature(False)
    if _promote(dt, *[_kind(p) for t in ts for p in t.params()]) != dt:
        raise MethodError("stream_with_logabsdet_jacobian: parameters would promote X's dtype")
    if not torch.cuda.is_available():
        raise RuntimeError("stream_with_logabsdet_jacobian streams through a ROCm GPU (torch.cuda.is_available() is False)")
    D, N = X.shape
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    Y = np.empty_like(X, order="F") if out is None else out
    if Y.shape != X.shape or Y.dtype != X.dtype or not Y.flags.f_contiguous:
        raise DimensionMismatch("out must be a column-major array like X")
    L = np.empty((1, N), dtype=X.dtype) if want_ladj else None
    keep = []
    arr = (_lib.Layer * max(1, len(ts)))()
    for i, t in enumerate(ts):
        ps = t._device_params(dev, dt, D)
        keep.extend(ps)
        arr[i].op = t.OP
        arr[i].k = t._k()
        for q, p in enumerate(ps):
            arr[i].p[q] = p.data_ptr()
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(_lib.lib().enf_flow_apply_host(
            _lib.ENF_F64 if dt == torch.float64 else _lib.ENF_F32, D, N, X.ctypes.data, D, Y.ctypes.data, D,
            L.ctypes.data if L is not None else None, 0, arr, len(ts), int(chunk_cols), stream))
    del keep
    return Y, L
