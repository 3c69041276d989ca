"""JohnsonSU distribution (src/johnson_trafo.jl:1-26,111-129) with the elementwise functions and
the sampler on the device (libenf.so: enf_johnsonsu_eval / enf_johnsonsu_sample, include/enf.h).

Mirrors the reference's Distributions.jl interface: ``pdf``, ``logpdf``, ``cdf``, ``logcdf``,
``ccdf``, ``logccdf``, ``quantile`` (elementwise over a tensor, Julia's broadcast ``pdf.(d, X)``),
``rand`` (the reference's rand(d, n) is Distributions' inverse-CDF fallback, quantile(d, rand())),
and the host-side statistics ``mean``, ``median``, ``var``, ``location`` (= mean) and ``scale``
(= var: the reference's definition, src/johnson_trafo.jl:21-22). Type promotion follows Julia's:
the result type is float(promote_type(eltype(x), partype(d))) (johnson_trafo.jl:30).
"""
from __future__ import annotations

import math

import numpy as np

from . import _lib
from .trafos import MethodError

_FNS = {"pdf": 0, "logpdf": 1, "cdf": 2, "logcdf": 3, "ccdf": 4, "logccdf": 5, "quantile": 6}


def _partype(vals):
    """Julia's promote() of the four parameters: Float32 only if every one is a float32."""
    return np.float32 if all(isinstance(v, (np.float32,)) or (isinstance(v, np.ndarray) and v.dtype == np.float32)
                             for v in vals) else np.float64


class JohnsonSU:
    """JohnsonSU(gamma, delta, xi, lambda); keyword defaults gamma=10, delta=3.5, xi=10, lambda=1
    (johnson_trafo.jl:9-12)."""

    def __init__(self, gamma=10.0, delta=3.5, xi=10.0, lambda_=1.0):
        vals = (gamma, delta, xi, lambda_)
        for v in vals:
            if not np.isscalar(v) and not (isinstance(v, np.ndarray) and v.ndim == 0):
                raise MethodError("JohnsonSU parameters are Real scalars (src/johnson_trafo.jl:1-6)")
        self.partype = _partype(vals)
        self.gamma, self.delta, self.xi, self.lambda_ = (self.partype(v) for v in vals)

    # ---- statistics (host; src/johnson_trafo.jl:15-26)
    def params(self):
        return (self.gamma, self.delta, self.xi, self.lambda_)

    def minimum(self):
        return -math.inf

    def maximum(self):
        return math.inf

    def mean(self):
        g, d, xi, l = (float(v) for v in self.params())
        return self.partype(xi - l * math.exp(d ** -2 / 2) * math.sinh(g / d))

    def median(self):
        g, d, xi, l = (float(v) for v in self.params())
        return self.partype(xi + l * math.sinh(-g / d))

    def var(self):
        g, d, xi, l = (float(v) for v in self.params())
        return self.partype(l ** 2 / 2 * (math.exp(d ** -2) - 1) * (math.exp(d ** -2) * math.cosh(2 * g / d) + 1))

    def location(self):
        return self.mean()

    def scale(self):
        return self.var()  # the reference defines scale(d) = var(d) (johnson_trafo.jl:22)

    # ---- elementwise functions (device)
    def _eval(self, fn: str, x):
        import torch

        scalar = not isinstance(x, (torch.Tensor, np.ndarray))
        if isinstance(x, torch.Tensor):
            if not x.is_cuda:
                raise MethodError("JohnsonSU functions take CUDA tensors or host arrays / scalars")
            X = x
        else:
            a = np.asarray(x)
            if a.dtype.kind not in "fiub":
                raise MethodError(f"{fn}(::JohnsonSU, x) needs real x, got {a.dtype}")
            X = torch.from_numpy(np.ascontiguousarray(a.astype(np.float64 if a.dtype.kind != "f" else a.dtype)))
            X = X.to("cuda")
        xt = np.float64 if X.dtype == torch.float64 else np.float32
        if X.dtype not in (torch.float32, torch.float64):
            X = X.to(torch.float64)
            xt = np.float64
        rt = np.promote_types(xt, self.partype)
        tdt = torch.float64 if rt == np.float64 else torch.float32
        Xc = X.to(tdt).contiguous()
        out = torch.empty_like(Xc)
        with torch.cuda.device(Xc.device):
            stream = torch.cuda.current_stream(Xc.device).cuda_stream
            _lib.check(_lib.lib().enf_johnsonsu_eval(
                _lib.ENF_F64 if tdt == torch.float64 else _lib.ENF_F32, _FNS[fn], Xc.numel(), Xc.data_ptr(),
                out.data_ptr(), float(self.gamma), float(self.delta), float(self.xi), float(self.lambda_), stream))
        if isinstance(x, torch.Tensor):
            return out
        res = out.cpu().numpy()
        return rt.type(res.reshape(())) if scalar else res

    def pdf(self, x):
        return self._eval("pdf", x)

    def logpdf(self, x):
        return self._eval("logpdf", x)

    def cdf(self, x):
        return self._eval("cdf", x)

    def logcdf(self, x):
        return self._eval("logcdf", x)

    def ccdf(self, x):
        return self._eval("ccdf", x)

    def logccdf(self, x):
        return self._eval("logccdf", x)

    def quantile(self, p):
        return self._eval("quantile", p)

    def rand(self, n: int, seed: int = 0, offset: int = 0, dtype=None, device="cuda"):
        """n draws as a CUDA tensor: quantile(u), u from Philox4x32-10 (key seed, counters from
        offset; include/enf.h enf_johnsonsu_sample). dtype defaults to partype(d)."""
        import torch

        dt = np.dtype(dtype or self.partype)
        if dt not in (np.dtype(np.float32), np.dtype(np.float64)):
            raise MethodError(f"rand(::JohnsonSU) supports float32/float64, got {dt}")
        tdt = torch.float64 if dt == np.float64 else torch.float32
        out = torch.empty(int(n), dtype=tdt, device=device)
        with torch.cuda.device(out.device):
            stream = torch.cuda.current_stream(out.device).cuda_stream
            _lib.check(_lib.lib().enf_johnsonsu_sample(
                _lib.ENF_F64 if tdt == torch.float64 else _lib.ENF_F32, int(n), out.data_ptr(), float(self.gamma),
                float(self.delta), float(self.xi), float(self.lambda_), int(seed) & (2 ** 64 - 1),
                int(offset) & (2 ** 64 - 1), stream))
        return out

    def __repr__(self):
        return f"JohnsonSU(gamma={self.gamma}, delta={self.delta}, xi={self.xi}, lambda={self.lambda_})"
