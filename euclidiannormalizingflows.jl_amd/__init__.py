"""MI355X-native (gfx950) batched bijector path of bat/EuclidianNormalizingFlows.jl.

Python host mirror of the reference's transform API (the reference host language, Julia, is not
installed in this image; the Julia ccall shim that binds the same C ABI is julia/ENFHip.jl).
All compute goes through libenf.so (include/enf.h): hand-written HIP kernels for gfx950.
"""
from ._lib import EnfError, version  # noqa: F401
from .comm import EnfComm  # noqa: F401
from .distributions import JohnsonSU  # noqa: F401
from .trafos import (  # noqa: F401
    CenterContract,
    CenterStretch,
    ComposedFunction,
    DimensionMismatch,
    HouseholderTrafo,
    JohnsonTrafo,
    JohnsonTrafoInv,
    MethodError,
    ScaleShiftTrafo,
    Trafo,
    compose,
    inverse,
    leaves,
    stream_with_logabsdet_jacobian,
    with_logabsdet_jacobian,
)

from .train import (  # noqa: F401
    ADAGrad,
    FlowState,
    WhiteningResult,
    allreduce_sum_,
    flow_vjp,
    minibatch_plan,
    mvnormal_negll_trafo,
    mvnormal_negll_trafograd,
    optimize_whitening,
)

__all__ = [
    "ADAGrad", "FlowState", "WhiteningResult", "allreduce_sum_", "flow_vjp", "minibatch_plan", "mvnormal_negll_trafo", "mvnormal_negll_trafograd",
    "optimize_whitening",
    "ScaleShiftTrafo", "CenterStretch", "CenterContract", "JohnsonTrafo", "JohnsonTrafoInv",
    "HouseholderTrafo", "ComposedFunction", "compose", "inverse", "stream_with_logabsdet_jacobian", "with_logabsdet_jacobian",
    "leaves", "Trafo", "MethodError", "DimensionMismatch", "EnfError", "version", "JohnsonSU", "EnfComm",
]
