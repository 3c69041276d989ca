"""CPU: libenf's host execution path (enf_flow_apply_cpu) -- SURVEY.md §8 config 1 ("ScaleShiftTrafo
D=1, N=1e3 fp64 on CPU, no GPU"). Host data (numpy arrays, CPU tensors, scalars) runs there; this file
needs no GPU. Checked like the GPU path: against the committed exact golden vectors and the oracle,
plus what only this path promises -- the reference's evaluation order (bit-identical elementwise maps,
the ∘-tree ladj association), scalar x::Real calls, thread-count independence."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden_flow
from parity import assert_as_accurate, check_vs_oracle, make_flow, rand_params

FLOW_FIXTURES = sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, "*.npz"))
                       if "scalars" not in f and "johnsonsu" not in f)


@pytest.mark.parametrize("name", FLOW_FIXTURES)
def test_golden_flow_cpu(enf, oracle, name):
    layers, X, Yx, Lx = load_golden_flow(name)
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), np.asfortranarray(X))
    assert isinstance(Y, np.ndarray) and Y.dtype == X.dtype
    Yt, Lt = oracle.flow_apply(layers, X)
    assert_as_accurate(Y, L, Yt, Lt, Yx, Lx, X.dtype, what=name)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("op", range(6))
@pytest.mark.parametrize("D", [1, 2, 5, 32])
def test_single_op_cpu_vs_oracle(enf, oracle, dtype, op, D):
    rng = np.random.default_rng(500 * op + D)
    layers = [(op, rand_params(rng, op, D, dtype, K=3 if op == 5 else 1))]
    X = rng.standard_normal((D, 1031)).astype(dtype)
    if op == 2:
        X *= 3
    X = np.asfortranarray(X)
    f = make_flow(enf, layers)
    Y, L = enf.with_logabsdet_jacobian(f, X)
    check_vs_oracle(oracle, layers, X, Y, L, dtype, what=f"cpu op{op} D{D}")
    if op != 5:  # the elementwise maps evaluate the reference's formulas in the same order: identical
        Yr, Lr = oracle.flow_apply(layers, X)
        assert np.array_equal(Y, Yr)
    assert np.array_equal(f(X), Y)


def test_config1_scaleshift_D1_fp64(enf):
    """Config 1 itself: y = muladd(x, a, b), ladj = log|a| in every column (scale_shift_trafo.jl:16-24)."""
    rng = np.random.default_rng(1)
    X = rng.standard_normal((1, 1000))
    a, b = np.array([-1.7]), np.array([0.25])
    Y, L = enf.with_logabsdet_jacobian(enf.ScaleShiftTrafo(a, b), X)
    assert Y.shape == (1, 1000) and L.shape == (1, 1000)
    # muladd (fma): within one rounding of the exact x*a + b
    assert np.all(np.abs(Y[0] - (X[0] * a[0] + b[0])) <= 2.0 ** -52 * (np.abs(X[0] * a[0]) + abs(b[0])))
    assert np.all(L == np.log(np.abs(a[0])))
    X2, L2 = enf.with_logabsdet_jacobian(enf.inverse(enf.ScaleShiftTrafo(a, b)), Y)
    assert np.allclose(X2, X, rtol=1e-15, atol=1e-15) and np.allclose(L2, -L, rtol=1e-15)


def test_composition_ladj_follows_the_compose_tree(enf):
    """f4 ∘ f3 ∘ f2 ∘ f1 (Julia's left-associated ∘): ChangesOfVariables adds inner + outer at every
    node, i.e. l1 + (l2 + (l3 + l4)) -- the CPU path reproduces that association bit for bit."""
    rng = np.random.default_rng(3)
    D, N = 6, 777
    layers = [(3, rand_params(rng, 3, D, np.float64)), (1, rand_params(rng, 1, D, np.float64)),
              (4, rand_params(rng, 4, D, np.float64)), (2, rand_params(rng, 2, D, np.float64))]
    X = np.asfortranarray(rng.standard_normal((D, N)))
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), X)
    ls, Z = [], X
    for op, ps in layers:
        Z, l = enf.with_logabsdet_jacobian(make_flow(enf, [(op, ps)]), Z)
        ls.append(l[0])
    assert np.array_equal(Z, Y)
    tree = ls[0] + (ls[1] + (ls[2] + ls[3]))
    assert np.array_equal(L[0], tree)
    left = ((ls[0] + ls[1]) + ls[2]) + ls[3]  # the GPU kernels' order: equal within rounding
    assert np.allclose(L[0], left, rtol=1e-14, atol=1e-14)


def _capi_apply(enf, X, layers_np, nthreads, Y=None, ladj=None, acc=0):
    lib = enf._lib
    D, N = X.shape
    arr = (lib.Layer * len(layers_np))()
    keep = []
    for i, (op, ps) in enumerate(layers_np):
        arr[i].op, arr[i].k = op, (np.asarray(ps[0]).reshape(D, -1).shape[1] if op == 5 else 0)
        for q, p in enumerate(ps):
            a = np.asfortranarray(np.broadcast_to(np.asarray(p, X.dtype), (D,)) if op != 5 else np.asarray(p, X.dtype))
            keep.append(a)
            arr[i].p[q] = a.ctypes.data
    Y = np.empty_like(X, order="F") if Y is None else Y
    ladj = np.zeros(N, X.dtype) if ladj is None else ladj
    dt = lib.ENF_F64 if X.dtype == np.float64 else lib.ENF_F32
    rc = lib.lib().enf_flow_apply_cpu(dt, D, N, X.ctypes.data, D, Y.ctypes.data, D, ladj.ctypes.data, acc, arr,
                                      len(layers_np), nthreads)
    return rc, Y, ladj


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_threads_inplace_accumulate(enf, dtype):
    """The result does not depend on the thread count (blocks are independent); X == Y in place and
    accumulate_ladj behave as enf_flow_apply's."""
    from test_gpu_train import mixed_layers

    rng = np.random.default_rng(4)
    D, N = 7, 10_007
    layers = mixed_layers(rng, D, dtype)
    X = np.asfortranarray(rng.standard_normal((D, N)).astype(dtype))
    rc1, Y1, L1 = _capi_apply(enf, X, layers, 1)
    rc0, Y0, L0 = _capi_apply(enf, X, layers, 0)
    assert rc1 == 0 and rc0 == 0
    assert np.array_equal(Y1, Y0) and np.array_equal(L1, L0)
    Xi = X.copy(order="F")
    base = np.full(N, 0.5, dtype)
    rc, Yi, Li = _capi_apply(enf, Xi, layers, 3, Y=Xi, ladj=base.copy(), acc=1)
    assert rc == 0 and Yi is Xi and np.array_equal(Xi, Y1)
    assert np.array_equal(Li, (base + L1).astype(dtype))


def test_scalar_calls(enf, oracle):
    """x::Real methods (johnson_trafo.jl:74-80, center_stretch.jl:37-43, scale_shift_trafo.jl:15):
    scalar parameters -> scalar y and ladj; vector parameters -> x broadcast (vector y, summed ladj)."""
    f = enf.JohnsonTrafo(4.0, 3.0, 2.0, 1.0)
    y, l = enf.with_logabsdet_jacobian(f, 0.5)
    assert isinstance(y, float) and isinstance(l, float)
    assert y == oracle.scalar("johnsontrafo", np.float64, 0.5, 4.0, 3.0, 2.0, 1.0)
    assert l == oracle.scalar("johnsontrafo_ladj", np.float64, 0.5, 4.0, 3.0, 2.0, 1.0)
    assert f(0.5) == y
    # integer x and parameters compute in Float64 (float(promote_type), johnson_trafo.jl:30)
    assert enf.JohnsonTrafo(1, 3, -4, 1)(0) == oracle.scalar("johnsontrafo", np.float64, 0.0, 1.0, 3.0, -4.0, 1.0)
    # Float32 x and Float32 parameters stay Float32
    y32 = enf.JohnsonTrafoInv(np.float32(1), np.float32(3), np.float32(-4), np.float32(0.5))(np.float32(0.3))
    assert isinstance(y32, np.float32)
    # vector parameters: broadcast of the scalar (test_johnson_trafo.jl:40-48 with x = fill(0.5, 2))
    fv = enf.JohnsonTrafo([4.0, 4.1], [3.0, 3.1], [2.0, 2.1], [1.0, 1.1])
    yv, lv = enf.with_logabsdet_jacobian(fv, 0.5)
    yw, lw = enf.with_logabsdet_jacobian(fv, np.array([0.5, 0.5]))
    assert np.array_equal(yv, yw) and lv == lw and yv.shape == (2,)
    # composition of scalar transforms
    g = enf.CenterContract(0.3, 1.5, 0.1) @ enf.CenterStretch(0.3, 1.5, 0.1)
    yg, lg = enf.with_logabsdet_jacobian(g, 0.7)
    assert abs(yg - 0.7) < 1e-14 and abs(lg) < 1e-14
    assert enf.ScaleShiftTrafo(2.0, 1.0)(3.0) == 7.0
    with pytest.raises(enf.MethodError):  # with_logabsdet_jacobian(::ScaleShiftTrafo, ::Real) is undefined
        enf.with_logabsdet_jacobian(enf.ScaleShiftTrafo(2.0, 1.0), 3.0)
    with pytest.raises(enf.MethodError):  # HouseholderTrafo takes vectors and matrices only
        enf.HouseholderTrafo(np.ones(3))(1.0)


def test_host_data_needs_no_gpu(enf, monkeypatch):
    """Config 1 "no GPU": host data never asks for a device (torch.cuda reporting no GPU changes
    nothing), and the result is the same."""
    import torch

    rng = np.random.default_rng(5)
    X = np.asfortranarray(rng.standard_normal((3, 100)))
    f = enf.JohnsonTrafo(rng.uniform(-1, 1, 3), rng.uniform(0.5, 2, 3), rng.uniform(-0.5, 0.5, 3), rng.uniform(0.5, 2, 3))
    Y, L = enf.with_logabsdet_jacobian(f, X)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    Y2, L2 = enf.with_logabsdet_jacobian(f, X)
    Yt, Lt = enf.with_logabsdet_jacobian(f, torch.from_numpy(X))
    assert np.array_equal(Y, Y2) and np.array_equal(L, L2)
    assert isinstance(Yt, torch.Tensor) and not Yt.is_cuda and np.array_equal(Yt.numpy(), Y)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_scaleshift_length1_a_ladj_counts_once(enf, dtype):
    """ScaleShiftTrafo([a], [b]) on D = 4 rows: ladj = sum(log.(abs.(f.a))) over a's own length, i.e.
    log|a| once per sample (src/scale_shift_trafo.jl:22; enf_layer.k = 1), not D log|a|; a length-D a
    keeps the sum over its D entries. Values computed by hand."""
    rng = np.random.default_rng(4)
    X = np.asfortranarray(rng.standard_normal((4, 7)).astype(dtype))
    f1 = enf.ScaleShiftTrafo(np.array([-2.5], dtype), np.array([0.25], dtype))
    Y, L = enf.with_logabsdet_jacobian(f1, X)
    assert np.allclose(Y, -2.5 * X.astype(np.float64) + 0.25, rtol=1e-6, atol=1e-6)
    assert np.allclose(np.asarray(L).reshape(-1), np.log(2.5), rtol=1e-6)
    a = np.array([0.5, -2.0, 3.0, 1.5], dtype)
    fD = enf.ScaleShiftTrafo(a, np.zeros(4, dtype))
    _, LD = enf.with_logabsdet_jacobian(fD, X)
    assert np.allclose(np.asarray(LD).reshape(-1), np.log(np.abs(a.astype(np.float64))).sum(), rtol=1e-6)
    assert f1._k() == 1 and fD._k() == 0


def test_capi_scaleshift_k_validated(enf):
    """enf_layer.k of a ScaleShift layer is 0 (length-D a) or 1 (length-1 a); anything else is refused."""
    lib = enf._lib
    a = np.array([2.0, 2.0]); b = np.zeros(2)
    X = np.zeros((3, 2)); Y = np.zeros((3, 2)); L = np.zeros(3)
    arr = (lib.Layer * 1)()
    arr[0].op, arr[0].p[0], arr[0].p[1] = lib.OP_SCALESHIFT, a.ctypes.data, b.ctypes.data
    for k, want in ((0, lib.ENF_OK), (1, lib.ENF_OK), (2, lib.ENF_ERR_INVALID), (-1, lib.ENF_ERR_INVALID)):
        arr[0].k = k
        rc = lib.lib().enf_flow_apply_cpu(lib.ENF_F64, 2, 3, X.ctypes.data, 2, Y.ctypes.data, 2, L.ctypes.data, 0,
                                          arr, 1, 1)
        assert rc == want, (k, rc)
        if rc == lib.ENF_OK:
            assert np.allclose(L, np.log(2.0) * (1 if k == 1 else 2))
