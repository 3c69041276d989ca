"""GPU tests of the round-3 capabilities:

* the gradient / VJP / whitening path at D > 64 (kernel rows up to 256 fp32 / 128 fp64; round 2 stopped
  at 64): enf_flow_negll_grad against the oracle's fp64 loss and its central differences at D = 100 and
  128, enf_flow_vjp against central differences, and an optimize_whitening epoch
  (src/optimize_whitening.jl:18-22,25-45 have no dimension bound);
* CenterStretch / CenterContract on the padded fragment path (src/center_stretch.jl:37-43,61-67 at a D
  that is a multiple of 16/sizeof(T) but not a power of two);
* ScaleShiftTrafo with a length-1 `a`: ladj = log|a| once and its gradient 1/a (src/scale_shift_trafo.jl:22,
  the sum over a's own length), values computed by hand;
* enf_flow_negll, the device reduction of mvnormal_negll_trafo (src/optimize_whitening.jl:7-15).
"""
import numpy as np
import pytest

from parity import check_vs_oracle, colmajor_cuda, loss_close, make_flow, rand_params, to_np

pytestmark = pytest.mark.gpu


def _fd_check(oracle, layers, X, g, D, idx, rel=1e-5, floor=1e-3):
    from test_gpu_train import flat, oracle_negll, unflat

    th0 = flat(layers, D)
    assert g.shape == th0.shape
    scale = np.abs(g).max()
    for i in idx:
        h = 1e-6 * max(1.0, abs(th0[i]))
        tp, tm = th0.copy(), th0.copy()
        tp[i] += h
        tm[i] -= h
        fd = (oracle_negll(oracle, unflat(layers, tp, D), X) - oracle_negll(oracle, unflat(layers, tm, D), X)) / (2 * h)
        assert abs(g[i] - fd) <= rel * (abs(fd) + floor * scale), (i, g[i], fd)


@pytest.mark.parametrize("D", [100, 128])
def test_negll_grad_large_D_finite_differences(enf, gpu, oracle, D):
    """fp64, every transform (mixed_layers: ScaleShift, chained Householder, CenterContract, Johnson,
    CenterStretch, JohnsonInv, reflection, Johnson) at D = 100 (kernel rows padded to 128) and 128:
    the loss equals the oracle's at 1e-12, the gradient its central differences on 240 coordinates
    spread over every parameter vector."""
    from test_gpu_train import mixed_layers, oracle_negll

    rng = np.random.default_rng(1000 + D)
    layers = mixed_layers(rng, D, np.float64)
    X = np.asfortranarray(0.8 * rng.standard_normal((D, 301)))
    negll, grads = enf.mvnormal_negll_trafograd(make_flow(enf, layers), colmajor_cuda(X), similar_fill_quirk=False)
    ref = oracle_negll(oracle, layers, X)
    assert np.isfinite(ref), ref  # (a finite-difference test: the loss must be finite)
    assert loss_close(negll, ref, 1e-12), (negll, ref)
    g = np.concatenate([np.asarray(a).reshape(-1, order="F") for per in grads for a in per])
    nvec = g.size // D  # parameter vectors of length D
    idx = [v * D + int(r) for v in range(nvec) for r in rng.choice(D, 240 // nvec + 1, replace=False)]
    _fd_check(oracle, layers, X, g, D, idx)


def test_negll_grad_D256_fp32(enf, gpu, oracle):
    """fp32 at D = 256 (one column per wave instruction; fp64 stops at 128): the loss against the oracle's
    fp64 loss of the same fp32 inputs, the gradient against its central differences on 64 coordinates
    (fp32 accuracy: 1e-3 of the gradient's scale)."""
    from test_gpu_train import oracle_negll

    rng = np.random.default_rng(256)
    D = 256
    layers = [(5, rand_params(rng, 5, D, np.float32)), (3, rand_params(rng, 3, D, np.float32)),
              (0, rand_params(rng, 0, D, np.float32)), (4, rand_params(rng, 4, D, np.float32))]
    X = np.asfortranarray((0.8 * rng.standard_normal((D, 2049))).astype(np.float32))
    n32, g32 = enf.mvnormal_negll_trafograd(make_flow(enf, layers), colmajor_cuda(X), similar_fill_quirk=False)
    l64 = [(op, [np.asarray(p, np.float64) for p in ps]) for op, ps in layers]
    X64 = np.asfortranarray(X.astype(np.float64))
    ref = oracle_negll(oracle, l64, X64)
    assert loss_close(n32, ref, 1e-4), (n32, ref)
    g = np.concatenate([np.asarray(x, np.float64).reshape(-1, order="F") for per in g32 for x in per])
    idx = [v * D + int(r) for v in range(g.size // D) for r in rng.choice(D, 6, replace=False)]
    _fd_check(oracle, l64, X64, g, D, idx, rel=1e-3, floor=0.1)


@pytest.mark.parametrize("D", [100, 128])
def test_vjp_large_D_vs_central_differences(enf, gpu, oracle, D):
    """enf_flow_vjp at D = 100 / 128 (every transform): dX against central differences of the oracle's
    <dY, Y> + dladj * ladj."""
    from test_gpu_train import mixed_layers
    from test_gpu_vjp import cotangent_fd

    rng = np.random.default_rng(2000 + D)
    layers = mixed_layers(rng, D, np.float64)
    N = 67
    X = np.asfortranarray(0.8 * rng.standard_normal((D, N)))
    dY, dl = rng.standard_normal((D, N)), rng.standard_normal(N)
    dX, _ = enf.flow_vjp(make_flow(enf, layers), colmajor_cuda(X), colmajor_cuda(dY), dl)
    fd = cotangent_fd(oracle, layers, X, dY, dl)
    err = np.abs(to_np(dX) - fd) / (np.abs(fd) + 1e-3 * np.abs(fd).max())
    assert err.max() < 2e-6, err.max()


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_optimize_whitening_large_D(enf, gpu, oracle, dtype):
    """One optimize_whitening epoch of 20 minibatches at D = 100 (4 x (J o H)): the first recorded negll
    is the oracle's loss of the initial parameters on that minibatch, the history is finite and falls."""
    from test_gpu_train import oracle_negll

    rng = np.random.default_rng(100)
    D = 100
    layers = []
    for _ in range(4):
        layers += [(5, rand_params(rng, 5, D, dtype)), (3, rand_params(rng, 3, D, dtype))]
    X = (rng.standard_normal((D, 20000)) * rng.uniform(0.5, 2, (D, 1))).astype(dtype)
    res = enf.optimize_whitening(colmajor_cuda(X), make_flow(enf, layers), enf.ADAGrad(), nbatches=20, nepochs=1)
    assert len(res.negll_history) == 20
    ref0 = oracle_negll(oracle, layers, np.asfortranarray(X[:, :1000].astype(np.float64)))
    assert abs(res.negll_history[0] - ref0) <= (1e-4 if dtype == np.float32 else 1e-10) * (abs(ref0) + 1)
    assert np.all(np.isfinite(res.negll_history))
    assert np.mean(res.negll_history[-5:]) < res.negll_history[0]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("D", [12, 100])
def test_padded_fragment_path_center_layers(enf, gpu, oracle, dtype, D):
    """CenterStretch / CenterContract (and every other op) on the padded fragment path: D = 12 and 100
    laid out as 16 and 128 rows (neutral Center records a = c = 0, b = 1 map the padded zeros to 0 with
    ladj 0), ragged tails, against the oracle."""
    if dtype == np.float32 and D % 4:
        pytest.skip("fp32 fragments hold 4 rows")
    rng = np.random.default_rng(3000 + D)
    layers = [(1, rand_params(rng, 1, D, dtype)), (5, rand_params(rng, 5, D, dtype, K=2)),
              (3, rand_params(rng, 3, D, dtype)), (2, rand_params(rng, 2, D, dtype)),
              (0, rand_params(rng, 0, D, dtype)), (1, rand_params(rng, 1, D, dtype)),
              (4, rand_params(rng, 4, D, dtype))]
    for N in (1, 63, 4097, 50_001):
        X = np.asfortranarray(rng.standard_normal((D, N)).astype(dtype))
        Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
        check_vs_oracle(oracle, layers, X, to_np(Y), to_np(L), dtype, what=f"padded center D{D} N{N}")
    # the inverse flow on the same path brings X back
    f = make_flow(enf, layers)
    Y, L = enf.with_logabsdet_jacobian(f, colmajor_cuda(X))
    Xb, Lb = enf.with_logabsdet_jacobian(enf.inverse(f), Y)
    tol = 2e-4 if dtype == np.float32 else 1e-9
    assert np.abs(to_np(Xb) - X).max() <= tol * (np.abs(X).max() + 1)
    assert np.abs(to_np(Lb) + to_np(L)).max() <= tol * (np.abs(to_np(L)).max() + 1)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_scaleshift_length1_a_ladj_and_gradient(enf, gpu, dtype):
    """ScaleShiftTrafo([a], [b]) at D = 5: Y = a x + b on every row, ladj = log|a| ONCE per sample
    (sum(log.(abs.(f.a))) over the length-1 vector, src/scale_shift_trafo.jl:22), and the gradient of
    mvnormal_negll_trafo w.r.t. a is sum_jd (a x + b) x / N - 1/a and w.r.t. b sum_jd (a x + b) / N,
    computed here by hand."""
    rng = np.random.default_rng(5)
    D, N = 5, 1000
    a, b = -1.7, 0.3
    f = enf.ScaleShiftTrafo(np.array([a], dtype), np.array([b], dtype))
    X = np.asfortranarray(rng.standard_normal((D, N)).astype(dtype))
    Y, L = enf.with_logabsdet_jacobian(f, colmajor_cuda(X))
    tol = 1e-6 if dtype == np.float32 else 1e-14
    assert np.allclose(to_np(Y), a * X.astype(np.float64) + b, rtol=tol, atol=tol)
    assert np.allclose(to_np(L).reshape(-1), np.log(abs(a)), rtol=tol, atol=tol)
    # host path (enf_flow_apply_cpu) agrees
    Yh, Lh = enf.with_logabsdet_jacobian(f, X)
    assert np.allclose(np.asarray(Lh).reshape(-1), np.log(abs(a)), rtol=tol, atol=tol)
    negll, grads = enf.mvnormal_negll_trafograd(f, colmajor_cuda(X), similar_fill_quirk=False)
    X64 = X.astype(np.float64)
    Y64 = a * X64 + b
    want_negll = ((Y64 ** 2 + np.log(2 * np.pi)) / 2).sum() / N - np.log(abs(a))
    want_ga = (Y64 * X64).sum() / N - 1.0 / a
    want_gb = Y64.sum() / N
    rt = 1e-4 if dtype == np.float32 else 1e-11
    assert abs(negll - want_negll) <= rt * (abs(want_negll) + 1)
    ga, gb = grads[0]
    assert np.shape(ga) == (1,) and np.shape(gb) == (1,)
    assert abs(float(ga[0]) - want_ga) <= rt * (abs(want_ga) + 1)
    assert abs(float(gb[0]) - want_gb) <= rt * (abs(want_gb) + 1)
    # the reference's recorded negll under Zygote omits the ScaleShift ladj (similar_fill's primal
    # zeros): + log|a| once, not D times
    nq, _ = enf.mvnormal_negll_trafograd(f, colmajor_cuda(X), similar_fill_quirk=True)
    assert abs(nq - (want_negll + np.log(abs(a)))) <= rt * (abs(want_negll) + 1)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("D", [5, 32, 300])
def test_mvnormal_negll_trafo_device_reduction(enf, gpu, oracle, dtype, D):
    """mvnormal_negll_trafo through enf_flow_negll (flow + reduction on the device, any D: 300 is past the
    gradient kernels' limit) against the oracle's fp64 loss of the same flow; at D <= 256 it also equals the
    gradient path's loss (enf_flow_negll_grad out[0])."""
    from test_gpu_train import oracle_negll

    rng = np.random.default_rng(4000 + D)
    layers = [(0, rand_params(rng, 0, D, dtype)), (5, rand_params(rng, 5, D, dtype, K=2)),
              (3, rand_params(rng, 3, D, dtype)), (2, rand_params(rng, 2, D, dtype)), (4, rand_params(rng, 4, D, dtype))]
    X = np.asfortranarray(0.8 * rng.standard_normal((D, 3001)).astype(dtype))
    f = make_flow(enf, layers)
    got = enf.mvnormal_negll_trafo(f, colmajor_cuda(X))
    l64 = [(op, [np.asarray(p, np.float64) for p in ps]) for op, ps in layers]
    ref = oracle_negll(oracle, l64, np.asfortranarray(X.astype(np.float64)))
    tol = 2e-5 if dtype == np.float32 else 1e-11
    assert abs(got - ref) <= tol * (abs(ref) + 1), (got, ref)
    if D <= 256:
        ng, _ = enf.mvnormal_negll_trafograd(f, colmajor_cuda(X), similar_fill_quirk=False)
        assert abs(got - ng) <= tol * (abs(ref) + 1)


def _hj64_layers(rng, D, pairs):
    layers = []
    for _ in range(pairs):
        layers += [(5, rand_params(rng, 5, D, np.float64)), (3, rand_params(rng, 3, D, np.float64))]
    return layers


@pytest.mark.parametrize("D", [32, 64, 128, 6, 24, 100])
@pytest.mark.parametrize("pairs", [1, 2, 4, 8, 9])
def test_hj64_program_vs_oracle(enf, gpu, oracle, D, pairs):
    """The compiled fp64 (J∘H)^n program (enf_flow_hj64.hip; n <= 8, n = 9 runs on the interpreter):
    forward + ladj at 1e-12 against the oracle (and the x87 evaluation), ragged tail, multi-tile waves,
    the plain call f(X) equal to the Y of the ladj call. D = 24 / 100 run on the padded layout (32 / 128,
    rows past D inert; round 3); D = 6 (layout 8) stays on the padded interpreter."""
    rng = np.random.default_rng(7000 + 100 * D + pairs)
    layers = _hj64_layers(rng, D, pairs)
    N = 100_003
    X = np.asfortranarray(rng.standard_normal((D, N)))
    f = make_flow(enf, layers)
    Y, L = enf.with_logabsdet_jacobian(f, colmajor_cuda(X))
    check_vs_oracle(oracle, layers, X, to_np(Y), to_np(L), np.float64, what=f"hj64 D{D} n{pairs}")
    assert np.array_equal(to_np(f(colmajor_cuda(X))), to_np(Y))


@pytest.mark.parametrize("D", [32, 100])
def test_hj64_program_edge_values_accumulate_inplace(enf, gpu, oracle, D):
    """fp64 program: huge (>= 2^26), infinite and NaN entries follow the reference (asinh64_tab's whole
    range, logprod64_tab's Inf / NaN); accumulate_ladj and Y aliasing X through the raw C ABI (D = 100:
    the padded layout)."""
    import torch

    from parity import col_err, ladj_err
    from test_gpu_parity import _raw_apply

    rng = np.random.default_rng(64)
    N = 20_001
    layers = _hj64_layers(rng, D, 4)
    X = rng.standard_normal((D, N))
    X[3, 7] = 3e30
    X[0, 100] = -1e25
    X[5, 101] = np.inf
    X[D - 1, 2000] = np.nan
    X[:, 4095] = 1e8
    X = np.asfortranarray(X)
    Yr, Lr = oracle.flow_apply(layers, X)
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    Y, L = to_np(Y), to_np(L).reshape(-1)
    assert np.array_equal(np.isnan(Y), np.isnan(Yr)) and np.array_equal(np.isnan(L), np.isnan(Lr))
    assert np.array_equal(np.isinf(Y), np.isinf(Yr)) and np.array_equal(np.isinf(L), np.isinf(Lr))
    fin = np.isfinite(Yr)
    assert col_err(np.where(fin, Y, 0), np.where(fin, Yr, 0)) < 1e-12
    finl = np.isfinite(Lr)
    assert ladj_err(L[finl], Lr[finl]) < 1e-12
    good = np.setdiff1d(np.arange(N), [7, 100, 101, 2000, 4095])
    check_vs_oracle(oracle, layers, np.asfortranarray(X[:, good]), Y[:, good], L[good], np.float64, what="hj64 edge")
    dev = [[torch.from_numpy(np.ascontiguousarray(p)).cuda() for p in ps] for _, ps in layers]
    lt = [(op, 1 if op == 5 else 0, [t.data_ptr() for t in ts]) for (op, _), ts in zip(layers, dev)]
    buf = colmajor_cuda(X).t().contiguous()
    L0 = torch.full((N,), 3.25, dtype=torch.float64, device="cuda")
    assert _raw_apply(enf, 1, D, N, buf.data_ptr(), D, buf.data_ptr(), D, L0.data_ptr(), 1, lt) == 0
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy().T, Y, equal_nan=True)
    Lb = L0.cpu().numpy() - 3.25
    assert np.all(np.abs(Lb[finl] - L[finl]) <= 1e-13 * (np.abs(L[finl]) + 3.25))
