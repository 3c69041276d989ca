"""GPU tests of the round-5 changes.

* The fp32 CenterContract ladj no longer clamps its two terms with min(., 1) (that turned a
  NaN input's ladj into log 2 where the reference's center_contract_ladj gives NaN, src/center_stretch.jl:17-22);
  NaN / +-Inf / huge columns of both Center transforms against the oracle.
* The config-5 step's reduction is one launch (enf_grad_tail.h grad_reduce_kernel) and the fused (J o H)^n
  gradient kernel takes two rows per lane with the flow's constant ladj computed once (enf_grad_hj.hip):
  the data-parallel step at a share of the minibatch (B > N > 0, the normalisation every real multi-rank step
  uses) equals the gradient of the share plus enf_whitening_apply(B) bit for bit, and the fused kernel
  on batches large enough that every wave strides over several tiles matches the fp64 generic kernel.
"""
import numpy as np
import pytest

from parity import check_vs_oracle, colmajor_cuda, loss_close, make_flow, rand_params, to_np

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("op", [1, 2])
@pytest.mark.parametrize("D", [2, 32])
def test_fp32_center_nan_inf_columns(enf, gpu, oracle, op, D):
    """fp32 CenterStretch (1) / CenterContract (2): NaN, +-Inf, huge and ordinary values in the same waves,
    against the oracle in fp32 (NaN where the reference is NaN, the same infinities, rtol 1e-5 elsewhere)."""
    rng = np.random.default_rng(5100 + 10 * op + D)
    ps = rand_params(rng, op, D, np.float32)
    N = 4099
    X = (rng.standard_normal((D, N)) * 2.0).astype(np.float32)
    special = np.array([np.nan, np.inf, -np.inf, 1e30, -1e30, 88.0, -88.0, 200.0, 0.0, -0.0], dtype=np.float32)
    for i, v in enumerate(special):
        X[:, 17 + 64 * i] = v        # whole columns
        X[i % D, 18 + 64 * i] = v    # one element of a column
    X = np.asfortranarray(X)
    layers = [(op, ps)]
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    Y, L = to_np(Y), to_np(L).reshape(-1)
    Yt, Lt = oracle.flow_apply(layers, X, nthreads=8)
    Lt = np.asarray(Lt).reshape(-1)
    # non-finite reference values: the same NaN / infinity, element by element
    assert np.array_equal(np.isnan(Y), np.isnan(Yt))
    assert np.array_equal(np.isnan(L), np.isnan(Lt)), np.nonzero(np.isnan(L) != np.isnan(Lt))
    inf = np.isinf(Yt)
    assert np.array_equal(Y[inf], Yt[inf])
    linf = np.isinf(Lt)
    assert np.array_equal(L[linf], Lt[linf])
    # a NaN input element makes its column's ladj NaN (the reference's log(abs(NaN)))
    nan_cols = np.unique(np.nonzero(np.isnan(X))[1])
    assert np.all(np.isnan(L[nan_cols]))
    fin = np.all(np.isfinite(X), axis=0) & np.all(np.isfinite(Yt), axis=0) & np.isfinite(Lt)
    check_vs_oracle(oracle, layers, np.asfortranarray(X[:, fin]), Y[:, fin], L[fin], np.float32,
                    what=f"op {op} D {D} finite columns")


def _hj_layers(rng, D, n, dtype=np.float32):
    layers = []
    for _ in range(n):
        layers += [(5, rand_params(rng, 5, D, dtype)), (3, rand_params(rng, 3, D, dtype))]
    return layers


@pytest.mark.parametrize("case", ["hj", "hj_d64", "chunked", "hj1_rows"])
def test_whitening_step_dp_share_equals_grad_plus_apply(enf, gpu, case):
    """enf_whitening_step_dp on a one-rank communicator with N = a share of the minibatch and B = the whole
    minibatch (B > N > 0) == enf_flow_negll_grad over the share + enf_whitening_apply(B): parameters, ADAGrad
    state and loss bit for bit, over 4 consecutive steps with different shares (the fused (J o H)^4 kernel at
    D = 32 and 64 -- rows over 64 KiB, reduced before the sum --, a chunked 20-layer flow, and J o H at D = 32 on
    2000 columns, whose gradient rows (at most 33 of 161 doubles) the sum carries themselves)."""
    import torch

    from euclidiannormalizingflows_jl_amd import _lib
    from euclidiannormalizingflows_jl_amd.train import FlowState, _workspace, householder_batches, trainable_runs
    from test_gpu_round4 import _long_flow

    rng = np.random.default_rng(5200)
    if case.startswith("hj"):
        D = 64 if case == "hj_d64" else 32
        layers = _hj_layers(rng, D, 1 if case == "hj1_rows" else 4)
    else:
        D = 8
        layers = [(op, ps) for op, ps in _long_flow(rng, D, np.float32) if op != 0]
    B = 2_000 if case == "hj1_rows" else 20_000
    X = colmajor_cuda((rng.standard_normal((D, B)) * 0.7).astype(np.float32))
    f = make_flow(enf, layers)
    opt = enf.ADAGrad()
    sa = FlowState(f, D, torch.float32, X.device, opt)
    sb = FlowState(f, D, torch.float32, X.device, opt)
    runs = np.ascontiguousarray(np.array(trainable_runs(sa), dtype=np.int64).reshape(-1))
    hbs = np.ascontiguousarray(np.array(householder_batches(sa), dtype=np.int64).reshape(-1))
    ws = _workspace(sa, B)
    out = torch.zeros(1 + sa.nparams, dtype=torch.float32, device=X.device)
    la = torch.zeros(1, dtype=torch.float64, device=X.device)
    lb = torch.zeros(1, dtype=torch.float64, device=X.device)
    L = _lib.lib()
    st = torch.cuda.current_stream().cuda_stream
    comm = enf.EnfComm.single()
    try:
        shares = ([(0, 7_001), (7_001, 20_000), (5_000, 5_003), (123, 19_999)] if B == 20_000 else
                  [(0, 701), (701, 2_000), (500, 503), (12, 1_999)])
        for it, (lo, hi) in enumerate(shares):
            N = hi - lo
            Xs = X[:, lo:hi]
            _lib.check(L.enf_whitening_step_dp(_lib.ENF_F32, D, N, Xs.data_ptr(), D, sa.layers(), len(sa.trafos),
                                               sa.theta.data_ptr(), sa.acc.data_ptr(), runs.ctypes.data, len(runs) // 2,
                                               hbs.ctypes.data, len(hbs) // 3, opt.eta, opt.epsilon, B, la.data_ptr(),
                                               comm.handle, ws.data_ptr(), ws.numel() * 8, st))
            out.zero_()
            _lib.check(L.enf_flow_negll_grad(_lib.ENF_F32, D, N, Xs.data_ptr(), D, sb.layers(), len(sb.trafos),
                                             out.data_ptr(), ws.data_ptr(), ws.numel() * 8, st))
            _lib.check(L.enf_whitening_apply(_lib.ENF_F32, D, sb.nparams, out.data_ptr(), B, sb.theta.data_ptr(),
                                             sb.acc.data_ptr(), runs.ctypes.data, len(runs) // 2, hbs.ctypes.data,
                                             len(hbs) // 3, opt.eta, opt.epsilon, lb.data_ptr(), st))
            torch.cuda.synchronize()
            assert torch.equal(sa.theta, sb.theta), it
            assert torch.equal(sa.acc, sb.acc), it
            assert float(la) == float(lb), (it, float(la), float(lb))
            assert np.isfinite(float(la)) and float(la) != 0.0
    finally:
        comm.close()


@pytest.mark.parametrize("D", [32, 64])
def test_hj_grad_kernel_striding_waves_vs_fp64(enf, gpu, oracle, D):
    """The fused (J o H)^4 fp32 gradient on a batch large enough that the grid is capped at the resident
    blocks and every wave strides over several tiles (N = 400 003, ragged tail), against the fp64 generic
    kernel; the loss (the constant ladj now subtracted once by the reduction) against the oracle's."""
    from test_gpu_train import oracle_negll

    rng = np.random.default_rng(5300 + D)
    L64 = _hj_layers(rng, D, 4, np.float64)
    L32 = [(op, [np.asarray(p, np.float32) for p in ps]) for op, ps in L64]
    N = 400_003
    X32 = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
    n32, g32 = enf.mvnormal_negll_trafograd(make_flow(enf, L32), colmajor_cuda(X32))
    n64, g64 = enf.mvnormal_negll_trafograd(make_flow(enf, L64), colmajor_cuda(X32.astype(np.float64)))
    sub = np.asfortranarray(X32[:, ::97])
    n32s, _ = enf.mvnormal_negll_trafograd(make_flow(enf, L32), colmajor_cuda(sub))
    assert loss_close(n32s, oracle_negll(oracle, L32, sub), 2e-5)
    assert loss_close(n32, n64, 1e-4)
    for p64, p32 in zip(g64, g32):
        for a, b in zip(p64, p32):
            a, b = np.ravel(a), np.ravel(b)
            assert np.max(np.abs(a - b)) < 1e-3 * (np.max(np.abs(a)) + 1e-3), (np.max(np.abs(a - b)), np.max(np.abs(a)))


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
def test_stream_copy_variants(enf, gpu, variant):
    """enf_stream_copy (the measurement copy bench.py's copy ceiling runs) copies every byte, including a tail
    that is not a whole 16-byte fragment, and rejects misaligned buffers."""
    import torch

    from euclidiannormalizingflows_jl_amd import _lib

    L = _lib.lib()
    n = 3 * (1 << 20) + 37
    src = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    dst = torch.zeros_like(src)
    _lib.check(L.enf_stream_copy(src.data_ptr(), dst.data_ptr(), n, variant, None))
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    assert L.enf_stream_copy(src.data_ptr() + 4, dst.data_ptr(), 64, variant, None) == _lib.ENF_ERR_INVALID


@pytest.mark.parametrize("D", [1, 2, 5, 32])
def test_negll_grad_vs_oracle_reverse_pass(enf, gpu, oracle, D):
    """The device gradient (enf_flow_negll_grad + the one-launch reduction) against the oracle's own reverse pass
    (oracle/enf_oracle_grad.c: the reference's Householder rrules and the derivatives of its formulas), fp64,
    every transform, chained and single reflections: entry by entry at 1e-10 of the gradient's scale."""
    rng = np.random.default_rng(5400 + D)
    layers = [(op, rand_params(rng, op, D, np.float64, K=2 if op == 5 else 1)) for op in [0, 5, 2, 3, 1, 4, 5, 3]]
    X = np.asfortranarray(0.8 * rng.standard_normal((D, 4001)))
    negll, grads = enf.mvnormal_negll_trafograd(make_flow(enf, layers), colmajor_cuda(X), similar_fill_quirk=False)
    g = np.concatenate([np.asarray(a).reshape(-1, order="F") for per in grads for a in per])
    n_ref, g_ref = oracle.negll_grad(layers, X)
    assert loss_close(negll, n_ref, 1e-12), (negll, n_ref)
    assert g.shape == g_ref.shape
    err = np.abs(g - g_ref) / (np.abs(g_ref) + 1e-3 * np.abs(g_ref).max())
    assert err.max() < 1e-10, (err.argmax(), g[err.argmax()], g_ref[err.argmax()])


@pytest.mark.parametrize("example", ["1d", "2d"])
def test_examples_training_vs_oracle(enf, gpu, oracle, example):
    """The reference examples' training (examples/nf_example_1d.jl:23-31: J o K o J o K on CenterStretch o
    Johnson data; nf_example_2d.jl:21-33: K o H o S on S o H o C data), fp64, ADAGrad, one epoch of 50
    minibatches on the device against the oracle's optimize_whitening: the loss history and the parameters agree
    to 1e-9 (the two sum their columns in different orders; ADAGrad amplifies that slowly)."""
    rng = np.random.default_rng(5500)
    if example == "1d":
        D = 1
        true = [(3, [np.array([10.0]), np.array([3.5]), np.array([10.0]), np.array([1.0])]),
                (1, [np.array([4.0]), np.array([1.0]), np.array([0.0])])]
        init = [(2, [np.array([0.0]), np.array([1.0]), np.array([0.0])]),
                (3, [np.array([0.0]), np.array([5.0]), np.array([0.0]), np.array([5.0])]),
                (2, [np.array([0.0]), np.array([1.0]), np.array([0.0])]),
                (3, [np.array([0.0]), np.array([5.0]), np.array([0.0]), np.array([5.0])])]
    else:
        D = 2
        true = [(1, [np.array([4.0, 4.1]), np.array([2.0, 2.1]), np.array([3.0, 3.1])]),
                (5, [np.array([1.0, 0.3])]),
                (0, [np.array([1.3, 0.4]), np.array([2.5, -1.2])])]
        init = [(0, [np.array([1.0, 1.0]), np.array([0.0, 0.0])]),
                (5, [rng.standard_normal(2)]),
                (2, [np.array([0.0, 0.0]), np.array([1.0, 1.0]), np.array([0.0, 0.0])])]
    XW = np.asfortranarray(rng.standard_normal((D, 5000)))
    X, _ = oracle.flow_apply(true, XW)
    X = np.asfortranarray(X)
    opt = enf.ADAGrad()  # Optimisers 0.2 defaults: eta = 0.1f0, epsilon = eps(Float32)
    # (the reference's recorded history, round 6: under Zygote the 2d flow's ScaleShift ladj is missing from it)
    th_ref, _, hist_ref = oracle.optimize_whitening(init, X, nbatches=50, nepochs=1, eta=opt.eta, epsilon=opt.epsilon,
                                                    zygote=True)
    r = enf.optimize_whitening(colmajor_cuda(X), make_flow(enf, init), opt, nbatches=50, nepochs=1)
    hist = np.asarray(r.negll_history)
    assert hist.shape == hist_ref.shape
    assert np.allclose(hist, hist_ref, rtol=1e-9, atol=0), np.abs(hist - hist_ref).max()
    th = r.optimizer_state.theta.cpu().numpy()
    assert np.allclose(th, th_ref, rtol=1e-9, atol=1e-12), np.abs(th - th_ref).max()


def _example_flows(example, rng):
    if example == "1d":
        init = [(2, [np.array([0.0]), np.array([1.0]), np.array([0.0])]),
                (3, [np.array([0.0]), np.array([5.0]), np.array([0.0]), np.array([5.0])]),
                (2, [np.array([0.0]), np.array([1.0]), np.array([0.0])]),
                (3, [np.array([0.0]), np.array([5.0]), np.array([0.0]), np.array([5.0])])]
        return 1, init
    init = [(0, [np.array([1.0, 1.0]), np.array([0.0, 0.0])]),
            (5, [rng.standard_normal(2)]),
            (2, [np.array([0.0, 0.0]), np.array([1.0, 1.0]), np.array([0.0, 0.0])])]
    return 2, init


@pytest.mark.parametrize("case", ["1d_B1000", "2d_B100", "2d_ragged", "f64_D5_multiblock", "hj_f32"])
def test_whitening_epoch_equals_steps(enf, gpu, case):
    """enf_whitening_epoch (round 5: an epoch of one-block minibatch steps in ONE launch, the batches walked by one
    block; other flows / sizes on the per-step path) equals the sequence of enf_whitening_step calls over the same
    minibatches bit for bit: parameters, ADAGrad state and every step's loss, over two epochs. Cases: the reference
    examples' flows at their batch sizes (the single-launch path; 2d takes the one-row-per-lane layout), a ragged
    last batch with another layout (mixed path), a multi-block fp64 flow and the fused fp32 (J o H)^2 kernel
    (per-step path inside the call)."""
    import torch

    from euclidiannormalizingflows_jl_amd import _lib
    from euclidiannormalizingflows_jl_amd.train import FlowState, _workspace, householder_batches, trainable_runs

    rng = np.random.default_rng(5600)
    if case in ("1d_B1000", "2d_B100", "2d_ragged"):
        D, layers = _example_flows(case[:2], rng)
        dtype = np.float64
        N, bs = {"1d_B1000": (5000, 1000), "2d_B100": (1000, 100), "2d_ragged": (1000, 300)}[case]
    elif case == "f64_D5_multiblock":
        D, dtype, N, bs = 5, np.float64, 6000, 2000
        layers = [(0, rand_params(rng, 0, D, dtype)), (5, rand_params(rng, 5, D, dtype)),
                  (3, rand_params(rng, 3, D, dtype)), (2, rand_params(rng, 2, D, dtype))]
    else:
        D, dtype, N, bs = 32, np.float32, 40_000, 10_000
        layers = []
        for _ in range(2):
            layers += [(5, rand_params(rng, 5, D, dtype)), (3, rand_params(rng, 3, D, dtype))]
    X = colmajor_cuda((0.8 * rng.standard_normal((D, N))).astype(dtype))
    f = make_flow(enf, layers)
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    L = _lib.lib()
    dt = _lib.ENF_F64 if dtype == np.float64 else _lib.ENF_F32
    opt = enf.ADAGrad()
    sa, sb = [FlowState(f, D, tdt, X.device, opt) for _ in range(2)]
    segs = trainable_runs(sa)
    hb = householder_batches(sa)
    runs = np.ascontiguousarray(np.array(segs, dtype=np.int64).reshape(-1))
    hbs = np.ascontiguousarray(np.array(hb, dtype=np.int64).reshape(-1))
    nb = (N + bs - 1) // bs
    ws = _workspace(sa, bs)
    la = torch.zeros(nb, dtype=torch.float64, device=X.device)
    lb = torch.zeros(nb, dtype=torch.float64, device=X.device)
    esz = 8 if dtype == np.float64 else 4
    for ep in range(2):
        _lib.check(L.enf_whitening_epoch(dt, D, N, X.data_ptr(), X.stride(1), bs, sa.layers(), len(sa.trafos),
                                         sa.theta.data_ptr(), sa.acc.data_ptr(), runs.ctypes.data, len(segs),
                                         hbs.ctypes.data, len(hb), opt.eta, opt.epsilon, la.data_ptr(), ws.data_ptr(),
                                         ws.numel() * 8, None))
        for j in range(nb):
            b0 = j * bs
            B = min(bs, N - b0)
            _lib.check(L.enf_whitening_step(dt, D, B, X.data_ptr() + b0 * X.stride(1) * esz, X.stride(1), sb.layers(),
                                            len(sb.trafos), sb.theta.data_ptr(), sb.acc.data_ptr(), runs.ctypes.data,
                                            len(segs), hbs.ctypes.data, len(hb), opt.eta, opt.epsilon,
                                            lb[j:].data_ptr(), ws.data_ptr(), ws.numel() * 8, None))
        torch.cuda.synchronize()
        assert torch.equal(la, lb), (ep, (la - lb).abs().max())
        assert torch.equal(sa.theta, sb.theta), ep
        assert torch.equal(sa.acc, sb.acc), ep
    assert torch.isfinite(la).all()


def test_optimize_whitening_epoch_equals_per_step(enf, gpu):
    """optimize_whitening on one rank (each epoch one enf_whitening_epoch call) equals the per-step loop
    (_per_step=True) bit for bit, eager and graph-captured, on the 2-D example's flow."""
    rng = np.random.default_rng(5700)
    D, init = _example_flows("2d", rng)
    X = colmajor_cuda(np.asfortranarray(rng.standard_normal((D, 3000))))
    res = []
    for kw in ({}, {"_per_step": True}, {"graph": True}):
        r = enf.optimize_whitening(X, make_flow(enf, init), enf.ADAGrad(), nbatches=30, nepochs=3, **kw)
        res.append((r.optimizer_state.theta.cpu().numpy(), r.optimizer_state.acc.cpu().numpy(),
                    np.asarray(r.negll_history)))
    for t, a, h in res[1:]:
        assert np.array_equal(res[0][0], t) and np.array_equal(res[0][1], a) and np.array_equal(res[0][2], h)
