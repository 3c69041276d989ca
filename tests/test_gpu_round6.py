"""GPU tests of the round-6 changes.

* The reference's recorded loss is the drop-in's default: under Zygote.pullback
  rrule(similar_fill) returns zeros as the primal (src/abstract_trafo.jl:30-33), so the negll that
  mvnormal_negll_trafograd returns and optimize_whitening records misses every ScaleShiftTrafo's ladj
  sum log|a| (src/scale_shift_trafo.jl:22-23). The library adds it on the device (the ENF_NEGLL_ZYGOTE dtype flag,
  include/enf.h) on every training path: the one-launch epoch, the per-step kernels, the data-parallel step and the
  chunked path; the offset is checked per step against the oracle's.
* Minibatch sizes round half to even (Julia's round(Int, N/nbatches), src/optimize_whitening.jl:31): the oracle
  used to round half away from zero; a tie size now matches the device.
* The cross-lane sums of enf_train.h (the xor tree and the permlane swaps written as inline asm with a hand-placed
  hazard pad) equal the __shfl_xor butterfly bit for bit at every group size (the round-5
  run-27 miscompile of the swap builtin gave wrong gradient sums).
* The gradient workspace of enf_flow_negll_grad_workspace(batchsize) suffices for a ragged last minibatch below
  the fused kernel's shape switch.
* Elementwise accuracy: the fraction of output elements within rtol * |y| of the
  high-precision value for configs 2 and 3, beside the reference algorithm's own (oracle at the data precision).
"""
import ctypes
import os

import numpy as np
import pytest

from parity import colmajor_cuda, loss_close, make_flow, rand_params, to_np

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _example_2d(rng):
    """examples/nf_example_2d.jl:12-33: X = (S o H o C)(randn), initial flow K o H o S (application order S, H, K)."""
    true = [(1, [np.array([4.0, 4.1]), np.array([2.0, 2.1]), np.array([3.0, 3.1])]),
            (5, [np.array([1.0, 0.3])]),
            (0, [np.array([1.3, 0.4]), np.array([2.5, -1.2])])]
    init = [(0, [np.array([1.0, 1.0]), np.array([0.0, 0.0])]),
            (5, [rng.standard_normal(2)]),
            (2, [np.array([0.0, 0.0]), np.array([1.0, 1.0]), np.array([0.0, 0.0])])]
    return true, init


@pytest.mark.parametrize("N,nbatches", [(250, 100), (1050, 100), (5000, 50)])
def test_minibatch_ties_vs_oracle(enf, gpu, oracle, N, nbatches):
    """N / nbatches = 2.5 and 10.5 are ties: Julia's round(Int, .) gives 2 and 10 (half to even), as the drop-in's
    minibatch_plan and now the oracle (round 5's llround gave 3 and 11). The 2-D example's training over those
    minibatches: history (as the reference records it) and parameters against the oracle's."""
    rng = np.random.default_rng(6000 + N)
    true, init = _example_2d(rng)
    X, _ = oracle.flow_apply(true, np.asfortranarray(rng.standard_normal((2, N))))
    X = np.asfortranarray(X)
    bs = max(int(round(N / nbatches)), 1)
    assert bs == {250: 2, 1050: 10, 5000: 100}[N]
    plan = enf.minibatch_plan(N, nbatches)
    assert max(B for B, _, _ in plan) == bs and len(plan) == -(-N // bs)
    opt = enf.ADAGrad()
    th_ref, _, hist_ref = oracle.optimize_whitening(init, X, nbatches=nbatches, nepochs=2, eta=opt.eta,
                                                    epsilon=opt.epsilon, zygote=True)
    r = enf.optimize_whitening(colmajor_cuda(X), make_flow(enf, init), opt, nbatches=nbatches, nepochs=2)
    hist = np.asarray(r.negll_history)
    assert hist.shape == hist_ref.shape == (2 * len(plan),)
    assert np.allclose(hist, hist_ref, rtol=1e-9, atol=1e-12), np.abs(hist - hist_ref).max()
    th = r.optimizer_state.theta.cpu().numpy()
    assert np.allclose(th, th_ref, rtol=1e-9, atol=1e-12), np.abs(th - th_ref).max()


@pytest.mark.parametrize("path", ["epoch", "per_step", "dp_comm", "dp_separate", "graph"])
def test_zygote_offset_is_scaleshift_ladj_per_step(enf, gpu, oracle, path):
    """The default history minus the similar_fill_quirk=False history is, step by step, sum log|a| of the
    ScaleShiftTrafo at the parameters that step started from -- the oracle's zygote=True minus zygote=False -- on
    every training path (the parameters themselves are identical with and without the quirk), and the default
    history is the oracle's recorded one."""
    rng = np.random.default_rng(6100)
    true, init = _example_2d(rng)
    init[0] = (0, [np.array([1.5, 1.6]), np.array([0.0, 0.0])])  # (a = 1 would make the first offset zero)
    X, _ = oracle.flow_apply(true, np.asfortranarray(rng.standard_normal((2, 3000))))
    X = np.asfortranarray(X)
    opt = enf.ADAGrad()
    _, _, hq = oracle.optimize_whitening(init, X, nbatches=30, nepochs=2, eta=opt.eta, epsilon=opt.epsilon,
                                         zygote=True)
    _, _, h0 = oracle.optimize_whitening(init, X, nbatches=30, nepochs=2, eta=opt.eta, epsilon=opt.epsilon)
    kw = {"epoch": {}, "per_step": {"_per_step": True}, "dp_separate": {"_dp_step": True}, "graph": {"graph": True},
          "dp_comm": {}}[path]
    comm = enf.EnfComm.single() if path == "dp_comm" else None
    try:
        if comm is not None:
            kw = {"comm": comm}
        ra = enf.optimize_whitening(colmajor_cuda(X), make_flow(enf, init), opt, nbatches=30, nepochs=2, **kw)
        rb = enf.optimize_whitening(colmajor_cuda(X), make_flow(enf, init), opt, nbatches=30, nepochs=2,
                                    similar_fill_quirk=False, **kw)
    finally:
        if comm is not None:
            comm.close()
    assert np.array_equal(to_np(ra.optimizer_state.theta), to_np(rb.optimizer_state.theta))
    ha, hb = np.asarray(ra.negll_history), np.asarray(rb.negll_history)
    assert np.allclose(ha - hb, hq - h0, rtol=1e-9, atol=1e-12), np.abs((ha - hb) - (hq - h0)).max()
    assert np.allclose(ha, hq, rtol=1e-9, atol=1e-12)
    assert abs(hq[0] - h0[0]) > 0.5  # (log 1.5 + log 1.6: the offset is not trivially zero)


@pytest.mark.parametrize("case", ["generic_f64", "f32_D32", "length1_a", "chunked_f32"])
def test_negll_zygote_flag_raw_capi(enf, gpu, case):
    """enf_flow_negll_grad with ENF_NEGLL_ZYGOTE OR'd into the dtype: out[0] is larger by N sum log|a| over the
    flow's ScaleShiftTrafos (a length-1 a counts once, src/scale_shift_trafo.jl:22), every gradient entry is the
    same bit for bit; the generic kernel, fp32, a length-1 a and the chunked path (20 layers)."""
    import torch

    from euclidiannormalizingflows_jl_amd import _lib
    from euclidiannormalizingflows_jl_amd.train import FlowState, _workspace

    rng = np.random.default_rng(6200)
    dtype = np.float64 if case == "generic_f64" else np.float32
    D = {"generic_f64": 5, "f32_D32": 32, "length1_a": 6, "chunked_f32": 8}[case]
    if case == "length1_a":
        f = enf.compose(enf.JohnsonTrafo(*rand_params(rng, 3, D, dtype)),
                        enf.ScaleShiftTrafo(np.array([1.7], dtype), rng.standard_normal(D).astype(dtype)))
        S = float(np.log(1.7))
    else:
        layers = [(0, rand_params(rng, 0, D, dtype)), (5, rand_params(rng, 5, D, dtype)),
                  (3, rand_params(rng, 3, D, dtype)), (0, rand_params(rng, 0, D, dtype))]
        if case == "chunked_f32":
            for _ in range(8):
                layers += [(5, rand_params(rng, 5, D, dtype)), (3, rand_params(rng, 3, D, dtype))]
        f = make_flow(enf, layers)
        S = float(sum(np.sum(np.log(np.abs(ps[0].astype(np.float64)))) for op, ps in layers if op == 0))
    N = 3001
    X = colmajor_cuda((0.7 * rng.standard_normal((D, N))).astype(dtype))
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    st = FlowState(f, D, tdt, X.device)
    ws = _workspace(st, N)
    L = _lib.lib()
    dt = _lib.ENF_F64 if dtype == np.float64 else _lib.ENF_F32
    outs = []
    for flag in (0, _lib.ENF_NEGLL_ZYGOTE):
        out = torch.zeros(1 + st.nparams, dtype=tdt, device=X.device)
        _lib.check(L.enf_flow_negll_grad(dt | flag, D, N, X.data_ptr(), X.stride(1), st.layers(), len(st.trafos),
                                         out.data_ptr(), ws.data_ptr(), ws.numel() * 8, None))
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy().astype(np.float64))
    assert np.array_equal(outs[0][1:], outs[1][1:])
    tol = 1e-12 if dtype == np.float64 else 2e-6
    assert abs((outs[1][0] - outs[0][0]) - N * S) <= tol * (abs(outs[0][0]) + N * abs(S) + 1), \
        (outs[1][0] - outs[0][0], N * S)
    # the drop-in's default returns the recorded value, similar_fill_quirk=False the true one
    nq, _ = enf.mvnormal_negll_trafograd(f, X)
    n0, _ = enf.mvnormal_negll_trafograd(f, X, similar_fill_quirk=False)
    assert loss_close(nq - n0, S, 1e-5 if dtype == np.float32 else 1e-10)


def test_epoch_large_batch_ragged_tail_workspace(enf, gpu):
    """enf_whitening_epoch on D = 32 fp32 (J o H)^2 with batchsize 60 000 (the fused gradient kernel's large-batch
    shape) over N = 100 000 columns: the last minibatch, 40 000 columns, takes the small-batch shape, which can need
    more partial rows than the large shape at 60 000. The workspace of enf_flow_negll_grad_workspace(batchsize), as
    the header documents, suffices (round 5 could reject that tail with 'workspace too small'), and the
    epoch equals the enf_whitening_step calls bit for bit."""
    import torch

    from euclidiannormalizingflows_jl_amd import _lib
    from euclidiannormalizingflows_jl_amd.train import FlowState, _workspace, householder_batches, trainable_runs

    rng = np.random.default_rng(6300)
    D, N, bs = 32, 100_000, 60_000
    layers = []
    for _ in range(2):
        layers += [(5, rand_params(rng, 5, D, np.float32)), (3, rand_params(rng, 3, D, np.float32))]
    X = colmajor_cuda((0.8 * rng.standard_normal((D, N))).astype(np.float32))
    f = make_flow(enf, layers)
    opt = enf.ADAGrad()
    sa, sb = [FlowState(f, D, torch.float32, X.device, opt) for _ in range(2)]
    segs, hb = trainable_runs(sa), householder_batches(sa)
    runs = np.ascontiguousarray(np.array(segs, dtype=np.int64).reshape(-1))
    hbs = np.ascontiguousarray(np.array(hb, dtype=np.int64).reshape(-1))
    ws = _workspace(sa, bs)
    L = _lib.lib()
    la = torch.zeros(2, dtype=torch.float64, device=X.device)
    lb = torch.zeros(2, dtype=torch.float64, device=X.device)
    _lib.check(L.enf_whitening_epoch(_lib.ENF_F32, D, N, X.data_ptr(), X.stride(1), bs, sa.layers(), len(sa.trafos),
                                     sa.theta.data_ptr(), sa.acc.data_ptr(), runs.ctypes.data, len(segs),
                                     hbs.ctypes.data, len(hb), opt.eta, opt.epsilon, la.data_ptr(), ws.data_ptr(),
                                     ws.numel() * 8, None))
    for j, (b0, B) in enumerate(((0, bs), (bs, N - bs))):
        _lib.check(L.enf_whitening_step(_lib.ENF_F32, D, B, X.data_ptr() + b0 * X.stride(1) * 4, X.stride(1),
                                        sb.layers(), len(sb.trafos), sb.theta.data_ptr(), sb.acc.data_ptr(),
                                        runs.ctypes.data, len(segs), hbs.ctypes.data, len(hb), opt.eta, opt.epsilon,
                                        lb[j:].data_ptr(), ws.data_ptr(), ws.numel() * 8, None))
    torch.cuda.synchronize()
    assert torch.equal(la, lb) and torch.isfinite(la).all()
    assert torch.equal(sa.theta, sb.theta) and torch.equal(sa.acc, sb.acc)


def _xlane_lib():
    path = os.path.join(ROOT, "tests", "xlane", "libenf_xlane.so")
    if not os.path.exists(path):
        pytest.fail(f"{path} is missing: build it with `make -C euclidiannormalizingflows.jl_amd/csrc xlane` "
                    "(__graft_entry__.build() does)")
    lib = ctypes.CDLL(path)
    lib.enf_xlane_check.restype = ctypes.c_int
    lib.enf_xlane_check.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return lib


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_cross_lane_primitives(enf, gpu, dtype):
    """enf_train.h's xor_tree over groups of P = 1 .. 64 lanes, add_xor_swap<16> / <32> (v_permlane16/32_swap as
    inline asm after an `s_nop 1` hazard pad) and lane_sum equal the __shfl_xor butterfly bit for bit, over inputs
    whose sums round differently in every association (tests/xlane/xlane.hip, a test-only library)."""
    import torch

    lib = _xlane_lib()
    rng = np.random.default_rng(6400)
    td = torch.float32 if dtype == np.float32 else torch.float64
    for trial in range(8):
        vals = (rng.standard_normal(64) * 10.0 ** rng.uniform(-8, 8, 64)).astype(dtype)
        x = torch.from_numpy(vals).cuda()
        for P in (1, 2, 4, 8, 16, 32, 64):
            out = torch.full((448,), float("nan"), dtype=td, device="cuda")
            assert lib.enf_xlane_check(0 if dtype == np.float32 else 1, P, x.data_ptr(), out.data_ptr(), None) == 0
            torch.cuda.synchronize()
            o = out.cpu().numpy().view(np.uint32 if dtype == np.float32 else np.uint64)
            assert np.array_equal(o[0:64], o[64:128]), (trial, P, "xor_tree")
            assert np.array_equal(o[128:192], o[192:256]), (trial, P, "permlane16 swap")
            assert np.array_equal(o[256:320], o[320:384]), (trial, P, "permlane32 swap")
            if dtype == np.float64:
                # lane_sum over D = P lanes: the full xor tree over the smallest power of two >= P (here P), every
                # lane < P gets the group-0 sum of the zero-padded values
                w = np.where(np.arange(64) < P, vals, 0.0)
                ref = torch.from_numpy(w).cuda()
                ref_out = torch.full((448,), float("nan"), dtype=td, device="cuda")
                assert lib.enf_xlane_check(1, P, ref.data_ptr(), ref_out.data_ptr(), None) == 0
                torch.cuda.synchronize()
                ro = ref_out.cpu().numpy().view(np.uint64)
                assert np.array_equal(o[384:384 + P], ro[64:64 + P]), (trial, P, "lane_sum")


def _elementwise(Y, Yh, rtol):
    rel = np.abs(Y.astype(np.float64) - Yh) / np.abs(Yh)
    fin = np.isfinite(rel)
    return float(np.mean(rel[fin] <= rtol)), float(np.max(rel[fin])), int(np.argmax(np.where(fin, rel, -1)))


def test_elementwise_report_config3(enf, gpu, oracle):
    """Config 3's flow (D = 32, 4 x (J o H), fp32, the survey's parameter distributions), N = 200 003: the fraction
    of elements with |y - y_hi| <= 1e-5 |y_hi| (north star's fp32 rtol read elementwise) is the reference algorithm's
    own to within 0.1 % (both ~99.5 %: the rest are outputs that cancel, where no fp32 evaluation has that relative
    accuracy), and every element with |y_hi| >= 0.5 meets it (as the reference's does)."""
    rng = np.random.default_rng(6500)
    D, N = 32, 200_003
    layers = []
    for _ in range(4):
        layers += [(5, [rng.standard_normal(D).astype(np.float32)]), (3, rand_params(rng, 3, D, np.float32))]
    X = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
    Y = to_np(enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))[0])
    Yh, _ = oracle.flow_apply_hi(layers, X)
    Yr, _ = oracle.flow_apply(layers, X, nthreads=8)
    f, worst, _ = _elementwise(Y, Yh, 1e-5)
    fr, worst_r, _ = _elementwise(Yr, Yh, 1e-5)
    print(f"config 3 elementwise rtol 1e-5: device {f:.6f} (worst {worst:.2e}), fp32 reference {fr:.6f} "
          f"(worst {worst_r:.2e})")
    assert f >= fr - 1e-3
    big = np.abs(Yh) >= 0.5
    assert np.all(np.abs(Y[big] - Yh[big]) <= 1e-5 * np.abs(Yh[big]))


def test_elementwise_report_config2_and_golden(enf, gpu, oracle):
    """Config 2 (D = 2, J o H, fp64, N = 1e6) against the oracle in extended precision: every element within rtol
    1e-12 of |y| where the fp64 reference algorithm is (its own failures are cancelling outputs), the fractions
    beside each other; the mpmath golden fixtures of configs 2 and 3 elementwise at 1e-12 / 1e-5."""
    from conftest import load_golden_flow

    rng = np.random.default_rng(6600)
    layers = [(5, rand_params(rng, 5, 2, np.float64)), (3, rand_params(rng, 3, 2, np.float64))]
    X = np.asfortranarray(rng.standard_normal((2, 1_000_000)))
    Y = to_np(enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))[0])
    Yh, _ = oracle.flow_apply_hi(layers, X)
    Yr, _ = oracle.flow_apply(layers, X)
    f, worst, _ = _elementwise(Y, Yh, 1e-12)
    fr, worst_r, _ = _elementwise(Yr, Yh, 1e-12)
    print(f"config 2 elementwise rtol 1e-12: device {f:.7f} (worst {worst:.2e}), fp64 reference {fr:.7f} "
          f"(worst {worst_r:.2e})")
    assert f >= fr - 1e-4
    ok_r = np.abs(Yr - Yh) <= 1e-12 * np.abs(Yh)
    big = ok_r & (np.abs(Yh) >= 0.5)
    assert np.all(np.abs(Y[big] - Yh[big]) <= 1e-12 * np.abs(Yh[big]))
    for name, rtol in (("config2_JoH_D2_float64", 1e-12), ("config3_flow8_D32_float32", 1e-5)):
        gl, Xg, Ye, _ = load_golden_flow(name)
        Yg = to_np(enf.with_logabsdet_jacobian(make_flow(enf, gl), colmajor_cuda(np.asfortranarray(Xg)))[0])
        fg, wg, _ = _elementwise(Yg, Ye, rtol)
        print(f"golden {name}: elementwise rtol {rtol:g}: {fg:.6f} (worst {wg:.2e})")
        m = np.abs(Ye) >= 0.5
        assert np.all(np.abs(Yg[m] - Ye[m]) <= rtol * np.abs(Ye[m])), name
