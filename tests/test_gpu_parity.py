"""GPU parity: libenf.so (through the host mirror and the raw C ABI) against the oracle and the
exact golden vectors. Tolerances and the normwise criterion: tests/parity.py."""
import ctypes
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden_flow
from parity import (RTOL, assert_as_accurate, assert_flow_close, check_vs_oracle, col_err, colmajor_cuda,
                    ladj_err, make_flow, make_trafo, rand_params, to_np)

pytestmark = pytest.mark.gpu

FLOW_FIXTURES = sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, "*.npz"))
                       if "scalars" not in f and "johnsonsu" not in f)


@pytest.mark.parametrize("name", FLOW_FIXTURES)
def test_golden_flow(enf, gpu, oracle, name):
    """Every committed fixture: GPU vs the exact (mpmath) reference formulas."""
    layers, X, Yx, Lx = load_golden_flow(name)
    f = make_flow(enf, layers)
    Y, L = enf.with_logabsdet_jacobian(f, colmajor_cuda(X))
    Yt, Lt = oracle.flow_apply(layers, X)
    assert_as_accurate(to_np(Y), to_np(L), Yt, Lt, Yx, Lx, X.dtype, what=name)


DS = [1, 2, 3, 4, 5, 8, 12, 16, 32, 36, 64, 100, 128, 256]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("op", range(6))
@pytest.mark.parametrize("D", DS)
def test_single_op_vs_oracle(enf, gpu, oracle, dtype, op, D):
    rng = np.random.default_rng(1000 * op + D)
    N = 4099
    K = 3 if op == 5 else 1
    layers = [(op, rand_params(rng, op, D, dtype, K))]
    X = rng.standard_normal((D, N)).astype(dtype)
    if op == 2:
        X *= 3
    X = np.asfortranarray(X)
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    check_vs_oracle(oracle, layers, X, to_np(Y), to_np(L), dtype, what=f"op{op} D{D}")
    # plain call f(X) gives the same Y
    Y2 = make_flow(enf, layers)(colmajor_cuda(X))
    assert np.array_equal(to_np(Y2), to_np(Y))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("D", [2, 24, 32, 64, 100, 128, 256])
def test_config3_pattern_vs_oracle(enf, gpu, oracle, dtype, D):
    """J4∘H4∘…∘J1∘H1 (SURVEY.md §8(d) config 3 pattern) on 200k samples."""
    rng = np.random.default_rng(7 + D)
    layers = []
    for _ in range(4):
        layers += [(5, rand_params(rng, 5, D, dtype)), (3, rand_params(rng, 3, D, dtype))]
    N = 200_003
    X = np.asfortranarray(rng.standard_normal((D, N)).astype(dtype))
    f = make_flow(enf, layers)
    Y, L = enf.with_logabsdet_jacobian(f, colmajor_cuda(X))
    check_vs_oracle(oracle, layers, X, to_np(Y), to_np(L), dtype, what=f"config3 D{D}")
    # inverse flow round trip
    X2, L2 = enf.with_logabsdet_jacobian(enf.inverse(f), Y)
    assert col_err(to_np(X2), X) < (1e-4 if dtype == np.float32 else 1e-11)
    assert ladj_err(-to_np(L2), to_np(L)) < 10 * RTOL[np.dtype(dtype)]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_mixed_ops_long_flow(enf, gpu, oracle, dtype):
    """Every op, Householder chains with several columns, > 16 layers / > 64 steps (several launches)."""
    rng = np.random.default_rng(99)
    D = 8
    layers = []
    for i in range(20):
        op = [5, 3, 0, 5, 2, 1, 4][i % 7]
        layers.append((op, rand_params(rng, op, D, dtype, K=5 if op == 5 else 1)))
    X = np.asfortranarray((0.5 * rng.standard_normal((D, 3001))).astype(dtype))
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    check_vs_oracle(oracle, layers, X, to_np(Y), to_np(L), dtype, what="mixed long flow")


@pytest.mark.parametrize("N", [1, 2, 3, 31, 32, 33, 127, 128, 129, 4097])
def test_tails(enf, gpu, oracle, N):
    """N not a multiple of the wave tile: the masked tail path."""
    rng = np.random.default_rng(N)
    for D in (1, 2, 32):
        layers = [(5, rand_params(rng, 5, D, np.float32)), (3, rand_params(rng, 3, D, np.float32))]
        X = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
        Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
        check_vs_oracle(oracle, layers, X, to_np(Y), to_np(L), np.float32, what=f"tail D{D} N{N}")


def test_batched_equals_per_column(enf, gpu):
    """test/test_johnson_trafo.jl:71-74, test/test_center_stretch.jl:64-67 (exact ==)."""
    rng = np.random.default_rng(5)
    for f in (enf.JohnsonTrafo([10.0, 11.0], [3.5, 3.6], [10.0, 11.0], [1.0, 1.1]),
              enf.CenterStretch([4.0, 4.1], [2.0, 2.1], [3.0, 3.1]),
              enf.JohnsonTrafo(np.float32([0.1, 0.2]), np.float32([1, 2]), np.float32([0, 1]), np.float32([1, 3]))):
        X = rng.standard_normal((2, 3))
        if isinstance(f.gamma if hasattr(f, "gamma") else f.a, np.ndarray) and f.gamma.dtype == np.float32:
            X = X.astype(np.float32)
        Y, L = enf.with_logabsdet_jacobian(f, colmajor_cuda(X))
        for j in range(3):
            y, l = enf.with_logabsdet_jacobian(f, colmajor_cuda(X)[:, j].contiguous())
            assert np.array_equal(to_np(y), to_np(Y)[:, j])
            assert to_np(l) == to_np(L)[0, j]
        X2, Li = enf.with_logabsdet_jacobian(enf.inverse(f), Y)
        assert col_err(to_np(X2), X) < 1e-5
        assert ladj_err(to_np(Li), -to_np(L)) < 1e-5


def test_householder_matrix_oracle(enf, gpu):
    """test/test_householder_trafo.jl:18-25,36-43: H(v) = I - 2vv'/(v'v); chain = H_K ... H_1."""
    rng = np.random.default_rng(3)
    v, X, V = rng.random(5), rng.random((5, 3)), rng.random((5, 3))
    Hm = lambda v: np.eye(5) - 2 * np.outer(v, v) / (v @ v)
    Y = to_np(enf.HouseholderTrafo(v)(colmajor_cuda(X)))
    assert np.allclose(Y, Hm(v) @ X, rtol=1e-13, atol=1e-14)
    YY = to_np(enf.HouseholderTrafo(v)(colmajor_cuda(Y)))
    assert np.allclose(YY, X, rtol=1e-13, atol=1e-14)
    chain = Hm(V[:, 2]) @ Hm(V[:, 1]) @ Hm(V[:, 0])
    Yc, L = enf.with_logabsdet_jacobian(enf.HouseholderTrafo(V), colmajor_cuda(X))
    assert np.allclose(to_np(Yc), chain @ X, rtol=1e-13, atol=1e-14)
    assert np.array_equal(to_np(L), np.zeros((1, 3)))
    Xr = to_np(enf.inverse(enf.HouseholderTrafo(V))(Yc))
    assert np.allclose(Xr, X, rtol=1e-13, atol=1e-14)
    # single sample: scalar 0 ladj (householder_trafo.jl:159)
    y, l = enf.with_logabsdet_jacobian(enf.HouseholderTrafo(V), colmajor_cuda(X)[:, 0].contiguous())
    assert float(l) == 0.0 and np.allclose(to_np(y), chain @ X[:, 0])


def test_vector_input_scalar_ladj(enf, gpu, oracle):
    """test/test_johnson_trafo.jl:40-48: vector x -> (y, sum of elementwise ladjs)."""
    import torch

    x = torch.tensor([0.5, 0.6], dtype=torch.float64, device="cuda")
    f = enf.JohnsonTrafo([4.0, 4.1], [3.0, 3.1], [2.0, 2.1], [1.0, 1.1])
    y, l = enf.with_logabsdet_jacobian(f, x)
    assert y.shape == (2,) and l.shape == ()
    ref_y = [oracle.scalar("johnsontrafo", np.float64, xv, g, d, xi, lm)
             for xv, g, d, xi, lm in zip([0.5, 0.6], [4.0, 4.1], [3.0, 3.1], [2.0, 2.1], [1.0, 1.1])]
    ref_l = sum(oracle.scalar("johnsontrafo_ladj", np.float64, xv, g, d, xi, lm)
                for xv, g, d, xi, lm in zip([0.5, 0.6], [4.0, 4.1], [3.0, 3.1], [2.0, 2.1], [1.0, 1.1]))
    assert np.allclose(to_np(y), ref_y, rtol=1e-14)
    assert abs(float(l) - ref_l) <= 1e-13 * (abs(ref_l) + 1)


def test_promotion_and_cpu_inputs(enf, gpu):
    """Julia promotion: float64 params on float32 data compute in float64; numpy in -> numpy out."""
    X = np.random.default_rng(0).standard_normal((2, 10)).astype(np.float32)
    Y, L = enf.with_logabsdet_jacobian(enf.JohnsonTrafo([1.0, 2.0], [1.0, 1.0], [0.0, 0.0], [1.0, 1.0]), X)
    assert isinstance(Y, np.ndarray) and Y.dtype == np.float64 and L.shape == (1, 10)
    Y32 = enf.JohnsonTrafo(np.float32([1, 2]), np.float32([1, 1]), np.float32([0, 0]), np.float32([1, 1]))(X)
    assert Y32.dtype == np.float32
    Yi = enf.JohnsonTrafo(4, 2, 3, 1)(X)  # Int params do not promote (test_johnson_trafo.jl:18)
    assert Yi.dtype == np.float32


def _raw_apply(enf, dtype, D, N, Xptr, ldx, Yptr, ldy, Lptr, acc, layers_t):
    lib = enf._lib
    arr = (lib.Layer * len(layers_t))()
    for i, (op, k, ptrs) in enumerate(layers_t):
        arr[i].op, arr[i].k = op, k
        for q, p in enumerate(ptrs):
            arr[i].p[q] = p
    return lib.lib().enf_flow_apply(dtype, D, N, Xptr, ldx, Yptr, ldy, Lptr, acc, arr, len(layers_t), None)


def test_capi_inplace_accumulate_strided(enf, gpu, oracle):
    """C ABI: Y == X in place, accumulate_ladj, leading dimensions > D, misaligned base."""
    import torch

    rng = np.random.default_rng(11)
    D, N = 32, 5000
    layers = [(5, rand_params(rng, 5, D, np.float32)), (3, rand_params(rng, 3, D, np.float32))]
    X = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
    Yr, Lr = oracle.flow_apply(layers, X)
    dev = [[torch.from_numpy(np.ascontiguousarray(np.asarray(p).reshape(D, -1, order="F").T)).cuda()
            for p in ps] for _, ps in layers]
    lt = [(op, (np.asarray(ps[0]).reshape(D, -1, order="F").shape[1] if op == 5 else 0), [t.data_ptr() for t in dv])
          for (op, ps), dv in zip(layers, dev)]
    # in place + accumulate onto 1.5
    buf = torch.from_numpy(np.ascontiguousarray(X.T)).cuda()
    lad = torch.full((N,), 1.5, dtype=torch.float32, device="cuda")
    assert _raw_apply(enf, 0, D, N, buf.data_ptr(), D, buf.data_ptr(), D, lad.data_ptr(), 1, lt) == 0
    torch.cuda.synchronize()
    assert_flow_close(buf.cpu().numpy().T, lad.cpu().numpy() - 1.5, Yr, Lr, np.float32, what="in-place")
    # strided: ldx = D + 3, ldy = D + 5 (generic kernel)
    Xs = torch.zeros((N, D + 3), dtype=torch.float32, device="cuda")
    Xs[:, :D] = torch.from_numpy(np.ascontiguousarray(X.T)).cuda()
    Ys = torch.zeros((N, D + 5), dtype=torch.float32, device="cuda")
    assert _raw_apply(enf, 0, D, N, Xs.data_ptr(), D + 3, Ys.data_ptr(), D + 5, lad.data_ptr(), 0, lt) == 0
    torch.cuda.synchronize()
    assert_flow_close(Ys[:, :D].cpu().numpy().T, lad.cpu().numpy(), Yr, Lr, np.float32, what="strided")
    # misaligned base pointer (4 bytes off a 16-B boundary): generic kernel
    raw = torch.zeros(N * D + 1, dtype=torch.float32, device="cuda")
    raw[1:] = torch.from_numpy(np.ascontiguousarray(X.T)).cuda().reshape(-1)
    Ym = torch.zeros_like(raw)
    assert _raw_apply(enf, 0, D, N, raw.data_ptr() + 4, D, Ym.data_ptr() + 4, D, None, 0, lt) == 0
    torch.cuda.synchronize()
    assert col_err(Ym[1:].reshape(N, D).cpu().numpy().T, Yr) < 1e-5
    # errors: partial overlap, bad op, N == 0 no-op
    assert _raw_apply(enf, 0, D, N, buf.data_ptr(), D, buf.data_ptr() + 4, D, None, 0, lt) == 1
    assert _raw_apply(enf, 0, D, N, buf.data_ptr(), D, Ys.data_ptr(), D, None, 0, [(9, 0, [0])]) == 1
    assert _raw_apply(enf, 0, D, 0, None, D, None, D, None, 0, lt) == 0


def test_edge_values_fp32(enf, gpu, oracle):
    """Huge, infinite and NaN inputs follow the reference's fp32 semantics (prod-overflow rare path)."""
    D = 4
    vals = np.float32([0.0, -0.0, 1e-30, 1e10, -1e10, 3e19, -3e38, np.inf, -np.inf, np.nan, 5.0, -7.0])
    N = 64
    X = np.zeros((D, N), np.float32)
    X.flat[: vals.size] = vals
    X.flat[vals.size: 2 * vals.size] = vals[::-1]
    X = np.asfortranarray(X)
    params = [np.float32([0.1, -0.2, 0.3, 0.0]), np.float32([1, 2, 0.5, 1]), np.float32([0, 0.1, -0.1, 0]),
              np.float32([1, 0.5, 2, 1])]
    Yr, Lr = oracle.flow_apply([(3, params)], X)
    Y, L = enf.with_logabsdet_jacobian(enf.JohnsonTrafo(*params), colmajor_cuda(X))
    Y, L = to_np(Y), to_np(L).reshape(-1)
    assert np.array_equal(np.isnan(Y), np.isnan(Yr)) and np.array_equal(np.isnan(L), np.isnan(Lr))
    fin = np.isfinite(Yr)
    assert np.array_equal(np.isinf(Y), np.isinf(Yr)) and np.all(np.sign(Y[~fin & ~np.isnan(Yr)]) ==
                                                                 np.sign(Yr[~fin & ~np.isnan(Yr)]))
    assert col_err(np.where(fin, Y, 0), np.where(fin, Yr, 0)) < 1e-5
    finl = np.isfinite(Lr)
    assert np.array_equal(np.isinf(L), np.isinf(Lr))
    assert ladj_err(L[finl], Lr[finl]) < 1e-5


def test_zero_samples_and_empty_flow(enf, gpu):
    import torch

    X = torch.zeros((3, 0), dtype=torch.float32, device="cuda")
    Y, L = enf.with_logabsdet_jacobian(enf.JohnsonTrafo(np.float32([1, 1, 1]), 1, 0, 1), X)
    assert Y.shape == (3, 0) and L.shape == (1, 0)


def test_full_size_round_trip_config3(enf, gpu):
    """Config 3 at full size (D=32, N=1e7, fp32): size-independent properties -- inverse(f)(f(X)) == X
    and ladj(inverse) == -ladj -- plus oracle parity on a strided sample of columns."""
    import torch

    import oracle as orc

    rng = np.random.default_rng(2026)
    D, N = 32, 10_000_000
    layers = []
    for _ in range(4):
        layers += [(5, rand_params(rng, 5, D, np.float32)), (3, rand_params(rng, 3, D, np.float32))]
    f = make_flow(enf, layers)
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    X = torch.randn((N, D), generator=g, device="cuda", dtype=torch.float32).t()
    Y, L = enf.with_logabsdet_jacobian(f, X)
    X2, L2 = enf.with_logabsdet_jacobian(enf.inverse(f), Y)
    # round trip, checked on the GPU in chunks to bound host memory
    worst = 0.0
    for c0 in range(0, N, 1_000_000):
        a, b = X[:, c0:c0 + 1_000_000], X2[:, c0:c0 + 1_000_000]
        scale = a.abs() + a.abs().amax(dim=0, keepdim=True)
        worst = max(worst, float(((b - a).abs() / scale).max()))
    assert worst < 1e-4, worst
    el = float(((L2 + L).abs() / (L.abs() + 1)).max())
    assert el < 1e-5, el
    idx = np.arange(0, N, 997)
    Xs = np.asfortranarray(X[:, idx].cpu().numpy())
    check_vs_oracle(orc, layers, Xs, Y[:, idx].cpu().numpy(), L[0, idx].cpu().numpy(), np.float32,
                    what="config3 sample")


def _hj_layers(rng, D, pairs):
    layers = []
    for _ in range(pairs):
        layers += [(5, rand_params(rng, 5, D, np.float32)), (3, rand_params(rng, 3, D, np.float32))]
    return layers


@pytest.mark.parametrize("D", [32, 64, 128, 24, 36, 100])
@pytest.mark.parametrize("pairs", [1, 2, 3, 4, 8, 9])
def test_hj_program_pairs_vs_oracle(enf, gpu, oracle, D, pairs):
    """The compiled (J∘H)^n program (enf_flow_hj.hip; n <= 8, n = 9 runs on the interpreter):
    forward + ladj, plain call f(X) and multi-tile waves (N > resident tiles) against the oracle.
    D = 24 / 36 / 100 run on the padded layout (32 / 64 / 128, rows past D inert; round 3)."""
    rng = np.random.default_rng(100 * D + pairs)
    layers = _hj_layers(rng, D, pairs)
    N = 300_007
    X = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
    f = make_flow(enf, layers)
    Y, L = enf.with_logabsdet_jacobian(f, colmajor_cuda(X))
    check_vs_oracle(oracle, layers, X, to_np(Y), to_np(L), np.float32, what=f"hj D{D} n{pairs}")
    assert np.array_equal(to_np(f(colmajor_cuda(X))), to_np(Y))


@pytest.mark.parametrize("D", [32, 100])
def test_hj_program_accumulate_inplace(enf, gpu, oracle, D):
    """accumulate_ladj = 1 and Y aliasing X through the raw C ABI on the compiled program (D = 100: the
    padded layout)."""
    import torch

    rng = np.random.default_rng(5)
    N = 50_001
    layers = _hj_layers(rng, D, 4)
    X = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
    Yr, Lr = oracle.flow_apply(layers, X)
    dev = [[torch.from_numpy(np.ascontiguousarray(p)).cuda() for p in ps] for _, ps in layers]
    lt = [(op, 1 if op == 5 else 0, [t.data_ptr() for t in ts]) for (op, _), ts in zip(layers, dev)]
    buf = colmajor_cuda(X).t().contiguous()  # N x D row-major == D x N column-major
    L0 = torch.full((N,), 3.25, dtype=torch.float32, device="cuda")
    assert _raw_apply(enf, 0, D, N, buf.data_ptr(), D, buf.data_ptr(), D, L0.data_ptr(), 1, lt) == 0
    torch.cuda.synchronize()
    assert col_err(buf.cpu().numpy().T, Yr) < 1e-5
    assert ladj_err(L0.cpu().numpy() - 3.25, Lr) < 1e-5


@pytest.mark.parametrize("D", [32, 64, 128, 24, 100])
def test_hj_program_exact_redo_edge_values(enf, gpu, oracle, D):
    """Columns with huge, infinite and NaN entries inside the compiled program: the tile is redone
    with the exact-range form; everything else in the batch is unaffected."""
    rng = np.random.default_rng(11)
    layers = _hj_layers(rng, D, 4)
    N = 4096
    X = rng.standard_normal((D, N)).astype(np.float32)
    bad = [7, 100, 101, 2000, 4095]
    X[3, 7] = 3e30
    X[0, 100] = -1e25
    X[5, 101] = np.inf
    X[D - 1, 2000] = np.nan
    X[:, 4095] = 1e3  # moderate but large |z|: product of q overflows, the fast form would lose it
    X = np.asfortranarray(X)
    Yr, Lr = oracle.flow_apply(layers, X)
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    Y, L = to_np(Y), to_np(L).reshape(-1)
    assert np.array_equal(np.isnan(Y), np.isnan(Yr)) and np.array_equal(np.isnan(L), np.isnan(Lr))
    assert np.array_equal(np.isinf(Y), np.isinf(Yr)) and np.array_equal(np.isinf(L), np.isinf(Lr))
    fin = np.isfinite(Yr)
    assert col_err(np.where(fin, Y, 0), np.where(fin, Yr, 0)) < 1e-5
    finl = np.isfinite(Lr)
    assert ladj_err(L[finl], Lr[finl]) < 1e-5
    good = np.setdiff1d(np.arange(N), bad)
    check_vs_oracle(oracle, layers, np.asfortranarray(X[:, good]), Y[:, good], L[good], np.float32, what="redo")


@pytest.mark.parametrize("chunk", [0, 1000, 4097, 70_001])
def test_host_streaming_equals_device_path(enf, gpu, oracle, chunk):
    """enf_flow_apply_host (host-resident batch, chunked through a device ring) gives exactly the
    device path's results: the same kernels per column, any chunking; in place on the host too; and
    (one chunking) the oracle's results on the first two chunks and the ragged tail."""
    rng = np.random.default_rng(31)
    D, N = 32, 200_003
    layers = _hj_layers(rng, D, 4)
    X = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
    f = make_flow(enf, layers)
    Yd, Ld = enf.with_logabsdet_jacobian(f, colmajor_cuda(X))
    Yh, Lh = enf.stream_with_logabsdet_jacobian(f, X, chunk_cols=chunk)
    assert np.array_equal(Yh, to_np(Yd)) and np.array_equal(Lh, to_np(Ld))
    Xi = X.copy(order="F")
    Yi, Li = enf.stream_with_logabsdet_jacobian(f, Xi, chunk_cols=chunk, out=Xi)
    assert Yi is Xi and np.array_equal(Xi, Yh) and np.array_equal(Li, Lh)
    if chunk == 4097:  # and against the oracle (not only HIP against HIP): the first two chunks and the ragged tail
        cols = np.r_[0:2 * chunk, N - 3000:N]
        check_vs_oracle(oracle, layers, np.asfortranarray(X[:, cols]), Yh[:, cols],
                        Lh[:, cols], np.float32, what="host streaming fp32")


def test_host_streaming_fp64_mixed_ops(enf, gpu, oracle):
    """Host streaming on the interpreter path (fp64, every op), against the oracle."""
    rng = np.random.default_rng(32)
    D, N = 5, 30_011
    layers = [(op, rand_params(rng, op, D, np.float64, K=2 if op == 5 else 1)) for op in (0, 5, 2, 3, 1, 4, 5, 3)]
    X = np.asfortranarray(rng.standard_normal((D, N)))
    Y, L = enf.stream_with_logabsdet_jacobian(make_flow(enf, layers), X, chunk_cols=7001)
    check_vs_oracle(oracle, layers, X, Y, L, np.float64, what="host streaming fp64")


@pytest.mark.parametrize("D", [2, 32])
def test_fp64_asinh_wide_range(enf, gpu, oracle, D):
    """The fp64 Johnson layer y = gamma + delta*asinh(z) (johnson_trafo.jl:31) with gamma = 0,
    delta = 1 against libm elementwise, 1e-12 relative, over 1e-320 .. 1e308, signed zeros (0 + -0
    is +0, as in the reference), Inf and NaN."""
    rng = np.random.default_rng(5)
    v = np.concatenate([np.logspace(-320, 308, 3000), rng.uniform(0.2, 0.3, 500), rng.uniform(9e3, 1.1e4, 500),
                        rng.standard_normal(1000) * 10, [0.0, 5e-324, 1e-300, 0.25, 0.2526, 1e4, 1.0000001e4,
                                                          1.7e308, np.inf, np.nan]])
    v = np.concatenate([v, -v])
    n = (v.size + D - 1) // D * D
    x = np.zeros(n)
    x[:v.size] = v
    X = np.asfortranarray(x.reshape(-1, D).T)
    one = np.ones(D)
    layers = [(3, [np.zeros(D), one, np.zeros(D), one])]  # y = asinh(x)
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    Y = to_np(Y)
    ref = 0.0 + 1.0 * np.arcsinh(X)
    fin = np.isfinite(ref) & (ref != 0)
    assert np.all(np.abs(Y[fin] - ref[fin]) <= 1e-12 * np.abs(ref[fin]))
    assert np.array_equal(np.isnan(Y), np.isnan(ref))
    inf = np.isinf(ref)
    assert np.array_equal(Y[inf], ref[inf])
    zero = ref == 0
    assert np.array_equal(np.signbit(Y[zero]), np.signbit(ref[zero]))
    Yr, Lr = oracle.flow_apply(layers, X)
    assert np.array_equal(np.isnan(to_np(L)).reshape(-1), np.isnan(Lr).reshape(-1))


@pytest.mark.parametrize("D", [2, 32])
def test_fp64_johnson_ulp_and_large_z_ladj(enf, gpu, oracle, D):
    """asinh64 (enf_math64.h) within 3 ulp of the correctly rounded asinh (x87 extended precision
    of the oracle's flow_apply_hi as the stand-in), and the ladj of columns whose 1 + z^2 product
    overflows double while each factor does not (|z| ~ 1e100: the kernel's per-segment product
    falls back to a sum of logs) equal to the reference's per-element sum; factors that overflow
    themselves (|z| > 1.4e154) give -Inf as the reference's log(1/sqrt(Inf)) does."""
    rng = np.random.default_rng(11)
    N = 4096
    X = rng.standard_normal((D, N)) * np.exp(rng.uniform(-30, 30, (D, N)))
    X[:, :64] = rng.uniform(0.5, 2.0, (D, 64)) * 1e100 * rng.choice([-1, 1], (D, 64))
    X[:, 64:80] = 1e200
    X = np.asfortranarray(X)
    one = np.ones(D)
    layers = [(3, [np.zeros(D), one, np.zeros(D), one])]  # y = asinh(x), ladj = -sum log(1+x^2)/2
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    Y, L = to_np(Y), to_np(L).reshape(-1)
    Yh, Lh = oracle.flow_apply_hi(layers, X)
    assert np.all(np.abs(Y - Yh) <= 3 * np.spacing(np.abs(Yh)))
    Yr, Lr = oracle.flow_apply(layers, X)
    assert np.all(np.isneginf(Lr[64:80])) and np.array_equal(L[64:80], Lr[64:80])
    fin = np.isfinite(Lr)
    assert fin[:64].all()
    assert np.all(np.abs(L[fin] - Lr[fin]) <= 1e-12 * (np.abs(Lr[fin]) + 1))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("D", [6, 12, 20, 100])
def test_padded_fragment_path(enf, gpu, oracle, dtype, D):
    """D a multiple of 16/sizeof(T) but not a power of two runs on the fragment kernel laid out as the
    next power of two (csrc/enf_internal.h frag_pad_dim): every op it takes (ScaleShift, Johnson,
    JohnsonInv, chained Householder) in one flow, tails of the wave tile, in place + accumulate through
    the raw C ABI, and ladj = NULL."""
    import torch

    if dtype == np.float32 and D % 4:
        pytest.skip("fp32 fragments hold 4 rows")
    rng = np.random.default_rng(D)
    layers = [(0, rand_params(rng, 0, D, dtype)), (5, rand_params(rng, 5, D, dtype, K=3)),
              (3, rand_params(rng, 3, D, dtype)), (5, rand_params(rng, 5, D, dtype)), (4, rand_params(rng, 4, D, dtype)),
              (3, rand_params(rng, 3, D, dtype))]
    for N in (1, 63, 4097, 70_001):
        X = np.asfortranarray(rng.standard_normal((D, N)).astype(dtype))
        Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
        check_vs_oracle(oracle, layers, X, to_np(Y), to_np(L), dtype, what=f"padded D{D} N{N}")
    dev = [[torch.from_numpy(np.ascontiguousarray(np.asarray(p).reshape(D, -1, order="F").T)).cuda() for p in ps]
           for _, ps in layers]
    lt = [(op, (np.asarray(ps[0]).reshape(D, -1, order="F").shape[1] if op == 5 else 0), [t.data_ptr() for t in dv])
          for (op, ps), dv in zip(layers, dev)]
    code = enf._lib.ENF_F32 if dtype == np.float32 else enf._lib.ENF_F64
    buf = torch.from_numpy(np.ascontiguousarray(X.T)).cuda()
    lad = torch.full((N,), 1.5, dtype=buf.dtype, device="cuda")
    assert _raw_apply(enf, code, D, N, buf.data_ptr(), D, buf.data_ptr(), D, lad.data_ptr(), 1, lt) == 0
    torch.cuda.synchronize()
    # same kernel arithmetic as the out-of-place call above: Y bit for bit, ladj + 1.5 up to its rounding
    Yo, Lo = to_np(Y), to_np(L).reshape(-1)
    assert np.array_equal(buf.cpu().numpy().T, Yo)
    eps = np.finfo(dtype).eps
    assert np.all(np.abs(lad.cpu().numpy() - (Lo + 1.5)) <= 2 * eps * (np.abs(Lo) + 1.5))
    Y2 = torch.zeros_like(buf)
    X2 = torch.from_numpy(np.ascontiguousarray(X.T)).cuda()
    assert _raw_apply(enf, code, D, N, X2.data_ptr(), D, Y2.data_ptr(), D, None, 0, lt) == 0
    torch.cuda.synchronize()
    assert np.array_equal(Y2.cpu().numpy(), buf.cpu().numpy())
