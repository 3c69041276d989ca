"""GPU parity of the dense-Householder MFMA kernel (enf_flow_wy.hip): a chained HouseholderTrafo with
k >= 8 reflections at D in {32, 64} runs as one orthogonal D x D product on the matrix cores
(SURVEY.md §8(f) item 3), the other layers of the flow elementwise in the same launch. Checked
against the oracle's reflection-by-reflection restatement of chained_householder_trafo
(src/householder_trafo.jl:71-78) in the same precision and in high precision (tests/parity.py)."""
import numpy as np
import pytest

from parity import RTOL, check_vs_oracle, col_err, colmajor_cuda, ladj_err, make_flow, rand_params, to_np

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("D", [32, 64])
@pytest.mark.parametrize("K", [8, 17, "D", "D+5", "2D+3"])
def test_dense_householder_vs_oracle(enf, gpu, oracle, dtype, D, K):
    """Pure chained HouseholderTrafo; k > D is split into dense steps of <= D reflections; N has a
    partial last tile."""
    k = {"D": D, "D+5": D + 5, "2D+3": 2 * D + 3}.get(K, K)
    rng = np.random.default_rng(100 * D + k)
    layers = [(5, rand_params(rng, 5, D, dtype, K=k))]
    X = np.asfortranarray(rng.standard_normal((D, 4099)).astype(dtype))
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    check_vs_oracle(oracle, layers, X, to_np(Y), to_np(L), dtype, what=f"H(k={k}) D{D}")
    assert np.array_equal(to_np(L), np.zeros((1, X.shape[1]), dtype=dtype))


def _inverse_layers(layers):
    """InverseFunctions.inverse of a composition as layer algebra (scale_shift_trafo.jl:26-30,
    center_stretch.jl:45,69, johnson_trafo.jl:82,107, householder_trafo.jl:153-154)."""
    out = []
    for op, ps in reversed(layers):
        if op == 0:
            a, b = ps
            ainv = (1 / a).astype(a.dtype)
            out.append((0, [ainv, (-ainv * b).astype(a.dtype)]))
        elif op in (1, 2, 3, 4):
            out.append(({1: 2, 2: 1, 3: 4, 4: 3}[op], ps))
        else:
            out.append((5, [np.asfortranarray(np.asarray(ps[0])[:, ::-1])]))
    return out


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("D", [32, 64])
def test_dense_householder_in_composed_flow(enf, gpu, oracle, dtype, D):
    """Every op around two dense steps and a single reflection, in one launch."""
    rng = np.random.default_rng(7 * D)
    ops = [(0, 1), (5, D), (3, 1), (1, 1), (5, 1), (4, 1), (5, 12), (2, 1), (3, 1)]
    layers = [(op, rand_params(rng, op, D, dtype, K=k)) for op, k in ops]
    for N in (1, 31, 33, 20_011):
        X = np.asfortranarray((0.7 * rng.standard_normal((D, N))).astype(dtype))
        f = make_flow(enf, layers)
        Y, L = enf.with_logabsdet_jacobian(f, colmajor_cuda(X))
        check_vs_oracle(oracle, layers, X, to_np(Y), to_np(L), dtype, what=f"composed D{D} N{N}")
        # the inverse flow (host-side parameter algebra) against the oracle on the same inverse
        # layers: fp32 Center layers may overflow on some columns, as the reference does
        Yn = to_np(Y)
        X2, L2 = enf.with_logabsdet_jacobian(enf.inverse(f), Y)
        check_vs_oracle(oracle, _inverse_layers(layers), Yn, to_np(X2), to_np(L2), dtype, what=f"inverse D{D} N{N}")


def test_dense_householder_inplace_accumulate(enf, gpu, oracle):
    """C ABI: X == Y in place and accumulate_ladj on the dense kernel."""
    import torch

    from test_gpu_parity import _raw_apply

    rng = np.random.default_rng(5)
    D, N = 32, 10_007
    layers = [(5, rand_params(rng, 5, D, np.float32, K=24)), (3, rand_params(rng, 3, D, np.float32))]
    X = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
    Yr, Lr = oracle.flow_apply(layers, X)
    dev = [[torch.from_numpy(np.ascontiguousarray(np.asarray(p).reshape(D, -1, order="F").T)).cuda()
            for p in ps] for _, ps in layers]
    lt = [(op, (np.asarray(ps[0]).reshape(D, -1, order="F").shape[1] if op == 5 else 0), [t.data_ptr() for t in dv])
          for (op, ps), dv in zip(layers, dev)]
    buf = torch.from_numpy(np.ascontiguousarray(X.T)).cuda()
    lad = torch.full((N,), -2.0, dtype=torch.float32, device="cuda")
    assert _raw_apply(enf, 0, D, N, buf.data_ptr(), D, buf.data_ptr(), D, lad.data_ptr(), 1, lt) == 0
    torch.cuda.synchronize()
    assert col_err(buf.cpu().numpy().T, Yr) < RTOL[np.dtype(np.float32)]
    assert ladj_err(lad.cpu().numpy() + 2.0, Lr) < RTOL[np.dtype(np.float32)]


def test_dense_householder_orthogonality_full_size(enf, gpu):
    """Size-independent property at 4e6 samples: a dense step preserves every column's norm, and
    H o H^-1 is the identity."""
    import torch

    rng = np.random.default_rng(9)
    D, N = 32, 4_000_000
    V = rand_params(rng, 5, D, np.float32, K=D)[0]
    f = enf.HouseholderTrafo(V)
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    X = torch.randn((N, D), device="cuda", generator=g).t()
    Y = f(X)
    nx, ny = torch.linalg.vector_norm(X.double(), dim=0), torch.linalg.vector_norm(Y.double(), dim=0)
    assert float(((ny - nx).abs() / nx).max()) < 3e-6
    X2 = enf.inverse(f)(Y)
    assert float(((X2 - X).abs().amax(dim=0) / X.abs().amax(dim=0)).max()) < 1e-5


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_dense_householder_nonfinite_columns(enf, gpu, oracle, dtype):
    """Columns with +-Inf / NaN entries come out as the reference's reflection chain makes them
    (all NaN from the second reflection on); the other columns of the tile are unaffected."""
    rng = np.random.default_rng(23)
    D = 32
    layers = [(5, rand_params(rng, 5, D, dtype, K=12)), (3, rand_params(rng, 3, D, dtype))]
    X = np.asfortranarray(rng.standard_normal((D, 300)).astype(dtype))
    X[3, 5] = np.inf
    X[0, 40] = -np.inf
    X[31, 41] = np.nan
    X[7, 299] = np.inf
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    Y, L = to_np(Y), to_np(L)
    Yr, Lr = oracle.flow_apply(layers, X)
    for c in (5, 40, 41, 299):
        assert np.isnan(Yr[:, c]).all() and np.isnan(Y[:, c]).all(), c
    assert np.array_equal(np.isnan(L), np.isnan(Lr.reshape(L.shape)))
    check_vs_oracle(oracle, layers, X, Y, L, dtype, what="non-finite columns")
