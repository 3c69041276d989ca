"""Config 2: JohnsonTrafo ∘ HouseholderTrafo at D = 2 in fp64 runs on its own
compiled kernel (csrc/enf_flow_d2.hip). Parity against the oracle (fp64 rtol 1e-12, BASELINE.json) over
every tail shape of its 128-column wave tile, elementwise accuracy over a wide input range, edge
values, in place / accumulate / no-ladj calls through the raw C ABI."""
import numpy as np
import pytest

from parity import check_vs_oracle, colmajor_cuda, make_flow, rand_params, to_np
from test_gpu_parity import _raw_apply

pytestmark = pytest.mark.gpu


def c2_layers(rng, dtype=np.float64):
    return [(5, rand_params(rng, 5, 2, dtype)), (3, rand_params(rng, 3, 2, dtype))]


@pytest.mark.parametrize("N", [1, 2, 63, 64, 65, 127, 128, 129, 255, 256, 257, 4097, 131_071, 1_000_003])
def test_c2_vs_oracle(enf, gpu, oracle, N):
    rng = np.random.default_rng(N)
    layers = c2_layers(rng)
    X = np.asfortranarray(rng.standard_normal((2, N)))
    f = make_flow(enf, layers)
    Y, L = enf.with_logabsdet_jacobian(f, colmajor_cuda(X))
    check_vs_oracle(oracle, layers, X, to_np(Y), to_np(L), np.float64, what=f"C2 N{N}")
    # f(X) (no ladj) gives the same Y
    assert np.array_equal(to_np(f(colmajor_cuda(X))), to_np(Y))


def test_c2_elementwise_wide_range(enf, gpu, oracle):
    """Elementwise against the oracle's fp64 evaluation of the same formulas: |y - y_ref| <= 1e-12 of
    the element's scale |gamma| + |delta asinh z| (the Householder step is shared arithmetic), the
    ladj within 1e-12 (|l| + 1); inputs over 1e-300 .. 1e300, both signs, zeros, Inf, NaN."""
    rng = np.random.default_rng(3)
    v = np.concatenate([np.logspace(-300, 300, 4000), rng.standard_normal(2000) * 3, [0.0, 1e-320, np.inf, np.nan]])
    v = np.concatenate([v, -v])
    rng.shuffle(v)
    X = np.asfortranarray(v[: v.size // 2 * 2].reshape(-1, 2).T)
    layers = c2_layers(rng)
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    Y, L = to_np(Y), to_np(L).reshape(-1)
    Yr, Lr = oracle.flow_apply(layers, X)
    Lr = Lr.reshape(-1)
    g = layers[1][1][0][:, None]
    scale = np.abs(g) + np.abs(Yr - g)
    fin = np.isfinite(Yr)
    assert np.all(np.abs(Y[fin] - Yr[fin]) <= 1e-12 * scale[fin])
    assert np.array_equal(np.isnan(Y), np.isnan(Yr))
    assert np.array_equal(Y[np.isinf(Yr)], Yr[np.isinf(Yr)])
    lf = np.isfinite(Lr)
    assert np.all(np.abs(L[lf] - Lr[lf]) <= 1e-12 * (np.abs(Lr[lf]) + 1))
    assert np.array_equal(np.isnan(L), np.isnan(Lr))
    assert np.array_equal(L[np.isinf(Lr)], Lr[np.isinf(Lr)])


def test_c2_capi_inplace_accumulate(enf, gpu, oracle):
    """Raw C ABI: in place (Y == X) with accumulate_ladj onto 1.5, and ladj = NULL."""
    import torch

    rng = np.random.default_rng(17)
    N = 300_001
    layers = c2_layers(rng)
    X = np.asfortranarray(rng.standard_normal((2, N)))
    Yr, Lr = oracle.flow_apply(layers, X)
    dev = [[torch.from_numpy(np.ascontiguousarray(np.asarray(p).reshape(2, -1, order="F").T)).cuda() for p in ps]
           for _, ps in layers]
    lt = [(op, 1 if op == 5 else 0, [t.data_ptr() for t in dv]) for (op, _), dv in zip(layers, dev)]
    f64 = enf._lib.ENF_F64
    buf = torch.from_numpy(np.ascontiguousarray(X.T)).cuda()
    lad = torch.full((N,), 1.5, dtype=torch.float64, device="cuda")
    assert _raw_apply(enf, f64, 2, N, buf.data_ptr(), 2, buf.data_ptr(), 2, lad.data_ptr(), 1, lt) == 0
    torch.cuda.synchronize()
    Y = buf.cpu().numpy().T
    L = lad.cpu().numpy()
    scale = np.abs(Yr) + np.abs(Yr).max(axis=0)
    assert np.all(np.abs(Y - Yr) <= 1e-12 * scale)
    assert np.all(np.abs((L - 1.5) - Lr.reshape(-1)) <= 1e-12 * (np.abs(Lr.reshape(-1)) + 2))
    Y2 = torch.zeros_like(buf)
    X2 = torch.from_numpy(np.ascontiguousarray(X.T)).cuda()
    assert _raw_apply(enf, f64, 2, N, X2.data_ptr(), 2, Y2.data_ptr(), 2, None, 0, lt) == 0
    torch.cuda.synchronize()
    assert np.array_equal(Y2.cpu().numpy().T, Y)
