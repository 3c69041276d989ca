"""GPU: the input VJP of a flow (enf_flow_vjp, host mirror flow_vjp).

The reference's rrules for the reflections (src/householder_trafo.jl:43-54 householder_trafo_pullback_x,
:105-124 chained_householder_trafo_pullback_x) are tested there against ForwardDiff Jacobians of the
explicit Householder matrices (test/test_householder_trafo.jl:27-33,49-55). Here: dX against the
explicit matrix product J' dY for single and chained reflections, and for every transform and
mixed compositions against central differences of the oracle's fp64 (Y, ladj); the parameter VJP
against central differences and against enf_flow_negll_grad (the loss is the cotangent dY = Y,
dladj = -1).
"""

import numpy as np
import pytest

from parity import colmajor_cuda, make_flow, rand_params, to_np

pytestmark = pytest.mark.gpu


def householder_matrix(v):
    v = np.asarray(v, np.float64)
    return np.eye(v.size) - 2.0 * np.outer(v, v) / (v @ v)


def cotangent_fd(oracle, layers, X, dY, dl, h=1e-6):
    """Central differences of S_j(X) = <dY_j, Y_j> + dl_j * ladj_j for every input coordinate: one
    row d of all columns is perturbed at once (the columns are independent)."""
    D, N = X.shape
    out = np.empty((D, N))
    for d in range(D):
        Xp, Xm = X.copy(), X.copy()
        hd = h * np.maximum(1.0, np.abs(X[d]))
        Xp[d] += hd
        Xm[d] -= hd
        Yp, Lp = oracle.flow_apply(layers, np.asfortranarray(Xp))
        Ym, Lm = oracle.flow_apply(layers, np.asfortranarray(Xm))
        Sp = (dY * Yp).sum(0) + dl * Lp
        Sm = (dY * Ym).sum(0) + dl * Lm
        out[d] = (Sp - Sm) / (2 * hd)
    return out


@pytest.mark.parametrize("D,k", [(5, 1), (5, 3), (32, 4), (64, 2)])
def test_vjp_householder_vs_explicit_matrices(enf, gpu, D, k):
    """dX = (H_k ... H_1)' dY with the explicit Householder matrices (householder_trafo_pullback_x,
    chained_householder_trafo_pullback_x); a reflection has ladj = 0, so dladj does not contribute."""
    rng = np.random.default_rng(100 + D + k)
    V = rng.standard_normal((D, k))
    f = enf.HouseholderTrafo(V if k > 1 else V[:, 0])
    X = rng.standard_normal((D, 333))
    dY = rng.standard_normal((D, 333))
    J = np.eye(D)
    for i in range(k):
        J = householder_matrix(V[:, i]) @ J
    want = J.T @ dY
    for dl in (None, rng.standard_normal(333)):
        dX, _ = enf.flow_vjp(f, colmajor_cuda(X), colmajor_cuda(dY), dl)
        assert np.allclose(to_np(dX), want, rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("op", [0, 1, 2, 3, 4, 5])
def test_vjp_each_transform_vs_central_differences(enf, gpu, oracle, op):
    rng = np.random.default_rng(200 + op)
    D, N = 6, 97
    layers = [(op, rand_params(rng, op, D, np.float64, K=2))]
    X = np.asfortranarray(rng.standard_normal((D, N)))
    dY, dl = rng.standard_normal((D, N)), rng.standard_normal(N)
    dX, _ = enf.flow_vjp(make_flow(enf, layers), colmajor_cuda(X), colmajor_cuda(dY), dl)
    fd = cotangent_fd(oracle, layers, X, dY, dl)
    err = np.abs(to_np(dX) - fd) / (np.abs(fd) + 1e-3 * np.abs(fd).max())
    assert err.max() < 2e-6, (op, err.max())


@pytest.mark.parametrize("D", [3, 8, 32])
def test_vjp_composed_flow_and_param_cotangent(enf, gpu, oracle, D):
    """A mixed composition (all six transforms, a chained reflection): dX against central differences;
    the parameter VJP against central differences of sum_j S_j over a parameter subset."""
    from test_gpu_train import flat, mixed_layers, unflat

    rng = np.random.default_rng(300 + D)
    layers = mixed_layers(rng, D, np.float64)
    N = 211
    X = np.asfortranarray(0.8 * rng.standard_normal((D, N)))
    dY, dl = rng.standard_normal((D, N)), rng.standard_normal(N)
    f = make_flow(enf, layers)
    dX, grads = enf.flow_vjp(f, colmajor_cuda(X), colmajor_cuda(dY), dl, param_grads=True)
    fd = cotangent_fd(oracle, layers, X, dY, dl)
    err = np.abs(to_np(dX) - fd) / (np.abs(fd) + 1e-3 * np.abs(fd).max())
    assert err.max() < 2e-6, err.max()
    G = np.concatenate([np.asarray(a, np.float64).reshape(-1, order="F") for per in grads for a in per])
    th0 = flat(layers, D)
    assert G.shape == th0.shape
    scale = np.abs(G).max()

    def S(th):
        Y, L = oracle.flow_apply(unflat(layers, th, D), X)
        return float((dY * Y).sum() + dl @ L)

    for i in rng.choice(th0.size, min(20, th0.size), replace=False):
        h = 1e-6 * max(1.0, abs(th0[i]))
        tp, tm = th0.copy(), th0.copy()
        tp[i] += h
        tm[i] -= h
        fdi = (S(tp) - S(tm)) / (2 * h)
        assert abs(G[i] - fdi) < 1e-5 * (abs(fdi) + 1e-3 * scale), (i, G[i], fdi)


def test_vjp_loss_cotangent_equals_negll_gradient(enf, gpu):
    """With dY = Y and dladj = -1 the pullback is the gradient of N * negll: the parameter VJP equals
    mvnormal_negll_trafograd * N (same kernel arithmetic), and dX is dS/dX."""
    from test_gpu_train import mixed_layers

    rng = np.random.default_rng(7)
    D, N = 8, 1500
    layers = mixed_layers(rng, D, np.float64)
    f = make_flow(enf, layers)
    X = colmajor_cuda(np.asfortranarray(rng.standard_normal((D, N))))
    Y, L = enf.with_logabsdet_jacobian(f, X)
    _, gvjp = enf.flow_vjp(f, X, Y, -np.ones(N), param_grads=True)
    _, gl = enf.mvnormal_negll_trafograd(f, X)
    for a, b in zip(gvjp, gl):
        for p, q in zip(a, b):
            assert np.allclose(np.asarray(p) / N, np.asarray(q), rtol=1e-12, atol=1e-14)


def test_vjp_fp32_matches_fp64(enf, gpu):
    from test_gpu_train import mixed_layers

    rng = np.random.default_rng(8)
    D, N = 32, 4097
    L64 = mixed_layers(rng, D, np.float64)
    L32 = [(op, [np.asarray(p, np.float32) for p in ps]) for op, ps in L64]
    X = rng.standard_normal((D, N))
    dY, dl = rng.standard_normal((D, N)), rng.standard_normal(N)
    d64, g64 = enf.flow_vjp(make_flow(enf, L64), colmajor_cuda(X), colmajor_cuda(dY), dl, param_grads=True)
    d32, g32 = enf.flow_vjp(make_flow(enf, L32), colmajor_cuda(X.astype(np.float32)),
                            colmajor_cuda(dY.astype(np.float32)), dl.astype(np.float32), param_grads=True)
    a, b = to_np(d64), to_np(d32).astype(np.float64)
    assert np.abs(a - b).max() < 1e-3 * np.abs(a).max()  # fp32 through 8 layers, |J| up to ~500
    for p64, p32 in zip(g64, g32):
        for u, v in zip(p64, p32):
            u, v = np.ravel(u), np.ravel(v)
            assert np.abs(u - v).max() < 1e-3 * (np.abs(u).max() + 1e-3)


def test_vjp_capi_in_place_null_ladj_and_errors(enf, gpu):
    """Through the C ABI: dX aliasing dY (same leading dimension), dladj = NULL, ragged N, no workspace
    without dparams; dX aliasing X is refused."""
    import torch

    rng = np.random.default_rng(9)
    D, N, ld = 5, 301, 7
    V = rng.standard_normal((D, 2))
    f = enf.HouseholderTrafo(V)
    Xs = torch.from_numpy(rng.standard_normal((N, ld))).cuda()   # column j at j*ld
    G = torch.from_numpy(rng.standard_normal((N, ld))).cuda()
    want = (householder_matrix(V[:, 1]) @ householder_matrix(V[:, 0])).T @ G.cpu().numpy()[:, :D].T
    st = enf.FlowState(f, D, torch.float64, Xs.device)
    L = enf._lib.lib()
    rc = L.enf_flow_vjp(enf._lib.ENF_F64, D, N, Xs.data_ptr(), ld, G.data_ptr(), ld, None, st.layers(), 1,
                        G.data_ptr(), ld, None, None, 0, None)
    assert rc == 0
    torch.cuda.synchronize()
    assert np.allclose(G.cpu().numpy()[:, :D].T, want, rtol=1e-13, atol=1e-13)
    rc = L.enf_flow_vjp(enf._lib.ENF_F64, D, N, Xs.data_ptr(), ld, G.data_ptr(), ld, None, st.layers(), 1,
                        Xs.data_ptr(), ld, None, None, 0, None)
    assert rc == enf._lib.ENF_ERR_INVALID
    dp = torch.zeros(st.nparams, dtype=torch.float64, device="cuda")
    rc = L.enf_flow_vjp(enf._lib.ENF_F64, D, N, Xs.data_ptr(), ld, G.data_ptr(), ld, None, st.layers(), 1,
                        G.data_ptr(), ld, dp.data_ptr(), None, 0, None)
    assert rc == enf._lib.ENF_ERR_INVALID  # dparams needs the workspace
