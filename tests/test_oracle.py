"""CPU: the oracle (CPU restatement of the reference) pinned by the reference's own known-answer
tests, its round-trip / Jacobian properties, and the exact mpmath golden vectors."""
import glob
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden_flow
from parity import RTOL, col_err, ladj_err


def julia_isapprox(a, b, T):
    """Julia's default isapprox: rtol = sqrt(eps(T))."""
    rtol = np.sqrt(np.finfo(T).eps)
    return abs(a - b) <= rtol * max(abs(a), abs(b))


def test_reference_kats(oracle):
    """test/test_center_stretch.jl:18-19, test/test_johnson_trafo.jl:21-22 (exact values by mpmath)."""
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        kats = json.load(f)
    for k in kats:
        T = np.dtype(k["T"]).type
        got = oracle.scalar(k["fn"], T, *k["args"])
        exact = float(k["exact"])
        if k["expected"] is not None:
            assert julia_isapprox(got, k["expected"], T), (k, got)
        # a few ulps of the result (log-type results: of max(|result|, 1))
        tol = 4 * np.finfo(T).eps * max(abs(exact), 1.0)
        assert abs(got - exact) <= tol, (k["fn"], got, exact)
        if "log_abs_derivative" in k:  # the ForwardDiff cross-checks at rtol 0.01
            assert abs(got - float(k["log_abs_derivative"])) <= 0.01 * abs(float(k["log_abs_derivative"]))


@pytest.mark.parametrize("dt", ["float64", "float32"])
def test_scalar_golden(oracle, dt):
    """Every scalar reference function on 160 random points, against mpmath (50 digits)."""
    z = np.load(os.path.join(GOLDEN, f"scalars_{dt}.npz"), allow_pickle=False)
    T = np.dtype(dt).type
    eps = np.finfo(T).eps
    for name in z.files:
        rows = z[name]
        for row in rows:
            args, exact = row[:-1], row[-1]
            got = oracle.scalar(name, T, *args)
            # formulas with cancellation (center_stretch's 1 - exp(|bx|), gamma + delta*asinh) lose
            # relative accuracy; measure against the size of the terms instead
            scale = max(abs(exact), 1.0)
            assert abs(got - exact) <= 64 * eps * scale, (name, args, got, exact)


FLOWS = sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, "*.npz")) if "scalars" not in f and "johnsonsu" not in f)


@pytest.mark.parametrize("name", FLOWS)
def test_flow_golden(oracle, name):
    """The batched reference algorithm (T precision) against the exact flows: the reference's own
    error, which is what the GPU is allowed up to K x (tests/parity.py); and the high-precision
    oracle (fp64 for fp32 data, x87 extended for fp64) against the exact values."""
    layers, X, Yx, Lx = load_golden_flow(name)
    Y, L = oracle.flow_apply(layers, X)
    rtol = RTOL[X.dtype]
    # the reference in its own precision is within 100x rtol even where it cancels (D = 1, 2)
    assert col_err(Y, Yx) < 100 * rtol and ladj_err(L, Lx) < 100 * rtol
    Yh, Lh = oracle.flow_apply_hi(layers, X)
    # (fixtures store the exact values rounded to float64: 1.1e-16 relative)
    assert col_err(Yh, Yx) < (1e-13 if X.dtype == np.float32 else 2.5e-16)
    assert ladj_err(Lh, Lx) < (1e-13 if X.dtype == np.float32 else 2.5e-16)


def test_round_trips(oracle):
    """test_center_stretch.jl:21-23, test_johnson_trafo.jl:24-26, householder :21,25,41."""
    rng = np.random.default_rng(0)
    X = rng.standard_normal(1000)
    Y = np.array([oracle.scalar("center_stretch", np.float64, x, 7, 2, 4) for x in X])
    Xr = np.array([oracle.scalar("center_contract", np.float64, y, 7, 2, 4) for y in Y])
    assert np.allclose(Xr, X, rtol=np.sqrt(np.finfo(float).eps))
    K = rng.standard_normal(10_000)
    Z = np.array([oracle.scalar("johnsontrafo_inv", np.float64, k, -2, 1, 0, 2.5) for k in K])
    Kr = np.array([oracle.scalar("johnsontrafo", np.float64, z, -2, 1, 0, 2.5) for z in Z])
    assert np.allclose(Kr, K, rtol=1e-8)
    # composed flow and its inverse
    D = 5
    layers = [(5, [rng.random((D, 3))]), (3, [rng.uniform(-1, 1, D), rng.uniform(0.5, 2, D),
                                             rng.uniform(-.5, .5, D), rng.uniform(.5, 2, D)]),
              (0, [rng.uniform(0.5, 2, D), rng.standard_normal(D)]), (2, [rng.uniform(0, 2, D), rng.uniform(.5, 2, D),
                                                                        rng.uniform(-.5, .5, D)])]
    Xm = np.asfortranarray(rng.standard_normal((D, 200)))
    Ym, Lm = oracle.flow_apply(layers, Xm)
    Xm2, Lm2 = oracle.flow_apply(oracle.inverse_layers(layers), Ym)
    assert np.allclose(Xm2, Xm, rtol=1e-9, atol=1e-10)
    assert np.allclose(Lm2, -Lm, rtol=1e-9, atol=1e-10)


def test_ladj_matches_logabsdet_jacobian(oracle):
    """ChangesOfVariables.test_with_logabsdet_jacobian: ladj == log|det J| (finite differences)."""
    rng = np.random.default_rng(1)
    D = 3
    layers = [(5, [rng.random((D, 2))]), (3, [rng.uniform(-1, 1, D), rng.uniform(0.5, 2, D),
                                             rng.uniform(-.5, .5, D), rng.uniform(.5, 2, D)]),
              (1, [rng.uniform(0, 2, D), rng.uniform(.5, 2, D), rng.uniform(-.5, .5, D)]),
              (4, [rng.uniform(-1, 1, D), rng.uniform(0.5, 2, D), rng.uniform(-.5, .5, D), rng.uniform(.5, 2, D)])]
    x0 = rng.standard_normal(D) * 0.7
    f = lambda x: oracle.flow_apply(layers, np.asfortranarray(x.reshape(D, 1)))[0][:, 0]
    h = 1e-6
    J = np.stack([(f(x0 + h * e) - f(x0 - h * e)) / (2 * h) for e in np.eye(D)], axis=1)
    _, L = oracle.flow_apply(layers, np.asfortranarray(x0.reshape(D, 1)))
    assert abs(L[0] - np.log(abs(np.linalg.det(J)))) < 1e-7


def test_householder_matrix(oracle):
    """test/test_householder_trafo.jl:18-25,38-43."""
    rng = np.random.default_rng(2)
    V, X = rng.random((5, 3)), np.asfortranarray(rng.random((5, 4)))
    H = lambda v: np.eye(5) - 2 * np.outer(v, v) / (v @ v)
    Y, L = oracle.flow_apply([(5, [V])], X)
    assert np.allclose(Y, H(V[:, 2]) @ H(V[:, 1]) @ H(V[:, 0]) @ X, rtol=1e-14, atol=1e-15)
    assert np.array_equal(L, np.zeros(4))


def test_batched_equals_per_column(oracle):
    """test_center_stretch.jl:64-67 / test_johnson_trafo.jl:71-74: exact equality."""
    rng = np.random.default_rng(3)
    layers = [(1, [np.array([4.0, 4.1]), np.array([2.0, 2.1]), np.array([3.0, 3.1])])]
    X = np.asfortranarray(rng.standard_normal((2, 3)))
    Y, L = oracle.flow_apply(layers, X)
    for j in range(3):
        y, l = oracle.flow_apply(layers, np.asfortranarray(X[:, j:j + 1]))
        assert np.array_equal(y[:, 0], Y[:, j]) and l[0] == L[j]


def test_negll(oracle):
    """mvnormal_negll_trafo (src/optimize_whitening.jl:7-15) on a known case."""
    Y = np.asfortranarray(np.zeros((2, 4)))
    L = np.full(4, 0.5)
    expect = -((-np.log(2 * np.pi) / 2) * 2 * 4 + 0.5 * 4) / 4
    assert abs(oracle.mvnormal_negll(Y, L) - expect) < 1e-14


def _unflat(layers, theta, D):
    res, o = [], 0
    for op, ps in layers:
        new = []
        for p in ps:
            n = np.asarray(p).size if op == 5 else D
            v = theta[o:o + n]
            new.append(v.reshape(D, -1, order="F") if op == 5 else v.copy())
            o += n
        res.append((op, new))
    return res


@pytest.mark.parametrize("D", [1, 2, 5])
def test_oracle_gradient_vs_central_differences(oracle, D):
    """The oracle's reverse pass (enf_oracle_grad.c: mvnormal_negll_trafograd restated with the reference's
    Householder rrules and the analytic derivatives of the elementwise formulas) against central differences of
    the oracle's own loss, on a flow of every transform (chained and single reflections); its loss equals
    mvnormal_negll of the forward flow exactly. (Zygote is third-party and absent: parity unpinned beyond this.)"""
    from parity import rand_params

    rng = np.random.default_rng(700 + D)
    layers = [(op, rand_params(rng, op, D, np.float64, K=2 if op == 5 else 1)) for op in [0, 5, 2, 3, 1, 4, 5, 3]]
    X = np.asfortranarray(0.8 * rng.standard_normal((D, 301)))
    negll, g = oracle.negll_grad(layers, X)
    Y, L = oracle.flow_apply(layers, X)
    assert negll == oracle.mvnormal_negll(Y, L)
    th = oracle.theta_of(layers, D)
    assert g.shape == th.shape

    def loss(theta):
        Yt, Lt = oracle.flow_apply(_unflat(layers, theta, D), X)
        return oracle.mvnormal_negll(Yt, Lt)

    fd = np.empty_like(th)
    for i in range(th.size):
        h = 1e-6 * max(1.0, abs(th[i]))
        tp, tm = th.copy(), th.copy()
        tp[i] += h
        tm[i] -= h
        fd[i] = (loss(tp) - loss(tm)) / (2 * h)
    err = np.abs(g - fd) / (np.abs(fd) + 1e-3 * np.abs(fd).max())
    assert err.max() < 2e-6, (err.argmax(), g[err.argmax()], fd[err.argmax()])
    # the x87 evaluation of the same reverse pass agrees to fp64 rounding
    _, g80 = oracle.negll_grad([(op, [np.asarray(p, np.longdouble) for p in ps]) for op, ps in layers],
                               X.astype(np.longdouble))
    assert np.allclose(g, np.asarray(g80, np.float64), rtol=1e-10, atol=1e-12 * np.abs(g).max())


def test_oracle_optimize_whitening_step(oracle):
    """One optimize_whitening epoch of the oracle == manual steps: per minibatch the oracle gradient, ADAGrad
    (acc from epsilon), then normalize! of every Householder column (src/optimize_whitening.jl:25-45,
    householder_trafo.jl:134-146)."""
    from parity import rand_params

    rng = np.random.default_rng(77)
    D = 2
    layers = [(0, rand_params(rng, 0, D, np.float64)), (5, rand_params(rng, 5, D, np.float64)),
              (2, rand_params(rng, 2, D, np.float64))]
    X = np.asfortranarray(rng.standard_normal((D, 1003)))
    th, acc, hist = oracle.optimize_whitening(layers, X, nbatches=4, nepochs=1, eta=0.1, epsilon=1e-8)
    assert hist.shape == (4,)  # round(1003/4) = 251 -> 251, 251, 251, 250
    t = oracle.theta_of(layers, D)
    a = np.full_like(t, 1e-8)
    for k, b0 in enumerate(range(0, 1003, 251)):
        n, g = oracle.negll_grad(_unflat(layers, t, D), np.asfortranarray(X[:, b0:b0 + 251]))
        assert n == hist[k]
        a = a + g * g
        t = t - 0.1 * g / (np.sqrt(a) + 1e-8)
        v = t[2 * D:3 * D]
        ss = 0.0
        for x in v:  # (the oracle's sum of squares, in order)
            ss += x * x
        t[2 * D:3 * D] = v / np.sqrt(ss)
    assert np.array_equal(th, t) and np.array_equal(acc, a)
