"""optimize_whitening / mvnormal_negll_trafograd semantics against the reference's Julia code
(src/optimize_whitening.jl:18-45, Optimisers.jl 0.2, Functors), and the data-parallel step on an
RCCL communicator of the C ABI captured into a HIP graph."""
import numpy as np
import pytest

from parity import colmajor_cuda, make_flow, rand_params, to_np

pytestmark = pytest.mark.gpu


def small_flow(rng, D=8, dtype=np.float64):
    return [(5, rand_params(rng, 5, D, dtype)), (3, rand_params(rng, 3, D, dtype)),
            (5, rand_params(rng, 5, D, dtype)), (3, rand_params(rng, 3, D, dtype))]


def test_optstate_is_copied_not_aliased(enf, gpu):
    """optimize_whitening.jl:28-34: trafo = deepcopy(initial_trafo), state = deepcopy(optstate). Two
    continuations from the same optstate give identical results; optstate is left untouched; the
    parameters come from initial_trafo (not from optstate)."""
    rng = np.random.default_rng(40)
    X = colmajor_cuda(rng.standard_normal((8, 4000)))
    f0 = make_flow(enf, small_flow(rng))
    r1 = enf.optimize_whitening(X, f0, enf.ADAGrad(), nbatches=4, nepochs=1)
    acc0 = r1.optimizer_state.acc.clone()
    th0 = r1.optimizer_state.theta.clone()
    a = enf.optimize_whitening(X, r1.result, enf.ADAGrad(), nbatches=4, nepochs=2, optstate=r1.optimizer_state)
    b = enf.optimize_whitening(X, r1.result, enf.ADAGrad(), nbatches=4, nepochs=2, optstate=r1.optimizer_state)
    assert np.array_equal(to_np(a.optimizer_state.theta), to_np(b.optimizer_state.theta))
    assert np.array_equal(to_np(a.optimizer_state.acc), to_np(b.optimizer_state.acc))
    assert a.negll_history == b.negll_history
    assert np.array_equal(to_np(r1.optimizer_state.acc), to_np(acc0))
    assert np.array_equal(to_np(r1.optimizer_state.theta), to_np(th0))
    assert a.optimizer_state.acc.data_ptr() != r1.optimizer_state.acc.data_ptr()
    # initial_trafo's parameters, optstate's accumulator: starting from f0 instead of r1.result differs
    c = enf.optimize_whitening(X, f0, enf.ADAGrad(), nbatches=4, nepochs=2, optstate=r1.optimizer_state)
    assert not np.array_equal(to_np(c.optimizer_state.theta), to_np(a.optimizer_state.theta))
    # ... and equals a fresh run whose accumulator is preset to optstate's
    d = enf.FlowState(f0, 8, a.optimizer_state.dtype, a.optimizer_state.device)
    d.acc.copy_(acc0)
    e = enf.optimize_whitening(X, f0, enf.ADAGrad(), nbatches=4, nepochs=2, optstate=d)
    assert np.array_equal(to_np(c.optimizer_state.theta), to_np(e.optimizer_state.theta))


def test_optstate_rule_and_layout_checks(enf, gpu):
    """The ADAGrad rule stored in the state is the one used (Optimisers leaves carry their rule);
    an optstate of another dtype or layout raises instead of feeding fp64 theta to fp32 kernels."""
    import torch

    rng = np.random.default_rng(41)
    layers = small_flow(rng)
    X = rng.standard_normal((8, 3000))
    st = enf.FlowState(make_flow(enf, layers), 8, torch.float64, torch.device("cuda:0"), enf.ADAGrad(eta=0.05))
    a = enf.optimize_whitening(colmajor_cuda(X), make_flow(enf, layers), enf.ADAGrad(eta=0.3), nbatches=3, nepochs=1,
                               optstate=st)
    b = enf.optimize_whitening(colmajor_cuda(X), make_flow(enf, layers), enf.ADAGrad(eta=0.05), nbatches=3, nepochs=1)
    assert np.array_equal(to_np(a.optimizer_state.theta), to_np(b.optimizer_state.theta))
    layers32 = [(op, [np.asarray(p, np.float32) for p in ps]) for op, ps in layers]
    with pytest.raises(ValueError):
        enf.optimize_whitening(colmajor_cuda(X.astype(np.float32)), make_flow(enf, layers32), enf.ADAGrad(),
                               nbatches=3, nepochs=1, optstate=st)
    with pytest.raises(ValueError):
        enf.optimize_whitening(colmajor_cuda(X), make_flow(enf, layers[:2]), enf.ADAGrad(), nbatches=3, nepochs=1,
                               optstate=st)


def test_scalar_and_length1_field_gradients(enf, gpu):
    """Zygote's gradient of a scalar field broadcast over the rows is one number, of a length-1
    vector field a length-1 vector: the sums over the rows of the per-row gradient."""
    rng = np.random.default_rng(42)
    D = 6
    X = colmajor_cuda(rng.standard_normal((D, 2000)))
    g, d, xi, lam = rand_params(rng, 3, D, np.float64)
    per_row = enf.JohnsonTrafo(np.full(D, 0.3), d, xi, lam)
    scalar = enf.JohnsonTrafo(0.3, d, xi, lam)
    len1 = enf.JohnsonTrafo(np.array([0.3]), d, xi, lam)
    n0, g0 = enf.mvnormal_negll_trafograd(per_row, X)
    n1, g1 = enf.mvnormal_negll_trafograd(scalar, X)
    n2, g2 = enf.mvnormal_negll_trafograd(len1, X)
    assert n0 == pytest.approx(n1, rel=1e-14) and n0 == pytest.approx(n2, rel=1e-14)
    assert isinstance(g1[0][0], float) and g1[0][0] == pytest.approx(float(np.sum(g0[0][0])), rel=1e-12)
    assert np.shape(g2[0][0]) == (1,) and g2[0][0][0] == pytest.approx(float(np.sum(g0[0][0])), rel=1e-12)


def test_length1_vector_field_is_one_trainable(enf, gpu):
    """Optimisers treats a length-1 vector as ONE trainable: it gets the gradient summed over the
    rows; the D device copies stay equal and the result keeps length 1."""
    rng = np.random.default_rng(43)
    D = 6
    X = colmajor_cuda(rng.standard_normal((D, 3000)) * 1.5 + 0.2)
    f = enf.ScaleShiftTrafo(np.array([1.1]), rng.standard_normal(D))
    r = enf.optimize_whitening(X, f, enf.ADAGrad(), nbatches=3, nepochs=2)
    th = to_np(r.optimizer_state.theta)
    assert np.all(th[:D] == th[0])
    assert np.shape(r.result.a) == (1,) and r.result.a[0] == th[0]
    # the same as a one-dimensional reference update: ADAGrad on the summed gradient
    eps, eta = float(np.finfo(np.float32).eps), float(np.float32(0.1))  # Python floats: all-float64 arithmetic
    acc, a, b = eps, 1.1, np.array(f.b, dtype=np.float64)
    accb = np.full(D, eps, dtype=np.float64)
    for _ in range(2):
        for lo, hi in ((0, 1000), (1000, 2000), (2000, 3000)):
            _, gr = enf.mvnormal_negll_trafograd(enf.ScaleShiftTrafo(np.array([a]), b), X[:, lo:hi])
            ga, gb = gr[0][0][0], gr[0][1]
            acc += ga * ga
            a -= eta * ga / (np.sqrt(acc) + eps)
            accb += gb * gb
            b = b - eta * gb / (np.sqrt(accb) + eps)
    assert th[0] == pytest.approx(a, rel=1e-12)
    assert np.allclose(th[D:], b, rtol=1e-12, atol=0)


def test_device_cache_follows_parameter_changes(enf, gpu):
    """The Python transforms are mutable (Julia's are not): reassigning a field or changing a
    parameter array in place must change the next result (no stale device copy)."""
    import torch

    rng = np.random.default_rng(44)
    D = 4
    X = colmajor_cuda(rng.standard_normal((D, 500)))
    g, d, xi, lam = rand_params(rng, 3, D, np.float64)
    f = enf.JohnsonTrafo(g.copy(), d, xi, lam)
    y0 = to_np(f(X))
    f.gamma = g + 1.0
    assert np.allclose(to_np(f(X)), y0 + 1.0, rtol=1e-12)
    f.gamma[:] = g - 2.0  # in place on the host array
    assert np.allclose(to_np(f(X)), y0 - 2.0, rtol=1e-12)
    t = torch.tensor(g, device="cuda")
    f.gamma = t
    assert np.allclose(to_np(f(X)), y0, rtol=1e-12)
    t.add_(0.5)  # in place on a device tensor
    assert np.allclose(to_np(f(X)), y0 + 0.5, rtol=1e-12)
    V = rng.standard_normal(D)
    h = enf.HouseholderTrafo(V)
    z0 = to_np(h(X))
    V[:] = -V  # the reflection is invariant under v -> -v: same result, but a fresh device copy
    assert np.allclose(to_np(h(X)), z0, rtol=1e-12)
    h.V = rng.standard_normal(D)
    assert not np.allclose(to_np(h(X)), z0)


def test_dp_step_rccl_graph_equals_eager(enf, gpu):
    """The data-parallel step (gradient, RCCL all-reduce through libenf's enf_comm on the kernels'
    stream, enf_whitening_apply) captured as one HIP graph per epoch is bit-identical to the eager
    launches on a real one-rank RCCL communicator, and to the torch.distributed-free _dp_step path."""
    rng = np.random.default_rng(45)
    D = 32
    layers = [(op, ps) for op, ps in small_flow(rng, D, np.float32)]
    X = colmajor_cuda(rng.standard_normal((D, 20_000)).astype(np.float32))
    comm = enf.EnfComm.single()
    try:
        runs = []
        for kw in ({"comm": comm, "graph": True}, {"comm": comm, "graph": False}, {"_dp_step": True}):
            r = enf.optimize_whitening(X, make_flow(enf, layers), enf.ADAGrad(), nbatches=5, nepochs=3, **kw)
            runs.append((to_np(r.optimizer_state.theta), to_np(r.optimizer_state.acc), r.negll_history))
        for th, acc, h in runs[1:]:
            assert np.array_equal(th, runs[0][0]) and np.array_equal(acc, runs[0][1]) and h == runs[0][2]
    finally:
        comm.close()
