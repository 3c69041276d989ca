"""CPU: host-side logic of the Julia-API mirror (no device compute): composition order, inverse
algebra, equality/hash, promotion rules and the reference's MethodError cases."""
import numpy as np
import pytest
import torch


def test_composition_order(enf):
    a, b, c = enf.JohnsonTrafo(1, 2, 3, 4), enf.HouseholderTrafo(np.ones(2)), enf.CenterStretch(1, 2, 3)
    f = a @ b @ c  # a ∘ b ∘ c: c applied first
    assert [type(t).__name__ for t in enf.leaves(f)] == ["CenterStretch", "HouseholderTrafo", "JohnsonTrafo"]
    assert enf.leaves(enf.compose(a, b, c)) == enf.leaves(f)


def test_inverse_algebra(enf):
    """src/scale_shift_trafo.jl:26-30, center_stretch.jl:45,69, johnson_trafo.jl:82,107,
    householder_trafo.jl:153-154, InverseFunctions: inverse(f ∘ g) = inverse(g) ∘ inverse(f)."""
    s = enf.ScaleShiftTrafo(np.array([2.0, -4.0]), np.array([1.0, 3.0]))
    si = enf.inverse(s)
    assert np.allclose(si.a, [0.5, -0.25]) and np.allclose(si.b, [-0.5, 0.75])
    assert isinstance(enf.inverse(enf.CenterStretch(1, 2, 3)), enf.CenterContract)
    assert isinstance(enf.inverse(enf.CenterContract(1, 2, 3)), enf.CenterStretch)
    j = enf.JohnsonTrafo(4, 2, 3, 1)
    assert isinstance(enf.inverse(j), enf.JohnsonTrafoInv)
    assert enf.inverse(enf.inverse(j)) == j
    v = enf.HouseholderTrafo(np.array([1.0, 2.0]))
    assert enf.inverse(v) is v
    V = np.arange(6.0).reshape(2, 3)
    assert np.array_equal(enf.inverse(enf.HouseholderTrafo(V)).V, V[:, ::-1])
    Vt = torch.arange(6.0).reshape(2, 3)
    assert torch.equal(enf.inverse(enf.HouseholderTrafo(Vt)).V, Vt.flip(1))
    f = j @ v
    fi = enf.inverse(f)
    assert [type(t).__name__ for t in enf.leaves(fi)] == ["JohnsonTrafoInv", "HouseholderTrafo"]


def test_equality_hash(enf):
    """test_center_stretch.jl:44-47 / test_johnson_trafo.jl:51-54: ==, isequal and hash of deepcopies."""
    import copy

    for f in (enf.CenterStretch([4.0, 4.1], [2.0, 2.1], [3.0, 3.1]),
              enf.JohnsonTrafo([10.0, 11.0], [3.5, 3.6], [10.0, 11.0], [1.0, 1.1]),
              enf.HouseholderTrafo(np.random.default_rng(0).random((5, 3)))):
        g = copy.deepcopy(f)
        assert f == g and f.isequal(g) and hash(f) == hash(g)
    assert enf.JohnsonTrafo(1, 2, 3, 4) != enf.JohnsonTrafoInv(1, 2, 3, 4)
    assert enf.CenterStretch(0.0, np.nan, 0.0).isequal(enf.CenterStretch(0.0, np.nan, 0.0))
    assert enf.CenterStretch(0.0, np.nan, 0.0) != enf.CenterStretch(0.0, np.nan, 0.0)


def test_defaults(enf):
    """@with_kw defaults (center_stretch.jl:25-29, johnson_trafo.jl:61-66)."""
    cs = enf.CenterStretch()
    assert (cs.a, cs.b, cs.c) == (0.0, 1.0, 0.0)
    j = enf.JohnsonTrafo()
    assert (j.gamma, j.delta, j.xi, j.lambda_) == (10.0, 3.5, 10.0, 1.0)


def test_promotion(enf):
    from euclidiannormalizingflows_jl_amd.trafos import _kind, _promote

    assert _promote(torch.float32, _kind(1), _kind(2)) == torch.float32          # Int params keep Float32
    assert _promote(torch.float32, _kind(1.5)) == torch.float64                  # Float64 literal promotes
    assert _promote(torch.float32, _kind(np.float32([1, 2]))) == torch.float32
    assert _promote(torch.float32, _kind([1.0, 2.0])) == torch.float64
    assert _promote(_kind(3)) == torch.float64                                   # float(Int) = Float64


def test_scaleshift_method_errors(enf):
    """with_logabsdet_jacobian(::ScaleShiftTrafo, x) exists only for vector a and matrix x."""
    with pytest.raises(enf.MethodError):
        enf.ScaleShiftTrafo(2.0, 1.0)._check_ladj_signature(False)
    with pytest.raises(enf.MethodError):
        enf.ScaleShiftTrafo(np.ones(2), np.zeros(2))._check_ladj_signature(True)
    enf.ScaleShiftTrafo(np.ones(2), np.zeros(2))._check_ladj_signature(False)


def test_no_cpu_fallback(enf):
    """Placement selects the path, nothing falls back: host data runs libenf's host implementation
    (enf_flow_apply_cpu) with or without a GPU; the device-only entry points (training, VJP, host
    streaming through the GPU) raise without one instead of computing elsewhere."""
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    Y = enf.JohnsonTrafo(1, 2, 3, 4)(np.zeros((2, 3), np.float32))
    assert isinstance(Y, np.ndarray) and Y.shape == (2, 3)
    X = np.zeros((2, 3), np.float32)
    f = enf.JohnsonTrafo(np.ones(2, np.float32), 2, 3, 4)
    for call in (lambda: enf.mvnormal_negll_trafograd(f, X), lambda: enf.flow_vjp(f, X, X),
                 lambda: enf.optimize_whitening(X, f, enf.ADAGrad(), nbatches=1, nepochs=1),
                 lambda: enf.stream_with_logabsdet_jacobian(f, np.asfortranarray(X))):
        with pytest.raises(RuntimeError, match="GPU"):
            call()


def test_package_does_not_import_oracle(enf):
    import sys
    import subprocess

    code = ("import sys; sys.path.insert(0, %r); from enf_pkg import load; load(); "
            "import euclidiannormalizingflows_jl_amd.trafos; "
            "print(any('oracle' in m for m in sys.modules))") % enf.__path__[0].rsplit("/", 1)[0]
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
    assert out.stdout.strip() == "False", out.stderr
