"""CPU: bench.py's layer-letter patterns and the inverse layer algebra of its --inverse leg (against the
reference's InverseFunctions.inverse methods, checked with the oracle: inverse(f)(f(X)) == X)."""
import numpy as np
import pytest


def test_parse_pattern():
    import bench

    assert bench.parse_pattern("HJ") == [(5, 1), (3, 1)]
    assert bench.parse_pattern("H4JSCKI") == [(5, 4), (3, 1), (0, 1), (1, 1), (2, 1), (4, 1)]
    for bad in ("", "X", "J2", "HJ-"):
        with pytest.raises(ValueError):
            bench.parse_pattern(bad)


@pytest.mark.parametrize("pattern", ["HJHJHJHJ", "SHC", "KHS", "JC", "KJKJ", "H3JIS"])
def test_inverse_layers_invert_the_flow(oracle, pattern):
    """bench.invert_layers (scale_shift_trafo.jl:26-30, center_stretch.jl:45,69, johnson_trafo.jl:82,107,
    householder_trafo.jl:153-154): the oracle's inverse flow maps the forward output back to X and its ladj is
    the negated forward ladj."""
    import bench

    D = 6
    layers = bench.build_flow(D, 4, np.float64, pattern=pattern)
    inv = bench.invert_layers(layers)
    assert bench.layer_letters(inv) == bench.layer_letters(bench.invert_layers(bench.invert_layers(inv)))
    rng = np.random.default_rng(3)
    X = np.asfortranarray(0.5 * rng.standard_normal((D, 200)))
    Y, L = oracle.flow_apply(layers, X)
    X2, L2 = oracle.flow_apply(inv, np.asfortranarray(Y))
    assert np.allclose(X2, X, rtol=1e-9, atol=1e-9)
    assert np.allclose(L2, -L, rtol=1e-9, atol=1e-9)
