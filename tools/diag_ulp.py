import sys, numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "tests"); sys.path.insert(0, "oracle")
from enf_pkg import load
enf = load()
import oracle
from parity import make_flow, colmajor_cuda, to_np
for D in (2, 32):
    rng = np.random.default_rng(11)
    N = 4096
    X = rng.standard_normal((D, N)) * np.exp(rng.uniform(-30, 30, (D, N)))
    X[:, :64] = rng.uniform(0.5, 2.0, (D, 64)) * 1e100 * rng.choice([-1, 1], (D, 64))
    X[:, 64:80] = 1e200
    X = np.asfortranarray(X)
    one = np.ones(D)
    layers = [(3, [np.zeros(D), one, np.zeros(D), one])]
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    Y = to_np(Y)
    Yh, Lh = oracle.flow_apply_hi(layers, X)
    ulp = np.abs(Y - Yh) / np.spacing(np.abs(Yh))
    idx = np.argsort(ulp.ravel())[-8:]
    print("D", D, "max ulp", ulp.max())
    for i in idx:
        print("  x=%r y=%r yh=%r ulp=%.2f" % (X.ravel()[i], Y.ravel()[i], Yh.ravel()[i], ulp.ravel()[i]))
