"""GPU tests of the round-4 changes to the host-batch ring (enf_flow_apply_host, the batch-ingest row of
SURVEY §8f) and of the compiled inverse program.

* The ring copies out of the caller's X on the host, which is not stream-ordered: it must first wait for
  the work already queued on the caller's stream (an async device-to-pinned copy into X queued
  just before the call was read stale).
* The ring stages through its own pinned slots and never page-locks caller memory (round 3, DESIGN §6:
  registering caller ranges reproduced the illegal-address fault); hipPointerGetAttributes on the caller's
  arrays after a call proves it.
"""
import ctypes

import numpy as np
import pytest

from parity import check_vs_oracle, colmajor_cuda, make_flow, rand_params, to_np

pytestmark = pytest.mark.gpu


def _hip():
    # the HIP runtime libenf.so runs on (already loaded: dlopen resolves the soname to it)
    return ctypes.CDLL("libamdhip64.so.7")


def _pointer_type(ptr):
    """(hipError, hipMemoryType) of a host pointer: 0 = unregistered, 1 = host (pinned / registered)."""
    buf = (ctypes.c_byte * 256)()
    hip = _hip()
    hip.hipPointerGetAttributes.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipPointerGetAttributes.restype = ctypes.c_int
    err = hip.hipPointerGetAttributes(ctypes.cast(buf, ctypes.c_void_p), ctypes.c_void_p(ptr))
    return err, ctypes.cast(buf, ctypes.POINTER(ctypes.c_int))[0]


def _hj_layers(rng, D, n, dtype=np.float32):
    layers = []
    for _ in range(n):
        layers.append((5, rand_params(rng, 5, D, dtype)))
        layers.append((3, rand_params(rng, 3, D, dtype)))
    return layers


def test_host_stream_waits_for_the_callers_stream(enf, gpu):
    """X is a pinned host array filled by a non-blocking device-to-host copy queued on the current stream
    right before the call (behind a long kernel): the ring must see the copied values, not the stale ones."""
    import torch

    rng = np.random.default_rng(41)
    D, N = 32, 300_007
    f = make_flow(enf, _hj_layers(rng, D, 2))
    src = torch.from_numpy(np.ascontiguousarray(rng.standard_normal((N, D)).astype(np.float32))).cuda()
    pinned = torch.zeros((N, D), dtype=torch.float32).pin_memory()  # stale content: zeros
    big = torch.randn(4096, 4096, device="cuda")
    for _ in range(8):  # keep the stream busy so the copy lands well after the call starts
        big = big @ big
        big = big / big.norm()
    pinned.copy_(src, non_blocking=True)
    X = pinned.numpy().T  # column-major (D, N) view of the pinned buffer
    Y, L = enf.stream_with_logabsdet_jacobian(f, X, chunk_cols=65_536)
    torch.cuda.synchronize()
    Yd, Ld = enf.with_logabsdet_jacobian(f, src.t())
    assert np.array_equal(Y, to_np(Yd)) and np.array_equal(L, to_np(Ld))


def test_host_stream_leaves_caller_memory_unregistered(enf, gpu):
    """After a streamed call the caller's pageable X, Y and ladj are not registered with the HIP runtime
    (hipPointerGetAttributes: an error or hipMemoryTypeUnregistered); a torch pinned buffer, the positive
    control, reads as host memory."""
    import torch

    rng = np.random.default_rng(42)
    D, N = 32, 100_003
    f = make_flow(enf, _hj_layers(rng, D, 1))
    X = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
    Y, L = enf.stream_with_logabsdet_jacobian(f, X, chunk_cols=20_000)
    for a in (X, Y, L):
        err, typ = _pointer_type(a.ctypes.data)
        assert err != 0 or typ == 0, (err, typ)
    pinned = torch.zeros(1024).pin_memory()
    err, typ = _pointer_type(pinned.data_ptr())
    assert err == 0 and typ == 1, (err, typ)


# ------------------------------------------------------------------------------ inverse program ----
def _inverse_layers(layers):
    """The layer list (innermost first) of inverse(f_n o ... o f_1): reversed, each layer inverted
    (johnson_trafo.jl:82 -> JohnsonTrafoInv with the same parameters, householder_trafo.jl:153-154: a single
    reflection is its own inverse)."""
    inv = {3: 4, 4: 3, 5: 5}
    return [(inv[op], ps) for op, ps in reversed(layers)]


@pytest.mark.parametrize("D", [24, 32, 64, 100, 128])
def test_inverse_program_vs_oracle(enf, gpu, oracle, D):
    """(J^-1, H)^4 -- what inverse(J4 o H4 o ... o J1 o H1) flattens to -- on the compiled inverse program
    (layouts 32 / 64 / 128, padded at D = 24 and 100), against the oracle at fp32 rtol 1e-5, ragged tail
    included."""
    rng = np.random.default_rng(7000 + D)
    fwd = _hj_layers(rng, D, 4)
    layers = _inverse_layers(fwd)
    N = 40_009
    # the inverse's natural inputs: forward outputs (normal samples pushed through the forward flow), plus
    # raw normal columns and a few columns large enough to overflow the fast path's q product (exact redo)
    X0 = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
    X, _ = oracle.flow_apply(fwd, X0, nthreads=8)
    X = np.asfortranarray(X.astype(np.float32))
    X[:, 1000:1400] = 0.5 * X0[:, 1000:1400]
    X[:, 7:11] *= 40.0
    X[:, 20] = np.inf
    X[3, 21] = np.nan
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    check_vs_oracle(oracle, layers, X, to_np(Y), to_np(L), np.float32, what=f"inverse program D={D}")
    # round trip through the compiled forward program on the columns that are forward outputs (the raw ones
    # expand through the sinh layers, and the forward reflections then cancel large entries)
    Xr, Lr = enf.with_logabsdet_jacobian(make_flow(enf, fwd), Y)
    ok = np.r_[22:1000, 1400:N]
    from parity import col_err, ladj_err
    assert col_err(to_np(Xr)[:, ok], X[:, ok]) < 1e-4
    assert ladj_err(to_np(Lr).reshape(-1)[ok], -to_np(L).reshape(-1)[ok]) < 1e-4
