"""Device-resident whitening training (optimize_whitening), backed by libenf.so.

Julia (src/optimize_whitening.jl)                        here
-------------------------------------------------------  -----------------------------------------------
mvnormal_negll_trafo(trafo, X)          :7-15             mvnormal_negll_trafo(trafo, X)
mvnormal_negll_trafograd(trafo, X)      :18-22            mvnormal_negll_trafograd(trafo, X) -> (negll, grads)
optimize_whitening(smpls, trafo, opt; nbatches,          optimize_whitening(smpls, trafo, opt, nbatches=100,
                   nepochs, optstate, negll_history)        nepochs=100, optstate=None, negll_history=None)
  :25-45                                                   -> WhiteningResult(result, optimizer_state,
                                                                              negll_history)
Optimisers.ADAGrad(eta=0.1f0, epsilon=eps(Float32))       ADAGrad(eta=0.1, epsilon=eps(float32))

Per training step (one minibatch): one fused forward+backward launch (enf_flow_negll_grad) over the
local samples, an optional cross-GPU sum of the (1 + P) loss/gradient values (torch.distributed,
which is RCCL on ROCm; no collective at world size 1), the ADAGrad update (enf_adagrad_step) on
the flat device parameter vector and the HouseholderTrafo column re-normalisation
(enf_householder_normalize, src/householder_trafo.jl:134-146), all on the device; the per-step
negll is written to a device history buffer and copied to the host once at the end.

Samples ``smpls`` are the reference's VectorOfSimilarVectors flattened: a (D, N) column-major
matrix (``flatview``). Minibatches are consecutive column ranges of
``round(N / nbatches)`` samples (Iterators.partition, the last one possibly shorter). Data-parallel
training is opt-in (``process_group=``, ``comm=`` or ``data_parallel=True``): every rank must hold
the SAME samples, takes an equal contiguous share of every minibatch, and the gradient is
normalised by the GLOBAL minibatch size, so every rank applies the identical update.

Trainable parameters are the array-valued fields (Optimisers/Functors treat scalar fields as
constants; Zygote still returns their gradient, summed to a number). A length-1 vector field
broadcast over the D rows is ONE trainable (its gradient is the sum over the rows; on the device
its D copies receive that same summed gradient, so they stay equal).

Reference quirk, reproduced by default: under Zygote the primal ladj of a ScaleShiftTrafo
is 0 (rrule(similar_fill), src/abstract_trafo.jl:30-33), so the negll that mvnormal_negll_trafograd returns and
optimize_whitening records in negll_history is the true negll + sum(log|a|) at the step's parameters (the
gradient is unaffected). ``similar_fill_quirk=False`` reports the true negll instead. The library computes the
offset on the device inside the step's own launches (the ENF_NEGLL_ZYGOTE dtype flag, include/enf.h).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from . import _lib
from .trafos import (HouseholderTrafo, ScaleShiftTrafo, Trafo, _as_cpu_array, _colmajor, _is_vector, _kind,
                     _ld, _promote, _to_device_matrix, compose, leaves)

LOG2PI = float(np.log(2 * np.pi))


@dataclass
class ADAGrad:
    """Optimisers.jl 0.2 ADAGrad: acc starts at epsilon; acc += g^2; x -= eta*g/(sqrt(acc) + epsilon)."""
    eta: float = float(np.float32(0.1))
    epsilon: float = float(np.finfo(np.float32).eps)


@dataclass
class WhiteningResult:
    result: object
    optimizer_state: "FlowState"
    negll_history: List[float]


class FlowState:
    """Flat device parameter vector of a flow (layout of enf_flow_param_count) + ADAGrad state."""

    def __init__(self, trafo, D: int, dtype, device, optimizer: Optional[ADAGrad] = None):
        self.trafos: List[Trafo] = leaves(trafo)
        self.D, self.dtype, self.device = D, dtype, device
        self.optimizer = optimizer or ADAGrad()  # the rule Optimisers.setup stores in the state's leaves
        segs, self.trainable, self.shapes = [], [], []
        for t in self.trafos:
            for name, p in zip(t.FIELDS, t.params()):
                if isinstance(t, HouseholderTrafo):
                    A = _as_cpu_array(p).astype(np.float64)
                    A = A.reshape(D, -1) if A.ndim == 2 else A.reshape(D, 1)
                    segs.append(np.asfortranarray(A).reshape(-1, order="F"))
                    self.shapes.append(("V", _as_cpu_array(p).shape))
                else:
                    segs.append(np.broadcast_to(_as_cpu_array(p).astype(np.float64), (D,)).copy())
                    self.shapes.append((name, _as_cpu_array(p).shape))
                self.trainable.append(_is_vector(p))
        sizes = [s.size for s in segs]
        self.offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        self.theta = torch.as_tensor(np.concatenate(segs), dtype=dtype, device=device)
        self.nparams = int(self.offsets[-1])
        self.acc = torch.full_like(self.theta, self.optimizer.epsilon)  # Optimisers.init(ADAGrad) = onevalue(epsilon, x)
        self._layers = self._make_layers()

    def tied_segments(self):
        """[start, end) of every trainable length-1 vector field expanded to D entries: one
        trainable whose gradient is the sum over the D rows."""
        return [(int(self.offsets[i]), int(self.offsets[i + 1])) for i, ((_, shape), tr) in
                enumerate(zip(self.shapes, self.trainable)) if tr and shape == (1,) and self.D > 1]

    def layout(self):
        return (self.D, self.dtype, [type(t).__name__ for t in self.trafos], self.shapes, self.trainable)

    def copy_optimizer_state_from(self, other: "FlowState") -> None:
        """Continue from another state (optimize_whitening.jl:28-29: state = deepcopy(optstate)):
        ADAGrad's accumulator and rule are copied, never aliased; the layouts must match."""
        if other.layout() != self.layout():
            raise ValueError("optstate does not match the flow: "
                             f"{other.layout()} vs {self.layout()} (D, dtype, transforms, field shapes)")
        self.acc = other.acc.detach().clone()
        self.optimizer = ADAGrad(other.optimizer.eta, other.optimizer.epsilon)

    def _make_layers(self):
        arr = (_lib.Layer * len(self.trafos))()
        esz = self.theta.element_size()
        base = self.theta.data_ptr()
        seg = 0
        for i, t in enumerate(self.trafos):
            arr[i].op = t.OP
            arr[i].k = t._k()
            for q in range(len(t.FIELDS)):
                arr[i].p[q] = base + int(self.offsets[seg]) * esz
                seg += 1
        return arr

    def layers(self):
        return self._layers

    def householder_columns(self):
        """(offset, k) of every Householder V in theta."""
        out, seg = [], 0
        for t in self.trafos:
            for _ in t.FIELDS:
                if isinstance(t, HouseholderTrafo):
                    out.append((int(self.offsets[seg]), t._k()))
                seg += 1
        return out

    def to_trafo(self):
        """Rebuild the composed transform from the device parameters (Functors reconstruction)."""
        th = self.theta.detach().cpu().numpy()
        rebuilt, seg = [], 0
        for t in self.trafos:
            vals = []
            for name in t.FIELDS:
                a = th[self.offsets[seg]:self.offsets[seg + 1]]
                _, shape = self.shapes[seg]
                if isinstance(t, HouseholderTrafo):
                    a = a.reshape(self.D, -1, order="F")
                    if len(shape) == 1:
                        a = a[:, 0]
                    vals.append(a.copy())
                elif self.trainable[seg]:
                    vals.append(a[:1].copy() if shape == (1,) else a.copy())
                else:
                    vals.append(getattr(t, name))
                seg += 1
            rebuilt.append(type(t)(*vals))
        return compose(*reversed(rebuilt))


def _dtype_of(trafo, X):
    return _promote(_kind(X), *[_kind(p) for t in leaves(trafo) for p in t.params()])


def _grad_call(state: FlowState, X: torch.Tensor, out: torch.Tensor, ws: torch.Tensor, zygote: bool = False):
    D, N = X.shape
    L = _lib.lib()
    dt = (_lib.ENF_F64 if state.dtype == torch.float64 else _lib.ENF_F32) | (_lib.ENF_NEGLL_ZYGOTE if zygote else 0)
    with torch.cuda.device(X.device):
        stream = torch.cuda.current_stream(X.device).cuda_stream
        _lib.check(L.enf_flow_negll_grad(dt, D, N, X.data_ptr(), _ld(X), state.layers(), len(state.trafos),
                                         out.data_ptr(), ws.data_ptr(), ws.numel() * ws.element_size(), stream))


def _workspace(state: FlowState, N: int):
    nb = ctypes.c_size_t()
    dt = _lib.ENF_F64 if state.dtype == torch.float64 else _lib.ENF_F32
    _lib.check(_lib.lib().enf_flow_negll_grad_workspace(dt, state.D, max(N, 1), state.layers(), len(state.trafos),
                                                        ctypes.byref(nb)))
    return torch.empty(max(1, nb.value // 8), dtype=torch.float64, device=state.device)


def mvnormal_negll_trafograd(trafo, X, similar_fill_quirk: bool = True):
    """(negll, gradient) of mvnormal_negll_trafo (src/optimize_whitening.jl:18-22).

    negll is the value the reference returns, i.e. under Zygote with the ScaleShiftTrafo ladj's primal taken as 0
    (+ sum log|a|, module docstring); similar_fill_quirk=False returns the true negll. The gradient is returned as a
    list per transform (application order) of per-field arrays."""
    M, _, _ = _to_device_matrix(X)
    dtype = _dtype_of(trafo, M)
    M = _colmajor(M, dtype)
    state = FlowState(trafo, M.shape[0], dtype, M.device)
    out = torch.zeros(1 + state.nparams, dtype=dtype, device=M.device)
    _grad_call(state, M, out, _workspace(state, M.shape[1]), zygote=similar_fill_quirk)
    N = M.shape[1]
    res = (out / N).cpu().numpy()
    negll = float(res[0])
    return negll, _tangent(state, res[1:])


def _tangent(state: "FlowState", g: np.ndarray):
    """Flat gradient (enf_flow_param_count layout) -> list per transform (application order) of
    per-field arrays, shaped as Zygote returns them: a Householder field as its D x k matrix, a
    scalar field broadcast over the rows as the sum, a length-1 vector field as a length-1 sum."""
    grads, seg = [], 0
    for t in state.trafos:
        per = []
        for _ in t.FIELDS:
            a = g[state.offsets[seg]:state.offsets[seg + 1]]
            _, shape = state.shapes[seg]
            if isinstance(t, HouseholderTrafo):
                a = a.reshape(state.D, -1, order="F")
            elif shape == ():
                a = float(np.sum(a))
            elif shape == (1,):
                a = np.array([np.sum(a)])
            per.append(a)
            seg += 1
        grads.append(per)
    return grads


def flow_vjp(trafo, X, dY, dladj=None, param_grads: bool = False):
    """Pullback of (Y, ladj) = with_logabsdet_jacobian(trafo, X) (enf_flow_vjp): returns
    (dX, dparams) with dX[:, j] = J_j' dY[:, j] + dladj[j] * grad_x ladj_j, the cotangent Zygote's
    pullback gives for X (src/householder_trafo.jl:43-54,105-124: the rrules' _pullback_x; broadcast
    AD of the elementwise maps), and -- with param_grads -- the parameter cotangent summed over the
    samples in mvnormal_negll_trafograd's per-transform layout (else None). dX has X's kind (device
    tensor or numpy) and the promoted dtype. dladj=None is a zero ladj cotangent."""
    M, restore, is_vec = _to_device_matrix(X)
    if is_vec:
        raise ValueError("flow_vjp: X must be a D x N matrix")
    dtype = _dtype_of(trafo, M)
    M = _colmajor(M, dtype)
    D, N = M.shape
    G, _, _ = _to_device_matrix(dY)
    if tuple(G.shape) != (D, N):
        raise ValueError(f"flow_vjp: dY has shape {tuple(G.shape)}, X is {(D, N)}")
    G = _colmajor(G.to(M.device), dtype)
    dl = None
    if dladj is not None:
        dl = torch.as_tensor(_as_cpu_array(dladj) if not isinstance(dladj, torch.Tensor) else dladj)
        dl = dl.reshape(-1).to(device=M.device, dtype=dtype).contiguous()
        if dl.numel() != N:
            raise ValueError(f"flow_vjp: dladj has {dl.numel()} entries for N = {N}")
    state = FlowState(trafo, D, dtype, M.device)
    dX = torch.empty((N, D), dtype=dtype, device=M.device).t()  # column-major D x N
    dp = torch.zeros(state.nparams, dtype=dtype, device=M.device) if param_grads else None
    ws = _workspace(state, N)  # (a flow beyond one gradient launch's bounds needs it for its checkpoints)
    with torch.cuda.device(M.device):
        _lib.check(_lib.lib().enf_flow_vjp(
            _lib.ENF_F64 if dtype == torch.float64 else _lib.ENF_F32, D, N, M.data_ptr(), _ld(M), G.data_ptr(), _ld(G),
            dl.data_ptr() if dl is not None else None, state.layers(), len(state.trafos), dX.data_ptr(), max(D, 1),
            dp.data_ptr() if dp is not None else None, ws.data_ptr() if ws is not None else None,
            ws.numel() * ws.element_size() if ws is not None else 0, torch.cuda.current_stream(M.device).cuda_stream))
    grads = _tangent(state, dp.cpu().numpy()) if param_grads else None
    orig_np, on_gpu, _ = restore
    if not on_gpu:
        dX = dX.cpu()
        if orig_np:
            dX = dX.numpy()
    return dX, grads


def mvnormal_negll_trafo(trafo, X) -> float:
    """-(sum(std_normal_logpdf.(Y)) + sum(ladj)) / nsamples (src/optimize_whitening.jl:7-15): the flow
    and the reduction on the device (enf_flow_negll, any flow with_logabsdet_jacobian takes); only the
    scalar comes back."""
    M, _, _ = _to_device_matrix(X)
    dtype = _dtype_of(trafo, M)
    M = _colmajor(M, dtype)
    D, N = M.shape
    state = FlowState(trafo, D, dtype, M.device)
    L = _lib.lib()
    dt = _lib.ENF_F64 if dtype == torch.float64 else _lib.ENF_F32
    nb = ctypes.c_size_t(0)
    _lib.check(L.enf_flow_negll_workspace(dt, D, N, ctypes.byref(nb)))
    ws = torch.empty(max(1, (nb.value + 7) // 8), dtype=torch.float64, device=M.device)
    out = torch.zeros(1, dtype=dtype, device=M.device)
    with torch.cuda.device(M.device):
        _lib.check(L.enf_flow_negll(dt, D, N, M.data_ptr(), _ld(M), state.layers(), len(state.trafos), out.data_ptr(),
                                    ws.data_ptr(), ws.numel() * 8, torch.cuda.current_stream(M.device).cuda_stream))
    return float((out / N).item())


def trainable_runs(state: "FlowState"):
    """[start, end) ranges of theta holding trainable parameters, adjacent segments merged (one
    enf_adagrad_step launch per run instead of one per parameter vector)."""
    runs = []
    for i, tr in enumerate(state.trainable):
        if not tr:
            continue
        s0, s1 = int(state.offsets[i]), int(state.offsets[i + 1])
        if runs and runs[-1][1] == s0:
            runs[-1] = (runs[-1][0], s1)
        else:
            runs.append((s0, s1))
    return runs


def householder_batches(state: "FlowState"):
    """Householder vectors of theta as (offset, count, stride) batches for
    enf_householder_normalize_strided: single equally spaced columns (the (J∘H)^n flows) become one
    batch, a HouseholderTrafo with a D x k matrix is one contiguous batch of k columns."""
    cols = state.householder_columns()
    if len(cols) > 1 and all(k == 1 for _, k in cols):
        offs = [o for o, _ in cols]
        st = offs[1] - offs[0]
        if st >= state.D and all(offs[i + 1] - offs[i] == st for i in range(len(offs) - 1)):
            return [(offs[0], len(offs), st)]
    return [(o, k, state.D) for o, k in cols]


def minibatch_plan(N: int, nbatches: int, rank: int = 0, world: int = 1):
    """Minibatches of optimize_whitening (src/optimize_whitening.jl:31-32: batchsize =
    round(Int, N/nbatches), Iterators.partition, the last batch possibly shorter) and this rank's
    contiguous share of each: a list of (B, lo, hi) with the batch size B and the column range
    [lo, hi) this rank processes. The shares of all ranks tile every batch exactly once."""
    batchsize = max(int(round(N / nbatches)), 1)
    plan = []
    for b0 in range(0, N, batchsize):
        B = min(b0 + batchsize, N) - b0
        plan.append((B, b0 + (B * rank) // world, b0 + (B * (rank + 1)) // world))
    return plan


def allreduce_sum_(buf: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """In-place cross-rank sum of the (1 + P) loss/gradient sums (torch.distributed: RCCL on ROCm,
    gloo on CPU); a no-op at world size 1. Every rank then normalises by the GLOBAL batch size."""
    if world > 1:
        import torch.distributed as dist

        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf


def optimize_whitening(smpls, initial_trafo, optimizer: Optional[ADAGrad] = None, nbatches: int = 100,
                       nepochs: int = 100, optstate: Optional[FlowState] = None,
                       negll_history: Optional[List[float]] = None, process_group=None,
                       similar_fill_quirk: bool = True, graph: bool = False, comm=None,
                       data_parallel: bool = False,
                       _dp_step: bool = False, _separate_update: bool = False,
                       _per_step: bool = False) -> WhiteningResult:
    """src/optimize_whitening.jl:25-45 on the device (see module docstring). negll_history holds what the reference
    records under Zygote (ScaleShiftTrafo's primal ladj taken as 0, src/abstract_trafo.jl:30-33: + sum log|a| at
    each step's parameters); similar_fill_quirk=False records the true negll. The updates are the same either way.

    optstate continues a previous run as the reference does (state = deepcopy(optstate), trafo =
    deepcopy(initial_trafo)): the parameters come from initial_trafo, the ADAGrad accumulator and rule
    from a copy of optstate (never modified); a layout mismatch raises ValueError.

    Data-parallel training is opt-in: process_group= (torch.distributed sum: RCCL on ROCm, gloo on
    CPU), comm= (an EnfComm: RCCL through libenf on the kernels' own stream) or data_parallel=True
    (the default group). All ranks must hold the same smpls.

    graph=True: the launches of one epoch are captured once into a HIP graph (torch.cuda.CUDAGraph)
    and the graph is replayed per epoch, which removes the host launch gaps between the launches of
    each minibatch step; the parameters, optimizer state and history are bit-identical to the eager
    loop (same kernels in the same order). With several ranks this needs comm= (the RCCL all-reduce
    is captured into the graph); a torch.distributed group stays eager.

    One rank (round 5): each epoch is ONE enf_whitening_epoch call -- a single launch when the minibatches fit the
    one-launch step (the reference examples' B = 100 / 1000 at D <= 2), else the per-step path inside the library.

    Test hooks: _dp_step=True runs the data-parallel step (gradient, all-reduce, enf_whitening_apply)
    on one rank; _separate_update=True replaces enf_whitening_apply by the separate
    enf_adagrad_step / enf_householder_normalize_strided calls (identical arithmetic); _per_step=True
    runs one enf_whitening_step call per minibatch instead of enf_whitening_epoch (identical arithmetic)."""
    import torch.distributed as dist

    M, _, _ = _to_device_matrix(smpls)
    D, N = M.shape
    dtype = _dtype_of(initial_trafo, M)
    M = _colmajor(M, dtype)
    state = FlowState(initial_trafo, D, dtype, M.device, optimizer)
    if optstate is not None:  # continue from a previous optimizer state (optimize_whitening.jl:28-29, 44)
        state.copy_optimizer_state_from(optstate)
    optimizer = state.optimizer
    world, rank = 1, 0
    if comm is not None:
        world, rank = comm.nranks, comm.rank
    elif process_group is not None or data_parallel:
        world = dist.get_world_size(process_group)
        rank = dist.get_rank(process_group)
    plan = minibatch_plan(N, nbatches, rank, world)
    batchsize = max(B for B, _, _ in plan)
    L = _lib.lib()
    dt = _lib.ENF_F64 if dtype == torch.float64 else _lib.ENF_F32
    dtq = dt | (_lib.ENF_NEGLL_ZYGOTE if similar_fill_quirk else 0)  # the training calls' dtype (loss reporting)
    out = torch.zeros(1 + state.nparams, dtype=dtype, device=M.device)
    ws = _workspace(state, batchsize)
    hist = torch.zeros(nepochs * len(plan), dtype=torch.float64, device=M.device)
    hbatches = householder_batches(state)
    segs = trainable_runs(state)
    tied = state.tied_segments()
    # one rank: the fused step (gradient, loss, ADAGrad and re-normalisation in three launches)
    fused = world == 1 and not tied and comm is None
    runs = np.ascontiguousarray(np.array(segs, dtype=np.int64).reshape(-1))
    hbs = np.ascontiguousarray(np.array(hbatches, dtype=np.int64).reshape(-1))
    if len(segs) > 64 or len(hbatches) > 16:
        fused = False
    # multi-rank update after the all-reduce: one enf_whitening_apply launch
    apply_fused = len(segs) <= 64 and len(hbatches) <= 16 and not _separate_update
    if _dp_step:
        fused = False
    def one_epoch(hbuf: torch.Tensor, stream: int) -> None:
        """Enqueue the steps of one epoch on `stream`; the loss of step j goes to hbuf[j]."""
        if fused and not _per_step:
            # the whole epoch in one call (enf_whitening_epoch: one launch when the minibatches fit the one-launch
            # step, else enf_whitening_step per batch; the same result bit for bit)
            _lib.check(L.enf_whitening_epoch(
                dtq, D, N, M.data_ptr(), _ld(M), batchsize, state.layers(), len(state.trafos), state.theta.data_ptr(),
                state.acc.data_ptr(), runs.ctypes.data, len(segs), hbs.ctypes.data, len(hbatches), optimizer.eta,
                optimizer.epsilon, hbuf.data_ptr(), ws.data_ptr(), ws.numel() * 8, stream))
            return
        for j, (B, lo, hi) in enumerate(plan):
            if fused and hi > lo:
                _lib.check(L.enf_whitening_step(
                    dtq, D, hi - lo, M[:, lo:hi].data_ptr(), _ld(M), state.layers(), len(state.trafos),
                    state.theta.data_ptr(), state.acc.data_ptr(), runs.ctypes.data, len(segs), hbs.ctypes.data,
                    len(hbatches), optimizer.eta, optimizer.epsilon, hbuf[j:].data_ptr(), ws.data_ptr(),
                    ws.numel() * 8, stream))
                continue
            if comm is not None and not tied and apply_fused:
                # data-parallel in one call: gradient of the share, RCCL sum of the kernels' double slice totals,
                # one tail launch (enf_whitening_step_dp; round 4)
                _lib.check(L.enf_whitening_step_dp(
                    dtq, D, hi - lo, M[:, lo:hi].data_ptr() if hi > lo else None, _ld(M), state.layers(),
                    len(state.trafos), state.theta.data_ptr(), state.acc.data_ptr(), runs.ctypes.data, len(segs),
                    hbs.ctypes.data, len(hbatches), optimizer.eta, optimizer.epsilon, B, hbuf[j:].data_ptr(),
                    comm.handle, ws.data_ptr(), ws.numel() * 8, stream))
                continue
            # data-parallel: local sums, cross-rank sum, then the update on every rank
            out.zero_()
            if hi > lo:
                Xb = M[:, lo:hi]
                _lib.check(L.enf_flow_negll_grad(dtq, D, hi - lo, Xb.data_ptr(), _ld(M), state.layers(),
                                                 len(state.trafos), out.data_ptr(), ws.data_ptr(),
                                                 ws.numel() * 8, stream))
            if comm is not None:
                comm.allreduce_sum_(out, stream)
            else:
                allreduce_sum_(out, world, process_group)
            for s0, s1 in tied:  # one trainable broadcast over D rows: every copy gets the summed gradient
                out[1 + s0:1 + s1] = out[1 + s0:1 + s1].sum()
            if apply_fused:  # loss, ADAGrad and re-normalisation in one launch (enf_whitening_apply)
                _lib.check(L.enf_whitening_apply(dt, D, state.nparams, out.data_ptr(), B, state.theta.data_ptr(),
                                                 state.acc.data_ptr(), runs.ctypes.data, len(segs), hbs.ctypes.data,
                                                 len(hbatches), optimizer.eta, optimizer.epsilon, hbuf[j:].data_ptr(),
                                                 stream))
            else:
                hbuf[j:j + 1].copy_(out[0:1] / B)
                g = out[1:]
                for s0, s1 in segs:
                    _lib.check(L.enf_adagrad_step(dt, s1 - s0, state.theta[s0:].data_ptr(),
                                                  state.acc[s0:].data_ptr(), g[s0:].data_ptr(), 1.0 / B,
                                                  optimizer.eta, optimizer.epsilon, stream))
                for off, k, ldv in hbatches:
                    _lib.check(L.enf_householder_normalize_strided(dt, D, k, state.theta[off:].data_ptr(), ldv,
                                                                   stream))

    P = len(plan)
    with torch.cuda.device(M.device):
        if graph and (world == 1 or comm is not None) and nepochs > 0:
            hep = torch.zeros(P, dtype=torch.float64, device=M.device)
            torch.cuda.synchronize(M.device)
            cg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(cg):  # captured on torch's capture stream; nothing runs yet
                one_epoch(hep, torch.cuda.current_stream(M.device).cuda_stream)
            for ep in range(nepochs):
                cg.replay()
                hist[ep * P:(ep + 1) * P].copy_(hep)
            torch.cuda.synchronize(M.device)
            del cg
        else:
            stream = torch.cuda.current_stream(M.device).cuda_stream
            for ep in range(nepochs):
                one_epoch(hist[ep * P:(ep + 1) * P], stream)
    h = hist.cpu().numpy().tolist()
    prev = list(negll_history) if negll_history is not None else []
    return WhiteningResult(state.to_trafo(), state, prev + h)
