"""Landmark-sharded LM across devices, one process per GPU over torch.distributed.

Every rank holds the whole problem but owns one time band of landmarks (landmarks ordered by their
earliest observing rig, cut into contiguous ranges balanced by observation count): it linearizes the
visual factors of its landmarks, eliminates them and forms its partial damped Schur-reduced system.
The root (rank 0) also owns every small factor (IMU, omega, random walks, priors), the constant-point
observations and the identity damping term.  Per LM iteration, everything is queued on the engine's
stream (deferred mode, vb_set_deferred) and the host reads the LM scalars ONCE:

  1. each rank: linearize (partial cost) -- or commit the linearization queued speculatively behind the
     previous iteration's cost pass
  2. each rank: partial reduced system S_r, RHS b_r                 (vb_assemble_reduced)
  3. S = sum S_r on the root: each rank sends the tiles its landmarks touch (point-to-point over
     RCCL/xGMI), b = sum b_r by reduce
  4. root: factor S, solve x_red                                    (vb_factor_solve_reduced)
  5. broadcast x_red (reduced order x 8 B)
  6. each rank: back-substitute its points (partial model reduction)
  7. box-plus (every rank applies the reduced step; points per shard) (partial step ratios)
  8. cost pass (partial cost + CostStats)
  9. the partial scalars of 1, 6, 7, 8 all-reduced in place on the engine stream, then the next
     iteration's linearization queued speculatively (vb_spec_linearize), then one host read
The LM decisions (Optimizer.cpp:834-1097, restated by vb_optimize) run identically on every rank from
the reduced scalars.  The bad-step path (step rescale, sub-step with the existing factor) reads its
scalars phase by phase, as the reference does (vb_gradient_dot_step partial scalar; vb_assemble_new_rhs
-> reduce -> root vb_solve_reduced -> broadcast -> vb_back_substitute_which(1)), and drops the
speculative linearization.

The controller is engine-agnostic: the HIP engine (device buffers, RCCL) in production, the CPU
oracle (host buffers, gloo) in the CPU tests.

Stream ordering, not host round trips: with the HIP engine, the loop runs with torch's current stream
set to the engine's own HIP stream (torch.cuda.ExternalStream over vb_stream).  RCCL then queues
each collective behind the engine kernels that produced its input, and the engine kernels that
consume its output queue behind the collective, so no exchange needs a stream or device
synchronisation; the host waits once per iteration, for the reduced LM scalars (with gloo, the
one-GPU test transport, every exchange is additionally staged through host memory).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import math
import os
import time

import numpy as np

from .engine import Settings, Summary


# ------------------------------------------------------------------ buffers as torch tensors
class _CudaArray:
    """Minimal __cuda_array_interface__ exporter for a device pointer (no copy)."""

    def __init__(self, ptr: int, n: int, typestr: str = "<f8"):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                         "version": 3, "strides": None}


def _tensor(ptr: int, n: int, device, int32: bool = False):
    import torch
    if n == 0:
        return torch.zeros(0, dtype=torch.int32 if int32 else torch.float64, device=device)
    if device is None or device.type == "cpu":
        ct = C.c_int32 if int32 else C.c_double
        return torch.from_numpy(np.ctypeslib.as_array((ct * n).from_address(ptr)))
    return torch.as_tensor(_CudaArray(ptr, n, "<i4" if int32 else "<f8"), device=device)


class ShardComm:
    """Collectives of the sharded LM.  `device` is where the engine's buffers live (a CUDA device
    for the HIP engine, None for the oracle).  With the nccl backend (RCCL) device tensors go over
    the wire directly; with gloo and device buffers they are staged through host memory."""

    def __init__(self, rank: int, world: int, device=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.rank, self.world, self.device = rank, world, device
        self.nccl = dist.get_backend() == "nccl"
        self.sdev = device if self.nccl else None  # where scalar tensors live
        # host waits for an LM scalar (a collective whose result the host reads): the measure of the
        # controller's pipelining (tests/test_distributed*.py count it per iteration)
        self.host_reads = 0

    # scalars
    def sum(self, *vals):
        t = self.torch.tensor(vals, dtype=self.torch.float64, device=self.sdev)
        self.dist.all_reduce(t)
        self.host_reads += 1
        return t.tolist()

    def max(self, v):
        t = self.torch.tensor([v], dtype=self.torch.float64, device=self.sdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        self.host_reads += 1
        return t.item()

    def all_gather_obj(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    # device / host buffers
    def _staged(self, t):
        return t if (self.nccl or t.device.type == "cpu") else t.cpu()

    def reduce_to_root(self, t):
        s = self._staged(t)
        self.dist.reduce(s, dst=0)
        if s is not t and self.rank == 0:
            t.copy_(s)

    def broadcast_from_root(self, t):
        s = self._staged(t)
        self.dist.broadcast(s, src=0)
        if s is not t:
            t.copy_(s)

    def sum_tiles_to_root(self, engine, tile_lists):
        """Sparse exchange: every non-root rank packs the tiles its partial system touches
        (engine.pack_shard_tiles) and sends them point-to-point; the root adds each rank's packed
        tiles into its tile store (engine.add_tiles).  tile_lists[r]: device int32 tensor of rank
        r's tile indices (root side)."""
        dist, torch = self.dist, self.torch
        if self.rank == 0:
            bufs, ops = [], []
            for r in range(1, self.world):
                n = int(tile_lists[r].numel())
                if n == 0:
                    continue
                b = torch.empty(n * 64 * 64, dtype=torch.float64, device=self.device if self.nccl else "cpu")
                bufs.append((r, n, b))
                ops.append(dist.P2POp(dist.irecv, b, r))
            if ops:
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
            for r, n, b in bufs:
                b = b.to(self.device)  # gloo: host -> device copy on the engine stream; nccl: no-op
                engine.add_tiles(tile_lists[r].data_ptr(), n, b.data_ptr())
        else:
            ptr, n = engine.pack_shard_tiles()
            if n:
                s = self._staged(_tensor(ptr, n, self.device))
                for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, s, 0)]):
                    w.wait()

    def sum_bands_to_root(self, full, bands):
        """full: this rank's matrix storage; bands[r] = (first, count) of rank r.  The root adds
        every other rank's band into its own storage (point-to-point, overlapped)."""
        dist = self.dist
        if self.rank == 0:
            bufs, ops = [], []
            for r in range(1, self.world):
                first, cnt = bands[r]
                if cnt == 0:
                    continue
                b = self.torch.empty(cnt, dtype=self.torch.float64,
                                     device=full.device if self.nccl else "cpu")
                bufs.append((first, cnt, b))
                ops.append(dist.P2POp(dist.irecv, b, r))
            if ops:
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
            for first, cnt, b in bufs:
                full[first:first + cnt] += b.to(full.device)
        else:
            first, cnt = bands[self.rank]
            if cnt:
                s = self._staged(full[first:first + cnt])
                for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, s.contiguous(), 0)]):
                    w.wait()


# ------------------------------------------------------------------ one scalar read per iteration
def word_bits(words):
    """two error bit words (int32, bits 0..30) -> 62 floats 0/1 (bit k of word i at 31 i + k): a MAX
    reduction of these over the ranks is the bitwise OR of the words (collectives have no bitwise-or)"""
    return [float((int(w) >> k) & 1) for w in words for k in range(31)]


def bits_word(bits):
    """inverse of word_bits (over MAX-reduced floats)"""
    return np.array([sum(int(round(float(bits[31 * i + k]))) << k for k in range(31)) for i in range(2)],
                    dtype=np.int32)


class _IterScalars:
    """The LM scalars of one iteration (vb_scalar_slots layout: [0] linearization cost, [1] cost pass
    cost, [2..4] CostStats, [8] max step ratio, [9] sum of squared ratios, [10] sum of ratios, [16] twice
    the model cost reduction), reduced over the ranks and read by the host ONCE per iteration.

    HIP engine (deferred mode, vb_set_deferred): the phase functions leave their partials in the
    engine's device slots.  With RCCL they are all-reduced in place on the engine stream (sum; the max
    ratio by max, the error words bitwise-ORed), the scalar point is marked (vb_mark_scalars) so work
    queued after it -- the next iteration's speculative linearization -- does not delay the read, and the
    host reads them once (vb_read_scalars).  With gloo (host-staged) the host reads the partials and the
    error words once and the reduction runs on host tensors; either way every rank decodes the same ORed
    words (vb_error_from_words), so all raise the same code and message.  Host engines (the oracle): the phase functions return their
    partials, collected here, reduced over gloo."""

    SUM = [0, 1, 2, 3, 4, 9, 10, 16]

    def __init__(self, engine, comm: ShardComm):
        self.e, self.c = engine, comm
        torch = comm.torch
        self.device = (hasattr(engine, "scalar_slots") and comm.device is not None
                       and comm.device.type != "cpu")
        if self.device:
            rp, ep = engine.scalar_slots()
            self.red = _tensor(rp, 24, comm.device)
            self.err = _tensor(ep, 2, comm.device, int32=True)
            small = engine.small_factor_count()
            self.spec = engine.spec_prepare()
            self.shifts = torch.arange(31, dtype=torch.int64, device=comm.device)
        else:
            self.host = np.zeros(17)
            small = 0  # the host engine's CostStats count every factor it evaluates
            self.spec = False
        # numTotal of the non-visual factors (the deferred cost pass leaves them out of red[2])
        self.n_small = int(sum(comm.all_gather_obj(small)))
        self.torch = torch

    def set(self, i, v):
        """a host engine's partial (device slots are written by the engine itself)"""
        if not self.device:
            self.host[i] = v

    def read(self, queue_after=None):
        """reduce + one host read; queue_after() is called once the scalars' point is queued (so the
        work it queues overlaps the read).  Returns the 17 reduced scalars (numTotal completed)."""
        c, torch = self.c, self.torch
        dist = c.dist
        if self.device and c.nccl:
            red, err = self.red, self.err
            # the error words are bit flags: ORed over the ranks as one 0/1 per bit reduced by MAX (RCCL
            # has no bitwise-or), in the same collective as the max step ratio
            bits = ((err.to(torch.int64).unsqueeze(1) >> self.shifts) & 1).to(torch.float64).flatten()
            mx = torch.cat([red[8:9], bits])
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            red[5:9].zero_()
            red[11:16].zero_()
            dist.all_reduce(red[0:17])
            red[8:9].copy_(mx[0:1])
            err.copy_((mx[1:].view(2, 31).to(torch.int64) << self.shifts).sum(1).to(torch.int32))
            if self.spec:
                self.e.mark_scalars()
            if queue_after:
                queue_after()
            # the code (and the engine's last_error text) of the ORed words: the same on every rank
            rc, v = self.e.read_scalars(17, check=False)
        else:
            words = None
            if self.device:
                if self.spec:
                    self.e.mark_scalars()
                if queue_after:
                    queue_after()
                rc, v = self.e.read_scalars(17, check=False)
                words = self.e.error_words()
            else:
                rc, v = 0, self.host.copy()
            t = torch.tensor([v[i] for i in self.SUM], dtype=torch.float64)
            bits = [] if words is None else word_bits(words)
            m = torch.tensor([v[8], -float(rc)] + bits, dtype=torch.float64)
            dist.all_reduce(t)
            dist.all_reduce(m, op=dist.ReduceOp.MAX)
            v = np.zeros(17)
            v[self.SUM] = t.numpy()
            v[8] = float(m[0])
            if words is None:  # host engines raise inside their calls; only a code travels
                rc = -int(round(float(m[1])))
            else:  # the ORed words, decoded as the RCCL path decodes them
                ored = bits_word(m[2:].tolist())
                rc = self.e.error_from_words(ored) if ored.any() else 0
        c.host_reads += 1
        if rc:  # every rank raises the same code with the same message (the error words ORed over the ranks)
            from .engine import VbError
            msg = self.e.last_error() if hasattr(self.e, "last_error") else ""
            raise VbError(rc, f"LM iteration failed (error words ORed over {c.world} ranks): {msg}")
        v = np.array(v, dtype=np.float64)
        v[2] += self.n_small
        return v


# ------------------------------------------------------------------ the sharded LM controller
class ShardedOptimizer:
    """Optimizer::optimize (Optimizer.cpp:768-1106) over landmark shards; mirrors vb_optimize."""

    def __init__(self, engine, comm: ShardComm):
        self.e, self.c = engine, comm
        self.n_params = engine.num_params()
        self.ext = self._engine_stream(engine, comm)
        self.n_factor = 0  # reduced factorizations run (the bench's roofline)
        first, cnt = engine.shard_tile_range()
        self.bands = comm.all_gather_obj((first, cnt))
        # HIP engine: exact tile sets (the nested-dissection order spreads a shard's contributions
        # over its subtree and the separators above it, so the enclosing band is wide)
        self.tile_lists = None
        if hasattr(engine, "shard_tiles") and comm.device is not None and comm.device.type != "cpu":
            lists = comm.all_gather_obj(engine.shard_tiles().tolist())
            self.tile_lists = [comm.torch.tensor(t, dtype=comm.torch.int32, device=comm.device) for t in lists]
        self.sync = getattr(engine, "synchronize", lambda: None)
        self.phases = _PhaseClock(self.ext)

    @staticmethod
    def _engine_stream(engine, comm):
        """torch.cuda.ExternalStream over the engine's HIP stream (None for host engines)."""
        if comm.device is None or comm.device.type == "cpu" or not hasattr(engine, "stream_ptr"):
            return None
        return comm.torch.cuda.ExternalStream(engine.stream_ptr(), device=comm.device)

    def on_engine_stream(self):
        """Context in which torch (and so RCCL) issues on the engine's stream."""
        if self.ext is None:
            return contextlib.nullcontext()
        return self.c.torch.cuda.stream(self.ext)

    def _buffers(self):
        m, nm, r, nr = self.e.reduced_buffers()
        dev = self.c.device
        return _tensor(m, nm, dev), _tensor(r, nr, dev)

    # LM building blocks ---------------------------------------------------------------
    def linearize(self, dont_retry):
        return self.c.sum(self.e.linearize(True, dont_retry))[0]

    def factor_solve_partial(self, lam):
        """damp + eliminate + exchange + factor + solve + back-substitute; returns this rank's partial
        model cost reduction (NaN in deferred mode: it stays in the engine's slot 16 as twice that)"""
        e, c = self.e, self.c
        self.n_factor += 1
        self.phases.mark("schur_ms")
        e.assemble_reduced(lam)
        self.phases.mark("factor_ms")
        S, b = self._buffers()
        if self.tile_lists is not None:
            self.sync_torch()
            c.sum_tiles_to_root(e, self.tile_lists)
        else:
            c.sum_bands_to_root(S, self.bands)
        c.reduce_to_root(b)
        self.sync_torch()
        if c.rank == 0:
            e.factor_solve_reduced()
        self.phases.mark("solve_ms")
        S, b = self._buffers()
        c.broadcast_from_root(b)
        self.sync_torch()
        return e.back_substitute(0)

    def damp_factor_solve(self, lam):
        return self.c.sum(self.factor_solve_partial(lam))[0]

    def gradient_dot_step(self, dont_retry):
        return self.c.sum(self.e.gradient_dot_step(dont_retry))[0]

    def solve_with_new_gradient(self):
        e, c = self.e, self.c
        e.assemble_new_rhs()
        _, b = self._buffers()
        c.reduce_to_root(b)
        self.sync_torch()
        if c.rank == 0:
            e.solve_reduced()
        _, b = self._buffers()
        c.broadcast_from_root(b)
        self.sync_torch()
        e.back_substitute(1)

    def apply_step(self, which):
        mx, sq, s = self.e.apply_step_raw(which)
        mx = self.c.max(mx)
        sq, s = self.c.sum(sq, s)
        n = max(1, self.n_params)
        return mx, math.sqrt(sq / n), s / n

    def cost(self, comparable):
        cost, st = self.e.cost(comparable)
        out = self.c.sum(cost, *st)
        return out[0], tuple(int(round(x)) for x in out[1:])

    def sync_torch(self):
        """Order torch's work before the engine's: a no-op on the engine's own stream."""
        if self.ext is None and self.c.device is not None and self.c.device.type != "cpu":
            self.c.torch.cuda.synchronize(self.c.device)

    # the loop ---------------------------------------------------------------------------
    def optimize(self, s: Settings | None = None) -> Summary:
        with self.on_engine_stream():
            return self._optimize(s)

    def _optimize(self, s: Settings | None = None) -> Summary:
        s = s or Settings.default()
        e = self.e
        damping = s.damping
        it, last_impr, last_troubled = 0, 0, -10
        initial_cost = final_cost = 0.0
        troubled_start_damping, troubled_start, n_troubled, largest_troubled = damping, 0, 0, 0
        n_rescaled = 0
        dont_retry = False
        deferred = hasattr(e, "set_deferred")
        sc = _IterScalars(e, self.c)
        self.spec_used = sc.spec
        spec_pending = False  # the next iteration's linearization was queued speculatively
        # per iteration: (host reads of LM scalars, whether it took the step-rescaling path)
        self.reads_per_iteration = []
        reads0 = self.c.host_reads

        def acceptable(st):
            rate = st[1] / (st[0] + 1.0)
            return rate < 0.03 and st[1] < st[2] * 2.0 + 50

        try:
            while True:
                # ---- queued: linearize, damp + eliminate + exchange + factor + solve, backup, box-plus,
                # cost pass; their scalars reduced over the ranks and read once (vb_optimize's pattern)
                if deferred:
                    e.set_deferred(True)
                used_spec = spec_pending
                if spec_pending:
                    e.spec_commit(True)  # the step stayed applied at full size: its linearization is ready
                    spec_pending = False
                else:
                    self.phases.mark("rs_update_ms")
                    if getattr(e, "rs_device", False):  # ark_vi_ba's preStepCallback (as vb_optimize)
                        e.update_rs_tables()
                    self.phases.mark("linearize_ms")
                    sc.set(0, e.linearize(True, dont_retry))
                sc.set(16, 2.0 * self.factor_solve_partial(damping))
                e.backup()
                self.phases.mark("step_ms")
                for i, x in zip((8, 9, 10), e.apply_step_raw(0)):
                    sc.set(i, x)
                self.phases.mark("cost_ms")
                cost, st = e.cost(True)
                sc.set(1, cost)
                for i, x in zip((2, 3, 4), st):
                    sc.set(i, x)
                self.phases.mark(None)
                speculate = sc.spec and it + 1 < s.max_num_iterations

                def queue_spec():
                    self.phases.mark("spec_linearize_ms")
                    e.spec_linearize(dont_retry)
                    self.phases.mark(None)
                v = sc.read(queue_spec if speculate else None)
                spec_pending = speculate
                if used_spec and hasattr(e, "spec_phase_ms"):
                    # this iteration's rebuild + linearization ran in the previous iteration's queue: their
                    # own device events (complete: they precede the cost pass just read), as vb_optimize
                    rs_ms, lin_ms = e.spec_phase_ms()
                    self.phases.add("rs_update_ms", rs_ms)
                    self.phases.add("linearize_ms", lin_ms)
                if deferred:
                    e.set_deferred(False)
                self.phases.close_iteration()
                n = max(1, self.n_params)
                prev_cost, new_cost, model_red = v[0], v[1], 0.5 * v[16]
                st = (int(round(v[2])), int(round(v[3])), int(round(v[4])))
                ratios = (v[8], math.sqrt(v[9] / n), v[10] / n)
                # ---- the LM decisions (Optimizer.cpp:834-1097), identical on every rank
                final_cost = prev_cost
                if it == 0:
                    initial_cost = prev_cost
                if model_red < 0:  # Optimizer.cpp:835-854 (see vb_optimize)
                    damping *= s.damping_adjust_on_fail
                cost_red = prev_cost - new_cost
                ratio_red_to_cost = cost_red / new_cost
                ratio_red_to_exp = cost_red / model_red
                applied = 1.0
                ok_rate = acceptable(st)
                rescaled = False
                if s.max_step_factor_attempts > 0 and (ratio_red_to_exp < s.min_relative_cost_reduction or not ok_rate):
                    rescaled, n_rescaled = True, n_rescaled + 1
                    back_red = self.gradient_dot_step(dont_retry)
                    sf = model_red / (model_red + back_red) if back_red > 0 else s.step_factor_decrease
                    for _ in range(s.max_step_factor_attempts):
                        applied *= sf
                        e.scale_step(sf)
                        e.restore()
                        self.apply_step(0)  # (its ratios are discarded, Optimizer.cpp:927)
                        cost_f, st_f = self.cost(True)
                        red_f = prev_cost - new_cost  # Optimizer.cpp:935
                        r_f = red_f / (model_red * applied)
                        if r_f >= s.min_relative_cost_reduction and acceptable(st_f):
                            new_cost, st, cost_red, ratio_red_to_exp, ok_rate = cost_f, st_f, red_f, r_f, True
                            break
                        if s.try_sub_step:
                            self.gradient_dot_step(dont_retry)
                            self.solve_with_new_gradient()
                            self.apply_step(1)
                            cost_s, st_s = self.cost(True)
                            red_s = prev_cost - cost_s
                            r_s = red_s / (model_red * applied)
                            if r_s >= s.min_relative_cost_reduction and acceptable(st_s):
                                new_cost, st, cost_red, ratio_red_to_exp, ok_rate = cost_s, st_s, red_s, r_s, True
                                break
                        dont_retry = True
                        sf = s.step_factor_decrease
                tol = (ratio_red_to_cost < s.relative_cost_tolerance or cost_red < s.absolute_cost_tolerance
                       or ratios[1] < s.variables_tolerance)
                rejected = new_cost > prev_cost or not ok_rate
                if spec_pending and (rejected or rescaled):  # it assumed the full step stays applied
                    e.spec_commit(False)
                    spec_pending = False
                if rejected:
                    if last_troubled != it - 1:
                        troubled_start_damping, troubled_start = damping, it
                    damping *= s.damping_adjust_on_fail
                    e.restore()
                    if damping > s.damping_max:
                        break
                    last_troubled = it
                else:
                    if last_troubled == it - 1 and troubled_start_damping < 1e1 and damping > 1e-3:
                        n_troubled += 1
                        largest_troubled = max(largest_troubled, it - troubled_start)
                    if ratio_red_to_exp >= s.min_relative_cost_reduction and applied > s.min_step_factor_for_good:
                        damping = max(damping * s.damping_adjust_on_good_step, s.damping_min)
                    else:
                        damping *= s.damping_adjust_on_average_step
                    final_cost = new_cost
                self.reads_per_iteration.append((self.c.host_reads - reads0, rescaled))
                reads0 = self.c.host_reads
                it += 1
                if not tol:
                    last_impr = it
                if it >= last_impr + s.stop_if_no_improvement_for and it >= last_troubled + s.distance_from_troubled_iteration:
                    break
                if it >= s.max_num_iterations:
                    break
        finally:
            if spec_pending:  # a convergence stop left it queued: never used
                e.spec_commit(False)
            if deferred:
                e.set_deferred(False)
            self.phases.close_iteration(final=True)
        out = Summary()
        out.initial_cost, out.final_cost = initial_cost, final_cost
        out.num_troubled_seqs, out.largest_troubled_seq, out.num_iterations = n_troubled, largest_troubled, it
        out.num_rescaled = n_rescaled
        return out


class _PhaseClock:
    """Per-phase device time of an LM iteration (vb_phase_times semantics), from torch.cuda events recorded
    on the engine's stream at the phase boundaries, without extra synchronisation: an iteration's marks are
    evaluated at the next iteration's close (or the final one), when the device has passed them.  A phase's
    time includes its collectives and any stream idle while the host stages them (gloo).  An iteration whose
    linearization was queued speculatively by the previous one has no rs_update / linearize marks: the
    controller adds that work's own device times (vb_spec_phase_ms) to it instead, so rs_update_ms and
    linearize_ms are this iteration's as in vb_phase_times, while spec_linearize_ms is the span the previous
    iteration's queue spent on it.  Host engines: nothing is recorded."""

    NAMES = ("rs_update_ms", "linearize_ms", "schur_ms", "factor_ms", "solve_ms", "step_ms", "cost_ms",
             "spec_linearize_ms")

    def __init__(self, ext):
        self.ext = ext
        self.ms = {k: 0.0 for k in self.NAMES}
        self.marks = []    # the iteration being queued
        self.pending = []  # the last closed iteration, evaluated at the next close
        self.extra, self.pending_extra = {}, {}  # phase times measured elsewhere (add())

    def mark(self, name):
        """The phase `name` starts here (None: nothing is timed from here)."""
        if self.ext is None:
            return
        import torch
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(self.ext)
        self.marks.append((name, ev))

    def add(self, name, ms):
        """device time of a phase of the iteration being queued, measured by the engine's own events"""
        if self.ext is not None:
            self.extra[name] = self.extra.get(name, 0.0) + ms

    def _evaluate(self, marks, extra):
        marks[-1][1].synchronize()
        ms = {k: 0.0 for k in self.NAMES}
        for (name, a), (_, b) in zip(marks, marks[1:]):
            if name is not None:
                ms[name] += a.elapsed_time(b)
        for name, v in extra.items():
            ms[name] += v
        ms["total_ms"] = marks[0][1].elapsed_time(marks[-1][1])
        self.ms = ms

    def close_iteration(self, final=False):
        if self.ext is None:
            return
        if self.pending:
            self._evaluate(self.pending, self.pending_extra)
        self.pending, self.marks = self.marks, []
        self.pending_extra, self.extra = self.extra, {}
        if final and self.pending:
            self._evaluate(self.pending, self.pending_extra)
            self.pending, self.pending_extra = [], {}


class PartitionedOptimizer(ShardedOptimizer):
    """The sharded LM with the reduced factorization itself distributed: every
    rank factors its nested-dissection subtree, rank 0 only the ROOT separators above them.  Engine
    built with set_partition(rank, world) (world a power of two; include/viba_hip.h).  Per reduced
    solve, instead of summing whole partial systems on rank 0:

      local: factor_part(0); solve_part(0)                 (subtree factor, forward solve)
      reduce ROOT tiles + ROOT rows of the forward vector to rank 0     (RCCL reduce, in place)
      rank 0: factor_part(1); solve_part(1)                (ROOT factor, forward + backward)
      broadcast ROOT rows of x; local: solve_part(2)       (subtree backward solve)
      all-reduce x (each rank contributes the rows it solved), back-substitute the landmarks
    """

    def __init__(self, engine, comm: ShardComm):
        self.e, self.c = engine, comm
        self.n_params = engine.num_params()
        self.ext = self._engine_stream(engine, comm)
        self.n_factor = 0
        self.tile_lists = None
        self.phases = _PhaseClock(self.ext)

    def _exchange(self, what, reduce):
        e, c = self.e, self.c
        ptr, n = e.part_exchange(what, 0)
        if n == 0:
            return
        t = _tensor(ptr, n, c.device)
        if reduce:
            c.reduce_to_root(t)
        else:
            c.broadcast_from_root(t)
        self.sync_torch()
        if reduce and c.rank != 0:
            return
        e.part_exchange(what, 1)

    def _solve(self, which):
        e, c = self.e, self.c
        e.solve_part(0)
        self._exchange(1, True)
        if c.rank == 0:
            e.solve_part(1)
        self._exchange(2, False)
        e.solve_part(2)
        ptr, n = e.share_x()
        x = _tensor(ptr, n, c.device)
        s = c._staged(x)
        c.dist.all_reduce(s)
        if s is not x:
            x.copy_(s)
        self.sync_torch()
        return e.back_substitute(which)

    def factor_solve_partial(self, lam):
        e, c = self.e, self.c
        self.n_factor += 1
        self.phases.mark("schur_ms")
        e.assemble_reduced(lam)
        self.phases.mark("factor_ms")
        e.factor_part(0)
        self._exchange(0, True)
        if c.rank == 0:
            e.factor_part(1)
        self.phases.mark("solve_ms")
        return self._solve(0)

    def solve_with_new_gradient(self):
        self.e.assemble_new_rhs()
        self._solve(1)


# ------------------------------------------------------------------ shard boundaries
def landmark_order(p):
    """Landmark order of vb_finalize (api.hip): registered points by earliest observing rig, ties by
    handle.  Returns (point handles in order, observations per landmark)."""
    fv = p.fvars[0]
    pts, poses = fv[:, 0].astype(np.int64), fv[:, 1].astype(np.int64)
    keep = p.const[0][pts] == 0
    pts, poses = pts[keep], poses[keep]
    n = len(p.const[0])
    first = np.full(n, np.iinfo(np.int64).max)
    np.minimum.at(first, pts, poses)
    cnt = np.bincount(pts, minlength=n)
    handles = np.flatnonzero(cnt > 0)
    order = handles[np.argsort(first[handles], kind="stable")]
    return order, cnt[order]


def shard_bounds(p, world: int):
    """Contiguous landmark ranges balanced by observation count."""
    _, cnt = landmark_order(p)
    cum = np.concatenate([[0], np.cumsum(cnt)])
    cuts = [0] + [int(np.searchsorted(cum, cum[-1] * k / world)) for k in range(1, world)] + [len(cnt)]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


# ------------------------------------------------------------------ bench entry (N > 1)
def run_sharded(args, rank: int, world: int, local: int):
    import json
    import sys

    import torch
    import torch.distributed as dist

    from . import synth
    from .engine import HipEngine

    def log(*a):
        if rank == 0:
            print(*a, file=sys.stderr, flush=True)

    # test-only overrides (a 1-GPU box): VIBA_DIST_BACKEND=gloo, VIBA_DIST_SAME_DEVICE=1
    backend = os.environ.get("VIBA_DIST_BACKEND", "nccl")
    if os.environ.get("VIBA_DIST_SAME_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)
    p = synth.generate(synth.config(args.config))
    # default: partitioned factorization (world a power of two); VIBA_MULTI=shard selects landmark
    # shards with the whole reduced system factored on rank 0
    # (world 1: the partition protocol has no subtree to hand out, so one rank runs as a single shard)
    mode = os.environ.get("VIBA_MULTI", "partition" if world > 1 and world & (world - 1) == 0 else "shard")
    if world == 1:
        mode = "shard"
    e = HipEngine(imu_calib_options=p.imu_calib_options, device=local, precision=getattr(args, "precision", "fp64"))
    if mode == "partition":
        e.set_partition(rank, world)
    else:
        lb, le = shard_bounds(p, world)[rank]
        e.set_landmark_shard(lb, le, rank == 0)
    synth.load_into(e, p, rs_device=getattr(args, "rs_tables", "device") == "device")
    st = e.problem_stats()
    comm = ShardComm(rank, world, dev)
    # the collectives' transport as it actually ran: RCCL (nccl backend) over xGMI, or gloo through host
    # memory (the one-GPU test box, VIBA_DIST_BACKEND=gloo)
    wire = "RCCL" if comm.nccl else "gloo (host-staged)"
    same_device = os.environ.get("VIBA_DIST_SAME_DEVICE") == "1"
    if mode == "partition":
        info = comm.all_gather_obj(e.part_info())
        log(f"[bench] {world} ranks, config {args.config}: {p.summary()}; partitioned factorization: subtree "
            f"columns {[i[0] for i in info]}, ROOT columns {info[0][1]} ({info[0][4]} tiles), contributions "
            f"local {[i[2] for i in info]} root {info[0][3]}")
        opt = PartitionedOptimizer(e, comm)
        parallelism = (f"nested-dissection subtree x{world} (landmarks, factor, solves per rank), ROOT separators "
                       f"on rank 0, {wire} reduce/broadcast of ROOT tiles and rows")
    else:
        log(f"[bench] {world} ranks, config {args.config}: {p.summary()}; landmark shards, Schur entries lm "
            f"{st[8]} obs {st[9]}")
        opt = ShardedOptimizer(e, comm)
        parallelism = f"landmark shards x{world}, {wire} tile exchange to rank 0"

    def settings(n):
        return Settings.default(max_num_iterations=n, stop_if_no_improvement_for=10**6,
                                distance_from_troubled_iteration=0)
    if args.warmup:
        opt.optimize(settings(args.warmup))
    # roofline: every fan-in launch of this rank timed with HIP events on the engine stream (family 4)
    e.profile_kernel(4)
    opt.n_factor = 0
    e.synchronize()
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    s = opt.optimize(settings(args.steps))
    e.synchronize()
    torch.cuda.synchronize(dev)
    dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()
    iters = s.num_iterations
    launches, kms = e.kernel_time()
    e.profile_kernel(-1)
    if mode == "partition":
        pi = e.part_info()
        contrib = pi[2] + pi[3]  # this rank's subtree schedule (+ the ROOT schedule on rank 0)
    else:
        contrib = st[6] if rank == 0 else 0
    flops = float(opt.n_factor) * contrib * 2.0 * 64 ** 3
    per_rank = comm.all_gather_obj((launches, kms, flops))
    phases = comm.all_gather_obj({k: round(v, 3) for k, v in opt.phases.ms.items()})
    reads = opt.reads_per_iteration
    ph = phases[0]
    dist_backend = dist.get_backend()
    dist.destroy_process_group()
    if rank != 0:
        return
    FP64_MFMA_PEAK_TF = 78.6
    l0, k0, f0 = per_rank[0]
    if l0 == 0 or k0 <= 0:  # no fan-in launch was event-timed on rank 0 (e.g. a graphed factorization)
        achieved = None
    else:
        achieved = f0 / (k0 * 1e-3) / 1e12
    roof = {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TF, "unit": "TFLOP/s",
            "frac": None if achieved is None else achieved / FP64_MFMA_PEAK_TF,
            # no PMC pass of a rank's own launches: the 1-GPU per-launch bytes cover the whole schedule's
            # levels, not a rank's subtree + ROOT levels, so they are not this line's traffic
            "traffic": None,
            "kernel": "fanin_kernel on rank 0 (its subtree + the ROOT separators), HIP events on the engine stream",
            "flops_per_launch": f0 / max(1, l0), "avg_launch_ms": k0 / max(1, l0), "launches": l0,
            "per_rank_tflops": [f / (k * 1e-3) / 1e12 if k > 0 else None for _, k, f in per_rank]}
    log(f"[bench] timed {iters} its in {elapsed:.3f}s; rank 0 last it: " +
        " ".join(f"{k[:-3]} {v:.2f}" for k, v in ph.items()) + f" ms; fan-in {achieved} TF/s")
    cpu = None
    if not args.no_cpu_baseline:
        e.close()
        try:
            from bench import cpu_baseline
            cpu = cpu_baseline(p, args.config, warmup=args.warmup)
        except Exception as ex:  # the baseline must never hide the GPU number
            log(f"[bench] cpu baseline failed: {ex}")
    out = {"metric": "LM iterations/sec on 10k-pose/300k-landmark VI-BA", "value": iters / elapsed,
           "unit": "LM iterations/s", "n_gpus": world, "steps": iters, "warmup": args.warmup,
           "ms_per_step": elapsed * 1e3 / max(1, iters), "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": "f64" if getattr(args, "precision", "fp64") == "fp64" else "f32/f64",
           "data": "synthetic (seeded Aria-like generator, csrc/synth.cpp)",
           "config": {"workload": f"config {args.config}: {st[0]} obs, {p.num_points} landmarks, "
                                  f"{p.vars[1].shape[0]} rigs, reduced order {st[3]}",
                      "parallelism": parallelism, "backend": dist_backend,
                      "ranks_share_one_gpu": same_device},
           "roofline": roof, "cpu_baseline": cpu,
           "phases_ms_rank0": ph, "phases_ms_per_rank": phases,
           # the controller's pipelining: host reads of LM scalars per timed iteration (1 unless the
           # iteration rescaled its step), and whether the next linearization was queued speculatively
           "host_reads_per_iteration": [int(n) for n, _ in reads], "speculative_linearization": bool(opt.spec_used),
           "cost": [s.initial_cost, s.final_cost]}
    print(json.dumps(out), flush=True)
