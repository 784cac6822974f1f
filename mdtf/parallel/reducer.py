"""Gradient aggregation across replicas over RCCL (xGMI) / gloo.

Replaces three reference mechanisms with collectives on flat buckets:

* ``Tower.average_gradients`` — in-graph mean of per-tower gradients
  (``distribute_tower.py:78-114``);
* ``SyncReplicasOptimizer`` — per-variable ConditionalAccumulators on the PS,
  ``replicas_to_aggregate`` of ``total_num_replicas`` (``distribute_train.py:146-160``);
* PS variable placement — variables round-robined over PS tasks, pulled by every
  worker every step (``distribute_train.py:109-110``).

Two modes:

``allreduce``
    every rank holds the full fp32 master and optimizer state; each bucket is
    all-reduced as soon as its last gradient lands (overlapping backward), then
    one fused optimizer launch per group.
``sharded``  ("PS shards", ZeRO-1 layout)
    each rank *is* the parameter server for ``1/N`` of every bucket: buckets
    are reduce-scattered during backward, the fused optimizer updates only the
    local shard of the fp32 master + state, and the refreshed compute weights
    (bf16 shadow, or fp32 master for fp32 groups) are all-gathered.  Per rank
    traffic ≈ the all-reduce's, the PS-CPU bottleneck and the separate
    parameter pull are gone.

Wire dtype (``comm_dtype``): fp32 (default) or bf16.  In bf16 mode each bucket's
fp32 gradients are cast into a persistent bf16 wire buffer, the collective runs
on half the bytes (xGMI rings are per-link bandwidth bound, so a bucket's
all-reduce / reduce-scatter time halves), and the result is widened back into
the fp32 gradient (allreduce) or the fp32 shard gradient the optimizer reads
(sharded).  Master weights and optimizer state stay fp32; only the summands on
the wire are rounded (relative error ~N * 2^-9 of the summed gradient, tested
in ``tests/test_distributed.py``).

Backup workers (``replicas_to_aggregate`` R < N): gradients of the first R
replicas to finish backward are aggregated, the rest contribute zeros (TF
drops them as stale).  On GPUs the arrival order is decided ON THE DEVICE: each
replica stamps the device clock when its backward has finished (a kernel on the
compute stream), the stamps are all-gathered and every replica ranks itself
(``csrc/backup.hip``; clock origins calibrated against the node's monotonic host clock, re-measured
every 1000 steps; single-node groups only, a multi-node group takes the store ticket).
The 0/1 mask scales the flat gradients before the bucket all-reduces, with no
host synchronize and no store round trip, so the step stays hipGraph-capturable.
On the CPU the order is an atomic counter in the cluster store.  Overlap is
disabled in this mode because the mask is only known after backward.  Unlike
TF's accumulators, stragglers are NOT skipped in time: every replica still joins
every collective (its contribution zeroed), so a slow replica delays the step;
backup workers here reproduce the gradient math (exactly R contributions per
step), not the latency hiding.  ``ps_mode='sync_ps'`` (``parallel/async_ps.py``)
reproduces both on dedicated PS ranks: each version is the mean of the first R
pushes computed on it and a late push is dropped, so a straggler never stalls
the other workers (``tests/test_distributed.py``, sync_ps straggler test).
"""
import os

import torch
import torch.distributed as dist
from ..train import variables as V



class _DoneThen(object):
    """An async collective's work handle whose ``wait`` also runs a follow-up (the shard copy of an emulated
    reduce-scatter)."""
    __slots__ = ("work", "then")

    def __init__(self, work, then):
        self.work, self.then = work, then

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
            self.then()
        return True


# gloo's reduce_scatter / all_gather move the same bytes as its all_reduce but cost 1.7-1.9x / 1.7x as much
# (2 ranks, 64 MiB: 122 / 114 ms vs 66 ms, profiles/sharded_vs_allreduce_r5.md); on gloo the sharded mode runs
# them as all_reduces (reduce-scatter: all_reduce + own shard; all-gather: all_reduce of the zero-padded
# shard).  RCCL keeps the native collectives (its all_reduce IS reduce-scatter + all-gather).
GLOO_VIA_ALLREDUCE = os.environ.get("MDTF_GLOO_RS_AR", "1") != "0"

class UpdateTarget(object):
    """Tensors one fused optimizer launch operates on."""
    __slots__ = ("group", "master", "grad", "shadow", "numel", "key", "decay")

    def __init__(self, group, master, grad, shadow, key):
        self.group = group
        self.master = master
        self.grad = grad
        self.shadow = shadow
        self.numel = master.numel()
        self.key = key
        self.decay = group.decay

    def state(self, name):
        return self.group.state_buffer("%s/%s" % (self.key, name), self.numel)


class _SliceTarget(UpdateTarget):
    """One bucket's slice of a group's shard buffers (sharded mode's per-bucket update during backward)."""
    __slots__ = ("off", "total")

    def __init__(self, group, master, grad, shadow, key, off, total):
        super(_SliceTarget, self).__init__(group, master, grad, shadow, key)
        self.off, self.total = off, total

    def state(self, name):
        return self.group.state_buffer("%s/%s" % (self.key, name), self.total)[self.off:self.off + self.numel]


def resolve_comm_dtype(comm_dtype=None):
    """``comm_dtype`` argument, else ``MDTF_COMM_DTYPE`` (fp32 | bf16); -> torch dtype."""
    name = comm_dtype if comm_dtype is not None else os.environ.get("MDTF_COMM_DTYPE", "fp32")
    if isinstance(name, torch.dtype):
        name = {torch.float32: "fp32", torch.bfloat16: "bf16"}.get(name, str(name))
    name = str(name).lower()
    if name in ("fp32", "float32", "float"):
        return torch.float32
    if name in ("bf16", "bfloat16"):
        return torch.bfloat16
    raise ValueError("comm_dtype must be fp32 or bf16, got %r" % (comm_dtype,))


class _NullCtx(object):
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def group_is_single_host(pg=None):
    """True when every rank of ``pg`` runs on this host.  Decided by exchanging host names over the group (a
    collective: every rank of ``pg`` calls it), not from torchrun's LOCAL_WORLD_SIZE / WORLD_SIZE, which the
    ClusterSpec launcher does not set: a multi-host group must never take the device-clock backup path, whose
    clocks are calibrated against one host's monotonic clock."""
    import socket
    if not (dist.is_available() and dist.is_initialized()):
        return True
    world = dist.get_world_size(pg)
    if world == 1:
        return True
    names = [None] * world
    dist.all_gather_object(names, socket.gethostname(), group=pg)
    return len(set(names)) == 1


class GradReducer(object):
    def __init__(self, space, process_group=None, mode="allreduce", overlap=True,
                 replicas_to_aggregate=None, store=None, comm_dtype=None):
        self.space = space
        self.comm_dtype = resolve_comm_dtype(comm_dtype)
        self._wire = {}                    # bucket index -> (bf16 full buffer, bf16 shard buffer or None)
        self.pg = process_group
        self.mode = mode
        self.distributed = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(process_group) if self.distributed else 1
        self.rank = dist.get_rank(process_group) if self.distributed else 0
        self.R = replicas_to_aggregate or self.world
        if self.R > self.world or self.R < 1:
            raise ValueError("replicas_to_aggregate=%d must be in [1, %d]" % (self.R, self.world))
        self.store = store
        # collectives run for world > 1; MDTF_FORCE_COLLECTIVES=1 also issues them on a 1-rank group
        # (exercises the RCCL + hipGraph capture path on a single GPU)
        self.collective = self.distributed and (self.world > 1 or
                                                os.environ.get("MDTF_FORCE_COLLECTIVES", "0") == "1")
        self.overlap = overlap and self.collective and self.R == self.world
        self.contributed = True
        self.num_contributors = self.world
        self._shards = {}
        # sharded + overlap: each bucket's shard is updated and all-gathered as soon as its reduce-scatter
        # lands, on a side stream (the capture stream inside a hipGraph capture), while backward continues (set per
        # step by the TrainOp: set_update_fn)
        self.eager_update = None
        self._upd_stream = None
        # backup workers decided on the device (GPU replicas): see the module docstring
        # device clocks are calibrated against ONE host clock, so only for a single-node group; multi-node
        # groups take the store ticket
        self.backup_device = (self.world > 1 and self.R < self.world and space.device is not None
                              and torch.device(space.device).type == "cuda"
                              and group_is_single_host(process_group))
        self._bk = None
        if mode not in ("allreduce", "sharded"):
            raise ValueError("mode must be 'allreduce' or 'sharded'")
        if mode == "sharded":
            self._init_shards()
        for v in space.variables:
            v.on_grad_ready = self._on_grad_ready if self.overlap else None

    # ------------------------------------------------------------------
    def _init_shards(self):
        for g in self.space.groups:
            off = 0
            for b in g.buckets:
                assert b.numel % self.world == 0, "bucket not padded to world size"
                b.shard_len = b.numel // self.world
                b.shard_offset = off
                off += b.shard_len
            n = off
            self._shards[id(g)] = {
                "master": torch.zeros(n, dtype=torch.float32, device=g.device),
                "grad": torch.zeros(n, dtype=torch.float32, device=g.device),
                "out": torch.zeros(n, dtype=g.shadow.dtype if g.shadow is not None else torch.float32,
                                   device=g.device),
            }
        self.load_shards_from_master()

    def load_shards_from_master(self):
        """(Re)initialise the owned fp32 master shard from the full master."""
        if self.mode != "sharded":
            return
        for g in self.space.groups:
            sh = self._shards[id(g)]
            for b in g.buckets:
                s = b.start + self.rank * b.shard_len
                sh["master"][b.shard_offset:b.shard_offset + b.shard_len].copy_(g.master[s:s + b.shard_len])

    # -- step protocol ---------------------------------------------------
    # MDTF_ZERO_SIDE=1: zero the flat fp32 gradient buffer on a side stream beside the forward pass (nothing reads or
    # writes gradients before backward; join_zero() makes the compute stream wait for it before the first backward
    # kernel).  Off by default: measured slower on both steps (ResNet-50 11241 vs 11389 img/s, BERT-base 6330 vs 6441
    # seq/s, alternating A/B, profiles/ab_r4.md) -- the fill's blocks take CU slots and HBM from the forward kernels.
    ZERO_SIDE = os.environ.get("MDTF_ZERO_SIDE", "0") == "1"

    def begin_step(self):
        dev = self.space.device
        V.begin_grad_epoch()               # store-first slots: a new step's first writes (train/variables.py)
        if self.ZERO_SIDE and dev is not None and torch.device(dev).type == "cuda":
            if getattr(self, "_zero_stream", None) is None:
                self._zero_stream = torch.cuda.Stream(dev)
            zs = self._zero_stream
            zs.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(zs):
                self.space.zero_grad(skip_stored=True)
            self._zero_pending = zs
        else:
            self.space.zero_grad(skip_stored=True)
        for v in self.space.variables:
            v.uses = 0
        for b in self.space.buckets:
            b.pending = len(b.variables)
            b.work = None
            b.launched = False
            b.updated = False
            b.gather = None

    def join_zero(self):
        """The compute stream waits for the side-stream gradient zeroing (before any gradient is written)."""
        zs = getattr(self, "_zero_pending", None)
        if zs is not None:
            torch.cuda.current_stream(self.space.device).wait_stream(zs)
            self._zero_pending = None

    def _on_grad_ready(self, var):
        b = var.bucket
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    def set_update_fn(self, fn):
        """``fn(target)`` runs the fused optimizer on one update target.  In sharded mode with overlapped
        reductions the reducer then updates and all-gathers every bucket during backward (the gather of the
        refreshed weights no longer waits for the whole backward, and never for the host)."""
        # Inside a hipGraph capture the per-bucket update and its all-gather are issued from the capturing (compute)
        # stream.  Cause of the round-2 segfault: ending a capture in which a side stream, forked from the capture
        # stream inside the autograd engine's device thread, ran the updates and issued the RCCL all-gathers made
        # hipStreamEndCapture segfault (reproduced in round 4 with MDTF_SHARDED_UPD_STREAM=1 inside capture,
        # gpurun_out/sharded_capture_r4c.log: SIGSEGV in torch.cuda.graphs capture_end); the same work issued from
        # the capture stream captures and replays bitwise equal to eager (tests/test_hip_graph.py).  The collectives
        # still run on RCCL's own stream beside backward; only the small fused update kernels run in line.
        # MDTF_SHARDED_CAPTURE_OVERLAP=0: no in-backward update inside a capture (gathers after the update).
        # Round 6: issuing the update from the capture stream right after the bucket's reduce-scatter made every
        # later backward kernel wait for that RS + update (the compute stream waited on the RS work in
        # _update_bucket, inside the bucket's own hook).  Inside a capture the update of bucket k is now issued when
        # bucket k+1 launches (MDTF_SHARDED_CAPTURE_UPD=lag, the default; the last one in end_backward): in the graph
        # the update node depends on RS_k and on the backward kernels issued before hook k+1, so RS_k runs beside a
        # whole bucket of backward and the compute stream only waits for an RS that has had that long to finish.
        # =fork runs the updates and all-gathers on a side stream the MAIN thread forks from the capture stream
        # before backward (fork_update_stream): still a hipStreamEndCapture segfault on ROCm 7 (r6,
        # tests/test_hip_graph.py sharded-fork, not run by default) -- the fork's thread was not the cause.
        # =inline is the round-5 behaviour.
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        self._capturing = capturing
        self._forked = False
        self._lagged = None
        self.launch_count = 0
        allowed = not capturing or os.environ.get("MDTF_SHARDED_CAPTURE_OVERLAP", "1") != "0"
        self.eager_update = fn if (self.mode == "sharded" and self.overlap and self.collective
                                   and self.R == self.world and allowed) else None

    CAPTURE_UPD = os.environ.get("MDTF_SHARDED_CAPTURE_UPD", "lag")

    def fork_update_stream(self):
        """Main thread, before backward, inside a capture: fork the update side stream from the capture stream
        (see set_update_fn).  A no-op outside a capture or when no in-backward update runs."""
        if self.eager_update is None or not getattr(self, "_capturing", False) or self.CAPTURE_UPD != "fork":
            return
        dev = self.space.device
        if self._upd_stream is None:
            self._upd_stream = torch.cuda.Stream(dev)
        self._upd_stream.wait_stream(torch.cuda.current_stream(dev))
        self._forked = True

    def _update_bucket(self, b):
        g = b.group
        sh = self._shards[id(g)]
        cuda = torch.device(g.device).type == "cuda"
        us = None
        # eager steps: a side stream forked here; inside a capture: the side stream the main thread forked before
        # backward (fork_update_stream), else the capture stream (see set_update_fn).  MDTF_SHARDED_UPD_STREAM=1
        # forks in this (autograd) thread inside a capture too: reproduces the round-4 EndCapture segfault.
        capt = getattr(self, "_capturing", False)
        env = os.environ.get("MDTF_SHARDED_UPD_STREAM", "")
        forked = capt and getattr(self, "_forked", False)
        side = cuda and (forked or env == "1" if capt else env != "0")
        self.bucket_updates = getattr(self, "bucket_updates", 0) + 1
        if capt:
            self.captured_bucket_updates = getattr(self, "captured_bucket_updates", 0) + 1
            # (bucket updated, buckets launched so far this step): lag mode updates bucket k after k+1 launched
            self.capture_update_log = getattr(self, "capture_update_log", []) + [
                (self.space.buckets.index(b), getattr(self, "launch_count", 0))]
            if not side:
                # the compute (capture) stream itself waits for this bucket's reduce-scatter
                self.capture_compute_waits = getattr(self, "capture_compute_waits", 0) + 1
        if side:
            if self._upd_stream is None:
                self._upd_stream = torch.cuda.Stream(g.device)
            us = self._upd_stream
            if not forked:
                us.wait_stream(torch.cuda.current_stream(g.device))
        ctx = torch.cuda.stream(us) if side else _NullCtx()
        with ctx, torch.no_grad():
            b.work.wait()                       # the update stream waits for this bucket's reduce-scatter
            b.work = None
            if self.comm_dtype != torch.float32:
                self._widen(b)
            o, n = b.shard_offset, b.shard_len
            total = sh["master"].numel()
            self.eager_update(_SliceTarget(g, sh["master"][o:o + n], sh["grad"][o:o + n],
                                           sh["out"][o:o + n] if g.shadow is not None else None, "shard", o, total))
            src = (sh["out"] if g.shadow is not None else sh["master"])[o:o + n]
            # .data: an alias with its own version counter -- the flat weight buffer's views are still saved by
            # backward nodes that have not run yet (the values they read are unchanged: this bucket's layers'
            # backward is complete), so the gather must not trip autograd's in-place check
            dst = (g.shadow if g.shadow is not None else g.master).data[b.start:b.end]
            b.gather = self._all_gather(dst, src)
        b.updated = True

    def _gloo_emulate(self):
        if not GLOO_VIA_ALLREDUCE or self.world == 1:
            return False
        if getattr(self, "_is_gloo", None) is None:
            self._is_gloo = dist.get_backend(self.pg) == "gloo"
        return self._is_gloo

    def _reduce_scatter(self, out, inp, async_op=True):
        """out (this rank's 1/world of inp) = sum over ranks of inp's shard.

        gloo emulation (GLOO_VIA_ALLREDUCE): all-reduces ``inp`` IN PLACE -- after the call the caller's gradient
        bucket holds the global sum, not the local gradient (the native reduce-scatter leaves it untouched).  Every
        caller passes the flat gradient bucket (or its bf16 wire copy), which nothing reads after its collective
        until begin_step zeroes it; a caller that needs the local gradient afterwards must pass a scratch copy."""
        if not self._gloo_emulate():
            return dist.reduce_scatter_tensor(out, inp, group=self.pg, async_op=async_op)
        n = out.numel()
        r = dist.get_rank(self.pg)
        w = dist.all_reduce(inp, group=self.pg, async_op=True)
        done = _DoneThen(w, lambda: out.copy_(inp[r * n:(r + 1) * n]))
        if not async_op:
            done.wait()
        return done

    def _all_gather(self, dst, src, async_op=True):
        """dst (world x src) = every rank's src, in rank order.

        gloo emulation: ``dst`` is zeroed and this rank's shard written before the async all-reduce, so until the
        returned work is waited on ``dst`` reads as zeros outside this rank's shard (neither old nor new values).
        Callers wait before any read: after_update / gather_full_* wait every gather, and the in-backward gathers
        target buckets whose layers' backward has completed."""
        if not self._gloo_emulate():
            return dist.all_gather_into_tensor(dst, src, group=self.pg, async_op=async_op)
        n = src.numel()
        r = dist.get_rank(self.pg)
        own = src.clone() if src.data_ptr() >= dst.data_ptr() and src.data_ptr() < dst.data_ptr() + dst.numel() * \
            dst.element_size() else src
        dst.zero_()
        dst[r * n:(r + 1) * n].copy_(own)
        w = dist.all_reduce(dst, group=self.pg, async_op=async_op)
        return w

    def _launch(self, b):
        if b.launched:
            return
        b.launched = True
        if not self.collective:
            return
        from ..ops import conv as _conv
        _conv.join_side_streams()          # side-stream weight gradients of this bucket are in
        g = b.group
        if self.comm_dtype != torch.float32:
            wire, wshard = self._wire_buffers(b)
            wire.copy_(g.grad[b.start:b.end])          # fp32 -> bf16 on the compute stream
            if self.mode == "allreduce":
                b.work = dist.all_reduce(wire, group=self.pg, async_op=True)
            else:
                b.work = self._reduce_scatter(wshard, wire)
        elif self.mode == "allreduce":
            b.work = dist.all_reduce(g.grad[b.start:b.end], group=self.pg, async_op=True)
        else:
            out = self._shards[id(g)]["grad"][b.shard_offset:b.shard_offset + b.shard_len]
            b.work = self._reduce_scatter(out, g.grad[b.start:b.end])
        if self.eager_update is not None:
            if getattr(self, "_capturing", False) and self.CAPTURE_UPD == "lag":
                prev, self._lagged = self._lagged, b
                self.launch_count = getattr(self, "launch_count", 0) + 1
                if prev is not None:
                    self._update_bucket(prev)
            else:
                self._update_bucket(b)

    def _flush_lagged(self):
        prev, self._lagged = getattr(self, "_lagged", None), None
        if prev is not None:
            self._update_bucket(prev)

    def _wire_buffers(self, b):
        """Persistent (graph-capture safe) bf16 wire buffers of one bucket."""
        ent = self._wire.get(id(b))
        if ent is None:
            g = b.group
            wire = torch.empty(b.numel, dtype=self.comm_dtype, device=g.device)
            wshard = (torch.empty(b.shard_len, dtype=self.comm_dtype, device=g.device)
                      if self.mode == "sharded" else None)
            ent = (wire, wshard)
            self._wire[id(b)] = ent
        return ent

    def _widen(self, b):
        """bf16 wire result -> the fp32 gradient the optimizer reads."""
        wire, wshard = self._wire[id(b)]
        g = b.group
        if self.mode == "allreduce":
            g.grad[b.start:b.end].copy_(wire)
        else:
            self._shards[id(g)]["grad"][b.shard_offset:b.shard_offset + b.shard_len].copy_(wshard)

    def _backup_buffers(self):
        """Stamp / offset / mask buffers, and the one-time calibration of every replica's device clock origin
        against the (shared) host clock: offset = device_ns - host_ns, all-gathered."""
        if self._bk is not None:
            return self._bk
        from ..ops import _native as N
        N.register("mdtf_stamp_realtime", [N.P, N.P])
        N.register("mdtf_backup_mask", [N.P, N.P, N.I, N.I, N.I, N.P, N.P])
        dev = torch.device(self.space.device)
        stamp = torch.zeros(1, dtype=torch.int64, device=dev)
        offsets = torch.zeros(self.world, dtype=torch.int64, device=dev)
        self._bk = {"stamp": stamp, "stamps": torch.zeros(self.world, dtype=torch.int64, device=dev),
                    "offsets": offsets, "mask": torch.ones(1, dtype=torch.float32, device=dev)}
        self._measure_clock_offsets()
        return self._bk

    def _measure_clock_offsets(self):
        """(Re)measure every replica's device-clock origin into the existing ``offsets`` buffer, in place, so a
        captured step graph that reads it sees the new values.  A collective over the group, host-synchronous:
        never called while a hipGraph is being captured."""
        import time
        from ..ops import _native as N
        bk = self._bk
        dev = torch.device(self.space.device)
        stamp = bk["stamp"]
        best = None
        for _ in range(5):                  # the tightest of a few host brackets around one device stamp
            torch.cuda.synchronize(dev)
            t0 = time.monotonic_ns()        # one system-wide clock for every rank of the node
            N.check(N.fn("mdtf_stamp_realtime")(N.ptr(stamp), N.stream_ptr()), "stamp_realtime")
            torch.cuda.synchronize(dev)
            t1 = time.monotonic_ns()
            if best is None or t1 - t0 < best[0]:
                best = (t1 - t0, int(stamp.item()) * 10 - (t0 + t1) // 2)
        off = torch.tensor([best[1]], dtype=torch.int64, device=dev)
        gathered = torch.zeros(self.world, dtype=torch.int64, device=dev)
        dist.all_gather(list(gathered.view(self.world, 1).unbind(0)), off, group=self.pg)
        bk["offsets"].copy_(gathered)
        torch.cuda.synchronize(dev)
        bk["at"] = None                         # set by the next step that uses the offsets

    BACKUP_RECALIBRATE_STEPS = 1000      # device-clock offsets re-measured this often (refclk drift)

    def refresh_backup_clock(self, step):
        """Host-side, between steps (also between hipGraph replays, which run no Python of the step): re-measure
        the clock offsets every BACKUP_RECALIBRATE_STEPS global steps.  Every replica reaches the same global step,
        so the collective re-measure is matched.  A step counter that went BACK (a restore after a recovery)
        restarts the period."""
        bk = self._bk
        if bk is None or not self.backup_device:
            return False
        at = bk.get("at")
        if at is None or step < at:
            bk["at"] = step
            return False
        if step - at < self.BACKUP_RECALIBRATE_STEPS:
            return False
        self._measure_clock_offsets()
        bk["at"] = step
        return True

    def _backup_mask_device(self, step=0):
        from ..ops import _native as N
        if not torch.cuda.is_current_stream_capturing():
            self.refresh_backup_clock(step)     # never inside a capture (host syncs and a collective)
        bk = self._backup_buffers()
        if bk.get("at") is None:
            bk["at"] = step
        N.check(N.fn("mdtf_stamp_realtime")(N.ptr(bk["stamp"]), N.stream_ptr()), "stamp_realtime")
        dist.all_gather(list(bk["stamps"].view(self.world, 1).unbind(0)), bk["stamp"], group=self.pg)
        N.check(N.fn("mdtf_backup_mask")(N.ptr(bk["stamps"]), N.ptr(bk["offsets"]), self.world, self.rank, self.R,
                                         N.ptr(bk["mask"]), N.stream_ptr()), "backup_mask")
        for g in self.space.groups:
            g.grad.mul_(bk["mask"])         # a backup replica contributes zeros (TF drops its push as stale)
        return bk["mask"]

    def end_backward(self, step=0):
        """Finish all reductions; returns the gradient scale (1/contributors)."""
        from ..ops import conv as _conv
        self.join_zero()
        _conv.join_side_streams()          # every weight gradient is in the flat buffer
        V.unclaimed_skips(self.space.variables)   # skipped slots no kernel wrote this step hold stale sums
        if self.backup_device:
            self.contributed = self._backup_mask_device(step)  # device 0/1 (read only when someone asks)
            self.num_contributors = self.R
        elif self.world > 1 and self.R < self.world:
            # the ticket is taken after this replica's backward has COMPLETED on the device (not
            # merely been enqueued), so "first R" means first R to finish computing
            if self.space.device is not None and torch.device(self.space.device).type == "cuda":
                torch.cuda.current_stream(self.space.device).synchronize()
            order = self.store.add("mdtf/sync_replicas/%d" % step, 1)
            self.contributed = order <= self.R
            if not self.contributed:
                self.space.zero_grad()     # a stale/backup replica: TF drops its gradients
            if self.rank == 0 and step >= 2:
                try:
                    self.store.delete_key("mdtf/sync_replicas/%d" % (step - 2))
                except Exception:
                    pass
            self.num_contributors = self.R
        else:
            self.num_contributors = self.world
        for b in self.space.buckets:
            if not b.launched:
                self._launch(b)
        self._flush_lagged()
        for b in self.space.buckets:
            if b.work is not None:
                b.work.wait()
                b.work = None
                if self.comm_dtype != torch.float32:
                    self._widen(b)
        if not self.collective and self.mode == "sharded":
            for g in self.space.groups:
                self._shards[id(g)]["grad"].copy_(self._gather_index(g, g.grad))
        return 1.0 / self.num_contributors

    def _gather_index(self, g, full):
        # world == 1: the shard is the whole bucket (minus nothing)
        return torch.cat([full[b.start:b.end] for b in g.buckets])

    def update_targets(self):
        if self.eager_update is not None and all(getattr(b, "updated", False) for b in self.space.buckets):
            return []                           # every bucket was updated during backward
        out = []
        for g in self.space.groups:
            if self.mode == "allreduce":
                out.append(UpdateTarget(g, g.master, g.grad, g.shadow, "full"))
            else:
                sh = self._shards[id(g)]
                out.append(UpdateTarget(g, sh["master"], sh["grad"], sh["out"] if g.shadow is not None else None,
                                        "shard"))
        return out

    def after_update(self):
        """Sharded mode: all-gather refreshed compute weights to every rank."""
        if self.mode != "sharded":
            return
        if self.eager_update is not None and all(getattr(b, "updated", False) for b in self.space.buckets):
            # the gathers were issued during backward: the compute stream (and a capture) joins them here,
            # a stream dependency, not a host wait
            for b in self.space.buckets:
                if b.gather is not None:
                    b.gather.wait()
                    b.gather = None
            if self._upd_stream is not None:
                torch.cuda.current_stream(self.space.device).wait_stream(self._upd_stream)
            return
        works = []
        for g in self.space.groups:
            sh = self._shards[id(g)]
            src = sh["out"] if g.shadow is not None else sh["master"]
            dst_full = g.shadow if g.shadow is not None else g.master
            for b in g.buckets:
                part = src[b.shard_offset:b.shard_offset + b.shard_len]
                dst = dst_full[b.start:b.end]
                if not self.collective:
                    dst.copy_(part)
                else:
                    works.append(self._all_gather(dst, part))
        for w in works:
            w.wait()

    # -- full-state helpers -------------------------------------------------
    def gather_full_master(self):
        """Make every rank's full fp32 master current (checkpointing, eval)."""
        if self.mode != "sharded":
            return
        for g in self.space.groups:
            if g.shadow is None:
                continue  # fp32 groups are gathered every step
            sh = self._shards[id(g)]
            for b in g.buckets:
                part = sh["master"][b.shard_offset:b.shard_offset + b.shard_len]
                dst = g.master[b.start:b.end]
                if self.world == 1:
                    dst.copy_(part)
                else:
                    self._all_gather(dst, part, async_op=False)

    def gather_full_state(self, target_key, name):
        """Full-size optimizer state buffer for checkpointing (sharded → gathered)."""
        out = []
        for g in self.space.groups:
            if self.mode == "allreduce":
                out.append(g.state_buffer("full/%s" % name, g.numel))
                continue
            sh_state = g.state_buffer("shard/%s" % name, self._shards[id(g)]["master"].numel())
            full = torch.zeros(g.numel, dtype=torch.float32, device=g.device)
            for b in g.buckets:
                part = sh_state[b.shard_offset:b.shard_offset + b.shard_len]
                if self.world == 1:
                    full[b.start:b.end].copy_(part)
                else:
                    self._all_gather(full[b.start:b.end], part, async_op=False)
            out.append(full)
        return out

    def scatter_full_state(self, name, fulls):
        """Inverse of :meth:`gather_full_state` (restore)."""
        for g, full in zip(self.space.groups, fulls):
            if self.mode == "allreduce":
                g.state_buffer("full/%s" % name, g.numel).copy_(full)
                continue
            sh_state = g.state_buffer("shard/%s" % name, self._shards[id(g)]["master"].numel())
            for b in g.buckets:
                s = b.start + self.rank * b.shard_len
                sh_state[b.shard_offset:b.shard_offset + b.shard_len].copy_(full[s:s + b.shard_len])

    def broadcast_parameters(self, src=0):
        """Chief → all: master weights and non-trainable variables (session init)."""
        if self.world > 1:
            for g in self.space.groups:
                dist.broadcast(g.master, src=self._global_src(src), group=self.pg)
        self.space.refresh_shadows()
        self.load_shards_from_master()

    def _global_src(self, src):
        if self.pg is None or self.pg == dist.group.WORLD:
            return src
        return dist.get_global_rank(self.pg, src)
