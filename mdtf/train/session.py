"""Sessions: ``tf.Session`` / ``MonitoredTrainingSession`` semantics on eager kernels.

Reference: ``distribute_train.py:169-206`` — ``MonitoredTrainingSession(master,
is_chief, checkpoint_dir, scaffold=Scaffold(init_op, init_fn), hooks=[StopAtStep,
SyncReplicas], save_checkpoint_secs=600, config, stop_grace_period_secs=60,
log_step_count_steps=100)`` then ``while not sess.should_stop(): sess.run(...)``.

Creation protocol (TF1 semantics):
  1. every TrainOp is finalised — variables re-homed into flat buffers, the
     gradient reducer bound to the worker process group (RCCL/gloo);
  2. the chief restores the latest checkpoint of ``checkpoint_dir`` if one
     exists, otherwise runs ``init_op`` / ``init_fn`` (warm start);
  3. the chief's state (weights, non-trainable variables, optimizer slots,
     global step) is broadcast to every replica — the "ready" barrier non-chief
     workers wait on (fix for SURVEY Q7: one global step, owned by the chief);
  4. hooks: ``begin`` → create → ``after_create_session``.
``close`` runs ``end`` on every hook (the checkpoint hook saves a final
checkpoint) and is safe to call twice.

Recovery (TF's ``_RecoverableSession``): a ``run`` that raises ``mdtf.errors.AbortedError`` /
``UnavailableError`` (or a transient store failure, ``mdtf.errors.as_recoverable``) re-creates the
session in this process — captured step graphs released, the latest checkpoint restored (else the
chief's broadcast state), hooks' ``after_create_session`` called again — and retries the step, up to
``max_recoveries`` times.

With several replicas the restore is a collective, so the replicas first AGREE, at a step boundary, that
one of them failed (reference ``distribute_train.py:169-180``: TF re-creates every worker's session when
a PS restart aborts them).  Every ``run`` does, on every replica and in the same place:
``before_run`` hooks -> one host all-reduce(MAX) of a code (0 ok, 1 recovery needed, 2 fatal) over a gloo
group of the replicas -> the step -> ``after_run`` hooks.  A recoverable error raised on ONE replica by a
hook, or inside the step once the step's collectives have been issued (a device error, a store failure), is
held and its code sent at the next agreement; then every replica re-creates its session from the chief's
latest checkpoint in process and they continue from the same global step (the failing replica retries the
run that raised).  A non-recoverable error in ``before_run`` still joins the agreement with code 2, so every
replica stops at that boundary instead of waiting in the next step's collectives.  An error that stops a
replica before it issues the step's collectives leaves its peers inside them: that ends in the collective
timeout / heartbeat watchdog and the job supervisor's restart (``mdtf.cluster.health.supervise``).

Multi-replica ``run`` calls must stay in lockstep (every replica calls ``run`` the same number of times, in the
same order): the agreement is a collective.  Fetch-only runs on one replica (the chief reading a variable)
belong outside the session (``Variable.value()``, ``Saver``).
"""
import os
import time

import torch

from ..utils import log as logger
from . import hooks as H
from . import step as S
from . import variables as V


class Scaffold(object):
    def __init__(self, init_op=None, init_feed_dict=None, init_fn=None, ready_op=None, local_init_op=None,
                 summary_op=None, saver=None, copy_from_scaffold=None):
        self.init_op = init_op
        self.init_feed_dict = init_feed_dict
        self.init_fn = init_fn
        self.ready_op = ready_op
        self.local_init_op = local_init_op
        self.summary_op = summary_op
        self.saver = saver

    def finalize(self):
        return self


def global_variables_initializer():
    """Variables are initialised at creation; kept for API parity (returns a no-op)."""
    return None


def _flatten(fetches):
    """Return (flat list, rebuild fn)."""
    if isinstance(fetches, (list, tuple)):
        parts = [_flatten(f) for f in fetches]
        flat = [x for p in parts for x in p[0]]

        def rebuild(vals, parts=parts, typ=type(fetches)):
            out, i = [], 0
            for p in parts:
                n = len(p[0])
                out.append(p[1](vals[i:i + n]))
                i += n
            return typ(out) if typ is not list else out
        return flat, rebuild
    if isinstance(fetches, dict):
        keys = list(fetches)
        parts = [_flatten(fetches[k]) for k in keys]
        flat = [x for p in parts for x in p[0]]

        def rebuild(vals, parts=parts, keys=keys):
            out, i = {}, 0
            for k, p in zip(keys, parts):
                n = len(p[0])
                out[k] = p[1](vals[i:i + n])
                i += n
            return out
        return flat, rebuild
    return [fetches], lambda vals: vals[0]


def _evaluate(f, ctx):
    if f is None:
        return None
    if isinstance(f, V.GlobalStep):
        return f.value()
    if isinstance(f, V.Variable):
        return S._host_value(f.master)
    if isinstance(f, S.Fetchable):
        return f.evaluate(ctx)
    if isinstance(f, torch.Tensor):
        return S._host_value(f)
    raise TypeError("Cannot fetch %r" % (f,))


class Session(object):
    """Plain session: ``run(fetches, feed_dict)`` with graph-like semantics."""

    def __init__(self, target="", graph=None, config=None):
        self.target = target
        self.config = config
        self._closed = False

    def run_raw(self, fetches, feed_dict=None):
        flat, rebuild = _flatten(fetches)
        ctx = S.RunContext(feed_dict, self)
        # train ops first: StepTensors fetched alongside read the training forward
        vals = [None] * len(flat)
        order = sorted(range(len(flat)), key=lambda i: 0 if isinstance(flat[i], S.TrainOp) else 1)
        for i in order:
            vals[i] = _evaluate(flat[i], ctx)
        return rebuild(vals)

    run = run_raw

    def close(self):
        self._closed = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def should_stop(self):
        return False


class MonitoredSession(Session):
    def __init__(self, hooks=None, is_chief=True, checkpoint_dir=None, scaffold=None, server=None,
                 stop_grace_period_secs=120, max_recoveries=None):
        super(MonitoredSession, self).__init__()
        self.max_recoveries = int(os.environ.get("MDTF_MAX_RECOVERIES", "3")) if max_recoveries is None \
            else int(max_recoveries)
        self.recoveries = 0
        self._hooks = list(hooks or [])
        self.is_chief = is_chief
        self.checkpoint_dir = checkpoint_dir
        self.scaffold = scaffold or Scaffold()
        self.server = server
        self._stop = False
        self.restored_from = None
        self._agree_pg = None          # gloo group of the replicas for the recovery agreement (world > 1)
        self._pending = None           # recoverable error (hook or step) held for the next agreement
        self._agree_buf = None
        self.agreements = 0
        self._agree_async = os.environ.get("MDTF_AGREE", "async") != "sync"
        self._agree_work = None        # async agreement in flight: (work, result tensor)
        self._posted_err = None
        for h in self._hooks:
            h.begin()
        self._create()
        for h in self._hooks:
            h.after_create_session(self, None)

    # -- creation ----------------------------------------------------------
    def _process_group(self):
        srv = self.server
        if srv is None:
            from ..cluster import server as srv_mod
            srv = srv_mod.current()
        if srv is not None and srv.worker_group is not None:
            return srv.worker_group, srv.store
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.group.WORLD, None
        return None, None

    def _create(self):
        import torch.distributed as dist
        pg, store = self._process_group()
        ops = S.train_ops()
        for op in ops:
            op.finalize(pg, store)
        V.get_store().frozen = True
        if V.get_global_step() is None:
            V.get_or_create_global_step()
        from .saver import Saver, latest_checkpoint
        distributed = dist.is_available() and dist.is_initialized() and pg is not None
        multi = distributed and dist.get_world_size(pg) > 1
        if multi and self._agree_pg is None and self.max_recoveries > 0:
            self._agree_pg = self._agreement_group(pg)
        # the chief picks the checkpoint; EVERY replica restores it (each takes its own
        # optimizer-state shard in sharded mode), so no restored state is broadcast
        ckpt = None
        if self.is_chief and self.checkpoint_dir:
            ckpt = latest_checkpoint(self.checkpoint_dir)
        if multi:
            box = [ckpt]
            src = dist.get_global_rank(pg, 0) if pg is not dist.group.WORLD else 0
            dist.broadcast_object_list(box, src=src, group=pg)
            ckpt = box[0]
        restored = False
        if ckpt:
            saver = self.scaffold.saver or Saver()
            reader = None
            if multi and not self._visible_everywhere(ckpt, pg):
                # node-local model_dir: only the chief can read the files; it broadcasts the
                # tensors and every replica restores from them (its own shard in sharded mode)
                from .saver import TensorDictReader, read_all
                box = [read_all(ckpt) if self.is_chief else None]
                src = dist.get_global_rank(pg, 0) if pg is not dist.group.WORLD else 0
                dist.broadcast_object_list(box, src=src, group=pg)
                reader = TensorDictReader(box[0])
                logger.info("checkpoint %s is not visible on every replica: restoring from the chief's copy" % ckpt)
            saver.restore(self, ckpt, reader=reader)
            self.restored_from = ckpt
            restored = True
            logger.info("Restored from checkpoint %s (global_step %d)" % (ckpt, V.get_global_step().value()))
            for op in ops:
                op.step_count = V.get_global_step().value()
        elif multi:
            self._broadcast_state(pg)
        else:
            for op in ops:
                op.reducer.load_shards_from_master()
        if self.is_chief and not restored and self.scaffold.init_fn is not None:
            self.scaffold.init_fn(self.scaffold, self)
            if multi:
                self._broadcast_state(pg)
        for op in ops:
            op.space.refresh_shadows()
            op.reducer.load_shards_from_master()

    @staticmethod
    def _agreement_group(pg):
        """A gloo (host) group over the same replicas: the per-step agreement never touches the device
        stream, so it neither syncs the host with the GPU nor enters a captured step graph."""
        import torch.distributed as dist
        if dist.get_backend(pg) == "gloo":
            return pg
        ranks = list(range(dist.get_world_size())) if pg is dist.group.WORLD else \
            [dist.get_global_rank(pg, i) for i in range(dist.get_world_size(pg))]
        return dist.new_group(ranks, backend="gloo", use_local_synchronization=True)

    AGREE_OK, AGREE_RECOVER, AGREE_FATAL = 0, 1, 2

    def _agree(self, code):
        """All-reduce(MAX) of this replica's code (0 ok, 1 recovery needed, 2 non-recoverable error): the
        worst code of any replica.  One 4-byte gloo all-reduce per step; its cost at 8 ranks is in
        ``profiles/agree_cost_r4.json`` (``bench/agree_cost.py``)."""
        import torch.distributed as dist
        t = self._agree_buf
        if t is None:
            t = self._agree_buf = torch.zeros(1, dtype=torch.int32)
        t.fill_(int(code))
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self._agree_pg)
        return int(t.item())

    @staticmethod
    def _visible_everywhere(ckpt, pg):
        """All-reduce(MIN) of 'this replica sees <ckpt>.index' over the group."""
        import os
        import torch.distributed as dist
        dev = V.get_store().device if dist.get_backend(pg) == "nccl" else "cpu"
        seen = torch.tensor([1 if os.path.exists(ckpt + ".index") else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(seen, op=dist.ReduceOp.MIN, group=pg)
        return bool(seen.item())

    def _broadcast_state(self, pg):
        """Chief (group rank 0) → every replica."""
        import torch.distributed as dist
        src = dist.get_global_rank(pg, 0) if pg is not dist.group.WORLD else 0
        store = V.get_store()
        for op in S.train_ops():
            for g in op.space.groups:
                dist.broadcast(g.master, src=src, group=pg)
                for key in sorted(g.state):     # same order on every rank
                    dist.broadcast(g.state[key], src=src, group=pg)
        for v in store.global_variables():
            if not v.trainable:
                dist.broadcast(v.master, src=src, group=pg)
        gs = torch.tensor([V.get_global_step().value()], dtype=torch.int64,
                          device=store.device if dist.get_backend(pg) == "nccl" else "cpu")
        dist.broadcast(gs, src=src, group=pg)
        V.get_global_step().assign(int(gs.item()))
        for op in S.train_ops():
            op.step_count = V.get_global_step().value()

    # -- running -----------------------------------------------------------
    def run(self, fetches, feed_dict=None, options=None, run_metadata=None):
        from .. import errors
        if self._agree_pg is not None:
            return self._run_agreed(fetches, feed_dict)
        while True:
            try:
                return self._run_once(fetches, feed_dict)
            except Exception as e:  # noqa: BLE001 - classified below
                err = errors.as_recoverable(e)
                if err is None or self.recoveries >= self.max_recoveries:
                    raise
                self.recoveries += 1
                logger.warn("session run failed with %s (%s); re-creating the session (recovery %d of %d)" % (
                    type(err).__name__, err, self.recoveries, self.max_recoveries))
                self._recreate()

    def _run_agreed(self, fetches, feed_dict):
        """Multi-replica run: hooks, step-boundary agreement, step (see the module docstring).

        ``MDTF_AGREE=async`` (default): the boundary's all-reduce is POSTED and the step runs while it travels;
        its result is read at the next boundary (one step later), where every replica sees the same code and
        acts on it together: the per-step cost is a post and a wait on a completed work instead of a blocking
        host round trip (``profiles/agree_cost_r4.json``).  A replica that must stop or recover still runs the
        step it posted the code with, so no peer is left inside that step's collectives.
        ``MDTF_AGREE=sync``: the all-reduce completes before the step (acted on at the same boundary)."""
        from .. import errors
        async_mode = self._agree_async
        while True:
            if self._stop:
                raise RuntimeError("Run called even after should_stop requested.")
            if async_mode and self._agree_work is not None:
                agreed = self._agree_result()        # the code posted one boundary ago
                if agreed >= self.AGREE_FATAL:
                    raise RuntimeError("a peer replica stopped on a non-recoverable error (agreed one step boundary "
                                       "later)")
                if agreed == self.AGREE_RECOVER:
                    self._recover_agreed()
                    continue
            pre = None
            fatal = None
            try:
                pre = self._before_run(fetches, feed_dict)
            except Exception as e:  # noqa: BLE001 - classified below
                err = errors.as_recoverable(e)
                if err is None:
                    fatal = e                # still join the agreement, so the peers stop too (no hang)
                else:
                    self._pending = self._pending or err
            code = self.AGREE_FATAL if fatal is not None else (
                self.AGREE_RECOVER if self._pending is not None else self.AGREE_OK)
            if async_mode:
                self._agree_post(code)
                if code == self.AGREE_RECOVER:
                    self._posted_err = self._posted_err or self._pending
                    self._pending = None     # posted; acted on when the result is read
            else:
                agreed = self._agree(code)
                self.agreements += 1
                if fatal is not None:
                    raise fatal
                if agreed >= self.AGREE_FATAL:
                    raise RuntimeError("a peer replica stopped on a non-recoverable error at this step boundary")
                if agreed == self.AGREE_RECOVER:
                    self._recover_agreed()
                    continue                 # retry this run on the restored state
            if pre is None:
                rc, extra, feed = None, {}, dict(feed_dict or {})
            else:
                rc, extra, feed = pre
            try:
                results = self.run_raw(self._all_fetches(fetches, extra), feed)
            except Exception as e:  # noqa: BLE001 - classified below
                err = errors.as_recoverable(e)
                if err is None:
                    raise
                # a recoverable error inside the step on this replica (e.g. a device or store error detected
                # once the step's collectives were issued): hold it, agree with the peers at their next step
                # boundary, recover there together and retry this run.  An error that stops this replica
                # BEFORE it issues the step's collectives leaves the peers waiting in them: that case ends in
                # the collective timeout / heartbeat watchdog and the supervisor's restart
                # (mdtf.cluster.health), as in TF when a worker dies mid-step.
                self._pending = err
                logger.warn("%s inside the step on this replica; recovery is agreed at the next step boundary"
                            % type(err).__name__)
                continue
            if fatal is not None:
                # async: the step ran (its collectives are matched on every replica); the peers stop at the next
                # boundary when they read code 2.  This replica stops now.
                raise fatal
            if rc is None:
                # async: a hook raised a recoverable error in before_run.  The step ran so the peers' collectives
                # are matched; this replica has no run context for it, so its after_run hooks are skipped, and the
                # posted RECOVER code re-creates every replica together at the next boundary.
                return results["__user__"]
            try:
                self._after_run(rc, extra, results)
            except Exception as e:  # noqa: BLE001 - classified below
                err = errors.as_recoverable(e)
                if err is None:
                    raise
                self._pending = err          # every replica finished this step's collectives: agree next run
                logger.warn("%s after the step on this replica; recovery is agreed at the next step boundary"
                            % type(err).__name__)
            if rc.stop_requested:
                self._stop = True
            return results["__user__"]

    def _agree_post(self, code):
        import torch.distributed as dist
        t = torch.full((1,), int(code), dtype=torch.int32)
        self._agree_work = (dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self._agree_pg, async_op=True), t)
        self.agreements += 1

    def _agree_result(self):
        work, t = self._agree_work
        self._agree_work = None
        work.wait()
        return int(t.item())

    def _recover_agreed(self):
        from .. import errors
        err = self._posted_err or self._pending or errors.AbortedError(
            message="a peer replica requested session recovery")
        self._pending = None
        self._posted_err = None
        if self.recoveries >= self.max_recoveries:
            raise err
        self.recoveries += 1
        logger.warn("replica recovery agreed (%s: %s); re-creating the session from the chief's checkpoint "
                    "(recovery %d of %d)" % (type(err).__name__, err, self.recoveries, self.max_recoveries))
        self._recreate()

    def _recreate(self):
        """Drop per-session device state and create again: restore the latest checkpoint, re-broadcast."""
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        S.release_graphs()
        self.restored_from = None
        self._create()
        for h in self._hooks:
            h.after_create_session(self, None)

    def _before_run(self, fetches, feed_dict):
        args = H.SessionRunArgs(fetches, feed_dict)
        rc = H.SessionRunContext(args, self)
        extra = {}
        feed = dict(feed_dict or {})
        for h in self._hooks:
            req = h.before_run(rc)
            if req is not None:
                extra[h] = req.fetches
                if req.feed_dict:
                    feed.update(req.feed_dict)
        return rc, extra, feed

    @staticmethod
    def _all_fetches(fetches, extra):
        all_fetches = {"__user__": fetches}
        for i, (h, f) in enumerate(extra.items()):
            all_fetches["__hook%d__" % i] = f
        return all_fetches

    def _after_run(self, rc, extra, results):
        for h in self._hooks:
            key = None
            if h in extra:
                key = "__hook%d__" % list(extra).index(h)
            h.after_run(rc, H.SessionRunValues(results.get(key) if key else None))

    def _run_once(self, fetches, feed_dict=None):
        if self._stop:
            raise RuntimeError("Run called even after should_stop requested.")
        rc, extra, feed = self._before_run(fetches, feed_dict)
        results = self.run_raw(self._all_fetches(fetches, extra), feed)
        self._after_run(rc, extra, results)
        if rc.stop_requested:
            self._stop = True
        return results["__user__"]

    def request_stop(self):
        self._stop = True

    def should_stop(self):
        return self._stop

    def _drain_agreement(self):
        """The last posted agreement (every replica posted one in its last run): complete it."""
        if self._agree_work is None:
            return
        try:
            if self._agree_result() != self.AGREE_OK:
                logger.warn("a recovery / stop request agreed at the last step boundary is dropped: the session "
                            "is closing")
        except Exception as e:  # noqa: BLE001 - closing anyway
            logger.warn("agreement drain at close failed: %s" % e)

    def close(self):
        if self._closed:
            return
        self._closed = True
        self._drain_agreement()
        for h in self._hooks:
            h.end(self)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        from . import step as step_mod
        step_mod.release_graphs()            # captured steps hold collectives of the current process group

    def __exit__(self, exc_type, exc, tb):
        if exc_type is None:
            self.close()
        else:
            self._closed = True
        return False


COLLECTIVE_SAVE_STEPS = 1000


def _collective_save(server=None):
    """True when a checkpoint save is a collective over the worker replicas (sharded mode, world > 1)."""
    if not any(getattr(op.optimizer, "mode", None) == "sharded" for op in S.train_ops()):
        return False
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return False
    srv = server
    if srv is None:
        from ..cluster import server as srv_mod
        srv = srv_mod.current()
    pg = srv.worker_group if srv is not None and srv.worker_group is not None else None
    return dist.get_world_size(pg) > 1


def MonitoredTrainingSession(master="", is_chief=True, checkpoint_dir=None, scaffold=None, hooks=None,
                             chief_only_hooks=None, save_checkpoint_secs=600, save_summaries_steps=100,
                             save_summaries_secs=None, config=None, stop_grace_period_secs=120,
                             log_step_count_steps=100, max_wait_secs=7200, save_checkpoint_steps=None,
                             summary_dir=None, server=None, max_recoveries=None):
    """TF1's MonitoredTrainingSession factory with the same default hooks.

    Sharded mode (``SyncReplicasOptimizer(mode='sharded')``, the PS-shard data-parallel path) with more
    than one replica makes ``Saver.save`` a collective: the optimizer shards and the fp32 masters are
    all-gathered.  TF's chief-only, time-triggered checkpoint hook would hang there (the other replicas
    never join) or fire on different steps per replica, so in that case the hook is installed on EVERY
    replica and triggered by step count (``save_checkpoint_steps``, else :data:`COLLECTIVE_SAVE_STEPS`).
    """
    scaffold = scaffold or Scaffold()
    all_hooks = list(hooks or [])
    collective = _collective_save(server)
    if (collective and checkpoint_dir and (save_checkpoint_secs or save_checkpoint_steps)
            and not any(isinstance(h, H.CheckpointSaverHook) for h in all_hooks)):
        steps = save_checkpoint_steps or COLLECTIVE_SAVE_STEPS
        if not save_checkpoint_steps:
            logger.warn("sharded replicas save collectively: save_checkpoint_secs=%s replaced by a step trigger "
                        "every %d steps on every replica" % (save_checkpoint_secs, steps))
        all_hooks.append(H.CheckpointSaverHook(checkpoint_dir, save_steps=steps, scaffold=scaffold))
        save_checkpoint_secs = save_checkpoint_steps = None
    if is_chief:
        all_hooks += list(chief_only_hooks or [])
        summary_dir = summary_dir or checkpoint_dir
        if log_step_count_steps and log_step_count_steps > 0:
            all_hooks.append(H.StepCounterHook(every_n_steps=log_step_count_steps))
        if summary_dir and (save_summaries_steps or save_summaries_secs):
            all_hooks.append(H.SummarySaverHook(save_steps=save_summaries_steps if not save_summaries_secs else None,
                                                save_secs=save_summaries_secs, output_dir=summary_dir))
        if checkpoint_dir and (save_checkpoint_secs or save_checkpoint_steps):
            all_hooks.append(H.CheckpointSaverHook(
                checkpoint_dir, save_secs=save_checkpoint_secs if not save_checkpoint_steps else None,
                save_steps=save_checkpoint_steps, scaffold=scaffold))
    return MonitoredSession(all_hooks, is_chief, checkpoint_dir, scaffold, server, stop_grace_period_secs,
                            max_recoveries=max_recoveries)
