"""Asynchronous parameter-server training (``--ps_mode=async``).

BASELINE config "ResNet-152 async parameter-server mode, 2 ps + 6 workers on one
node".  The reference only has the synchronous SyncReplicas path
(``distribute_train.py:146-160``) with its ``replicas_to_aggregate`` flag; its
PS tasks hold variables in host memory behind TF gRPC (``distribute.py:81``).

MI355X design:

* every PS task is a rank with its own GPU; the variables placed on it by
  ``replica_device_setter`` (greedy by bytes) live in *its* HBM as flat fp32
  master + optimizer-state buffers, grouped exactly like each worker's
  ``FlatParamSpace`` groups for that PS (so a group travels as ONE contiguous
  message, no packing);
* workers run forward/backward on their own GPU and exchange with every PS by
  point-to-point RCCL send/recv over xGMI (gloo on CPU): push fp32 gradients,
  receive the updated compute weights (bf16 shadow, or fp32 for fp32 groups);
* the data plane never touches the cluster store: every PS keeps one posted
  receive of a 2-word request header ``[kind, version]`` per worker and polls
  them; a ``push`` header is followed by the worker's gradients (bf16 on the
  wire: half the bytes, widened into the fp32 gradient the optimizer reads),
  received into per-worker buffers so several workers' payloads stream in
  concurrently, and applied in completion order (no aggregation, no barrier)
  with the fused optimizer kernel; the reply is the PS version + the refreshed
  compute weights;
* workers overlap: the push of step t and its reply travel while forward and
  backward of step t+1 run on the weights already held (the reply lands in a
  staging copy, swapped in before the next push) -- one step of built-in
  staleness, the classic async-PS trade;
* staleness (PS version at apply time minus the version the gradient was
  computed from) is measured per update and reported, with the PS's busy /
  idle split;
* ``global_step`` = updates applied by PS 0 (every push reaches every PS),
  returned in each reply; workers stop at ``total_step`` and send a ``done``
  header; PS tasks exit when every worker is done (the reference's done-queue,
  ``distribute_train.py:86-90``);
* the chief pulls the fp32 masters from every PS and writes a sharded
  tensor-bundle checkpoint (one data file per PS task — the TF layout).
"""
import json
import os
import time

import torch
import torch.distributed as dist

from ..train import variables as V
from ..utils import log as logger
from .flat import FlatParamSpace
from .reducer import UpdateTarget

_PREFIX = "mdtf/async"


def _groups_by_ps(space_groups, num_ps):
    out = {p: [] for p in range(num_ps)}
    for g in space_groups:
        out[g.ps_task].append(g)
    return out


class _PSGroupedSpace(FlatParamSpace):
    """FlatParamSpace whose groups never mix variables of different PS tasks."""

    def __init__(self, variables, device, compute_dtype, num_ps):
        from .flat import FlatGroup
        import collections
        self.device = device
        self.compute_dtype = compute_dtype
        by_key = collections.OrderedDict()
        for v in reversed(list(variables)):
            shadow = compute_dtype if (compute_dtype is not None and not v.keep_fp32
                                       and compute_dtype != torch.float32) else None
            by_key.setdefault((int(v.ps_task or 0) % num_ps, shadow, bool(v.apply_weight_decay)), []).append(v)
        self.groups = []
        for (p, sd, dec), vs in sorted(by_key.items(), key=lambda kv: (kv[0][0], str(kv[0][1]), kv[0][2])):
            g = FlatGroup(vs, device, sd, dec)
            g.ps_task = p
            self.groups.append(g)
        self.variables = list(variables)


def _varspec(variables):
    # pad_rows travels too: the PS must rebuild the same flat layout (e.g. BERT's tied decoder reserves zero rows
    # after the word embedding and the MLM bias), or every chief send / push / pull would differ in size
    return [{"name": v.name, "shape": list(v.shape), "keep_fp32": bool(v.keep_fp32),
             "decay": bool(v.apply_weight_decay), "ps": int(v.ps_task or 0),
             "pad_rows": int(getattr(v, "pad_rows", 0) or 0)} for v in variables]


K_PULL, K_PUSH, K_DONE, K_MASTER = 0, 1, 2, 3


class _Posted(object):
    """A posted receive whose completion is polled without blocking, on both backends.  An RCCL work answers
    ``is_completed()`` from its HIP event; a gloo receive completes only inside ``wait()`` (its
    ``is_completed()`` stays False), so a helper thread waits on it and the poll reads a flag.  A failed
    receive (peer died, gloo timeout) is re-raised from ``done()`` / ``wait()`` in the service loop, so the PS
    fails for the supervisor to restart instead of polling forever."""
    __slots__ = ("work", "ev", "err", "wake")

    def __init__(self, work, threaded, wake=None):
        self.work = work
        self.ev = None
        self.err = None
        self.wake = wake
        if threaded:
            import threading
            self.ev = threading.Event()
            threading.Thread(target=self._wait, daemon=True).start()

    def _wait(self):
        try:
            self.work.wait()
        except BaseException as e:  # noqa: BLE001 - handed to the service loop
            self.err = e
        finally:
            self.ev.set()
            if self.wake is not None:
                self.wake.set()

    def done(self):
        if self.ev is not None:
            if not self.ev.is_set():
                return False
            if self.err is not None:
                raise self.err
            return True
        return self.work.is_completed()

    def wait(self):
        if self.ev is not None:
            self.ev.wait()
            if self.err is not None:
                raise self.err
        else:
            self.work.wait()


def service_loop(workers, post_header, read_header, post_payload, serve, apply_batch, threaded, st,
                 idle_wait_s=0.002):
    """The PS request loop, backend-independent (RCCL: ``threaded=False``, works polled with
    ``is_completed()``; gloo: helper threads).

    ``post_header(w)`` / ``post_payload(w)`` post the receives of worker ``w``'s next header / push payload
    (works; a list for the payload); ``read_header(w)`` -> ``(kind, version)`` of the header that completed;
    ``serve(w, kind, version)`` handles a non-push request (False once ``w`` is done); ``apply_batch(batch)``
    applies the completed pushes ``[(w, version), ...]``.  Returns when every worker is done.  ``st["idle"]``
    accumulates the seconds spent waiting with nothing to do."""
    wake = None
    if threaded:
        import threading
        wake = threading.Event()

    def posted(work):
        return _Posted(work, threaded, wake)

    req = {w: posted(post_header(w)) for w in workers}
    inflight = {}
    done = 0
    while done < len(workers):
        if wake is not None:
            wake.clear()                  # any completion after this point is seen by the wait below
        progressed = False
        for w in workers:
            r = req.get(w)
            if r is None or not r.done():
                continue
            progressed = True
            r.wait()
            kind, wver = read_header(w)
            if kind == K_PUSH:
                inflight[w] = ([posted(x) for x in post_payload(w)], wver)
                req[w] = None                 # re-posted once the update is applied
                continue
            if serve(w, kind, wver):
                req[w] = posted(post_header(w))
            else:
                req[w] = None
                done += 1
        ready = [w for w, (rs, _) in inflight.items() if all(x.done() for x in rs)]
        if ready:
            progressed = True
            batch = []
            for w in ready:
                rs, wver = inflight.pop(w)
                for x in rs:
                    x.wait()
                batch.append((w, wver))
            apply_batch(batch)
            for w, _ in batch:
                req[w] = posted(post_header(w))
        if not progressed:
            ti = time.time()
            if wake is not None:
                wake.wait(idle_wait_s)        # woken by the helper thread of the next completed receive
            else:
                os.sched_yield()              # RCCL: the next poll is an event query, no GIL contention
            st["idle"] += time.time() - ti
    return st


class _TimedStore(object):
    """Proxy of the cluster store that counts and times every call made through it."""

    def __init__(self, store):
        self._store = store
        self.calls = 0
        self.wait_s = 0.0

    def __getattr__(self, name):
        fn = getattr(self._store, name)
        if not callable(fn):
            return fn

        def timed(*a, **k):
            t = time.time()
            try:
                return fn(*a, **k)
            finally:
                self.calls += 1
                self.wait_s += time.time() - t
        return timed
WIRE = torch.bfloat16            # gradient wire dtype (MDTF_ASYNC_WIRE=fp32 for full-precision pushes)


def _wire_dtype():
    import os
    return torch.float32 if os.environ.get("MDTF_ASYNC_WIRE", "bf16") == "fp32" else WIRE


def _hdr(device):
    return torch.zeros(2, dtype=torch.int64, device=device)


# ---------------------------------------------------------------------------
# parameter-server side
# ---------------------------------------------------------------------------
def run_parameter_server(op, server, sync_replicas=None, total_step=None):
    """PS role of the Train operator in async mode: a store-free request loop over all workers.

    ``sync_replicas = R`` (ps_mode ``sync_ps``): SyncReplicasOptimizer semantics on the same data plane
    (distribute_train.py:146-160): the PS accumulates the pushes computed on its CURRENT version, applies their
    mean as ONE update once R have arrived, and only then replies to those R workers.  A push computed on an
    older version -- a backup worker that lost the race -- is dropped (TF discards stale gradients) and answered at
    once with the current weights, so a straggler never holds the other workers back: that is the latency hiding
    of ``replicas_to_aggregate < total_num_replicas``.  From ``total_step`` on every push is answered at once."""
    from ..runtime.train import configure_store_for
    import os
    store = server.store
    ps = server.task_index
    num_ps = server.layout.num_ps
    vstore = configure_store_for(server)
    device = vstore.device
    cdev = device if device.type == "cuda" else torch.device("cpu")
    spec = json.loads(store.get("%s/varspec" % _PREFIX).decode())
    variables = []
    for s in spec:
        if s["ps"] % num_ps != ps:
            continue
        t = torch.zeros(s["shape"], dtype=torch.float32, device=device)
        v = V.Variable(s["name"], t, trainable=True, keep_fp32=s["keep_fp32"])
        v.apply_weight_decay = s["decay"]
        v.ps_task = ps
        v.pad_rows = int(s.get("pad_rows", 0))
        variables.append(v)
    space = _PSGroupedSpace(variables, device, vstore.compute_dtype, num_ps)
    groups = [g for g in space.groups]
    chief = server.layout.rank_of("worker", 0, 0)
    for g in groups:                      # initial values from the chief
        dist.recv(g.master, src=chief)
    space.refresh_shadows()
    optimizer = op.optimizer
    wire = _wire_dtype()
    workers = [server.layout.rank_of("worker", w, r) for w in range(server.layout.num_workers)
               for r in range(server.layout.towers_per_worker)]
    hdr = {w: _hdr(cdev) for w in workers}
    gbuf = {}                             # worker -> per-group wire buffers (payloads of several workers in flight)
    vt = torch.zeros(1, dtype=torch.int64, device=cdev)
    st = {"version": 0, "done": 0, "stale_sum": 0, "stale_max": 0, "updates": 0, "apply": 0.0, "idle": 0.0,
          "applies": 0, "batched_max": 0, "dropped": 0}
    accepted = []                         # sync_ps: workers whose push on the current version waits for the mean
    timed_store = _TimedStore(store)
    server.store = timed_store            # any store call made while serving is timed (the data plane makes none)
    t0 = time.time()

    def bufs(w):
        if w not in gbuf:
            gbuf[w] = [torch.empty(g.numel, dtype=wire if g.shadow is not None else torch.float32, device=device)
                       for g in groups]
        return gbuf[w]

    def reply(w):
        vt.fill_(st["version"])
        dist.send(vt, dst=w)
        for g in groups:
            dist.send(g.shadow if g.shadow is not None else g.master, dst=w)

    def apply_sync(batch):
        """sync_ps: accept pushes on the current version until R are in, apply their mean once, reply to them;
        drop (and answer at once) every push computed on an older version or after the last step."""
        ta = time.time()
        for w, wver in batch:
            if wver == st["version"] and len(accepted) < sync_replicas and (total_step is None
                                                                           or st["version"] < total_step):
                accepted.append(w)
            else:
                st["dropped"] += 1
                reply(w)
        if len(accepted) >= sync_replicas:
            step = st["version"]
            with torch.no_grad():
                for gi, g in enumerate(groups):
                    g.grad.copy_(gbuf[accepted[0]][gi])
                    for w in accepted[1:]:
                        g.grad.add_(gbuf[w][gi])
                    optimizer.update(UpdateTarget(g, g.master, g.grad, g.shadow, "full"),
                                     optimizer.learning_rate(step), 1.0 / len(accepted), step)
            st["version"] += 1
            st["updates"] += 1
            st["applies"] += 1
            st["batched_max"] = max(st["batched_max"], len(accepted))
            for w in accepted:
                reply(w)
            del accepted[:]
        st["apply"] += time.time() - ta

    def apply_batch(batch):
        """Every payload that completed since the last apply, as consecutive updates in ONE fused pass per group
        (chunks of MAX_MULTI); then one reply per worker with the weights after the chunk."""
        from ..ops.optim import MAX_MULTI
        if sync_replicas:
            return apply_sync(batch)
        ta = time.time()
        for c0 in range(0, len(batch), MAX_MULTI):
            chunk = batch[c0:c0 + MAX_MULTI]
            steps = [st["version"] + i for i in range(len(chunk))]
            with torch.no_grad():
                for gi, g in enumerate(groups):
                    optimizer.update_multi(UpdateTarget(g, g.master, g.grad, g.shadow, "full"),
                                           [gbuf[w][gi] for w, _ in chunk], steps)
            for w, wver in chunk:
                stale = st["version"] - wver
                st["stale_sum"] += stale
                st["stale_max"] = max(st["stale_max"], stale)
                st["updates"] += 1
                st["version"] += 1
            st["applies"] += 1
            st["batched_max"] = max(st["batched_max"], len(chunk))
            for w, _ in chunk:
                reply(w)
        st["apply"] += time.time() - ta

    def serve(w, kind, wver):
        """Handle a non-push request; returns False when the worker is done."""
        if kind == K_DONE:
            st["done"] += 1
            return False
        if kind == K_MASTER:
            for g in groups:
                dist.send(g.master, dst=w)
        else:
            reply(w)
        return True

    # ONE service loop for RCCL and gloo: a posted header receive per worker, polled; a push's payload receives
    # stay in flight while other workers are served; completed payloads are applied together
    threaded = dist.get_backend() != "nccl"
    service_loop(workers, lambda w: dist.irecv(hdr[w], src=w), lambda w: tuple(hdr[w].tolist()),
                 lambda w: [dist.irecv(b, src=w) for b in bufs(w)], serve, apply_batch, threaded, st)
    server.store = store
    updates = st["updates"]
    stale_sum, stale_max = st["stale_sum"], st["stale_max"]
    t_apply, t_idle = st["apply"], st["idle"]
    dt = time.time() - t0
    stats = {"ps": ps, "updates": updates, "mean_staleness": stale_sum / max(updates, 1), "max_staleness": stale_max,
             "updates_per_sec": updates / max(dt, 1e-9), "apply_s": round(t_apply, 3), "idle_s": round(t_idle, 3),
             "wall_s": round(dt, 3), "store_wait_s": round(timed_store.wait_s, 6), "store_calls": timed_store.calls,
             "applies": st["applies"], "batched_max": st["batched_max"], "wire": str(wire).replace("torch.", ""),
             "poll": "threaded-gloo" if threaded else "rccl-is_completed",
             "mode": "sync_ps R=%d" % sync_replicas if sync_replicas else "async", "dropped": st["dropped"]}
    store.set("%s/ps%d/stats" % (_PREFIX, ps), json.dumps(stats))
    out_dir = os.environ.get("MDTF_BENCH_OUT")
    if out_dir:
        with open(os.path.join(out_dir, "ps%d.json" % ps), "w") as f:
            json.dump(stats, f)
    logger.info("async PS %d: %s" % (ps, stats))
    server.signal_done()
    return stats


# ---------------------------------------------------------------------------
# worker side
# ---------------------------------------------------------------------------
class AsyncWorker(object):
    def __init__(self, op, server, tower, grads_and_vars, total_step, sync=False):
        self.op = op
        self.sync = sync                  # sync_ps: wait for the PS reply before the next step (no pipelining)
        self.server = server
        self.tower = tower
        self.total_step = total_step
        self.store = server.store
        self.num_ps = server.layout.num_ps
        if self.num_ps < 1:
            raise ValueError("async PS mode needs at least one ps task")
        self.rank = server.rank
        self.ps_ranks = [server.layout.rank_of("ps", p) for p in range(self.num_ps)]
        vstore = V.get_store()
        self.vars = [v for _, v in grads_and_vars]
        for v in self.vars:
            v.ps_task = int(v.ps_task or 0) % self.num_ps
        self.space = _PSGroupedSpace(self.vars, vstore.device, vstore.compute_dtype, self.num_ps)
        vstore.flat = self.space
        vstore.frozen = True
        self.by_ps = _groups_by_ps(self.space.groups, self.num_ps)
        self.version = [0] * self.num_ps
        dev = vstore.device
        cdev = dev if dev.type == "cuda" else torch.device("cpu")
        self._vt = [torch.zeros(1, dtype=torch.int64, device=cdev) for _ in range(self.num_ps)]
        self._h = [_hdr(cdev) for _ in range(self.num_ps)]
        wire = _wire_dtype()
        self._wire = {id(g): torch.empty(g.numel, dtype=wire if g.shadow is not None else torch.float32, device=dev)
                      for g in self.space.groups}
        self._stage = {id(g): torch.empty(g.numel, dtype=g.shadow.dtype if g.shadow is not None else torch.float32,
                                          device=dev) for g in self.space.groups}
        self.steps_done = 0

    def _send_hdr(self, kind, version=None):
        version = self.version if version is None else version
        for p, pr in enumerate(self.ps_ranks):
            self._h[p][0] = kind
            self._h[p][1] = version[p]
            dist.send(self._h[p], dst=pr)

    def _post_reply(self, into_staging):
        """Receive requests for every PS's reply (version + compute weights)."""
        reqs = []
        for p, pr in enumerate(self.ps_ranks):
            reqs.append(dist.irecv(self._vt[p], src=pr))
            for g in self.by_ps[p]:
                dst = self._stage[id(g)] if into_staging else (g.shadow if g.shadow is not None else g.master)
                reqs.append(dist.irecv(dst, src=pr))
        return reqs

    def _finish_reply(self, reqs, from_staging):
        for r in reqs:
            r.wait()
        for p in range(self.num_ps):
            self.version[p] = int(self._vt[p].item())
        if from_staging:
            for g in self.space.groups:
                (g.shadow if g.shadow is not None else g.master).copy_(self._stage[id(g)])

    def _push(self, version):
        """Cast this step's gradients onto the wire buffers and send them (header first) to every PS, labelled
        with ``version``: the PS versions of the weights forward/backward ran on."""
        self._send_hdr(K_PUSH, version)
        for g in self.space.groups:
            self._wire[id(g)].copy_(g.grad)
        reqs = []
        for p, pr in enumerate(self.ps_ranks):
            for g in self.by_ps[p]:
                reqs.append(dist.isend(self._wire[id(g)], dst=pr))
        return reqs

    def _exchange(self, kind):
        """Blocking request/reply (initial pull)."""
        self._send_hdr(kind)
        self._finish_reply(self._post_reply(False), False)

    def pull_masters(self):
        """Chief: fetch the authoritative fp32 masters from every PS (checkpointing)."""
        self._send_hdr(K_MASTER)
        for p, pr in enumerate(self.ps_ranks):
            for g in self.by_ps[p]:
                dist.recv(g.master, src=pr)

    def run(self, post_fn=None, args=(), kwargs=None):
        from ..train import step as S
        from ..train.saver import Saver
        server = self.server
        is_chief = server.is_chief
        if is_chief:
            self.store.set("%s/varspec" % _PREFIX, json.dumps(_varspec(self.vars)))
            for p, pr in enumerate(self.ps_ranks):
                for g in self.by_ps[p]:
                    dist.send(g.master, dst=pr)
        self._exchange(K_PULL)
        loss_h = self.tower.program
        t0 = time.time()
        window = t0
        last = None
        import os
        bench_warmup = int(os.environ.get("MDTF_BENCH_WARMUP", "0"))
        # fault injection for tests: MDTF_STRAGGLER=worker:<task>:<seconds> makes that worker sleep every step;
        # worker:<task>:x<k> sleeps k times its own forward/backward time of the step (slower by a factor k + 1
        # whatever the machine's load, so a test's "late" does not depend on how busy the host is)
        slow = os.environ.get("MDTF_STRAGGLER", "").split(":")
        mine = len(slow) == 3 and slow[0] == "worker" and int(slow[1]) == self.op.task_index
        delay, delay_x = 0.0, 0.0
        if mine:
            if slow[2].startswith("x"):
                delay_x = float(slow[2][1:])
            else:
                delay = float(slow[2])
        t_bench = None
        pending = None                    # (push send requests, reply receive requests) of the previous step
        step = 0
        while True:
            if self.steps_done == bench_warmup and t_bench is None:
                if V.get_store().device.type == "cuda":
                    torch.cuda.synchronize()
                t_bench = time.time()
            if self.sync and self.version[0] >= self.total_step:
                break                         # sync_ps: the last answer already carried the final version
            ctx = S.RunContext({})
            for v in self.vars:
                v.uses = 0
            self.space.zero_grad()
            # forward/backward of this step overlaps the previous push and its reply (into staging)
            t_fb = time.time()
            out = loss_h.forward(ctx, grad=True)
            out["loss"].backward()
            if delay:
                time.sleep(delay)
            elif delay_x:
                if V.get_store().device.type == "cuda":
                    torch.cuda.synchronize()
                time.sleep(delay_x * (time.time() - t_fb))
            from ..ops import conv as _conv
            _conv.join_side_streams()
            used = list(self.version)         # the weights this gradient was computed on
            if pending is not None:
                for r in pending[0]:
                    r.wait()
                self._finish_reply(pending[1], True)
            step = self.version[0]            # updates applied by PS 0 == the global step
            if step >= self.total_step:
                pending = None
                break
            pending = (self._push(used), self._post_reply(True))
            if self.sync:
                # synchronous replicas: the next step runs on the weights the PS answers with (the mean of the
                # first R pushes of this version, or the current weights if this push came too late)
                for r in pending[0]:
                    r.wait()
                self._finish_reply(pending[1], True)
                pending = None
            self.steps_done += 1
            last = out["loss"]
            if self.steps_done % 10 == 0:
                lv = float(last)
                now = time.time()
                logger.info("async step %d (local %d), loss = %.8f (%.1f examples/sec local)" % (
                    step, self.steps_done, lv, 10 * self.op.batch_size / max(now - window, 1e-9)))
                window = now
            if step + 1 >= self.total_step and pending is not None:
                for r in pending[0]:
                    r.wait()
                self._finish_reply(pending[1], True)
                pending = None
                if self.version[0] >= self.total_step:
                    break
        if V.get_store().device.type == "cuda":
            torch.cuda.synchronize()
        out_dir = os.environ.get("MDTF_BENCH_OUT")
        if out_dir and t_bench is not None:
            timed = self.steps_done - bench_warmup
            with open(os.path.join(out_dir, "worker%d.json" % self.op.task_index), "w") as f:
                json.dump({"steps": timed, "seconds": time.time() - t_bench, "batch": self.op.batch_size,
                           "staleness": getattr(self, "staleness", None), "steps_done": self.steps_done}, f)
        if is_chief and self.op.model_dir:
            self.pull_masters()
            V.get_or_create_global_step().assign(self.version[0])
            Saver(sharded=True, save_optimizer_state=False).save(None, "%s/model.ckpt" % self.op.model_dir.rstrip("/"),
                                                                 global_step=V.get_global_step())
        self._send_hdr(K_DONE)
        self.last_loss = last
        server.signal_done()
        if post_fn is not None:
            post_fn(args, kwargs or {})
        return self.steps_done
