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
* a PS applies each worker's gradient as soon as it arrives (no aggregation,
  no barrier) with the fused optimizer kernel; request order is the arrival
  order recorded by an atomic ticket counter in the cluster store;
* staleness (PS version at apply time minus the version the gradient was
  computed from) is measured per update and reported;
* ``global_step`` counts applied worker updates (store counter); workers stop
  at ``total_step`` and send a "done" ticket; PS tasks exit when every worker
  is done (the reference's done-queue, ``distribute_train.py:86-90``);
* the chief pulls the fp32 masters from every PS and writes a sharded
  tensor-bundle checkpoint (one data file per PS task — the TF layout).
"""
import json
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
    return [{"name": v.name, "shape": list(v.shape), "keep_fp32": bool(v.keep_fp32),
             "decay": bool(v.apply_weight_decay), "ps": int(v.ps_task or 0)} for v in variables]


def _ticket(store, ps, msg):
    n = store.add("%s/ps%d/n" % (_PREFIX, ps), 1)
    store.set("%s/ps%d/t/%d" % (_PREFIX, ps, n), msg)


# ---------------------------------------------------------------------------
# parameter-server side
# ---------------------------------------------------------------------------
def run_parameter_server(op, server):
    """PS role of the Train operator in async mode."""
    from ..runtime.train import configure_store_for
    store = server.store
    ps = server.task_index
    num_ps = server.layout.num_ps
    vstore = configure_store_for(server)
    device = vstore.device
    spec = json.loads(store.get("%s/varspec" % _PREFIX).decode())
    variables = []
    for s in spec:
        if s["ps"] % num_ps != ps:
            continue
        t = torch.zeros(s["shape"], dtype=torch.float32, device=device)
        v = V.Variable(s["name"], t, trainable=True, keep_fp32=s["keep_fp32"])
        v.apply_weight_decay = s["decay"]
        v.ps_task = ps
        variables.append(v)
    space = _PSGroupedSpace(variables, device, vstore.compute_dtype, num_ps)
    groups = [g for g in space.groups]
    chief = server.layout.rank_of("worker", 0, 0)
    for g in groups:                      # initial values from the chief
        dist.recv(g.master, src=chief)
    space.refresh_shadows()
    optimizer = op.optimizer
    version = 0
    done = 0
    n = 0
    num_workers = server.layout.num_worker_ranks
    stale_sum, stale_max, updates = 0, 0, 0
    vt = torch.zeros(1, dtype=torch.int64, device=device if device.type == "cuda" else "cpu")
    t0 = time.time()
    while done < num_workers:
        n += 1
        key = "%s/ps%d/t/%d" % (_PREFIX, ps, n)
        store.wait([key])
        rank_s, kind, wver = store.get(key).decode().split(":")
        store.delete_key(key)
        r = int(rank_s)
        if kind == "done":
            done += 1
            continue
        if kind == "push":
            for g in groups:
                dist.recv(g.grad, src=r)
            lr = optimizer.learning_rate(version)
            with torch.no_grad():
                for g in groups:
                    optimizer.update(UpdateTarget(g, g.master, g.grad, g.shadow, "full"), lr, 1.0, version)
            stale = version - int(wver)
            stale_sum += stale
            stale_max = max(stale_max, stale)
            updates += 1
            version += 1
        if kind == "master":
            for g in groups:
                dist.send(g.master, dst=r)
            continue
        vt.fill_(version)
        dist.send(vt, dst=r)
        for g in groups:
            dist.send(g.shadow if g.shadow is not None else g.master, dst=r)
    dt = time.time() - t0
    stats = {"ps": ps, "updates": updates, "mean_staleness": stale_sum / max(updates, 1), "max_staleness": stale_max,
             "updates_per_sec": updates / max(dt, 1e-9)}
    store.set("%s/ps%d/stats" % (_PREFIX, ps), json.dumps(stats))
    logger.info("async PS %d: %s" % (ps, stats))
    server.signal_done()
    return stats


# ---------------------------------------------------------------------------
# worker side
# ---------------------------------------------------------------------------
class AsyncWorker(object):
    def __init__(self, op, server, tower, grads_and_vars, total_step):
        self.op = op
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
        self._vt = [torch.zeros(1, dtype=torch.int64, device=dev if dev.type == "cuda" else "cpu")
                    for _ in range(self.num_ps)]
        self.steps_done = 0

    def _exchange(self, kind):
        reqs = []
        for p in range(self.num_ps):
            _ticket(self.store, p, "%d:%s:%d" % (self.rank, kind, self.version[p]))
        for p, pr in enumerate(self.ps_ranks):
            if kind == "push":
                for g in self.by_ps[p]:
                    reqs.append(dist.isend(g.grad, dst=pr))
            reqs.append(dist.irecv(self._vt[p], src=pr))
            for g in self.by_ps[p]:
                reqs.append(dist.irecv(g.shadow if g.shadow is not None else g.master, src=pr))
        for r in reqs:
            r.wait()
        for p in range(self.num_ps):
            self.version[p] = int(self._vt[p].item())
        for g in self.space.groups:
            if g.shadow is not None:
                pass  # the bf16 compute weights were received directly; fp32 masters stay on the PS

    def pull_masters(self):
        """Chief: fetch the authoritative fp32 masters from every PS (checkpointing)."""
        for p in range(self.num_ps):
            _ticket(self.store, p, "%d:master:0" % self.rank)
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
        self._exchange("pull")
        gs_key = "%s/global_step" % _PREFIX
        loss_h = self.tower.program
        t0 = time.time()
        window = t0
        last = None
        import os
        bench_warmup = int(os.environ.get("MDTF_BENCH_WARMUP", "0"))
        t_bench = None
        while True:
            if self.steps_done == bench_warmup and t_bench is None:
                if V.get_store().device.type == "cuda":
                    torch.cuda.synchronize()
                t_bench = time.time()
            ctx = S.RunContext({})
            for v in self.vars:
                v.uses = 0
            self.space.zero_grad()
            out = loss_h.forward(ctx, grad=True)
            out["loss"].backward()
            from ..ops import conv as _conv
            _conv.join_side_streams()
            self._exchange("push")
            self.steps_done += 1
            step = self.store.add(gs_key, 1)
            last = out["loss"]
            if step % 10 == 0:
                lv = float(last)
                now = time.time()
                logger.info("async step %d (local %d), loss = %.8f (%.1f examples/sec local)" % (
                    step, self.steps_done, lv, 10 * self.op.batch_size / max(now - window, 1e-9)))
                window = now
            if step >= self.total_step:
                break
        if V.get_store().device.type == "cuda":
            torch.cuda.synchronize()
        out_dir = os.environ.get("MDTF_BENCH_OUT")
        if out_dir and t_bench is not None:
            timed = self.steps_done - bench_warmup
            with open(os.path.join(out_dir, "worker%d.json" % self.op.task_index), "w") as f:
                json.dump({"steps": timed, "seconds": time.time() - t_bench, "batch": self.op.batch_size,
                           "staleness": getattr(self, "staleness", None)}, f)
        if is_chief and self.op.model_dir:
            self.pull_masters()
            V.get_or_create_global_step().assign(self.store.add(gs_key, 0))
            Saver(sharded=True, save_optimizer_state=False).save(None, "%s/model.ckpt" % self.op.model_dir.rstrip("/"),
                                                                 global_step=V.get_global_step())
        for p in range(self.num_ps):
            _ticket(self.store, p, "%d:done:0" % self.rank)
        self.last_loss = last
        server.signal_done()
        if post_fn is not None:
            post_fn(args, kwargs or {})
        return self.steps_done
