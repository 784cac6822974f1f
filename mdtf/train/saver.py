"""``tf.train.Saver`` on tensor-bundle V2 files (see ``mdtf/ckpt``).

Saved tensors use TF names: variables by scope path, ``global_step``
(int64), optimizer slots ``<var>/Momentum`` or ``<var>/Adam``/``<var>/Adam_1``
and the Adam ``beta1_power``/``beta2_power`` scalars.  With ``sharded=True``
one data file per PS task is written and each variable goes to the shard of
the PS task ``replica_device_setter`` assigned it to (the reference's PS
variable placement, ``distribute_train.py:109-110``).

In PS-shard (``mode='sharded'``) training the fp32 masters/slots of each rank
are partial; ``save``/``restore`` gather/scatter them collectively, so in that
mode every replica must call them (``MonitoredTrainingSession`` installs the
checkpoint hook on every replica with a step-based trigger).
"""
import glob
import os

import torch

from ..ckpt import checkpoint_state as CS
from ..ckpt.tensor_bundle import BundleReader, BundleWriter
from ..utils import log as logger
from . import step as S
from . import variables as V


def latest_checkpoint(checkpoint_dir):
    return CS.latest_checkpoint(checkpoint_dir)


class TensorDictReader(object):
    """BundleReader look-alike over an in-memory ``{name: tensor}`` dict."""

    def __init__(self, tensors):
        self.tensors = tensors

    def __contains__(self, name):
        return name in self.tensors

    def keys(self):
        return list(self.tensors)

    def get_tensor(self, name):
        return self.tensors[name]


def read_all(save_path):
    r = BundleReader(save_path)
    return {k: r.get_tensor(k) for k in r.keys()}


def _is_writer():
    import torch.distributed as dist
    from ..cluster import server as srv_mod
    srv = srv_mod.current()
    if srv is not None:
        return srv.is_chief
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


class Saver(object):
    def __init__(self, var_list=None, max_to_keep=5, sharded=False, keep_checkpoint_every_n_hours=10000.0,
                 save_optimizer_state=True):
        self.var_list = var_list
        self.max_to_keep = max_to_keep
        self.sharded = sharded
        self.save_optimizer_state = save_optimizer_state
        self._last = []

    def _variables(self):
        store = V.get_store()
        if self.var_list is None:
            return store.global_variables()
        out = []
        for v in (self.var_list.values() if isinstance(self.var_list, dict) else self.var_list):
            out.append(store.vars[v] if isinstance(v, str) else v)
        return out

    def _named_tensors(self):
        """name -> (tensor, ps_shard).  Collective in PS-shard mode."""
        tensors = {}
        step = V.get_global_step().value() if V.get_global_step() is not None else 0
        for op in S.train_ops():
            if op.reducer is not None:
                op.reducer.gather_full_master()
        for v in self._variables():
            tensors[v.name] = (v.master, v.ps_task or 0)
        if V.get_global_step() is not None:
            tensors["global_step"] = (torch.tensor(step, dtype=torch.int64), 0)
        if self.save_optimizer_state:
            for op in S.train_ops():
                if op.reducer is None:
                    continue
                for state, suffix in op.optimizer.slot_checkpoint_names():
                    fulls = op.reducer.gather_full_state(None, state)
                    for g, full in zip(op.space.groups, fulls):
                        for var in g.variables:
                            o = var.flat_offset
                            tensors["%s/%s" % (var.name, suffix)] = (full[o:o + var.numel()].view(var.shape),
                                                                     var.ps_task or 0)
                for k, val in op.optimizer.extra_checkpoint_scalars(op.step_count).items():
                    tensors[k] = (torch.tensor(val, dtype=torch.float32), 0)
        return tensors

    def save(self, sess, save_path, global_step=None, write_state=True):
        tensors = self._named_tensors()
        if global_step is not None:
            gs = int(global_step.value() if isinstance(global_step, V.GlobalStep) else global_step)
            prefix = "%s-%d" % (save_path, gs)
        else:
            prefix = save_path
        if not _is_writer():
            return prefix
        num_shards = 1
        if self.sharded:
            num_shards = max(s for _, s in tensors.values()) + 1
        w = BundleWriter(prefix, num_shards)
        for name in sorted(tensors):
            t, shard = tensors[name]
            w.add(name, t, shard if self.sharded else 0)
        w.finish()
        if write_state:
            d = os.path.dirname(prefix) or "."
            st = CS.read_state(d)
            same = os.path.abspath(prefix)
            paths = [p for p in (st["all_model_checkpoint_paths"] if st else [])
                     if os.path.abspath(p) != same] + [prefix]
            if self.max_to_keep and len(paths) > self.max_to_keep:
                for old in paths[:-self.max_to_keep]:
                    for f in glob.glob(old + ".index") + glob.glob(old + ".data-*"):
                        os.remove(f)
                paths = paths[-self.max_to_keep:]
            CS.write_state(d, prefix, paths)
        return prefix

    def restore(self, sess, save_path, reader=None):
        """``reader``: any object with ``in`` / ``get_tensor`` (e.g. :class:`TensorDictReader` of tensors
        the chief read and broadcast when ``save_path`` is not visible on this replica)."""
        r = reader if reader is not None else BundleReader(save_path)
        store = V.get_store()
        missing = []
        with torch.no_grad():
            for v in self._variables():
                if v.name in r:
                    v.master.copy_(r.get_tensor(v.name).to(v.master.dtype).to(v.master.device))
                else:
                    missing.append(v.name)
            if "global_step" in r and V.get_global_step() is not None:
                V.get_global_step().assign(int(r.get_tensor("global_step").item()))
            for op in S.train_ops():
                if op.reducer is None:
                    continue
                op.step_count = V.get_global_step().value() if V.get_global_step() is not None else op.step_count
                for state, suffix in op.optimizer.slot_checkpoint_names():
                    fulls = []
                    for g in op.space.groups:
                        full = torch.zeros(g.numel, dtype=torch.float32, device=g.device)
                        for var in g.variables:
                            key = "%s/%s" % (var.name, suffix)
                            if key in r:
                                o = var.flat_offset
                                full[o:o + var.numel()].copy_(r.get_tensor(key).reshape(-1).to(full.device))
                        fulls.append(full)
                    op.reducer.scatter_full_state(state, fulls)
                op.space.refresh_shadows()
                op.reducer.load_shards_from_master()
        for v in store.global_variables():
            v.refresh_shadow()
        if missing:
            logger.warn("restore: %d variables not found in %s: %s" % (len(missing), save_path, missing[:8]))
        return missing

    def recover_last_checkpoints(self, paths):
        self._last = list(paths)
