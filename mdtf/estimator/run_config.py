"""``RunConfig`` — estimator run configuration with a deterministic ``uid()``.

Reference: ``distribute_utils.py:23-54`` subclasses ``tf.contrib.learn.RunConfig``
only to fix ``uid()`` (sorted, address-free field dump so two equal configs
compare equal).  This is a standalone config object with the same fields the
estimator/session layer consumes, parsed from ``TF_CONFIG`` when present
(``{"cluster": {...}, "task": {"type": "worker", "index": 0}}``) so a
TF-style launcher keeps working.
"""
import collections
import json
import os

from ..cluster.cluster_spec import ClusterSpec

# properties users may change between runs without changing the config identity
_DEFAULT_UID_WHITE_LIST = [
    "tf_random_seed", "save_summary_steps", "save_checkpoints_steps", "save_checkpoints_secs",
    "session_config", "keep_checkpoint_max", "keep_checkpoint_every_n_hours", "log_step_count_steps",
]


class RunConfig(object):
    def __init__(self, model_dir=None, tf_random_seed=None, save_summary_steps=100, save_checkpoints_steps=None,
                 save_checkpoints_secs=600, session_config=None, keep_checkpoint_max=5,
                 keep_checkpoint_every_n_hours=10000, log_step_count_steps=100, cluster_spec=None,
                 task_type=None, task_id=None):
        if save_checkpoints_steps is not None and save_checkpoints_secs not in (None, 600):
            raise ValueError("save_checkpoints_steps and save_checkpoints_secs are mutually exclusive")
        if save_checkpoints_steps is not None:
            save_checkpoints_secs = None
        self._model_dir = model_dir
        self._tf_random_seed = tf_random_seed
        self._save_summary_steps = save_summary_steps
        self._save_checkpoints_steps = save_checkpoints_steps
        self._save_checkpoints_secs = save_checkpoints_secs
        self._session_config = session_config
        self._keep_checkpoint_max = keep_checkpoint_max
        self._keep_checkpoint_every_n_hours = keep_checkpoint_every_n_hours
        self._log_step_count_steps = log_step_count_steps
        tf_config = json.loads(os.environ.get("TF_CONFIG", "{}") or "{}")
        if cluster_spec is None and tf_config.get("cluster"):
            cluster_spec = ClusterSpec(tf_config["cluster"])
        task = tf_config.get("task", {})
        self._cluster_spec = cluster_spec if cluster_spec is not None else ClusterSpec({})
        self._task_type = task_type or task.get("type") or ("worker" if self._cluster_spec.jobs else None)
        self._task_id = int(task_id if task_id is not None else task.get("index", 0))
        jobs = self._cluster_spec.jobs
        self._num_ps_replicas = self._cluster_spec.num_tasks("ps") if "ps" in jobs else 0
        nw = self._cluster_spec.num_tasks("worker") if "worker" in jobs else 0
        nw += self._cluster_spec.num_tasks("chief") if "chief" in jobs else 0
        self._num_worker_replicas = max(nw, 1)
        if "chief" in jobs:
            self._is_chief = self._task_type == "chief"
        else:
            self._is_chief = self._task_type in (None, "worker") and self._task_id == 0
        self._master = ""

    # read-only properties in TF style
    model_dir = property(lambda s: s._model_dir)
    tf_random_seed = property(lambda s: s._tf_random_seed)
    save_summary_steps = property(lambda s: s._save_summary_steps)
    save_checkpoints_steps = property(lambda s: s._save_checkpoints_steps)
    save_checkpoints_secs = property(lambda s: s._save_checkpoints_secs)
    session_config = property(lambda s: s._session_config)
    keep_checkpoint_max = property(lambda s: s._keep_checkpoint_max)
    keep_checkpoint_every_n_hours = property(lambda s: s._keep_checkpoint_every_n_hours)
    log_step_count_steps = property(lambda s: s._log_step_count_steps)
    cluster_spec = property(lambda s: s._cluster_spec)
    task_type = property(lambda s: s._task_type)
    task_id = property(lambda s: s._task_id)
    is_chief = property(lambda s: s._is_chief)
    num_ps_replicas = property(lambda s: s._num_ps_replicas)
    num_worker_replicas = property(lambda s: s._num_worker_replicas)
    master = property(lambda s: s._master)

    def replace(self, **kwargs):
        """A copy with some fields replaced (``tf.estimator.RunConfig.replace``)."""
        import copy
        new = copy.copy(self)
        for k, v in kwargs.items():
            if not hasattr(new, "_" + k):
                raise ValueError("RunConfig has no property %r" % k)
            setattr(new, "_" + k, v)
        if kwargs.get("save_checkpoints_steps") is not None:
            new._save_checkpoints_secs = None
        return new

    def uid(self, whitelist=None):
        """Deterministic identity string of every field not in ``whitelist``.

        Same contract as ``distribute_utils.py:24-54``: sorted ``key=repr``
        pairs, the cluster spec rendered as a sorted dict (never an object
        address).
        """
        if whitelist is None:
            whitelist = _DEFAULT_UID_WHITE_LIST
        state = {k: v for k, v in self.__dict__.items() if not k.startswith("__")}
        for k in whitelist:
            state.pop("_" + k, None)
        ordered = collections.OrderedDict(sorted(state.items(), key=lambda t: t[0]))
        if "_cluster_spec" in ordered:
            ordered["_cluster_spec"] = collections.OrderedDict(sorted(ordered["_cluster_spec"].as_dict().items(),
                                                                      key=lambda t: t[0]))
        return ", ".join("%s=%r" % (k, v) for k, v in ordered.items())
