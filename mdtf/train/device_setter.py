"""Variable placement policies (``tf.train.replica_device_setter`` analogues).

Reference: ``replica_device_setter(worker_device, ps_device, cluster)``
round-robins variables over the PS tasks in creation order
(``distribute_train.py:109-110``); ``local_device_setter`` round-robins them
over local devices (``distribute_utils.py:118-145``).

Here compute placement is fixed (one process per GPU); the setters record
*ownership*: which PS task / shard a variable belongs to.  That drives the
sharded checkpoint layout (one data file per PS task) and is reported by
``--log_device_placement``.
"""
from ..utils import log as logger


class _RoundRobinStrategy(object):
    def __init__(self, num_tasks):
        self._num_tasks = max(int(num_tasks), 1)
        self._next = 0

    def __call__(self, var):
        t = self._next
        self._next = (self._next + 1) % self._num_tasks
        return t


class GreedyLoadBalancingStrategy(object):
    """Place each variable on the least-loaded task (by bytes)."""

    def __init__(self, num_tasks):
        self._loads = [0] * max(int(num_tasks), 1)

    def __call__(self, var):
        t = min(range(len(self._loads)), key=lambda i: self._loads[i])
        self._loads[t] += var.numel() * var.master.element_size()
        return t


class DeviceSetter(object):
    def __init__(self, num_tasks, ps_device, worker_device, strategy=None, log=False):
        self.num_tasks = num_tasks
        self.ps_device = ps_device
        self.worker_device = worker_device
        self.strategy = strategy or _RoundRobinStrategy(num_tasks)
        self.log = log
        self.placements = {}

    def __call__(self, var):
        t = self.strategy(var) if self.num_tasks > 0 else 0
        var.ps_task = t
        var.device_hint = "%s/task:%d" % (self.ps_device, t) if self.num_tasks > 0 else self.worker_device
        self.placements[var.name] = var.device_hint
        if self.log:
            logger.info("placement: %s -> %s" % (var.name, var.device_hint))


def replica_device_setter(ps_tasks=0, ps_device="/job:ps", worker_device="/job:worker", merge_devices=True,
                          cluster=None, ps_ops=None, ps_strategy=None):
    if cluster is not None:
        from ..cluster import ClusterSpec
        cl = cluster if isinstance(cluster, ClusterSpec) else ClusterSpec(cluster)
        ps_tasks = cl.num_tasks("ps") if "ps" in cl.jobs else 0
    from ..config.flags import FLAGS
    try:
        log = FLAGS.log_device_placement
    except Exception:
        log = False
    return DeviceSetter(ps_tasks, ps_device.split("/cpu")[0].split("/gpu")[0], worker_device,
                        ps_strategy or _RoundRobinStrategy(ps_tasks), log)


def local_device_setter(num_devices=1, ps_device_type='cpu', worker_device='/cpu:0', ps_ops=None,
                        ps_strategy=None):
    """Variables round-robin over local devices (``distribute_utils.py:118-145``)."""
    if ps_strategy is not None and not callable(ps_strategy):
        raise TypeError("ps_strategy must be callable")
    return DeviceSetter(num_devices, "/%s" % ps_device_type, worker_device,
                        ps_strategy or _RoundRobinStrategy(num_devices))
