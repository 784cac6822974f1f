"""ClusterSpec: the ps/worker job description (``tf.train.ClusterSpec`` analogue).

Reference usage: ``distribute.py:57-80`` splits the ``ps_hosts`` /
``worker_hosts`` strings on ',' and builds ``ClusterSpec({"ps": ..., "worker": ...})``;
``distribute_train.py:77`` calls ``cluster.num_tasks("worker")``.

Fix: entries are stripped and validated as ``host:port``
(``"127.0.0.1: 22"`` → ``127.0.0.1:22``).

Rank layout (one OS process per GPU): a worker *task* with ``gpu_num`` GPUs is a
group of ``gpu_num`` ranks ("towers").  In sync mode only worker towers form the
collective group; parameter-server tasks host the rendezvous store and the
shutdown barrier.  In async mode PS tasks own one GPU each and are ranks
``0..P-1`` of the world, followed by the worker towers.
"""
import collections


def parse_host_list(spec):
    """Parse ``"h1:p1, h2: p2"`` (or a list) into ``["h1:p1", "h2:p2"]``."""
    if spec is None:
        return []
    items = spec.split(",") if isinstance(spec, str) else list(spec)
    out = []
    for raw in items:
        s = str(raw).replace(" ", "").strip()
        if not s:
            continue
        if ":" not in s:
            raise ValueError("cluster address %r is not host:port" % raw)
        host, port = s.rsplit(":", 1)
        if not host:
            raise ValueError("cluster address %r has an empty host" % raw)
        try:
            p = int(port)
        except ValueError:
            raise ValueError("cluster address %r has a non-integer port" % raw)
        if not 0 < p < 65536:
            raise ValueError("cluster address %r has an out-of-range port" % raw)
        out.append("%s:%d" % (host, p))
    return out


def split_address(addr):
    host, port = addr.rsplit(":", 1)
    return host, int(port)


class ClusterSpec(object):
    """Mapping job name -> ordered list of ``host:port`` task addresses."""

    def __init__(self, cluster):
        if isinstance(cluster, ClusterSpec):
            cluster = cluster.as_dict()
        self._jobs = collections.OrderedDict()
        for job in sorted(cluster):
            tasks = cluster[job]
            if isinstance(tasks, dict):
                tasks = [tasks[k] for k in sorted(tasks)]
            self._jobs[job] = parse_host_list(tasks)

    @classmethod
    def from_hosts(cls, ps_hosts, worker_hosts):
        return cls({"ps": parse_host_list(ps_hosts), "worker": parse_host_list(worker_hosts)})

    @property
    def jobs(self):
        return list(self._jobs)

    def num_tasks(self, job_name):
        if job_name not in self._jobs:
            raise ValueError("No such job in cluster: %r" % job_name)
        return len(self._jobs[job_name])

    def task_indices(self, job_name):
        return list(range(self.num_tasks(job_name)))

    def job_tasks(self, job_name):
        return list(self._jobs[job_name])

    def task_address(self, job_name, task_index):
        tasks = self._jobs.get(job_name)
        if tasks is None or not 0 <= task_index < len(tasks):
            raise ValueError("No task %r in job %r" % (task_index, job_name))
        return tasks[task_index]

    def as_dict(self):
        return {job: list(tasks) for job, tasks in self._jobs.items()}

    def __eq__(self, other):
        return isinstance(other, ClusterSpec) and self.as_dict() == other.as_dict()

    def __repr__(self):
        return "ClusterSpec(%r)" % self.as_dict()

    # -- rendezvous --------------------------------------------------------
    def coordinator_address(self):
        """The task hosting the rendezvous store: ps/0, else worker/0."""
        if self._jobs.get("ps"):
            return self._jobs["ps"][0]
        if self._jobs.get("worker"):
            return self._jobs["worker"][0]
        raise ValueError("cluster has no ps or worker task")


class RankLayout(object):
    """Maps (job, task, tower) <-> collective ranks and local GPU indices."""

    def __init__(self, cluster, gpu_num, async_ps=False):
        self.cluster = cluster
        self.gpu_num = max(int(gpu_num or 0), 0)
        self.towers_per_worker = max(self.gpu_num, 1)
        self.async_ps = bool(async_ps)
        self.num_ps = cluster.num_tasks("ps") if "ps" in cluster.jobs else 0
        self.num_workers = cluster.num_tasks("worker") if "worker" in cluster.jobs else 0
        self.num_worker_ranks = self.num_workers * self.towers_per_worker
        self.ps_offset = 0
        self.worker_offset = self.num_ps if self.async_ps else 0
        self.world_size = self.worker_offset + self.num_worker_ranks

    def rank_of(self, job_name, task_index, tower=0):
        if job_name == "ps":
            if not self.async_ps:
                return None  # sync-mode PS tasks are not collective members
            return self.ps_offset + task_index
        if not 0 <= tower < self.towers_per_worker:
            raise ValueError("tower %d out of range (gpu_num=%d)" % (tower, self.gpu_num))
        return self.worker_offset + task_index * self.towers_per_worker + tower

    def worker_rank_of(self, task_index, tower=0):
        """Rank inside the worker-only group (the gradient-reduction group)."""
        return task_index * self.towers_per_worker + tower

    def describe(self, rank):
        if rank < self.worker_offset:
            return ("ps", rank - self.ps_offset, 0)
        r = rank - self.worker_offset
        return ("worker", r // self.towers_per_worker, r % self.towers_per_worker)

    def worker_ranks(self):
        return list(range(self.worker_offset, self.worker_offset + self.num_worker_ranks))

    @property
    def num_processes(self):
        """Every process of the job: one per PS task plus one per worker tower."""
        return self.num_ps + self.num_worker_ranks

    def process_index(self, job_name, task_index, tower=0):
        """Dense id over ALL processes (PS tasks first) -- heartbeat ids, independent of the ps mode."""
        if job_name == "ps":
            return task_index
        return self.num_ps + task_index * self.towers_per_worker + tower

    def ps_ranks(self):
        return list(range(self.ps_offset, self.ps_offset + self.num_ps)) if self.async_ps else []

    def local_device_index(self, job_name, task_index, tower=0):
        """GPU index on this task's host: ps tasks (async) first, then worker towers."""
        host = split_address(self.cluster.task_address(job_name, task_index))[0]
        idx = 0
        if self.async_ps:
            for t in range(self.num_ps):
                if job_name == "ps" and t == task_index:
                    return idx
                if split_address(self.cluster.task_address("ps", t))[0] == host:
                    idx += 1
        for t in range(self.num_workers):
            if job_name == "worker" and t == task_index:
                return idx + tower
            if split_address(self.cluster.task_address("worker", t))[0] == host:
                idx += self.towers_per_worker
        raise ValueError("task %s/%d not in cluster" % (job_name, task_index))
