"""Server: per-process cluster membership (``tf.train.Server`` analogue).

Reference: ``distribute.py:81`` starts an in-process gRPC server per task and
every worker↔PS byte moves over TCP through PS CPU memory.  Here:

* the coordinator task (ps/0, else worker/0) hosts a ``torch.distributed``
  ``TCPStore`` — rendezvous, the done-queue shutdown barrier
  (``distribute_train.py:43-46,86-90,202-205``), backup-worker arrival counters
  and rank-failure heartbeats all live there;
* every worker *tower* (one process per GPU) joins the collective group
  (RCCL over xGMI on MI355X, gloo on CPU) — that group carries the gradient
  reduction and parameter broadcast;
* in async-PS mode the PS tasks own one GPU each and join the world group too.

``Server.target`` mirrors TF's ``grpc://host:port`` string.

Under ``torchrun`` (``RANK``/``WORLD_SIZE`` in the environment) use
:meth:`Server.from_env`: the node is one worker task whose ``gpu_num`` is the
local world size and no PS task exists.
"""
import datetime
import os
import time

from ..config import constants
from ..utils import log as logger
from .cluster_spec import ClusterSpec, RankLayout, split_address

_CURRENT = None


def current():
    """The Server of this process (None before one is created)."""
    return _CURRENT


def _set_current(server):
    global _CURRENT
    _CURRENT = server


class Server(object):
    def __init__(self, cluster, job_name, task_index, gpu_num=None, local_rank=None,
                 async_ps=None, start=True, backend=None, store_timeout_s=constants.STORE_TIMEOUT_S):
        if not isinstance(cluster, ClusterSpec):
            cluster = ClusterSpec(cluster)
        if job_name not in ("ps", "worker"):
            raise ValueError("job_name must be 'ps' or 'worker', got %r" % (job_name,))
        if task_index is None:
            raise ValueError("task_index must be set (flag --task_index or @task_index)")
        self.cluster = cluster
        self.job_name = job_name
        self.task_index = int(task_index)
        cluster.task_address(job_name, self.task_index)  # validates
        if async_ps is None:
            from ..config.flags import FLAGS
            async_ps = FLAGS.ps_mode in ("async", "sync_ps")
        self.layout = RankLayout(cluster, gpu_num if gpu_num is not None else 0, async_ps=async_ps)
        if local_rank is None:
            local_rank = int(os.environ.get("MDTF_LOCAL_RANK", "0"))
        self.local_rank = local_rank
        self.backend = backend
        self.store_timeout_s = store_timeout_s
        self.store = None
        self.rank = self.layout.rank_of(job_name, self.task_index, local_rank if job_name == "worker" else 0)
        self.world_size = self.layout.world_size
        self.worker_group = None
        self.heartbeat = None
        self._torchrun = False
        self._started = False
        _set_current(self)
        if start:
            self.start()

    # ------------------------------------------------------------------
    @classmethod
    def from_env(cls, backend=None, start=True):
        """Build the Server from torchrun-style environment variables."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        local_rank = int(os.environ.get("LOCAL_RANK", str(rank % local_world)))
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", str(constants.DEFAULT_PORT)))
        nnodes = max(world // max(local_world, 1), 1)
        workers = ["%s:%d" % (addr, port + i) for i in range(nnodes)]
        srv = cls(ClusterSpec({"ps": [], "worker": workers}), "worker", rank // local_world,
                  gpu_num=local_world, local_rank=local_rank, async_ps=False, start=False, backend=backend)
        srv._torchrun = True
        srv.rank, srv.world_size = rank, world
        if start:
            srv.start()
        return srv

    @property
    def target(self):
        return "mdtf://%s" % self.cluster.coordinator_address()

    @property
    def is_chief(self):
        return self.job_name == "worker" and self.task_index == 0 and self.local_rank == 0

    @property
    def is_coordinator(self):
        if self._torchrun:
            return self.rank == 0
        if self.layout.num_ps:
            return self.job_name == "ps" and self.task_index == 0
        return self.job_name == "worker" and self.task_index == 0 and self.local_rank == 0

    @property
    def num_workers(self):
        return self.layout.num_workers

    def device(self):
        """torch.device this process computes on."""
        import torch
        if self.job_name == "ps" and not self.layout.async_ps:
            return torch.device("cpu")
        if not torch.cuda.is_available():
            return torch.device("cpu")
        if self._torchrun:
            # (local ranks beyond the visible devices share them: the MDTF_DIST_BACKEND=gloo rehearsal of an
            # N-rank job on fewer GPUs; a real launch has one device per local rank)
            return torch.device("cuda", self.local_rank % max(torch.cuda.device_count(), 1))
        idx = self.layout.local_device_index(self.job_name, self.task_index, self.local_rank)
        return torch.device("cuda", idx % max(torch.cuda.device_count(), 1))

    # ------------------------------------------------------------------
    def start(self):
        if self._started:
            return
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MDTF_RANK_TAG", "[%s:%d%s]" % (
            self.job_name, self.task_index, "/%d" % self.local_rank if self.layout.gpu_num > 1 else ""))
        # surface RCCL errors / dead peers as exceptions instead of silent hangs
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        # RCCL prints the failing call before it aborts a process (silent otherwise)
        os.environ.setdefault("NCCL_DEBUG", "WARN")
        # flight recorder on: hipGraph capture waits until the RCCL watchdog has retired every eager
        # work (train/graph.py _drain_comm_watchdog reads the recorder's active entries)
        os.environ.setdefault("TORCH_FR_BUFFER_SIZE", "2000")
        timeout = datetime.timedelta(seconds=self.store_timeout_s)
        if self._torchrun:
            # MDTF_DIST_BACKEND=gloo: multi-rank rehearsal on a box with fewer GPUs than ranks (RCCL needs one
            # device per rank); the step then cannot be graph-captured and runs eagerly (train/graph.py)
            backend = self.backend or os.environ.get("MDTF_DIST_BACKEND") or (
                "nccl" if torch.cuda.is_available() else "gloo")
            if backend == "nccl":
                torch.cuda.set_device(self.local_rank)
            if not dist.is_initialized():
                dist.init_process_group(backend, timeout=timeout)
            self.store = dist.distributed_c10d._get_default_store()
            self.worker_group = dist.group.WORLD
            self._started = True
            # torchrun's elastic agent already tears the job down when a rank dies;
            # the heartbeat watchdog is opt-in there (MDTF_HEARTBEAT=1)
            if os.environ.get("MDTF_HEARTBEAT") == "1":
                self._start_heartbeat(dist.get_rank(), dist.get_world_size())
            return
        host, port = split_address(self.cluster.coordinator_address())
        self.store = dist.TCPStore(host, port, is_master=self.is_coordinator, timeout=timeout,
                                   wait_for_workers=False)
        if self.rank is not None:
            # MDTF_DIST_BACKEND=gloo: several tasks sharing one GPU (the 1-GPU async-PS rehearsal)
            backend = self.backend or os.environ.get("MDTF_DIST_BACKEND") or (
                "nccl" if torch.cuda.is_available() else "gloo")
            dev = self.device()
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
            else:
                backend = "gloo"
            dist.init_process_group(backend, store=dist.PrefixStore("mdtf/pg", self.store),
                                    rank=self.rank, world_size=self.world_size, timeout=timeout)
            if self.layout.async_ps:
                self.worker_group = dist.new_group(self.layout.worker_ranks())
            else:
                self.worker_group = dist.group.WORLD
        self._started = True
        self._start_heartbeat(self.layout.process_index(self.job_name, self.task_index,
                                                        self.local_rank if self.job_name == "worker" else 0),
                              self.layout.num_processes)
        logger.info("Server started: %s task %d (rank %s of %d) target %s" % (
            self.job_name, self.task_index, self.rank, self.world_size, self.target))

    def _start_heartbeat(self, hb_id, hb_world):
        from . import health
        enabled, interval, timeout = health.heartbeat_settings()
        if enabled and hb_world > 1 and self.store is not None:
            self.heartbeat = health.Heartbeat(self.store, hb_id, hb_world, interval=interval, timeout=timeout)
            self.heartbeat.start()

    # -- done-queue barrier (distribute_train.py:43-46, 86-90, 202-205) ---
    def signal_done(self):
        """A worker tower reports completion (the reference's done-queue enqueue)."""
        if self.heartbeat is not None:
            self.heartbeat.stop(done=True)      # finished, not failed
        n = self.store.add("mdtf/done_queue0", 1)
        logger.info("done token enqueued (%d received)" % n)
        return n

    def done_count(self):
        return self.store.add("mdtf/done_queue0", 0)

    def wait_for_workers(self, num_tokens=None, poll_s=0.05, timeout_s=None):
        """Block until every worker tower has signalled done.

        Fix for SURVEY Q8: every PS waits for *all* tokens (the reference's PS
        tasks shared one queue and split the tokens, so some never exited).
        """
        if num_tokens is None:
            num_tokens = self.layout.num_worker_ranks
        t0 = time.time()
        while self.done_count() < num_tokens:
            if timeout_s is not None and time.time() - t0 > timeout_s:
                raise TimeoutError("only %d of %d done tokens after %.0fs" % (
                    self.done_count(), num_tokens, timeout_s))
            time.sleep(poll_s)

    def join(self):
        """PS role: serve until all workers are done (tf.train.Server.join)."""
        self.wait_for_workers()

    def shutdown(self):
        import torch.distributed as dist
        if self.heartbeat is not None:
            self.heartbeat.stop(done=True)
        if dist.is_initialized() and not self._torchrun:
            dist.destroy_process_group()
        _set_current(None)
