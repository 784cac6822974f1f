"""Tower launcher: one OS process per GPU.

The reference drives ``gpu_num`` GPUs from one worker process as in-graph
"towers" (``distribute_train.py:116-139``).  On MI355X each GPU gets its own
process (RCCL rank).  When a worker task is started the reference way
(``python distribute.py --job_name=worker --task_index=0`` with
``@gpu_num(gpu_num=4)``) :func:`maybe_spawn_towers` turns that process into a
launcher *before any GPU is touched*: it starts ``gpu_num`` child processes of
the same command line with ``MDTF_LOCAL_RANK=t`` and exits with the worst
child exit code.  Children are started with ``subprocess`` — never ``exec`` —
so the parent never replaces itself.

Also provides :func:`launch_local_cluster`, used by tests and examples to start
a whole ps+worker ClusterSpec on localhost.
"""
import os
import signal
import socket
import subprocess
import sys
import time

from ..utils import log as logger

ENV_LOCAL_RANK = "MDTF_LOCAL_RANK"
ENV_LOCAL_WORLD = "MDTF_LOCAL_WORLD_SIZE"


def under_torchrun():
    return "RANK" in os.environ and "WORLD_SIZE" in os.environ and "LOCAL_RANK" in os.environ


def is_tower_child():
    return ENV_LOCAL_RANK in os.environ


def maybe_spawn_towers(job_name, gpu_num, argv=None):
    """If this worker must drive >1 GPU, become a launcher; never returns then."""
    if job_name != "worker" or (gpu_num or 0) <= 1 or is_tower_child() or under_torchrun():
        return
    argv = list(sys.argv if argv is None else argv)
    procs = []
    for t in range(gpu_num):
        env = dict(os.environ)
        env[ENV_LOCAL_RANK] = str(t)
        env[ENV_LOCAL_WORLD] = str(gpu_num)
        procs.append(subprocess.Popen([sys.executable] + argv, env=env))
    logger.info("launched %d tower processes: %s" % (gpu_num, [p.pid for p in procs]))
    code = wait_all(procs)
    sys.exit(code)


def wait_all(procs, poll_s=0.2):
    """Wait for all children; if one fails, terminate the rest (fail fast)."""
    codes = {}
    try:
        while len(codes) < len(procs):
            for p in procs:
                if p.pid in codes:
                    continue
                rc = p.poll()
                if rc is not None:
                    codes[p.pid] = rc
                    if rc != 0:
                        logger.error("tower process %d exited with %d; stopping siblings" % (p.pid, rc))
                        for q in procs:
                            if q.poll() is None:
                                q.send_signal(signal.SIGTERM)
            time.sleep(poll_s)
    except KeyboardInterrupt:
        for q in procs:
            if q.poll() is None:
                q.send_signal(signal.SIGTERM)
        raise
    bad = [c for c in codes.values() if c != 0]
    return bad[0] if bad else 0


def free_port(host="127.0.0.1"):
    s = socket.socket()
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def cluster_commands(script_argv, num_ps, num_workers, host="127.0.0.1"):
    """argv lists of every ps/worker task of a localhost ClusterSpec (fresh ports)."""
    ports = [free_port(host) for _ in range(num_ps + num_workers)]
    ps_hosts = ",".join("%s:%d" % (host, p) for p in ports[:num_ps]) or "none"
    worker_hosts = ",".join("%s:%d" % (host, p) for p in ports[num_ps:])
    cmds = []
    for job, n in (("ps", num_ps), ("worker", num_workers)):
        for i in range(n):
            cmds.append([sys.executable] + list(script_argv) + [
                "--job_name=%s" % job, "--task_index=%d" % i,
                "--ps_hosts=%s" % ps_hosts, "--worker_hosts=%s" % worker_hosts])
    return cmds


def launch_local_cluster(script_argv, num_ps, num_workers, extra_env=None, host="127.0.0.1",
                         timeout_s=600, cwd=None, max_restarts=0, log_dir=None):
    """Start ``num_ps`` ps + ``num_workers`` worker tasks of ``script_argv`` locally.

    Every task receives ``--job_name/--task_index/--ps_hosts/--worker_hosts``.
    Returns the list of exit codes (ps tasks first).  With ``max_restarts > 0``
    the job runs under :func:`mdtf.cluster.health.supervise`: a failed task
    stops the job and the whole job is restarted (resuming from its latest
    checkpoint), and the codes are those of the last attempt.
    """
    if max_restarts:
        from . import health
        codes, attempts = health.supervise(cluster_commands(script_argv, num_ps, num_workers, host),
                                           env=extra_env, max_restarts=max_restarts, timeout_s=timeout_s, cwd=cwd,
                                           log_dir=log_dir)
        launch_local_cluster.last_attempts = attempts
        return codes
    env = dict(os.environ)
    env.update(extra_env or {})
    procs = [subprocess.Popen(cmd, env=env, cwd=cwd)
             for cmd in cluster_commands(script_argv, num_ps, num_workers, host)]
    deadline = time.time() + timeout_s
    codes = []
    for p in procs:
        remaining = max(deadline - time.time(), 1)
        try:
            codes.append(p.wait(timeout=remaining))
        except subprocess.TimeoutExpired:
            for q in procs:
                if q.poll() is None:
                    q.kill()
            raise
    return codes


def main(argv=None):
    """``python -m mdtf.cluster.launcher --num_ps 1 --num_workers 2 [--max_restarts N] script.py [args]``:
    run a whole ps+worker job on this host, optionally supervised (restart on failure)."""
    import argparse
    p = argparse.ArgumentParser(description=main.__doc__)
    p.add_argument("--num_ps", type=int, default=1)
    p.add_argument("--num_workers", type=int, default=1)
    p.add_argument("--max_restarts", type=int, default=0)
    p.add_argument("--timeout_s", type=float, default=None)
    p.add_argument("script", nargs=argparse.REMAINDER)
    a = p.parse_args(argv)
    if not a.script:
        p.error("missing script")
    codes = launch_local_cluster(a.script, a.num_ps, a.num_workers, timeout_s=a.timeout_s or 10 ** 9,
                                 max_restarts=a.max_restarts)
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


if __name__ == "__main__":
    sys.exit(main())
