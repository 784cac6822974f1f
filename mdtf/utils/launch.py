"""One-process-per-GPU launch contract of the benchmark scripts (``bench.py``, ``bench/*_bench.py``).

``python bench.py --gpus N`` must measure N GPUs whether or not the caller used torchrun:

* under ``torch.distributed.run`` (``RANK``/``WORLD_SIZE`` in the environment) the rank count must
  equal ``--gpus``; a mismatch exits non-zero instead of silently timing a different job;
* without it and N > 1, the script re-launches itself as a ``torch.distributed.run`` CHILD process
  (rendezvous on 127.0.0.1, a free port) and exits with the child's code.  This happens before
  anything touches the GPU, and the parent never ``exec``s: the child is an ordinary subprocess.
"""
import os
import socket
import subprocess
import sys


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def under_launcher():
    return "RANK" in os.environ and "WORLD_SIZE" in os.environ


def ensure_ranks(n_gpus, script, argv=None):
    """Make the current job have exactly ``n_gpus`` ranks (see module docstring).

    Returns normally when the current process is one of the right number of ranks (or n_gpus == 1
    outside a launcher); otherwise spawns the launcher child and ``sys.exit``s with its code."""
    argv = list(sys.argv[1:] if argv is None else argv)
    if under_launcher():
        world = int(os.environ["WORLD_SIZE"])
        if world != n_gpus:
            sys.stderr.write("launch mismatch: --gpus %d but WORLD_SIZE=%d; refusing to report a %d-rank "
                             "measurement as %d GPUs\n" % (n_gpus, world, world, n_gpus))
            sys.exit(3)
        return
    if n_gpus <= 1:
        return
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n_gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(script)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC for RCCL on this host driver
    sys.stdout.flush()
    rc = subprocess.call(cmd, env=env)
    sys.exit(rc)
