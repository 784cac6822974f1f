"""Failure detection, fault injection and restart supervision.

The reference has none of this (SURVEY §5 "Failure detection"): its PS blocks
forever on the done-queue when a worker dies, and TF1's recoverable session is
the only recovery path.  Here:

* :class:`Heartbeat` — every task of a job (ps and worker ranks) bumps a
  counter ``mdtf/hb/<rank>`` in the job's TCPStore every ``interval`` seconds
  and watches everyone else's counter.  A peer whose counter has not moved for
  ``timeout`` seconds (measured on the watcher's own monotonic clock, so host
  clock skew does not matter) is declared failed: the watcher logs it, records
  ``mdtf/hb/failed`` and terminates its own process with
  :data:`EXIT_PEER_FAILURE`.  Hard exit is deliberate: a rank blocked inside an
  RCCL collective on a dead peer cannot be unwound from Python, and the
  supervisor restarts the whole job from the last checkpoint anyway.  A task
  that finishes normally marks itself ``done`` so it is never reported.
* :class:`FaultInjectionHook` — a SessionRunHook that kills (or hangs) the
  process of one chosen task at a given global step, driven by environment
  variables (``MDTF_FAULT_STEP``, ``MDTF_FAULT_TASK=worker:1``,
  ``MDTF_FAULT_MODE=exit|hang|abort|unavailable``; abort/unavailable raise the TF error in-process,
  which the MonitoredSession recovers from without a restart); it only fires on the first attempt
  (``MDTF_RESTART_ATTEMPT=0``) so a restarted job runs clean.
* :func:`supervise` — runs a set of task commands, and when any of them fails,
  stops the rest and restarts the whole set (up to ``max_restarts`` times)
  with ``MDTF_RESTART_ATTEMPT`` incremented; the chief then resumes from the
  latest checkpoint in ``model_dir`` (MonitoredTrainingSession restore).
"""
import os
import signal
import subprocess
import threading
import time

from ..train import hooks as H
from ..train import variables as V
from ..utils import log as logger

EXIT_PEER_FAILURE = 75
EXIT_INJECTED_FAULT = 76
ENV_ATTEMPT = "MDTF_RESTART_ATTEMPT"


class Heartbeat(object):
    def __init__(self, store, rank, world_size, interval=1.0, timeout=30.0, prefix="mdtf/hb", on_failure=None):
        self.store = store
        self.rank = rank
        self.world = world_size
        self.interval = float(interval)
        self.timeout = float(timeout)
        self.prefix = prefix
        self.on_failure = on_failure
        self._stop = threading.Event()
        self._thread = None
        self._seen = {}          # rank -> (last counter value, monotonic time it changed)
        self.failed_rank = None

    def _key(self, r):
        return "%s/%d" % (self.prefix, r)

    def start(self):
        if self._thread is not None:
            return self
        self.store.set(self._key(self.rank), "0")
        now = time.monotonic()
        for r in range(self.world):
            if r != self.rank:
                self._seen[r] = (None, now)
        self._thread = threading.Thread(target=self._run, name="mdtf-heartbeat", daemon=True)
        self._thread.start()
        return self

    def _run(self):
        beat = 0
        while not self._stop.wait(self.interval):
            beat += 1
            try:
                self.store.set(self._key(self.rank), str(beat))
                self._check()
            except Exception as e:      # the store host itself died
                if self._stop.is_set():
                    return
                self._fail(None, "coordination store unreachable: %s" % (e,))
                return

    def _check(self):
        now = time.monotonic()
        for r in list(self._seen):
            key = self._key(r)
            if not self.store.check([key]):
                val = None
            else:
                val = self.store.get(key).decode()
            if val == "done":
                self._seen.pop(r)
                continue
            last, t = self._seen[r]
            if val is None:
                # not started yet (slow imports / staggered launch): the clock runs from its first beat
                self._seen[r] = (None, now)
            elif val != last:
                self._seen[r] = (val, now)
            elif now - t > self.timeout:
                self._fail(r, "no heartbeat from rank %d for %.1fs" % (r, now - t))
                return

    def _fail(self, r, why):
        self.failed_rank = r
        logger.error("rank %d: %s -- peer failure, aborting this rank" % (self.rank, why))
        try:
            self.store.set("%s/failed" % self.prefix, str(r))
        except Exception:
            pass
        if self.on_failure is not None:
            self.on_failure(r)
        else:
            os._exit(EXIT_PEER_FAILURE)

    def stop(self, done=True):
        self._stop.set()
        if done:
            try:
                self.store.set(self._key(self.rank), "done")
            except Exception:
                pass
        if self._thread is not None:
            self._thread.join(timeout=self.interval * 2 + 1)


def heartbeat_settings():
    """(enabled, interval, timeout) from MDTF_HEARTBEAT / _INTERVAL / _TIMEOUT."""
    enabled = os.environ.get("MDTF_HEARTBEAT", "1") not in ("0", "false", "off")
    return (enabled, float(os.environ.get("MDTF_HEARTBEAT_INTERVAL", "1.0")),
            float(os.environ.get("MDTF_HEARTBEAT_TIMEOUT", "300.0")))


class FaultInjectionHook(H.SessionRunHook):
    """Kill or hang this process at ``step`` if it is the chosen task (first attempt only)."""

    def __init__(self, job_name, task_index, step=None, task=None, mode=None):
        self.step = int(step if step is not None else os.environ.get("MDTF_FAULT_STEP", "-1"))
        task = task if task is not None else os.environ.get("MDTF_FAULT_TASK", "worker:0")
        self.mode = mode or os.environ.get("MDTF_FAULT_MODE", "exit")
        self.armed = (self.step >= 0 and task == "%s:%d" % (job_name, task_index)
                      and int(os.environ.get(ENV_ATTEMPT, "0")) == 0)

    @classmethod
    def from_env(cls, job_name, task_index):
        if "MDTF_FAULT_STEP" not in os.environ:
            return None
        h = cls(job_name, task_index)
        return h if h.armed else None

    def before_run(self, run_context):
        if not self.armed or V.get_global_step().value() < self.step:
            return None
        if self.mode.endswith("_before_run"):
            # a recoverable error raised by a hook BEFORE the step (the async agreement still runs the step)
            from .. import errors
            self.armed = False
            cls = errors.AbortedError if self.mode.startswith("abort") else errors.UnavailableError
            logger.error("injected before_run fault at global step %d (%s)" % (V.get_global_step().value(),
                                                                             self.mode))
            raise cls(message="injected %s at global step %d" % (self.mode, V.get_global_step().value()))
        if not self.mode.endswith("_in_step"):
            return None
        # raise from INSIDE the train op (after its collectives and update), not from a hook
        from .. import errors
        from ..train import step as S
        self.armed = False
        cls = errors.AbortedError if self.mode.startswith("abort") else errors.UnavailableError

        def fault(step):
            logger.error("injected in-step fault at global step %d (%s)" % (step, self.mode))
            raise cls(message="injected %s inside the step at global step %d" % (self.mode, step))
        S.STEP_FAULTS.append(fault)
        return None

    def after_run(self, run_context, run_values):
        if (not self.armed or self.mode.endswith("_in_step") or self.mode.endswith("_before_run")
                or V.get_global_step().value() < self.step):
            return
        logger.error("injected fault at global step %d (%s)" % (V.get_global_step().value(), self.mode))
        if self.mode in ("abort", "unavailable"):
            # in-process recoverable fault: the MonitoredSession re-creates itself from the checkpoint
            from .. import errors
            self.armed = False
            cls = errors.AbortedError if self.mode == "abort" else errors.UnavailableError
            raise cls(message="injected %s at global step %d" % (self.mode, V.get_global_step().value()))
        if self.mode == "hang":
            while True:
                time.sleep(3600)
        os._exit(EXIT_INJECTED_FAULT)


def _stop_all(procs, grace_s=5.0):
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    t0 = time.time()
    for p in procs:
        try:
            p.wait(timeout=max(grace_s - (time.time() - t0), 0.1))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def supervise(commands, env=None, max_restarts=0, timeout_s=None, cwd=None, poll_s=0.2, log_dir=None):
    """Run ``commands`` (lists of argv) as one job; restart all of them on any failure.

    ``log_dir``: each task's stdout+stderr goes to ``task<i>.attempt<a>.log`` there.
    Returns ``(exit_codes, attempts)`` of the last attempt.
    """
    base_env = dict(os.environ)
    base_env.update(env or {})
    deadline = time.time() + timeout_s if timeout_s else None
    attempt = 0
    while True:
        e = dict(base_env)
        e[ENV_ATTEMPT] = str(attempt)
        logs = []
        if log_dir:
            os.makedirs(log_dir, exist_ok=True)
            logs = [open(os.path.join(log_dir, "task%d.attempt%d.log" % (i, attempt)), "w")
                    for i in range(len(commands))]
        procs = [subprocess.Popen(c, env=e, cwd=cwd, stdout=logs[i] if logs else None,
                                  stderr=subprocess.STDOUT if logs else None) for i, c in enumerate(commands)]
        failed = None
        while True:
            codes = [p.poll() for p in procs]
            bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                failed = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if deadline and time.time() > deadline:
                _stop_all(procs)
                raise TimeoutError("job did not finish within %.0fs" % timeout_s)
            time.sleep(poll_s)
        for f in logs:
            f.close()
        if failed is None:
            return [p.returncode for p in procs], attempt
        logger.error("task %d exited with %d (attempt %d); stopping the job" % (failed[0], failed[1], attempt))
        _stop_all(procs)
        if attempt >= max_restarts:
            return [p.returncode for p in procs], attempt
        attempt += 1
        logger.info("restarting the job (attempt %d of %d)" % (attempt, max_restarts))
