"""Session-run hooks (``tf.train.SessionRunHook`` family).

Reference: ``MonitoredTrainingSession`` is created with
``StopAtStepHook(last_step=total_step)`` and the SyncReplicas hook
(``distribute_train.py:169-180``) and implicitly adds CheckpointSaver (600 s),
StepCounter (every 100 steps) and SummarySaver hooks; ``ExamplesPerSecondHook``
is defined in ``distribute_utils.py:57-116``.  All of them are provided here
with the TF hook protocol (begin / after_create_session / before_run /
after_run / end).
"""
import json
import math
import os
import time

import torch

from ..utils import log as logger
from . import variables as V


class SessionRunArgs(object):
    def __init__(self, fetches=None, feed_dict=None, options=None):
        self.fetches = fetches
        self.feed_dict = feed_dict
        self.options = options


class SessionRunValues(object):
    def __init__(self, results, options=None, run_metadata=None):
        self.results = results
        self.options = options
        self.run_metadata = run_metadata


class SessionRunContext(object):
    def __init__(self, original_args, session):
        self.original_args = original_args
        self.session = session
        self._stop_requested = False

    def request_stop(self):
        self._stop_requested = True

    @property
    def stop_requested(self):
        return self._stop_requested


class SessionRunHook(object):
    def begin(self):
        pass

    def after_create_session(self, session, coord=None):
        pass

    def before_run(self, run_context):
        return None

    def after_run(self, run_context, run_values):
        pass

    def end(self, session):
        pass


class SecondOrStepTimer(object):
    def __init__(self, every_secs=None, every_steps=None):
        if (every_secs is None) == (every_steps is None):
            raise ValueError("exactly one of every_secs and every_steps should be provided")
        self._every_secs, self._every_steps = every_secs, every_steps
        self._last_time, self._last_step = None, None

    def should_trigger_for_step(self, step):
        if self._last_step is None:
            return True
        if step == self._last_step:
            return False
        if self._every_secs is not None:
            return time.time() >= self._last_time + self._every_secs
        return step >= self._last_step + self._every_steps

    def update_last_triggered_step(self, step):
        now = time.time()
        if self._last_time is None:
            elapsed = (None, None)
        else:
            elapsed = (now - self._last_time, step - self._last_step)
        self._last_time, self._last_step = now, step
        return elapsed

    def last_triggered_step(self):
        return self._last_step


class StopAtStepHook(SessionRunHook):
    def __init__(self, num_steps=None, last_step=None):
        if (num_steps is None) == (last_step is None):
            raise ValueError("One of num_steps or last_step must be specified.")
        self._num_steps, self._last_step = num_steps, last_step

    def after_create_session(self, session, coord=None):
        gs = V.get_global_step()
        if self._last_step is None:
            self._last_step = gs.value() + self._num_steps
        if gs.value() >= self._last_step:
            session.request_stop()

    def after_run(self, run_context, run_values):
        if V.get_global_step().value() >= self._last_step:   # '>=' fixes SURVEY Q12
            run_context.request_stop()


class StepCounterHook(SessionRunHook):
    """Logs ``global_step/sec`` every N steps (TF StepCounterHook)."""

    def __init__(self, every_n_steps=100, every_n_secs=None, output_dir=None, summary_writer=None):
        self._timer = SecondOrStepTimer(every_secs=every_n_secs,
                                        every_steps=every_n_steps if every_n_secs is None else None)
        self._writer = summary_writer
        self.last_rate = None

    def after_run(self, run_context, run_values):
        step = V.get_global_step().value()
        if self._timer.should_trigger_for_step(step):
            dt, ds = self._timer.update_last_triggered_step(step)
            if dt:
                self.last_rate = ds / dt
                logger.info("global_step/sec: %g" % self.last_rate)
                if self._writer is not None:
                    self._writer.add_scalar("global_step/sec", self.last_rate, step)


class ExamplesPerSecondHook(SessionRunHook):
    """Average and current examples/sec (``distribute_utils.py:57-116``).

    ``batch_size`` should be the *global* batch for a whole-job rate.
    """

    def __init__(self, batch_size, every_n_steps=100, every_n_secs=None, sync_fn=None):
        if (every_n_steps is None) == (every_n_secs is None):
            raise ValueError("exactly one of every_n_steps and every_n_secs should be provided.")
        self._timer = SecondOrStepTimer(every_secs=every_n_secs, every_steps=every_n_steps)
        self._step_train_time = 0.0
        self._total_steps = 0
        self._batch_size = batch_size
        self._sync = sync_fn
        self.average_examples_per_sec = None
        self.current_examples_per_sec = None

    def after_run(self, run_context, run_values):
        step = V.get_global_step().value()
        if self._timer.should_trigger_for_step(step):
            if self._sync is not None:
                self._sync()
            elapsed_time, elapsed_steps = self._timer.update_last_triggered_step(step)
            if elapsed_time:
                steps_per_sec = elapsed_steps / elapsed_time
                self._step_train_time += elapsed_time
                self._total_steps += elapsed_steps
                self.average_examples_per_sec = self._batch_size * (self._total_steps / self._step_train_time)
                self.current_examples_per_sec = steps_per_sec * self._batch_size
                logger.info("Average examples/sec: %g (%g), step = %g" % (
                    self.average_examples_per_sec, self.current_examples_per_sec, self._total_steps))


class LoggingTensorHook(SessionRunHook):
    def __init__(self, tensors, every_n_iter=None, every_n_secs=None, formatter=None):
        self._tensors = tensors if isinstance(tensors, dict) else {getattr(t, "name", str(i)): t
                                                                   for i, t in enumerate(tensors)}
        self._timer = SecondOrStepTimer(every_secs=every_n_secs,
                                        every_steps=every_n_iter if every_n_secs is None else None)
        self._formatter = formatter
        self._should = False

    def before_run(self, run_context):
        self._should = self._timer.should_trigger_for_step(V.get_global_step().value())
        return SessionRunArgs(self._tensors) if self._should else None

    def after_run(self, run_context, run_values):
        if self._should and run_values.results:
            self._timer.update_last_triggered_step(V.get_global_step().value())
            vals = {k: (float(v) if hasattr(v, "__float__") and getattr(v, "ndim", 0) == 0 else v)
                    for k, v in run_values.results.items()}
            logger.info(self._formatter(vals) if self._formatter else
                        ", ".join("%s = %s" % kv for kv in vals.items()))


class NanTensorHook(SessionRunHook):
    def __init__(self, loss_tensor, fail_on_nan_loss=True):
        self._loss = loss_tensor
        self._fail = fail_on_nan_loss

    def before_run(self, run_context):
        return SessionRunArgs(self._loss)

    def after_run(self, run_context, run_values):
        v = float(run_values.results)
        if math.isnan(v) or math.isinf(v):
            if self._fail:
                raise RuntimeError("Model diverged with loss = NaN.")
            logger.warn("Model diverged with loss = NaN.")
            run_context.request_stop()


class CheckpointSaverHook(SessionRunHook):
    """Saves tensor-bundle checkpoints every N secs/steps and at the end."""

    def __init__(self, checkpoint_dir, save_secs=None, save_steps=None, saver=None, checkpoint_basename="model.ckpt",
                 scaffold=None, listeners=None):
        if save_secs is None and save_steps is None:
            save_secs = 600
        self._dir = checkpoint_dir
        self._timer = SecondOrStepTimer(every_secs=save_secs, every_steps=save_steps if save_secs is None else None)
        self._saver = saver
        self._scaffold = scaffold
        self._path = os.path.join(checkpoint_dir, checkpoint_basename)
        self._session = None
        self._listeners = listeners or []

    def _get_saver(self):
        if self._saver is None:
            from .saver import Saver
            self._saver = (self._scaffold.saver if self._scaffold is not None and self._scaffold.saver else Saver())
        return self._saver

    def after_create_session(self, session, coord=None):
        self._session = session
        step = V.get_global_step().value()
        self._timer.update_last_triggered_step(step)

    def after_run(self, run_context, run_values):
        step = V.get_global_step().value()
        if self._timer.should_trigger_for_step(step):
            self._timer.update_last_triggered_step(step)
            self._save(run_context.session, step)

    def end(self, session):
        step = V.get_global_step().value()
        if step != self._timer.last_triggered_step():
            self._save(session, step)

    def _save(self, session, step):
        logger.info("Saving checkpoints for %d into %s." % (step, self._path))
        for lst in self._listeners:
            lst.before_save(session, step)
        self._get_saver().save(session, self._path, global_step=step)
        for lst in self._listeners:
            lst.after_save(session, step)


class SummarySaverHook(SessionRunHook):
    """Writes scalar summaries (``tf.summary.scalar`` values) every N steps."""

    def __init__(self, save_steps=100, save_secs=None, output_dir=None, summary_writer=None, scaffold=None,
                 summary_op=None):
        self._timer = SecondOrStepTimer(every_secs=save_secs, every_steps=save_steps if save_secs is None else None)
        self._writer = summary_writer
        self._dir = output_dir

    def begin(self):
        if self._writer is None and self._dir:
            from ..utils.summary import FileWriter
            self._writer = FileWriter(self._dir)

    def after_run(self, run_context, run_values):
        step = V.get_global_step().value()
        if self._writer is not None and self._timer.should_trigger_for_step(step):
            self._timer.update_last_triggered_step(step)
            from ..utils import summary
            for name, val in summary.collect_step_scalars().items():
                self._writer.add_scalar(name, val, step)
            self._writer.flush()

    def end(self, session):
        if self._writer is not None:
            self._writer.close()


class SyncReplicasHook(SessionRunHook):
    """Companion hook of SyncReplicasOptimizer (``make_session_run_hook``).

    TF's hook starts the chief queue runner and the initial tokens; here the
    synchronisation is collective, so the hook only records whether this
    replica's gradients were aggregated in the last step (backup workers).
    """

    def __init__(self, opt, is_chief):
        self._opt = opt
        self.is_chief = is_chief
        self._dropped = 0
        self._dropped_dev = None       # device-side count when the contributor mask lives on the GPU

    @property
    def dropped_steps(self):
        """Steps whose gradients were not aggregated (a host read only when asked for)."""
        extra = int(self._dropped_dev.item()) if self._dropped_dev is not None else 0
        return self._dropped + extra

    def after_run(self, run_context, run_values):
        from . import step as step_mod
        for op in step_mod.train_ops():
            if op.optimizer is not self._opt:
                continue
            c = op.last_contributed
            if isinstance(c, torch.Tensor):
                # GPU backup workers: count on the device, no host sync per step
                miss = (c.reshape(-1)[:1] == 0).to(torch.int64)
                self._dropped_dev = miss if self._dropped_dev is None else self._dropped_dev + miss
            elif not c:
                self._dropped += 1


class ProfilerHook(SessionRunHook):
    """Captures a torch.profiler trace (ROCm/roctracer) for steps [start, start+n)."""

    def __init__(self, output_dir, start_step=10, num_steps=5):
        self._dir, self._start, self._n = output_dir, start_step, num_steps
        self._prof = None

    def before_run(self, run_context):
        step = V.get_global_step().value()
        if step == self._start and self._prof is None:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts)
            self._prof.__enter__()
        return None

    def after_run(self, run_context, run_values):
        step = V.get_global_step().value()
        if self._prof is not None and step >= self._start + self._n:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self._prof.__exit__(None, None, None)
            os.makedirs(self._dir, exist_ok=True)
            path = os.path.join(self._dir, "trace_step%d.json" % step)
            self._prof.export_chrome_trace(path)
            with open(os.path.join(self._dir, "kernels_step%d.txt" % step), "w") as f:
                f.write(self._prof.key_averages().table(sort_by="self_cuda_time_total"
                                                        if torch.cuda.is_available() else "self_cpu_time_total",
                                                        row_limit=60))
            self._prof = None


class FinalOpsHook(SessionRunHook):
    def __init__(self, final_ops, final_ops_feed_dict=None):
        self._ops, self._feed = final_ops, final_ops_feed_dict
        self.final_ops_values = None

    def end(self, session):
        self.final_ops_values = session.run_raw(self._ops, self._feed)


class JsonMetricsHook(SessionRunHook):
    """Appends {step, fetched values} JSON lines (machine-readable training log)."""

    def __init__(self, path, tensors, every_n_steps=10):
        self._path, self._tensors, self._every = path, tensors, every_n_steps

    def before_run(self, run_context):
        if V.get_global_step().value() % self._every == 0:
            return SessionRunArgs(self._tensors)
        return None

    def after_run(self, run_context, run_values):
        if run_values.results is None:
            return
        rec = {"step": V.get_global_step().value()}
        for k, v in run_values.results.items():
            rec[k] = float(v)
        with open(self._path, "a") as f:
            f.write(json.dumps(rec) + "\n")
