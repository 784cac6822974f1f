"""Command-line flag system (absl / ``tf.app.flags`` equivalent, no TF).

Reference: ``distribute_flags.py:9-62`` defines the flags through
``tf.app.flags``.  This module offers the same ``DEFINE_*`` API and a lazily
parsed global ``FLAGS`` object: the first attribute read parses ``sys.argv``
(like TF, because the reference's decorators read ``FLAGS.job_name`` at import
time, ``distribute.py:39-40``).  Unknown command-line arguments are tolerated
so user scripts can add their own argparse handling.

Fixes vs the reference: the thread-pool flags are defined as
``intra_op_parallelism_threads`` / ``inter_op_parallelism_threads`` (no
trailing spaces) and are wired into ``torch.set_num_threads`` by
:func:`apply_thread_flags`.
"""
import argparse
import sys
import threading


def _str2bool(v):
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y", "on"):
        return True
    if s in ("0", "false", "f", "no", "n", "off"):
        return False
    raise argparse.ArgumentTypeError("expected a boolean, got %r" % v)


class _FlagValues(object):
    """Holds flag definitions and lazily parsed values."""

    def __init__(self):
        object.__setattr__(self, "_defs", {})
        object.__setattr__(self, "_values", {})
        object.__setattr__(self, "_parsed", False)
        object.__setattr__(self, "_lock", threading.RLock())
        object.__setattr__(self, "_argv", None)

    # -- definition -------------------------------------------------------
    def _define(self, name, default, help_str, kind):
        with self._lock:
            self._defs[name] = (default, help_str, kind)
            if self._parsed:
                # late definition: parse this flag from the remembered argv
                self._values[name] = self._parse_one(name, default, kind)

    def _parse_one(self, name, default, kind):
        p = argparse.ArgumentParser(add_help=False)
        self._add(p, name, default, kind)
        ns, _ = p.parse_known_args(self._argv or [])
        return getattr(ns, name)

    @staticmethod
    def _add(p, name, default, kind):
        if kind is bool:
            p.add_argument("--" + name, nargs="?", const=True, default=default, type=_str2bool)
            p.add_argument("--no" + name, dest=name, action="store_false")
        else:
            p.add_argument("--" + name, default=default, type=kind)

    # -- parsing ----------------------------------------------------------
    def __call__(self, argv=None):
        """Parse ``argv`` (defaults to ``sys.argv[1:]``); returns unparsed args."""
        with self._lock:
            argv = list(sys.argv[1:] if argv is None else argv)
            p = argparse.ArgumentParser(add_help=False)
            for name, (default, _, kind) in self._defs.items():
                self._add(p, name, default, kind)
            ns, rest = p.parse_known_args(argv)
            object.__setattr__(self, "_argv", argv)
            self._values.clear()
            self._values.update(vars(ns))
            object.__setattr__(self, "_parsed", True)
            return rest

    def _ensure(self):
        if not self._parsed:
            self.__call__()

    def reset(self, argv=None):
        """Re-parse from scratch (tests)."""
        object.__setattr__(self, "_parsed", False)
        if argv is not None:
            self.__call__(argv)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        self._ensure()
        if name in self._values:
            return self._values[name]
        raise AttributeError("flag --%s is not defined" % name)

    def __setattr__(self, name, value):
        self._ensure()
        if name not in self._defs:
            raise AttributeError("flag --%s is not defined" % name)
        self._values[name] = value

    def __contains__(self, name):
        return name in self._defs

    def flag_values_dict(self):
        self._ensure()
        return dict(self._values)


FLAGS = _FlagValues()


def DEFINE_string(name, default, help_str=""):
    FLAGS._define(name, default, help_str, str)


def DEFINE_integer(name, default, help_str=""):
    FLAGS._define(name, default, help_str, int)


def DEFINE_float(name, default, help_str=""):
    FLAGS._define(name, default, help_str, float)


def DEFINE_boolean(name, default, help_str=""):
    FLAGS._define(name, default, help_str, bool)


DEFINE_bool = DEFINE_boolean

# ---------------------------------------------------------------------------
# The reference's flag set (distribute_flags.py:10-62), plus framework knobs.
# ---------------------------------------------------------------------------
DEFINE_boolean('use_fp16', False, "Train the model with reduced-precision compute (bf16 on MI355X).")
DEFINE_string('project_name', 'Your project name', "String to save the project name.")
DEFINE_string('job_name', '', "One of ps and worker")
DEFINE_string('ps_hosts', '', "Comma separated host:port list of parameter servers.")
DEFINE_string('worker_hosts', '', "Comma separated host:port list of workers.")
DEFINE_integer('task_index', None, "Task index within the job; task 0 of the workers is the chief.")
DEFINE_integer('replicas_to_aggregate', None,
               "Number of replicas to aggregate before a parameter update (default: all workers).")
DEFINE_integer('intra_op_parallelism_threads', 0, "Host threads for intra-op parallelism (0 = auto).")
DEFINE_integer('inter_op_parallelism_threads', 0, "Host threads for inter-op parallelism (0 = auto).")
DEFINE_boolean('log_device_placement', False, "Log the device every variable is placed on.")
DEFINE_integer('input_image_height', 224, "Input image height.")
DEFINE_integer('input_image_width', 224, "Input image width.")
DEFINE_integer('sample_number', 100000, "Total sample numbers to train.")
DEFINE_float('train_learning_rate', 0.001, "Value of initial learning rate.")
DEFINE_string('learning_rate_json', 'YOUR LEARNING RATE SAVING PATH', "Path of the learning-rate json file.")
# framework extensions
DEFINE_string("data_load_option", "tfrecords", "DistributeExperiment input mode: tfrecords | placeholder | datapath | synthetic.")
DEFINE_string('ps_mode', 'sync', "Parameter-server mode: sync (RCCL reduce-scatter/all-gather), async, or sync_ps "
              "(dedicated PS ranks aggregating the first replicas_to_aggregate pushes per version; late pushes of "
              "backup workers are dropped, so a straggler does not stall the step).")
DEFINE_string('model_dir', '', "Override @model_dir (checkpoint directory).")
DEFINE_string('data_dir', '', "Override @data_dir (input data).")
DEFINE_string('mode', '', "Override @current_mode (Train / Eval).")
DEFINE_integer('epochs', 0, "Override @epoch_num when > 0.")
DEFINE_integer('save_checkpoint_steps', 0, "Checkpoint every N global steps (0: every save_checkpoint_secs).")
DEFINE_integer('save_checkpoint_secs', 600, "Checkpoint period in seconds (chief), as MonitoredTrainingSession.")
DEFINE_boolean('hip_graph', False, "Capture the synchronous training step in a hipGraph and replay it (mdtf.train.graph).")


def apply_thread_flags():
    """Wire the thread-pool flags into torch."""
    import torch
    if FLAGS.intra_op_parallelism_threads > 0:
        torch.set_num_threads(FLAGS.intra_op_parallelism_threads)
    if FLAGS.inter_op_parallelism_threads > 0:
        try:
            torch.set_num_interop_threads(FLAGS.inter_op_parallelism_threads)
        except RuntimeError:
            pass  # can only be set once, before any inter-op work started
