"""Input pipeline: the reference's data-loader extension points on eager tensors.

Reference: ``distribute_input.py:19-208`` — ``InputOptions``, the ``Dataloader``
ABC and the ``TFRecordDataLoader`` / ``DataPathDataLoader`` /
``PlaceholderDataLoader`` templates whose abstract hooks users implement.

Graph-free design: ``load_train_batch`` returns *handles*
(:class:`~mdtf.train.step.SourceOutput` or placeholders) that the session
resolves once per ``run``.  Batches are produced by background threads
(records from the native shuffling loader, parsed + decoded + stacked),
staged in pinned host memory and copied to HBM with non-blocking DMA.

Fixes: Q14 — user hooks may be written with a single underscore
(``_decode_raw_data``) or with the reference's name-mangled spelling
(``_TFRecordDataLoader__decode_raw_data``, or ``__decode_raw_data`` inside the
subclass); Q15 — the non-shuffled batch path uses ``num_thread``; Q16 — the
DataPath reader reads from the name queue; Q10 — the placeholder sample queue
is built once and every tower is fed.
"""
import abc
import enum
import multiprocessing
import queue
import threading

import numpy as np
import torch

from ..config import constants
from ..config.flags import FLAGS
from ..train import step as S
from . import example as E
from . import tfrecord as TFR


class InputOptions(enum.Enum):
    TF_RECORD = 0
    PLACEHOLDER = 1
    DATAPATHLOADER = 2
    SYNTHETIC = 3


def _find_hook(obj, base_names):
    """Locate a user hook under its plain, single-underscore or mangled names."""
    candidates = []
    for name in base_names:
        candidates += [name, "_" + name]
        for cls in type(obj).__mro__:
            candidates.append("_%s__%s" % (cls.__name__, name))
    for c in candidates:
        fn = getattr(obj, c, None)
        if callable(fn):
            return fn
    return None


def _require_hook(obj, name):
    fn = _find_hook(obj, [name])
    if fn is None:
        raise NotImplementedError("%s must implement %s (or _%s)" % (type(obj).__name__, name, name))
    return fn


def _to_tensor(x):
    if isinstance(x, torch.Tensor):
        return x
    return torch.as_tensor(np.asarray(x))


def _stack(examples):
    """List of per-example tuples -> tuple of batched (pinned) tensors."""
    cols = list(zip(*examples))
    out = []
    for col in cols:
        t = torch.stack([_to_tensor(c) for c in col])
        if torch.cuda.is_available():
            t = t.pin_memory()
        out.append(t)
    return tuple(out)


class _Prefetcher(object):
    """Background batch producer: ``num_threads`` threads fill a bounded queue."""

    def __init__(self, make_batch, depth=4, num_threads=1):
        self._make = make_batch
        self._q = queue.Queue(maxsize=depth)
        self._stop = False
        self._threads = [threading.Thread(target=self._run, daemon=True) for _ in range(max(num_threads, 1))]
        for t in self._threads:
            t.start()

    def _run(self):
        while not self._stop:
            try:
                b = self._make()
            except StopIteration:
                self._q.put(StopIteration)
                return
            except Exception as e:  # surface producer errors to the consumer
                self._q.put(e)
                return
            self._q.put(b)

    def __call__(self):
        b = self._q.get()
        if b is StopIteration:
            raise StopIteration("input exhausted")
        if isinstance(b, Exception):
            raise b
        return b

    def close(self):
        self._stop = True


class Dataloader(metaclass=abc.ABCMeta):
    """Base of every data loader (``distribute_input.py:25-69``).

    Injected by the entrypoint: ``batch_size``, ``sample_number``, ``data_dir``,
    ``gpu_num`` (and ``features`` for TFRecord loaders).
    """
    type = "Dataloader"
    batch_size = 32
    sample_number = 0
    data_dir = ""
    gpu_num = 1

    @abc.abstractmethod
    def load_train_batch(self, name_queue=None, *args, **kwargs):
        """Return (raw_data, ground_truth) handles for training."""

    @abc.abstractmethod
    def load_eval_batch(self, *args, **kwargs):
        """Return (raw_data, ground_truth) handles for evaluation."""

    def _generate_image_batch(self, example_list, min_queue_examples, num_thread, shuffle=True):
        """Batch a per-example producer (``example_list``: callable -> tuple).

        ``shuffle=True``: a shuffle buffer of ``min_queue_examples + 3*batch``
        examples, sampled uniformly (``tf.train.shuffle_batch``); else FIFO.
        """
        produce = example_list
        bs = self.batch_size
        capacity = max(int(min_queue_examples), 0) + 3 * bs
        rng = np.random.default_rng(getattr(self, "seed", 0))
        lock = threading.Lock()
        pool = []

        def make_batch():
            out = []
            with lock:
                if shuffle:
                    while len(pool) < min(capacity, max(bs, int(min_queue_examples))):
                        pool.append(produce())
                    for _ in range(bs):
                        i = int(rng.integers(len(pool)))
                        out.append(pool[i])
                        pool[i] = produce()
                else:
                    for _ in range(bs):
                        out.append(produce())
            return _stack(out)
        threads = max(1, min(int(num_thread), 4))
        src = S.BatchSource(_Prefetcher(make_batch, depth=4, num_threads=threads if not shuffle else 1),
                            name=type(self).__name__)
        self._source = src
        return src

    def _batch_outputs(self, source, n=2):
        return source.outputs(n)


class TFRecordDataLoader(Dataloader, metaclass=abc.ABCMeta):
    """TFRecord input (``distribute_input.py:72-106``).

    User hook: ``_decode_raw_data(raw_features, height, width, *args) ->
    [raw_data, ground_truth]`` for ONE example (numpy/tensors).
    """
    type = "TFRecordDataLoader"
    features = None
    num_reader_threads = 4

    def load_train_batch(self, name_queue=None, *args, **kwargs):
        if name_queue is None:
            raise RuntimeError("Cannot find get the queue from tf-record.")
        return self.load_batch_from_tfrecord(name_queue, *args, **kwargs)

    def load_eval_batch(self, name_queue=None, *args, **kwargs):
        if name_queue is None:
            name_queue = TFR.string_input_producer([self.data_dir], shuffle=False)
        return self.load_batch_from_tfrecord(name_queue, *args, shuffle=False, **kwargs)

    def load_batch_from_tfrecord(self, filename_queue, *args, shuffle=True, **kwargs):
        height = FLAGS.input_image_height
        width = FLAGS.input_image_width
        if self.features is None:
            raise ValueError("TFRecordDataLoader needs features (@current_feature)")
        decode = _require_hook(self, "decode_raw_data")
        files = filename_queue.files if isinstance(filename_queue, TFR.NameQueue) else TFR.expand_paths(filename_queue)
        reader = TFR.ShuffledRecordLoader(files, epochs=getattr(filename_queue, "num_epochs", None), shuffle=shuffle,
                                          capacity=4096, num_threads=self.num_reader_threads)
        self._reader = reader
        features = self.features

        def produce():
            rec = reader.next()
            parsed = E.parse_single_example(rec, features)
            return tuple(decode(parsed, height, width, *args))
        min_q = int(self.sample_number * constants.MIN_FRACTION_OF_EXAMPLE_IN_QUEUE) if shuffle else 0
        min_q = min(min_q, 10000)
        src = self._generate_image_batch(produce, min_q, multiprocessing.cpu_count() * 2, shuffle=shuffle)
        return src.outputs(2)


class DataPathDataLoader(Dataloader, metaclass=abc.ABCMeta):
    """User-defined reader over a name queue (``distribute_input.py:109-148``).

    Hooks: ``create_name_queue(data_dir)``, ``_create_reader()`` (object with
    ``read(name_queue) -> (key, value)``), ``_parse_raw_data(value) ->
    [raw_data, ground_truth]``.
    """
    type = "DataPathDataLoader"

    def load_train_batch(self, name_queue=None, *args, **kwargs):
        assert name_queue is not None, "name queue cannot be None for DataPathDataLoader!"
        reader = _require_hook(self, "create_reader")()
        parse = _require_hook(self, "parse_raw_data")

        def produce():
            _, value = reader.read(name_queue)     # Q16: read from the name queue
            return tuple(parse(value))
        min_q = min(int(self.sample_number * constants.MIN_FRACTION_OF_EXAMPLE_IN_QUEUE), 10000)
        return self._generate_image_batch(produce, min_q, multiprocessing.cpu_count() * 2, shuffle=True).outputs(2)

    def load_eval_batch(self, *args, **kwargs):
        nq = self.create_name_queue(self.data_dir)
        reader = _require_hook(self, "create_reader")()
        parse = _require_hook(self, "parse_raw_data")

        def produce():
            _, value = reader.read(nq)
            return tuple(parse(value))
        return self._generate_image_batch(produce, 0, 1, shuffle=False).outputs(2)

    @abc.abstractmethod
    def create_name_queue(self, data_dir):
        """Return a name queue (e.g. ``string_input_producer(paths)``)."""


class PlaceholderDataLoader(Dataloader, metaclass=abc.ABCMeta):
    """Feed-dict input (``distribute_input.py:151-208``).

    Hooks: ``_create_placeholder() -> (raw_ph, gt_ph)``,
    ``_put_names_dict_into_queue(queue)``, ``decode_data_from_path_name(paths)
    -> {'raw_data': ..., 'ground_truth': ...}``.
    """
    type = "PlaceholderDataLoader"

    def load_train_batch(self, name_queue=None, *args, **kwargs):
        ph = _require_hook(self, "create_placeholder")(*args, **kwargs)
        self.placeholders = tuple(ph)
        return self.placeholders

    def load_eval_batch(self, *args, **kwargs):
        return self.load_train_batch(None, *args, **kwargs)

    def load_queue_for_placeholder(self, *args, **kwargs):
        q = getattr(self, "_sample_queue", None)
        if q is None:   # Q10: build once, keep cycling
            q = queue.Queue()
            _require_hook(self, "put_names_dict_into_queue")(q, *args, **kwargs)
            self._sample_queue = q
        return q

    @abc.abstractmethod
    def decode_data_from_path_name(self, paths, *args, **kwargs):
        """Return {'raw_data': array, 'ground_truth': array} for one sample."""

    def load_placeholder_data(self, sample_path_queue, *args, **kwargs):
        raw_batch, gt_batch = [], []
        for _ in range(self.batch_size):
            paths = sample_path_queue.get()
            data = self.decode_data_from_path_name(paths, *args, **kwargs)
            raw_batch.append(data['raw_data'])
            gt_batch.append(data['ground_truth'])
            sample_path_queue.put(paths)
        return np.stack([np.asarray(r) for r in raw_batch]), np.stack([np.asarray(g) for g in gt_batch])


class SyntheticDataLoader(Dataloader):
    """Device-resident random batches of a fixed shape (benchmarks, smoke tests).

    ``shape`` excludes the batch dim; labels are uniform in ``[0, num_classes)``.
    The batch is generated once on the device and reused every step (the
    standard synthetic-data benchmark protocol: no H2D in the timed loop).
    """
    type = "SyntheticDataLoader"

    def __init__(self, shape=(224, 224, 3), num_classes=1000, dtype=torch.float32, label_shape=(), seed=0,
                 label_dtype=torch.int64, resample=False):
        self.shape = tuple(shape)
        self.num_classes = num_classes
        self.dtype = dtype
        self.label_shape = tuple(label_shape)
        self.seed = seed
        self.label_dtype = label_dtype
        self.resample = resample
        self._batch = None

    def _make(self):
        from ..train import variables as V
        dev = V.get_store().device
        g = torch.Generator(device="cpu").manual_seed(self.seed)
        x = torch.randn((self.batch_size,) + self.shape, generator=g).to(self.dtype)
        if self.label_dtype.is_floating_point:
            y = torch.randn((self.batch_size,) + self.label_shape, generator=g)
        else:
            y = torch.randint(0, self.num_classes, (self.batch_size,) + self.label_shape, generator=g)
        return x.to(dev), y.to(self.label_dtype).to(dev)

    def _next(self):
        if self._batch is None or self.resample:
            self._batch = self._make()
        return self._batch

    def load_train_batch(self, name_queue=None, *args, **kwargs):
        return S.BatchSource(self._next, name="synthetic").outputs(2)

    def load_eval_batch(self, *args, **kwargs):
        return self.load_train_batch()
