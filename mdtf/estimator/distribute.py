"""``DistributeEstimator`` and ``DistributeExperiment`` — the reference's two
alternative front ends, made to work.

* ``DistributeEstimator`` (``distribute_estimator.py:13-35``): an
  :class:`~mdtf.estimator.Estimator` that also carries an input class, given
  as ``input_class=`` or by the ``@current_input(input='ClassName')`` class
  annotation (resolved through the annotation registry / ``mdtf.data``), and an
  optional separate ``eval_model_fn`` used by ``evaluate``.
* ``DistributeExperiment`` (``distribute_experiment.py:11-83``): Train or Eval
  driven by user callables ``train_fn(dataloader, input_mode, pre, post)`` /
  ``eval_fn(dataloader, pre, post)``.  The load option comes from
  ``FLAGS.data_load_option`` (defined here, unlike the reference, whose
  undefined flag made the class unusable); data loaders are given directly or
  named by ``@current_input(train_input=..., eval_input=...)``.
"""
from ..config import annotations
from ..config.flags import FLAGS
from ..data import loaders as L
from .estimator import Estimator, ModeKeys

_OPTIONS = {
    "tfrecords": L.InputOptions.TF_RECORD,
    "placeholder": L.InputOptions.PLACEHOLDER,
    "datapath": L.InputOptions.DATAPATHLOADER,
    "synthetic": L.InputOptions.SYNTHETIC,
}


def current_input(**kwds):
    """Class annotation naming the input class(es): keys ``input``, ``train_input``, ``eval_input``."""
    allowed = ("input", "train_input", "eval_input")
    for k in kwds:
        if k not in allowed:
            raise TypeError("current_input got unknown key %r (allowed: %s)" % (k, ", ".join(allowed)))

    def decorate(f):
        for k, v in kwds.items():
            setattr(f, k, v)
        return f
    return decorate


def _resolve_class(name):
    if not isinstance(name, str):
        return name
    import mdtf.data as data_pkg
    for mod in (data_pkg, L):
        cls = getattr(mod, name, None)
        if cls is not None:
            return cls
    reg = annotations._REGISTRY.get(name)
    if reg is not None:
        return reg
    import sys
    main = sys.modules.get("__main__")
    cls = getattr(main, name, None)
    if cls is None:
        raise ValueError("input class %r not found (register it with mdtf.annotations.register_class)" % name)
    return cls


class DistributeEstimator(Estimator):
    def __init__(self, model_fn, eval_model_fn=None, config=None, params=None, input_class=None, model_dir=None):
        super(DistributeEstimator, self).__init__(model_fn, model_dir=model_dir, config=config, params=params)
        if input_class is None:
            name = getattr(type(self), "input", None) or getattr(DistributeEstimator, "input", None)
            if not name:
                raise ValueError("Please either pass your input class or use annotation @current_input")
            input_class = _resolve_class(name)
        self.input_class = input_class
        self.eval_model_fn = eval_model_fn

    def _model_fn_for(self, mode):
        if mode == ModeKeys.EVAL and self.eval_model_fn is not None:
            return self.eval_model_fn
        return self._model_fn


class DistributeExperiment(object):
    def __init__(self, mode, train_fn=None, train_dataloader=None, eval_fn=None, eval_dataloader=None,
                 features=None):
        self.mode = mode
        if train_fn is None and eval_fn is None:
            raise ValueError("At least provide a function for processing")
        option = FLAGS.data_load_option
        if option not in _OPTIONS:
            raise ValueError("Please specify a valid data load option %s as --data_load_option." % sorted(_OPTIONS))
        self.input_mode = _OPTIONS[option]
        if mode == "Train":
            if train_fn is None:
                raise ValueError("In Train mode, train_fn cannot be None")
            self.train_fn = train_fn
            self.train_dataloader = train_dataloader or self._loader("train_input", features)
        elif mode == "Eval":
            if eval_fn is None:
                raise ValueError("In Eval mode, eval_fn must be provided.")
            self.eval_fn = eval_fn
            self.eval_dataloader = eval_dataloader or self._loader("eval_input", features)
        else:
            raise ValueError("Please provide either Train or Eval as mode.")

    def _loader(self, key, features):
        name = getattr(type(self), key, None) or getattr(DistributeExperiment, key, None)
        if not name:
            raise ValueError("In %s mode, a %s data loader must be provided." % (self.mode, key))
        cls = _resolve_class(name)
        loader = annotations.instantiate(cls)
        if self.input_mode == L.InputOptions.TF_RECORD:
            if features is None:
                raise ValueError("Please provide features for parsing the tf-record.")
            loader.features = features
        return loader

    def train(self, pre_train_fn=None, post_train_fn=None):
        return self.train_fn(self.train_dataloader, self.input_mode, pre_train_fn, post_train_fn)

    def evaluation(self, pre_eval_fn=None, post_evaluation_fn=None):
        return self.eval_fn(self.eval_dataloader, pre_eval_fn, post_evaluation_fn)

    def run(self):
        if self.mode == "Train":
            return self.train()
        return self.evaluation()
