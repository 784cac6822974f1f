"""Annotation (decorator) based configuration — the reference's IoC layer.

Reference: ``distribute_annotations.py:8-339`` — sixteen decorator factories
that each copy whitelisted keyword arguments onto the decorated function/class,
plus two reflection helpers.  Here every decorator is produced by one factory
(:func:`_annotation`) from a table of (decorator name -> accepted keys).

Behavioural fixes:
  * Q1 — the reference silently drops unknown keys (so the sample's
    ``ps_hosts(ps_host=...)`` configured nothing).  We raise ``TypeError`` for
    unknown keys; the singular/plural host aliases are accepted explicitly.
  * Q6 — ``get_advice`` values must be callables (or ``None``).
  * ``get_instance_from_annotation`` resolves classes from the given module,
    the explicit class registry, or ``__main__``; it accepts class objects and
    instances as well as names, and runs a zero-argument ``__init__`` when one
    exists (the reference always skipped ``__init__``).
"""
import inspect
import sys

_REGISTRY = {}


def register_class(cls=None, name=None):
    """Register a user class (Model/Loss/Dataloader/...) for name lookup.

    Usable as ``@register_class`` or ``@register_class(name="Alias")``.
    """
    def deco(c):
        _REGISTRY[name or c.__name__] = c
        return c
    if cls is None:
        return deco
    return deco(cls)


def _annotation(deco_name, keys, aliases=None, validate=None):
    keys = tuple(keys)
    aliases = dict(aliases or {})

    def factory(**kwds):
        resolved = {}
        for k, v in kwds.items():
            k2 = aliases.get(k, k)
            if k2 not in keys:
                raise TypeError("@%s does not accept %r (accepted: %s)" % (deco_name, k, ", ".join(keys)))
            if validate is not None:
                validate(k2, v)
            resolved[k2] = v

        def decorate(f):
            for k, v in resolved.items():
                setattr(f, k, v)
            return f
        return decorate

    factory.__name__ = deco_name
    factory.__qualname__ = deco_name
    factory.__doc__ = "Annotation @%s(%s): stores the value(s) as attribute(s) of the decorated object." % (
        deco_name, ", ".join("%s=..." % k for k in keys))
    return factory


def _callable_or_none(key, value):
    if value is not None and not callable(value):
        raise TypeError("advice %r must be a callable or None, got %r (SURVEY Q6)" % (key, type(value).__name__))


# -- function-level annotations on main (distribute_annotations.py:8-315) ----
current_model = _annotation("current_model", ["model"])
current_input = _annotation("current_input", ["input"])
current_mode = _annotation("current_mode", ["mode"])
current_feature = _annotation("current_feature", ["features"])
gpu_num = _annotation("gpu_num", ["gpu_num"])
ps_hosts = _annotation("ps_hosts", ["ps_hosts"], aliases={"ps_host": "ps_hosts"})
worker_hosts = _annotation("worker_hosts", ["worker_hosts"], aliases={"worker_host": "worker_hosts"})
job_name = _annotation("job_name", ["job_name"])
task_index = _annotation("task_index", ["task_index"])
batch_size = _annotation("batch_size", ["batch_size"])
sample_number = _annotation("sample_number", ["sample_number"])
epoch_num = _annotation("epoch_num", ["epoch_num"])
model_dir = _annotation("model_dir", ["model_dir"])
data_dir = _annotation("data_dir", ["data_dir"])
optimizer = _annotation("optimizer", ["optimizer"])
loss = _annotation("loss", ["loss"])
# framework extensions (no reference counterpart)
ps_mode = _annotation("ps_mode", ["ps_mode"])
eval_steps = _annotation("eval_steps", ["eval_steps"])
save_checkpoint = _annotation("save_checkpoint", ["save_checkpoint_secs", "save_checkpoint_steps"])

# -- class-level annotations on the operator (Train/Eval) --------------------
# The reference whitelists the misspelt 'post_processs_fn' (:100) while Train.run
# reads 'post_process_fn' (distribute_train.py:218); accept both, store the latter.
get_advice = _annotation(
    "get_advice",
    ["pre_fn", "post_fn", "pre_process_fn", "post_process_fn", "init_fn"],
    aliases={"post_processs_fn": "post_process_fn"},
    validate=_callable_or_none)
parse_data_dir = _annotation("parse_data_dir", ["parse_data_dir_fn"], validate=_callable_or_none)


def get_value_from_annotation(obj, attr, default=inspect.Parameter.empty):
    """Return ``obj.<attr>``; raise ``ValueError`` when absent (``:336-339``)."""
    if hasattr(obj, attr):
        return getattr(obj, attr)
    if default is not inspect.Parameter.empty:
        return default
    raise ValueError("Annotation @%s is required on %r" % (attr, getattr(obj, "__name__", obj)))


def _lookup_class(name, module):
    candidates = []
    if module is not None:
        candidates.append(module if isinstance(module, dict) else vars(module))
    candidates.append(_REGISTRY)
    main = sys.modules.get("__main__")
    if main is not None:
        candidates.append(vars(main))
    for space in candidates:
        if name in space:
            return space[name]
    raise ValueError("Cannot resolve class %r (looked in %s, the class registry and __main__)" % (
        name, getattr(module, "__name__", "the given namespace")))


def instantiate(cls):
    """Instantiate ``cls``: run ``__init__`` only if it takes no required args.

    The reference always used ``cls.__new__(cls)`` (``:331-333``), which skips
    ``__init__`` but still enforces ``abc`` abstract methods.
    """
    init = cls.__init__
    if init is object.__init__:
        return cls()
    try:
        sig = inspect.signature(init)
    except (TypeError, ValueError):
        return cls.__new__(cls)
    required = [p for p in list(sig.parameters.values())[1:]
                if p.default is inspect.Parameter.empty
                and p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD, p.KEYWORD_ONLY)]
    if required:
        obj = cls.__new__(cls)
        if getattr(obj, "__abstractmethods__", None) or getattr(cls, "__abstractmethods__", None):
            raise TypeError("Can't instantiate abstract class %s" % cls.__name__)
        return obj
    return cls()


def get_instance_from_annotation(obj, attr, module=None):
    """Resolve the class named by ``obj.<attr>`` and return an instance.

    ``obj.<attr>`` may be a class name (string), a class, or an instance.
    """
    value = get_value_from_annotation(obj, attr)
    if isinstance(value, str):
        cls = _lookup_class(value, module)
    elif inspect.isclass(value):
        cls = value
    else:
        return value
    if getattr(cls, "__abstractmethods__", None):
        raise TypeError("Can't instantiate abstract class %s with abstract methods %s" % (
            cls.__name__, ", ".join(sorted(cls.__abstractmethods__))))
    return instantiate(cls)
