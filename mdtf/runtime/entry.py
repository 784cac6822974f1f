"""Annotation-driven entrypoint (the body of the reference's ``distribute.py:46-132``).

User script::

    @annotations.current_model(model='MyModel')
    @annotations.optimizer(optimizer=mdtf.train.AdamOptimizer(0.001))
    ...
    def main(argv):
        mdtf.runtime.entry.run_from_annotations(main)

    if __name__ == '__main__':
        mdtf.app.run(main)

Steps (reference numbering): 1) cluster description from annotations/flags,
2) operator parameters, 3) data loader (reflection + type dispatch +
injection), 4) operator class (``Train``/``Eval``), 5) attribute injection,
then ``operator.run()``.  Before any GPU work the worker becomes a tower
launcher when ``gpu_num > 1`` (one process per GPU).
"""
import os
import sys

from ..cluster import ClusterSpec, Server, launcher
from ..config import annotations
from ..config.flags import FLAGS, apply_thread_flags
from ..data import loaders as Input
from ..utils import log as logger
from .eval import Eval
from .net import Net
from .train import Train

_OPERATORS = {"Train": Train, "Eval": Eval}


def register_operator(name, cls):
    _OPERATORS[name] = cls


def _maybe(main, key, default=None):
    return annotations.get_value_from_annotation(main, key, default)


def _flag_or(main, key):
    val = _maybe(main, key, None)
    flag = getattr(FLAGS, key, None)
    if flag not in (None, ""):
        return flag              # explicit command line wins (tests / launchers)
    return val


def run_from_annotations(main, module=None):
    """Build and run the operator described by ``main``'s annotations."""
    apply_thread_flags()
    ps_hosts = _flag_or(main, "ps_hosts") or ""
    if str(ps_hosts).strip().lower() == "none":          # explicit "no parameter server" on the command line
        ps_hosts = ""
    worker_hosts = _flag_or(main, "worker_hosts")
    job_name = _flag_or(main, "job_name")
    task_index = _flag_or(main, "task_index")
    if not worker_hosts:
        raise ValueError("worker_hosts must be given (@worker_hosts or --worker_hosts)")
    if job_name not in ("ps", "worker"):
        raise ValueError("job_name must be 'ps' or 'worker' (@job_name or --job_name)")
    cluster = ClusterSpec.from_hosts(ps_hosts, worker_hosts)
    gpu_num = int(_maybe(main, "gpu_num", 0) or 0)
    launcher.maybe_spawn_towers(job_name, gpu_num)     # no return if this process became a launcher
    if job_name == "ps" and (_maybe(main, "ps_mode", None) or FLAGS.ps_mode) not in ("async", "sync_ps"):
        os.environ["HIP_VISIBLE_DEVICES"] = ""          # sync-mode PS hosts no GPU work (distribute.py:61-62)

    optimizer = _maybe(main, "optimizer", None)
    mode = annotations.get_value_from_annotation(main, "mode")
    if mode not in _OPERATORS:
        raise ValueError("mode must be set in the annotation @current_mode (one of %s)" % sorted(_OPERATORS))
    batch_size = annotations.get_value_from_annotation(main, "batch_size")
    epoch_num = annotations.get_value_from_annotation(main, "epoch_num")
    sample_number = annotations.get_value_from_annotation(main, "sample_number")
    data_dir = _maybe(main, "data_dir", "")
    model_dir = _maybe(main, "model_dir", "")
    if model_dir and not os.path.exists(model_dir):
        os.makedirs(model_dir, exist_ok=True)                  # create instead of failing
    loss = annotations.get_instance_from_annotation(main, "loss", module)
    server = Server(cluster, job_name=job_name, task_index=task_index, gpu_num=gpu_num,
                    async_ps=(_maybe(main, "ps_mode", None) or FLAGS.ps_mode) in ("async", "sync_ps"))

    data_loader = annotations.get_instance_from_annotation(main, "input", module)
    ltype = getattr(data_loader, "type", None)
    if ltype == "TFRecordDataLoader":
        if not hasattr(main, "features"):
            raise ValueError("Please use @current_feature to create your features for data_loader")
        data_loader.features = annotations.get_value_from_annotation(main, "features")
        input_mode = Input.InputOptions.TF_RECORD
    elif ltype == "PlaceholderDataLoader":
        input_mode = Input.InputOptions.PLACEHOLDER
    elif ltype == "DataPathDataLoader":
        input_mode = Input.InputOptions.DATAPATHLOADER
    elif ltype == "SyntheticDataLoader":
        input_mode = Input.InputOptions.SYNTHETIC
    else:
        raise ValueError("Data loader %s has unknown type %r; subclass one of TFRecordDataLoader, "
                         "PlaceholderDataLoader, DataPathDataLoader, SyntheticDataLoader" % (
                             type(data_loader).__name__, ltype))
    data_loader.batch_size = batch_size
    data_loader.sample_number = sample_number
    data_loader.data_dir = data_dir
    data_loader.gpu_num = gpu_num

    cls = _OPERATORS[mode]
    operator = cls.__new__(cls)
    for k in ("pre_fn", "post_fn", "pre_process_fn", "post_process_fn", "init_fn", "parse_data_dir_fn"):
        if hasattr(cls, k):
            setattr(operator, k, getattr(cls, k))
    if optimizer is None:
        from ..train.optimizer import AdamOptimizer
        optimizer = AdamOptimizer(0.001)
    inject = dict(task_index=task_index, job_name=job_name, optimizer=optimizer, server=server, cluster=cluster,
                  data_loader=data_loader, input_mode=input_mode, batch_size=batch_size, epoch_num=epoch_num,
                  sample_number=sample_number, model_dir=model_dir, data_dir=data_dir, loss=loss, gpu_num=gpu_num)
    for k, v in inject.items():
        setattr(operator, k, v)
    for k in ("ps_mode", "eval_steps", "save_checkpoint_secs", "save_checkpoint_steps"):
        if hasattr(main, k):
            setattr(operator, k, getattr(main, k))
    if job_name != "ps":
        model = annotations.get_instance_from_annotation(main, "model", module)
        operator.net = Net(model=model)
    try:
        result = operator.run()
    finally:
        server.shutdown()
    return result
