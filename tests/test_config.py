"""Flags, annotations and reflection (reference distribute_flags.py / distribute_annotations.py)."""
import abc

import pytest

from mdtf.config import annotations as A
from mdtf.config import flags as F


def test_flags_parse_and_defaults():
    fv = F._FlagValues()
    fv._define("job_name", "", "", str)
    fv._define("task_index", None, "", int)
    fv._define("use_fp16", False, "", bool)
    rest = fv(["--job_name=worker", "--task_index", "3", "--use_fp16", "--unknown=1"])
    assert fv.job_name == "worker" and fv.task_index == 3 and fv.use_fp16 is True
    assert rest == ["--unknown=1"]
    fv.reset(["--nouse_fp16"])
    assert fv.use_fp16 is False and fv.job_name == ""


def test_reference_flag_names_exist():
    for name in ["use_fp16", "project_name", "job_name", "ps_hosts", "worker_hosts", "task_index",
                 "replicas_to_aggregate", "intra_op_parallelism_threads", "inter_op_parallelism_threads",
                 "log_device_placement", "input_image_height", "input_image_width", "sample_number",
                 "train_learning_rate", "learning_rate_json"]:
        assert name in F.FLAGS


def test_annotations_set_attributes():
    @A.current_model(model="MyModel")
    @A.gpu_num(gpu_num=4)
    @A.ps_hosts(ps_hosts="127.0.0.1:22")
    @A.batch_size(batch_size=35)
    def main():
        pass
    assert main.model == "MyModel" and main.gpu_num == 4 and main.ps_hosts == "127.0.0.1:22"
    assert A.get_value_from_annotation(main, "batch_size") == 35
    with pytest.raises(ValueError):
        A.get_value_from_annotation(main, "epoch_num")


def test_unknown_keys_rejected_and_alias_accepted():
    # the reference silently dropped ps_host=...; we accept the alias and reject junk
    @A.ps_hosts(ps_host="1.2.3.4:5")
    def main():
        pass
    assert main.ps_hosts == "1.2.3.4:5"
    with pytest.raises(TypeError):
        A.gpu_num(gpus=4)


def test_get_advice_requires_callables():
    with pytest.raises(TypeError):
        A.get_advice(pre_fn="print(...)")                # must be a callable (or None)

    def f(*a):
        return 1

    @A.get_advice(pre_fn=f, post_processs_fn=f)          # reference spelling accepted
    class Op(object):
        pass
    assert Op.pre_fn is f and Op.post_process_fn is f


class _Base(metaclass=abc.ABCMeta):
    @abc.abstractmethod
    def go(self):
        pass


class _Impl(_Base):
    def __init__(self):
        self.inited = True

    def go(self):
        return 1


class _NeedsArgs(_Base):
    def __init__(self, a):
        self.a = a

    def go(self):
        return 2


def test_reflection_instantiation():
    import sys
    mod = sys.modules[__name__]

    @A.current_model(model="_Impl")
    def main():
        pass
    obj = A.get_instance_from_annotation(main, "model", mod)
    assert isinstance(obj, _Impl) and obj.inited
    main.model = "_NeedsArgs"
    obj = A.get_instance_from_annotation(main, "model", mod)   # reference semantics: __new__ only
    assert isinstance(obj, _NeedsArgs) and not hasattr(obj, "a")
    main.model = "_Base"
    with pytest.raises(TypeError):
        A.get_instance_from_annotation(main, "model", mod)
    main.model = _Impl
    assert isinstance(A.get_instance_from_annotation(main, "model"), _Impl)
    main.model = "DoesNotExist"
    with pytest.raises(ValueError):
        A.get_instance_from_annotation(main, "model", mod)


def test_registry_lookup():
    @A.register_class
    class RegisteredLoss(object):
        pass

    @A.loss(loss="RegisteredLoss")
    def main():
        pass
    assert type(A.get_instance_from_annotation(main, "loss")).__name__ == "RegisteredLoss"
