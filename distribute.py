#!/usr/bin/env python
"""Entrance of a distributed training job — the reference's ``distribute.py``, on mdtf.

Launch one process per task, exactly like the reference (``distribute.py:1-136``):

    python distribute.py --job_name=ps     --task_index=0
    python distribute.py --job_name=worker --task_index=0

With ``@gpu_num(n > 1)`` a worker task starts ``n`` tower processes (one per
GPU); ``torchrun`` launches are also accepted.  This sample is BASELINE config
1: LeNet on MNIST-shaped data, 1 parameter server + 1 worker on localhost
(synthetic data unless ``--data_dir`` points at MNIST TFRecords written with
``examples/make_mnist_tfrecords.py``).  User classes are found by reflection
in this module (``__main__``), the mdtf class registry, or the module given to
``run_from_annotations``.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mdtf  # noqa: E402
from mdtf.config import annotations  # noqa: E402
from mdtf.config.flags import FLAGS  # noqa: E402
from mdtf.data import example as E  # noqa: E402
from mdtf.data.loaders import SyntheticDataLoader, TFRecordDataLoader  # noqa: E402
from mdtf.models import LeNet  # noqa: E402
from mdtf.runtime import Loss  # noqa: E402
from mdtf.runtime.entry import run_from_annotations  # noqa: E402


class MyModel(LeNet):
    """LeNet-5 style CNN (conv5x5-32, pool, conv5x5-64, pool, fc512, fc10)."""


class MyLoss(Loss):
    def loss(self, predict, ground_truth):
        return mdtf.nn.sparse_softmax_cross_entropy_with_logits(ground_truth, predict).mean()


class MyDataLoader(SyntheticDataLoader):
    """MNIST-shaped synthetic batches (28x28x1, 10 classes)."""

    def __init__(self):
        super(MyDataLoader, self).__init__(shape=(28, 28, 1), num_classes=10, resample=False)


class MnistTFRecordLoader(TFRecordDataLoader):
    """MNIST TFRecords: ``image_raw`` (784 uint8 bytes) + ``label`` (int64)."""

    def _decode_raw_data(self, raw_features, height, width, *args):
        img = E.decode_raw(raw_features["image_raw"], np.uint8).astype(np.float32).reshape(28, 28, 1) / 255.0
        return [torch.from_numpy(img), torch.tensor(int(raw_features["label"]), dtype=torch.int64)]


FEATURES = {"image_raw": E.FixedLenFeature([], E.string), "label": E.FixedLenFeature([], E.int64)}


@annotations.current_model(model='MyModel')
@annotations.optimizer(optimizer=mdtf.train.AdamOptimizer(0.001))
@annotations.loss(loss='MyLoss')
@annotations.current_mode(mode='Train')
@annotations.current_input(input='MyDataLoader')
@annotations.current_feature(features=FEATURES)
@annotations.gpu_num(gpu_num=0)
@annotations.ps_hosts(ps_hosts="127.0.0.1:2222")
@annotations.worker_hosts(worker_hosts="127.0.0.1:2223")
@annotations.job_name(job_name=FLAGS.job_name)
@annotations.task_index(task_index=FLAGS.task_index)
@annotations.batch_size(batch_size=32)
@annotations.sample_number(sample_number=3200)
@annotations.epoch_num(epoch_num=1)
@annotations.model_dir(model_dir="/tmp/mdtf_mnist")
@annotations.data_dir(data_dir="")
def main(argv):
    if FLAGS.model_dir:
        main.model_dir = FLAGS.model_dir
    if FLAGS.data_dir:
        main.data_dir = FLAGS.data_dir
        main.input = "MnistTFRecordLoader"
    if FLAGS.mode:
        main.mode = FLAGS.mode
    if FLAGS.epochs:
        main.epoch_num = FLAGS.epochs
    run_from_annotations(main)
    return 0


if __name__ == '__main__':
    mdtf.app.run(main)
