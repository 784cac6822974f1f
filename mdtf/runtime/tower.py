"""``Tower``: one data-parallel replica of the model.

Reference: ``distribute_tower.py:16-152``.  A TF tower is a copy of the model
graph on ``/gpu:i`` sharing variables through scope reuse; its gradients are
averaged in-graph by ``average_gradients``.  Here a tower is one process/GPU
(rank).  ``process`` records the tower computation as a
:class:`~mdtf.train.step.TowerProgram`, runs the variable-building pass, and
returns handles for the loss and logits; ``average_gradients`` of handles is
the cross-replica mean that the bucketed RCCL reducer performs during the
step.  Called with real tensors it computes the mean directly (the math of
``:78-114``).
"""
import re

import torch

from ..config import constants
from ..train import step as S
from ..train import variables as V
from ..utils import summary


class Tower(object):
    def __init__(self, net, scope, tower_grades, raw_data, ground_truth, loss, optimizer, pre_process_fn=None,
                 batch_size=None):
        self.net = net
        self.scope = scope
        self.tower_grades = tower_grades
        self.raw_data = raw_data
        self.ground_truth = ground_truth
        self.loss = loss
        self.optimizer = optimizer
        self.pre_process_fn = pre_process_fn
        self.batch_size = batch_size or 1
        self.program = None

    def get_gradient(self, loss):
        return self.optimizer.compute_gradients(loss)

    def _forward(self, post_process_fn, args, kwargs):
        scope = self.scope.rstrip("/")

        def fn(raw, gt):
            if self.pre_process_fn is not None:          # applied to the pair
                raw, gt = self.pre_process_fn(raw, gt, args, kwargs)
            with V.name_scope(scope):
                logits = self.net.process(raw, args, kwargs)
                if post_process_fn is not None:
                    logits = post_process_fn(logits)
                self._ground_truth_value = gt
                self.loss_to_scope(logits, gt)
                losses = V.get_collection('losses', scope)
                total = losses[0]
                for l in losses[1:]:
                    total = total + l
            for i, l in enumerate(losses):
                summary.scalar("%s/loss_%d" % (scope, i), l)
            summary.scalar("%s/total_loss" % scope, total)
            return {"loss": total, "logits": logits}
        return fn

    def tower_loss(self, post_process_fn=None, *args, **kwargs):
        prog = S.TowerProgram(self._forward(post_process_fn, args, kwargs), (self.raw_data, self.ground_truth),
                              name=self.scope.rstrip("/") or "tower")
        self.program = prog
        prog.build(self.batch_size)
        return prog.output("loss"), prog.output("logits")

    def process(self, post_process_fn=None, *args, **kwargs):
        """Record the tower, create its variables, compute gradient handles.

        Returns ``(summaries, loss, logits)`` like ``distribute_tower.py:32-58``.
        """
        with V.variable_scope(V.get_variable_scope(), reuse=None):
            loss, logits = self.tower_loss(post_process_fn, *args, **kwargs)
        V.get_variable_scope().reuse_variables()
        summaries = V.get_collection(V.GraphKeys.SUMMARIES, self.scope)
        grads = self.get_gradient(loss)
        self.tower_grades.append(grads)
        return summaries, loss, logits

    def __loss(self, result, ground_truth):
        return self.loss.loss(result, ground_truth)

    def loss_to_scope(self, result, ground_truth=None):
        gt = self.ground_truth if ground_truth is None else ground_truth
        l = self.__loss(result, gt)
        V.add_to_collection('losses', l)
        losses = V.get_collection('losses')
        total = losses[0]
        for x in losses[1:]:
            total = total + x
        return total

    @staticmethod
    def average_gradients(tower_grads):
        """Mean gradient per shared variable over towers.

        With gradient handles (the normal training path) the per-variable
        results are the reducer's averaged flat-buffer slots; with tensors the
        mean is computed here.
        """
        average_grads = []
        for grad_and_vars in zip(*tower_grads):
            g0, v0 = grad_and_vars[0]
            if isinstance(g0, S.GradRef):
                average_grads.append((g0, v0))
                continue
            grads = [torch.as_tensor(g).unsqueeze(0) for g, _ in grad_and_vars]
            average_grads.append((torch.cat(grads, 0).mean(0), v0))
        return average_grads

    @staticmethod
    def tower_fn(tower):
        return tower.process()


def strip_tower_prefix(name):
    return re.sub('%s_[0-9]*/' % constants.TOWER_NAME, '', name)
