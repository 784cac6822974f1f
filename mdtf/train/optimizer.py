"""Optimizers (TF1 ``tf.train.*Optimizer`` API) on fused flat-buffer kernels.

Reference: ``@optimizer(optimizer=tf.train.AdamOptimizer(0.001))``
(``distribute.py:26``), the default Adam(1e-3) (``distribute.py:112``) and
``SyncReplicasOptimizer`` (``distribute_train.py:146-160``).

``compute_gradients`` / ``apply_gradients`` / ``minimize`` return *handles*
(see :mod:`mdtf.train.step`): the work runs when a session runs the returned
train op.  Updates are applied by one fused HIP launch per parameter group
(:mod:`mdtf.ops.optim`).  Optimizer slots keep TF's checkpoint names
(``<var>/Momentum``, ``<var>/Adam``, ``<var>/Adam_1``, ``beta1_power``,
``beta2_power``).
"""
import torch
from ..ops import optim as K
from . import step as step_mod


def _lr_value(lr, global_step):
    if callable(lr):
        return float(lr(global_step))
    if hasattr(lr, "learning_rate"):        # mdtf.utils.learning_rate.LearningRate
        return float(lr.learning_rate)
    return float(lr)


class Optimizer(object):
    slot_names = ()

    def __init__(self, learning_rate, use_locking=False, name="Optimizer", weight_decay=0.0):
        self._lr = learning_rate
        self._name = name
        self.use_locking = use_locking
        self.weight_decay = float(weight_decay)

    def get_name(self):
        return self._name

    def learning_rate(self, global_step=0):
        return _lr_value(self._lr, global_step)

    # -- TF graph-building API (deferred) -------------------------------
    def compute_gradients(self, loss, var_list=None):
        return step_mod.compute_gradients(loss, var_list)

    def apply_gradients(self, grads_and_vars, global_step=None, name=None):
        return step_mod.TrainOp(self, grads_and_vars, global_step)

    def minimize(self, loss, global_step=None, var_list=None, name=None):
        if isinstance(loss, torch.Tensor):
            # inside an Estimator model_fn (re-run eagerly every step): the estimator
            # turns this request into ONE TrainOp over the recorded program's loss
            from ..estimator.estimator import current_capture
            cap = current_capture()
            if cap is None:
                raise TypeError("minimize() of a concrete tensor is only valid inside an Estimator model_fn; "
                                "use the loss handle returned by Tower.process()")
            return cap.record(self, global_step, var_list)
        return self.apply_gradients(self.compute_gradients(loss, var_list), global_step, name)

    # -- fused update over one UpdateTarget ------------------------------
    def update(self, target, lr, grad_scale, step, dyn=None):
        """One fused launch over ``target``.  ``dyn``: optional device tensor
        ``[lr, lr_t, grad_scale]`` overriding the scalars (hipGraph replay)."""
        raise NotImplementedError

    def step_size(self, lr, step):
        """The per-step ``lr_t`` the kernel applies (Adam folds its bias correction in)."""
        return lr

    def update_multi(self, target, grads, steps, grad_scale=1.0):
        """Apply ``grads`` (<= 8, in order) to ``target`` as consecutive updates at global ``steps``, in ONE
        fused pass (async parameter server).  Default: one ``update`` per gradient."""
        for g, st in zip(grads, steps):
            target.grad.copy_(g)
            self.update(target, self.learning_rate(st), grad_scale, st)

    def _wd(self, target):
        return self.weight_decay if target.decay else 0.0

    def slot_checkpoint_names(self):
        """(state name, TF slot suffix) pairs."""
        return []

    def extra_checkpoint_scalars(self, step):
        return {}


class GradientDescentOptimizer(Optimizer):
    def __init__(self, learning_rate, use_locking=False, name="GradientDescent", weight_decay=0.0):
        super(GradientDescentOptimizer, self).__init__(learning_rate, use_locking, name, weight_decay)

    def update(self, target, lr, grad_scale, step, dyn=None):
        K.sgd_(target.master, target.grad, target.shadow, lr, grad_scale, self._wd(target), dyn=dyn)

    def update_multi(self, target, grads, steps, grad_scale=1.0):
        lrs = [self.learning_rate(s) for s in steps]
        K.apply_multi_("sgd", target.master, grads, None, None, target.shadow, lrs, lrs, grad_scale=grad_scale,
                       weight_decay=self._wd(target))


class MomentumOptimizer(Optimizer):
    def __init__(self, learning_rate, momentum=0.9, use_locking=False, name="Momentum", use_nesterov=False,
                 weight_decay=0.0):
        super(MomentumOptimizer, self).__init__(learning_rate, use_locking, name, weight_decay)
        self.momentum = float(momentum)
        self.use_nesterov = use_nesterov

    def update(self, target, lr, grad_scale, step, dyn=None):
        K.momentum_(target.master, target.grad, target.state("momentum"), target.shadow, lr, self.momentum,
                    grad_scale, self._wd(target), self.use_nesterov, dyn=dyn)

    def update_multi(self, target, grads, steps, grad_scale=1.0):
        lrs = [self.learning_rate(s) for s in steps]
        K.apply_multi_("momentum", target.master, grads, target.state("momentum"), None, target.shadow, lrs, lrs,
                       momentum=self.momentum, grad_scale=grad_scale, weight_decay=self._wd(target),
                       flag=self.use_nesterov)

    def slot_checkpoint_names(self):
        return [("momentum", "Momentum")]


class AdamOptimizer(Optimizer):
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, use_locking=False, name="Adam",
                 weight_decay=0.0, decoupled_weight_decay=False, bias_correction=True):
        super(AdamOptimizer, self).__init__(learning_rate, use_locking, name, weight_decay)
        self.beta1, self.beta2, self.epsilon = float(beta1), float(beta2), float(epsilon)
        self.decoupled = decoupled_weight_decay
        self.bias_correction = bias_correction

    def update(self, target, lr, grad_scale, step, dyn=None):
        K.adam_(target.master, target.grad, target.state("m"), target.state("v"), target.shadow, lr,
                self.beta1, self.beta2, self.epsilon, step + 1, grad_scale, self._wd(target), self.decoupled,
                self.bias_correction, dyn=dyn)

    def step_size(self, lr, step):
        return K.adam_lr_t(lr, self.beta1, self.beta2, step + 1, self.bias_correction)

    def update_multi(self, target, grads, steps, grad_scale=1.0):
        lrs = [self.learning_rate(s) for s in steps]
        lrts = [self.step_size(lr, s) for lr, s in zip(lrs, steps)]
        K.apply_multi_("adam", target.master, grads, target.state("m"), target.state("v"), target.shadow, lrs, lrts,
                       beta1=self.beta1, beta2=self.beta2, epsilon=self.epsilon, grad_scale=grad_scale,
                       weight_decay=self._wd(target), flag=self.decoupled)

    def slot_checkpoint_names(self):
        return [("m", "Adam"), ("v", "Adam_1")]

    def extra_checkpoint_scalars(self, step):
        return {"beta1_power": self.beta1 ** (step + 1), "beta2_power": self.beta2 ** (step + 1)}


class AdamWeightDecayOptimizer(AdamOptimizer):
    """BERT's optimizer: Adam without bias correction + decoupled weight decay."""

    def __init__(self, learning_rate, weight_decay_rate=0.01, beta_1=0.9, beta_2=0.999, epsilon=1e-6,
                 name="AdamWeightDecayOptimizer"):
        super(AdamWeightDecayOptimizer, self).__init__(learning_rate, beta_1, beta_2, epsilon, name=name,
                                                       weight_decay=weight_decay_rate,
                                                       decoupled_weight_decay=True, bias_correction=False)


class SyncReplicasOptimizer(Optimizer):
    """Synchronous data-parallel wrapper (``tf.train.SyncReplicasOptimizer``).

    ``replicas_to_aggregate`` of ``total_num_replicas`` gradients are averaged
    per step (backup workers when smaller).  ``mode='allreduce'`` reduces with
    overlapped bucketed all-reduce; ``mode='sharded'`` makes every rank the
    parameter server of 1/N of each bucket (reduce-scatter + local fused update
    + all-gather) — the MI355X-native form of PS variable sharding.
    ``bucket_bytes`` (default ``MDTF_BUCKET_MB`` or 32 MiB of fp32 gradients) sets the
    collective granularity; ``comm_dtype='bf16'`` halves the bytes on the wire.
    """

    def __init__(self, opt, replicas_to_aggregate=None, total_num_replicas=None, variable_averages=None,
                 variables_to_average=None, use_locking=False, name="sync_replicas", mode="allreduce",
                 bucket_bytes=None, overlap=True, hip_graph=None, comm_dtype=None):
        super(SyncReplicasOptimizer, self).__init__(opt._lr, use_locking, name, opt.weight_decay)
        self._opt = opt
        self.replicas_to_aggregate = replicas_to_aggregate
        self.total_num_replicas = total_num_replicas
        self.mode = mode
        self.bucket_bytes = bucket_bytes
        self.overlap = overlap
        self.hip_graph = hip_graph   # None: MDTF_HIP_GRAPH / --hip_graph decide (mdtf.train.graph)
        # gradient wire dtype: None -> MDTF_COMM_DTYPE (fp32 default) | "bf16" (mdtf.parallel.reducer)
        self.comm_dtype = comm_dtype

    def learning_rate(self, global_step=0):
        return self._opt.learning_rate(global_step)

    def update(self, target, lr, grad_scale, step, dyn=None):
        self._opt.update(target, lr, grad_scale, step, dyn=dyn)

    def update_multi(self, target, grads, steps, grad_scale=1.0):
        self._opt.update_multi(target, grads, steps, grad_scale)

    def step_size(self, lr, step):
        return self._opt.step_size(lr, step)

    def slot_checkpoint_names(self):
        return self._opt.slot_checkpoint_names()

    def extra_checkpoint_scalars(self, step):
        return self._opt.extra_checkpoint_scalars(step)

    def apply_gradients(self, grads_and_vars, global_step=None, name=None):
        op = step_mod.TrainOp(self, grads_and_vars, global_step, sync=True)
        return op

    def make_session_run_hook(self, is_chief, num_tokens=-1):
        from .hooks import SyncReplicasHook
        return SyncReplicasHook(self, is_chief)

    def get_init_tokens_op(self, num_tokens=-1):
        return None

    def get_chief_queue_runner(self):
        return None


# aliases with TF spellings
Adam = AdamOptimizer
Momentum = MomentumOptimizer
GradientDescent = GradientDescentOptimizer
