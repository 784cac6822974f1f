"""``Train`` operator: the between-graph-replication training run loop.

Mirrors ``distribute_train.py:22-221`` step by step (PS role blocks on the
done-queue; worker builds towers, averages gradients, wraps the optimizer in
``SyncReplicasOptimizer``, runs ``MonitoredTrainingSession`` until the
``StopAtStepHook``), on the MI355X design: one process per GPU, gradient
reduction over RCCL, fused optimizer kernels.

Attributes injected by the entrypoint (``distribute.py:110-127``): task_index,
job_name, optimizer, server, cluster, data_loader, input_mode, batch_size,
epoch_num, sample_number, model_dir, data_dir, net, loss, gpu_num.

Fixes: Q6 (advice must be callables), Q7 (one chief-owned global
step broadcast at session creation), Q8 (every PS waits for all done tokens),
Q9 (``pre_process_fn`` returns the (raw, gt) pair), Q10 (placeholder sample
queue built once), Q11 (examples/sec uses the real window time; the log also
reports the whole-job rate), Q12 (``>=`` on the final step + end-of-run
barrier), Q13 (``total_step`` counts *aggregated* updates; each consumes
``batch_size`` examples per replica).
"""
import time

import torch

from ..config import annotations
from ..config.flags import FLAGS
from ..data.loaders import InputOptions
from ..data import tfrecord as TFR
from ..train import device_setter as DS
from ..train import hooks as H
from ..train import optimizer as O
from ..train import session as SESS
from ..train import variables as V
from ..utils import log as logger
from .tower import Tower


def configure_store_for(server):
    """Point the variable store at this replica's device and compute dtype."""
    store = V.get_store()
    dev = server.device() if server is not None else torch.device("cpu")
    store.device = dev
    # MI355X: bf16 compute on MFMA with fp32 master weights is the native mode on the GPU
    # (the reference's --use_fp16 switch); CPU replicas compute in fp32 (or bf16 with --use_fp16).
    if dev.type == "cuda":
        store.compute_dtype = torch.bfloat16
    else:
        store.compute_dtype = torch.bfloat16 if FLAGS.use_fp16 else None
    return store


@annotations.get_advice()
class Train(object):
    def _ps_mode(self):
        mode = getattr(self, "ps_mode", None) or FLAGS.ps_mode
        if mode in ("async", "sync_ps"):
            return mode
        if mode in ("allreduce", "sharded"):
            return mode
        # 'sync': PS tasks present -> PS-shard semantics; else plain all-reduce DP
        return "sharded" if self.cluster.num_tasks("ps") > 0 else "allreduce"

    def train(self, pre_fn=None, post_fn=None, init_fn=None, pre_process_fn=None, post_process_fn=None,
              parse_data_dir_fn=None, *args, **kwargs):
        server = self.server
        is_chief = server.is_chief
        replicas_to_aggregate = FLAGS.replicas_to_aggregate
        total_step = self.epoch_num * (self.sample_number // self.batch_size)
        num_workers = self.cluster.num_tasks("worker")
        num_replicas = server.layout.num_worker_ranks
        data_dir = self.data_dir if parse_data_dir_fn is None else parse_data_dir_fn(self.data_dir)
        ps_mode = self._ps_mode()

        # ------------------------------------------------------------ PS role
        if self.job_name == "ps":
            if ps_mode in ("async", "sync_ps"):
                from ..parallel.async_ps import run_parameter_server
                r = None
                if ps_mode == "sync_ps":
                    r = replicas_to_aggregate or num_replicas
                run_parameter_server(self, server, sync_replicas=r, total_step=total_step)
                return
            server.join()
            return

        # -------------------------------------------------------- worker role
        store = configure_store_for(server)
        pre_train_result = None if pre_fn is None else pre_fn(args, kwargs)
        global_step = V.get_or_create_global_step()
        worker_device = "/job:worker/task:%d" % self.task_index
        tower_grads, tower_losses = [], []
        with V.device(DS.replica_device_setter(worker_device=worker_device, ps_device="/job:ps/cpu:0",
                                               cluster=self.cluster)):
            with V.variable_scope(V.get_variable_scope()):
                i = server.local_rank
                with V.name_scope("tower_%d" % i) as scope:
                    raw_data, ground_truth = self._inputs(data_dir)
                    tower = Tower(self.net, scope, tower_grads, raw_data, ground_truth, self.loss, self.optimizer,
                                  pre_process_fn=pre_process_fn, batch_size=self.batch_size)
                    summaries, loss, logits = tower.process(post_process_fn, pre_train_result)
                    tower_losses.append(loss)
        grads = Tower.average_gradients(tower_grads)
        loss = tower_losses[0]

        if ps_mode in ("async", "sync_ps"):
            from ..parallel.async_ps import AsyncWorker
            return AsyncWorker(self, server, tower, grads, total_step, sync=ps_mode == "sync_ps").run(
                post_fn, args, kwargs)

        if replicas_to_aggregate is None:
            replicas_to_aggregate = num_replicas
        optimizer = O.SyncReplicasOptimizer(self.optimizer, replicas_to_aggregate=replicas_to_aggregate,
                                            total_num_replicas=num_replicas, name="sync_replicas", mode=ps_mode)
        train_op = optimizer.apply_gradients(grads, global_step=global_step)
        sync_replicas_hook = optimizer.make_session_run_hook(is_chief)

        if is_chief:
            logger.info("Worker %d: Initializing session..." % self.task_index)
        else:
            logger.info("Worker %d: Waiting for session to be initialized..." % self.task_index)
        save_secs = getattr(self, "save_checkpoint_secs", None) or FLAGS.save_checkpoint_secs
        save_steps = getattr(self, "save_checkpoint_steps", None) or FLAGS.save_checkpoint_steps or None
        hooks = [H.StopAtStepHook(last_step=total_step), sync_replicas_hook]
        from ..cluster.health import FaultInjectionHook
        fault = FaultInjectionHook.from_env(self.job_name, self.task_index)
        if fault is not None:
            hooks.append(fault)
        # sharded replicas save collectively: the session factory then puts a step-triggered
        # checkpoint hook on every replica (session.MonitoredTrainingSession)
        ckpt_kwargs = dict(save_checkpoint_secs=save_secs if not save_steps else None,
                           save_checkpoint_steps=save_steps)
        with SESS.MonitoredTrainingSession(master=server.target, is_chief=is_chief,
                                           checkpoint_dir=self.model_dir or None,
                                           scaffold=SESS.Scaffold(init_op=SESS.global_variables_initializer(),
                                                                  init_fn=init_fn),
                                           hooks=hooks, config=None, stop_grace_period_secs=60,
                                           log_step_count_steps=100, server=server, **ckpt_kwargs) as sess:
            logger.info("Worker %d: Session initialization complete." % self.task_index)
            self.session = sess
            sample_queue = None
            if self.input_mode == InputOptions.PLACEHOLDER:
                sample_queue = self.data_loader.load_queue_for_placeholder(data_dir)
            window_start, window_step = time.time(), global_step.value()
            step = global_step.value()
            while not sess.should_stop():
                if self.input_mode == InputOptions.PLACEHOLDER:
                    raw_b, gt_b = self.data_loader.load_placeholder_data(sample_queue)
                    _, step, loss_value = sess.run([train_op, global_step, loss],
                                                   feed_dict={raw_data: raw_b, ground_truth: gt_b})
                else:
                    _, step, loss_value = sess.run([train_op, global_step, loss])
                if step % 10 == 0:
                    lv = float(loss_value)                      # syncs the device once per window
                    now = time.time()
                    steps = max(step - window_step, 1)
                    duration = (now - window_start) / steps
                    examples_per_sec = self.batch_size / duration if duration > 0 else 0.0
                    logger.info('step %d, loss = %.8f (%.1f examples/sec; %.3f sec/batch; job %.1f examples/sec)' % (
                        step, lv, examples_per_sec, duration, examples_per_sec * num_replicas))
                    window_start, window_step = now, step
                if step >= total_step:
                    break
            self.last_loss = loss_value
        server.signal_done()
        logger.info('kill_ps_enqueue_op done....')
        if post_fn is not None:
            post_fn(args, kwargs)

    def _inputs(self, data_dir):
        mode = self.input_mode
        if mode == InputOptions.TF_RECORD:
            q = TFR.string_input_producer([data_dir], shuffle=True)
            return self.data_loader.load_train_batch(q)
        if mode == InputOptions.PLACEHOLDER:
            return self.data_loader.load_train_batch()
        if mode == InputOptions.DATAPATHLOADER:
            q = self.data_loader.create_name_queue(data_dir)
            return self.data_loader.load_train_batch(q)
        if mode == InputOptions.SYNTHETIC:
            return self.data_loader.load_train_batch()
        raise ValueError("unknown input mode %r" % (mode,))

    def run(self):
        self.train(pre_fn=getattr(self, "pre_fn", None),
                   post_fn=getattr(self, "post_fn", None),
                   pre_process_fn=getattr(self, "pre_process_fn", None),
                   post_process_fn=getattr(self, "post_process_fn", None),
                   init_fn=getattr(self, "init_fn", None),
                   parse_data_dir_fn=getattr(self, "parse_data_dir_fn", None))
