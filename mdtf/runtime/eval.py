"""``Eval`` operator — a real evaluation loop (the reference's is a stub,
``distribute_eval.py:13-23``).

Builds the model forward from ``data_loader.load_eval_batch()`` under the same
variable names, restores the latest checkpoint from ``model_dir`` (waiting for
one up to ``checkpoint_wait_secs``), runs ``eval_steps`` batches in inference
mode (BN uses moving statistics) and reports mean loss and — when the logits
are class scores and the ground truth integer labels — top-1 accuracy.  Eval
tasks of a multi-replica job shard the batches and all-reduce the sums.
"""
import time

import torch

from ..config.flags import FLAGS
from ..data.loaders import InputOptions
from ..train import saver as SV
from ..train import step as S
from ..train import variables as V
from ..utils import log as logger
from .tower import Tower


class Eval(object):
    def __init__(self, data_loader=None, input_mode=None):
        self.data_loader = data_loader
        self.input_mode = input_mode

    def eval(self, pre_eval_fn=None, post_eval_fn=None, pre_process_fn=None, post_process_fn=None, *args, **kwargs):
        from .train import configure_store_for
        server = getattr(self, "server", None)
        if server is not None and self.job_name == "ps":
            return None
        configure_store_for(server)
        pre = pre_eval_fn(args, kwargs) if pre_eval_fn is not None else None
        if self.input_mode == InputOptions.PLACEHOLDER:
            raw, gt = self.data_loader.load_eval_batch()
        else:
            raw, gt = self.data_loader.load_eval_batch()
        tower = Tower(self.net, "tower_0/", [], raw, gt, self.loss, None, pre_process_fn=pre_process_fn,
                      batch_size=self.batch_size)
        with S.training_mode(False):
            loss_h, logits_h = tower.tower_loss(post_process_fn, pre)
        V.get_store().frozen = True           # variables exist now: later forwards reuse them
        V.get_or_create_global_step()
        ckpt = self._wait_for_checkpoint()
        if ckpt is not None:
            SV.Saver(save_optimizer_state=False).restore(None, ckpt)
            logger.info("Eval: restored %s (global_step %d)" % (ckpt, V.get_global_step().value()))
        else:
            logger.warn("Eval: no checkpoint in %r; evaluating the initial weights" % (self.model_dir,))
        steps = int(getattr(self, "eval_steps", 0) or max(self.sample_number // max(self.batch_size, 1), 1))
        total_loss, correct, count = 0.0, 0.0, 0.0
        sample_queue = None
        if self.input_mode == InputOptions.PLACEHOLDER:
            sample_queue = self.data_loader.load_queue_for_placeholder(self.data_dir)
        for _ in range(steps):
            feed = None
            if sample_queue is not None:
                rb, gb = self.data_loader.load_placeholder_data(sample_queue)
                feed = {raw: rb, gt: gb}
            ctx = S.RunContext(feed)
            try:
                out = tower.program.forward(ctx, grad=False)
            except StopIteration:
                break
            lv = out["loss"].detach().float()
            logits = out["logits"]
            labels = tower._ground_truth_value
            total_loss += float(lv)
            if logits.dim() == 2 and labels is not None and not labels.is_floating_point() and labels.dim() == 1:
                correct += float((logits.argmax(-1) == labels.to(logits.device)).sum())
                count += labels.numel()
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and server is not None and server.worker_group is not None:
            t = torch.tensor([total_loss, correct, count, float(steps)], dtype=torch.float64,
                             device=V.get_store().device if V.get_store().device.type == "cuda" else "cpu")
            dist.all_reduce(t, group=server.worker_group)
            total_loss, correct, count, steps = t.tolist()
        self.metrics = {"loss": total_loss / max(steps, 1),
                        "accuracy": (correct / count) if count else None,
                        "global_step": V.get_global_step().value(), "steps": int(steps)}
        logger.info("Eval: %s" % self.metrics)
        if server is not None:
            server.signal_done()
        if post_eval_fn is not None:
            post_eval_fn(args, kwargs)
        return self.metrics

    def _wait_for_checkpoint(self):
        md = getattr(self, "model_dir", None)
        wait = float(getattr(self, "checkpoint_wait_secs", 0))
        t0 = time.time()
        while True:
            ckpt = SV.latest_checkpoint(md) if md else None
            if ckpt or time.time() - t0 >= wait:
                return ckpt
            time.sleep(1.0)

    def run(self):
        return self.eval(pre_eval_fn=getattr(self, "pre_fn", None), post_eval_fn=getattr(self, "post_fn", None),
                         pre_process_fn=getattr(self, "pre_process_fn", None),
                         post_process_fn=getattr(self, "post_process_fn", None))
