import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import mdtf
from mdtf.models import Bert, BertPretrainingLoss, SyntheticBertLoader
from mdtf.runtime import Net, Tower
from mdtf.train import variables as V
store = V.get_store(); store.device = torch.device("cuda"); store.compute_dtype = torch.bfloat16
ld = SyntheticBertLoader(128, 20); ld.batch_size = 64
raw, gt = ld.load_train_batch()
base = mdtf.train.AdamWeightDecayOptimizer(1e-4, weight_decay_rate=0.01)
tg = []
t = Tower(Net(Bert("base", seq_len=128, max_predictions=20)), "tower_0/", tg, raw, gt, BertPretrainingLoss(20), base, batch_size=64)
_, loss, _ = t.process()
opt = mdtf.train.SyncReplicasOptimizer(base, hip_graph=False)
op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
for _ in range(3): sess.run(op)
torch.cuda.synchronize()
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    sess.run(op); torch.cuda.synchronize()
for name in ("aten::copy_", "aten::fill_", "aten::add_", "aten::add", "aten::cat", "aten::zeros", "aten::to", "aten::_to_copy"):
    evs=[e for e in prof.key_averages(group_by_stack_n=6) if e.key == name]
    for e in sorted(evs, key=lambda e: -e.count)[:4]:
        st=[s for s in e.stack if "mdtf" in s or "bert" in s][:4]
        print(name, e.count, " | ".join(st))
