import os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch
import test_kernels_gpu as T
T.setup_module(T)
for be in ("mdtf2", "miopen", "mdtf"):
    os.environ["MDTF_CONV"] = be
    for model in ("tinyres", "tiny"):
        saved = T._Tiny
        if model == "tinyres":
            T._Tiny = T._TinyRes
        torch.manual_seed(3)
        x = torch.randn(16, 12, 12, 64)
        y = torch.randint(0, 16, (16,))
        lc, gc = T._tiny_step("cpu", None, x, y)
        lg, gg = T._tiny_step(T.DEV, torch.bfloat16, x, y)
        T._Tiny = saved
        errs = sorted(((T._rel(gg[k], gc[k]), k) for k in gc), reverse=True)[:5]
        print(be, model, "loss rel %.2e" % (abs(lc - lg) / lc), ["%s %.3f" % (k, e) for e, k in errs], flush=True)
