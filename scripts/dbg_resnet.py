import os, sys, torch
root = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, root); sys.path.insert(0, os.path.join(root, "tests"))
import test_kernels_gpu as T
torch.manual_seed(9)
x = torch.randn(16, 64, 64, 3); y = torch.randint(0, 16, (16,))
for mode in ("mdtf", "miopen"):
    os.environ["MDTF_CONV"] = mode
    l_cpu, b_cpu, a_cpu = T._one_step("cpu", None, x, y)
    l_gpu, b_gpu, a_gpu = T._one_step("cuda", torch.bfloat16, x, y)
    print(mode, "loss", l_cpu, l_gpu)
    bad = []
    for name in a_cpu:
        d_cpu = a_cpu[name] - b_cpu[name]; d_gpu = a_gpu[name] - b_gpu[name]
        if d_cpu.norm() < 1e-6: continue
        e = T._rel(d_gpu, d_cpu)
        bad.append((e, name))
    bad.sort(reverse=True)
    for e, n in bad[:12]: print("  %.3f %s" % (e, n))
    print("  median", sorted(bad)[len(bad)//2])
