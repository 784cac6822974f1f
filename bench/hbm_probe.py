import torch, statistics
def timeit(fn, reps=20):
    for _ in range(3): fn()
    ts=[]
    for _ in range(reps):
        a,b=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); b.synchronize(); ts.append(a.elapsed_time(b))
    return statistics.median(ts)
n=256*56*56*256
x=torch.randn(n,device='cuda').bfloat16(); r=torch.randn(n,device='cuda').bfloat16(); y=torch.empty_like(x)
t=timeit(lambda: y.copy_(x)); print("copy   %.3f ms %.2f TB/s"%(t, 4*n/t/1e9))
t=timeit(lambda: torch.add(x,r,out=y)); print("add    %.3f ms %.2f TB/s"%(t, 6*n/t/1e9))
t=timeit(lambda: x.sum()); print("sum    %.3f ms %.2f TB/s"%(t, 2*n/t/1e9))
t=timeit(lambda: y.zero_()); print("zero   %.3f ms %.2f TB/s"%(t, 2*n/t/1e9))
