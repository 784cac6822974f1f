#!/usr/bin/env python
"""Do independent branches of a captured hipGraph run concurrently on this ROCm?  (The RCCL
gradient all-reduces of a captured training step sit on a forked stream; they overlap backward only
if graph branches execute concurrently.)  Two spin kernels: eager on two streams, then captured
on a fork/join pair of streams; prints the times relative to one spin."""
import time

import torch


def spin_ms(cycles):
    torch.cuda.synchronize()
    t = time.perf_counter()
    torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3


def main():
    torch.cuda.init()
    cyc = 50_000_000
    spin_ms(cyc)
    one = min(spin_ms(cyc) for _ in range(3))
    s1 = torch.cuda.Stream()

    def two():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(s1):
            torch.cuda._sleep(cyc)
        cur.wait_stream(s1)

    torch.cuda.synchronize()
    t = time.perf_counter()
    two()
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t) * 1e3
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        two()
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t) * 1e3
    print("one spin %.1f ms | two streams eager %.1f ms (%.2fx) | captured fork/join graph %.1f ms (%.2fx)" % (
        one, eager, eager / one, graph, graph / one))


if __name__ == "__main__":
    main()
