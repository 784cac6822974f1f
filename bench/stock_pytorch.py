#!/usr/bin/env python
"""Comparator: stock PyTorch-ROCm ResNet-50 v1.5 training (BASELINE.md "comparator").

Plain ``torch.nn`` ResNet-50 v1.5, channels_last, bf16 autocast with fp32
weights, ``torch.optim.SGD(momentum=0.9, foreach)``, DDP over RCCL when
launched with torchrun — i.e. what a PyTorch user gets from MIOpen/hipBLASLt
without this framework.  Same synthetic data / batch / timing protocol as
``bench.py``; prints one JSON line.
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    def __init__(self, cin, width, stride):
        super().__init__()
        cout = width * 4
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        s = x if self.down is None else self.down(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        return F.relu(self.bn3(self.conv3(y)) + s)


class ResNet50(nn.Module):
    def __init__(self, blocks=(3, 4, 6, 3), num_classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        layers, cin = [], 64
        for s, n in enumerate(blocks):
            w = 64 * 2 ** s
            for u in range(n):
                layers.append(Bottleneck(cin, w, 2 if (u == 0 and s > 0) else 1))
                cin = w * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        x = self.layers(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=256)
    args = p.parse_args()
    distributed = int(os.environ.get("WORLD_SIZE", "1")) > 1
    if distributed:
        dist.init_process_group("nccl")
        rank, world = dist.get_rank(), dist.get_world_size()
        torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
    else:
        rank, world = 0, 1
    dev = torch.device("cuda")
    model = ResNet50().to(dev).to(memory_format=torch.channels_last)
    if distributed:
        model = nn.parallel.DistributedDataParallel(model, device_ids=[dev.index], bucket_cap_mb=32,
                                                    gradient_as_bucket_view=True)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5, foreach=True)
    x = torch.randn(args.batch, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], device=dev)
    if distributed:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el)
    if rank == 0:
        print(json.dumps({"metric": "stock-pytorch resnet50 images/sec", "value": world * args.batch * args.steps / el,
                          "n_gpus": world, "ms_per_step": 1000 * el / args.steps, "per_gpu_batch": args.batch,
                          "loss": float(loss)}), flush=True)


if __name__ == "__main__":
    main()
