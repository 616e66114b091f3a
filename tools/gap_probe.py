#!/usr/bin/env python3
"""Inter-kernel gap probe (run under rocprofv3 --kernel-trace; tools/gpu_gap.sh). Each
iteration first queues ~0.5 ms of work on s1 so the host has queued everything after it
before the GPU gets there (the gaps are then the GPU's, not the host's), then tiny
torch kernels on s1: (a) back to back, (b) a timing event recorded between them, (c) a
non-timing event between them, (d) a wait on an event s2 completed long ago, (e) a wait
on an event s2 records after ~50 us of work. tools/gap_probe_parse.py prints the median
gap before each position."""
import torch

s1 = torch.cuda.Stream()
s2 = torch.cuda.Stream()
x = torch.zeros(1024, device="cuda")
big = torch.zeros(1 << 24, device="cuda")
mid = torch.zeros(1 << 22, device="cuda")
ev_t = torch.cuda.Event(enable_timing=True)
ev_n = torch.cuda.Event()
ev_old = torch.cuda.Event()
with torch.cuda.stream(s2):
    x.add_(0)
    ev_old.record(s2)
torch.cuda.synchronize()
for it in range(60):
    with torch.cuda.stream(s1):
        for _ in range(40):
            big.mul_(1.0)  # holds the queue while the host runs ahead
        x.add_(1)          # a1
        x.add_(1)          # a2
        ev_t.record(s1)
        x.add_(1)          # b
        ev_n.record(s1)
        x.add_(1)          # c
        s1.wait_event(ev_old)
        x.add_(1)          # d
    with torch.cuda.stream(s2):
        for _ in range(8):
            mid.mul_(1.0)
        ev_n.record(s2)
    with torch.cuda.stream(s1):
        s1.wait_event(ev_n)
        x.add_(1)          # e
    torch.cuda.synchronize()
print("done")
