#!/usr/bin/env python3
"""Event-record cost by HIP event flags (run under rocprofv3 --kernel-trace; tools/gpu_gap2.sh).
Like tools/gap_probe.py: ~0.5 ms of holder work on s1 so the host runs ahead, then tiny
kernels with, between them, a record of an event created with (f) hipEventDisableTiming,
(g) + hipEventDisableSystemFence, (h) + hipEventReleaseToDevice; then (i)-(k): s1 waits on
an event of each kind that s2 records after ~50 us of work (gap after the wait)."""
import ctypes as C

import torch

hip = C.CDLL("libamdhip64.so")
hip.hipEventCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
hip.hipStreamWaitEvent.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
DT, DSF, RTD = 0x2, 0x20000000, 0x40000000


def mk(flags):
    e = C.c_void_p()
    assert hip.hipEventCreateWithFlags(C.byref(e), flags) == 0
    return e


s1 = torch.cuda.Stream()
s2 = torch.cuda.Stream()
x = torch.zeros(1024, device="cuda")
big = torch.zeros(1 << 24, device="cuda")
mid = torch.zeros(1 << 22, device="cuda")
evs = [mk(DT), mk(DT | DSF), mk(DT | RTD)]
wevs = [mk(DT), mk(DT | DSF), mk(DT | RTD)]
torch.cuda.synchronize()
h1, h2 = s1.cuda_stream, s2.cuda_stream
for it in range(60):
    with torch.cuda.stream(s1):
        for _ in range(40):
            big.mul_(1.0)
        x.add_(1)          # a1
        x.add_(1)          # a2
        for e in evs:
            assert hip.hipEventRecord(e, h1) == 0
            x.add_(1)      # f, g, h
    for e in wevs:
        with torch.cuda.stream(s2):
            for _ in range(8):
                mid.mul_(1.0)
            assert hip.hipEventRecord(e, h2) == 0
        assert hip.hipStreamWaitEvent(h1, e, 0) == 0
        with torch.cuda.stream(s1):
            x.add_(1)      # i, j, k
    torch.cuda.synchronize()
print("done")
