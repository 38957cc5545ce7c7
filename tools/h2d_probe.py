#!/usr/bin/env python3
"""Host-to-device copy rates on the GPU box (PCIe-inclusive rate):
   python3 tools/h2d_probe.py [GB]
one page-locked host buffer (the size of the bench's sc16 / fc32 step), copied to HBM as one hipMemcpyAsync, and as
N chunks spread over S copy streams, each timed over a few repetitions; prints one JSON line."""
import json
import sys
import time

import torch


def rate(host, dev, chunks, streams, reps=4):
    n = host.numel()
    ss = [torch.cuda.Stream() for _ in range(streams)]
    step = (n + chunks - 1) // chunks
    torch.cuda.synchronize()
    best = 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        for c in range(chunks):
            a, b = c * step, min(n, (c + 1) * step)
            with torch.cuda.stream(ss[c % streams]):
                dev[a:b].copy_(host[a:b], non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, n / (time.perf_counter() - t0) / 1e9)
    return round(best, 2)


def main():
    out = {}
    for gb in [float(x) for x in sys.argv[1:]] or [1.536, 3.072]:
        n = int(gb * 1e9)
        host = torch.empty(n, dtype=torch.uint8).pin_memory()
        host.fill_(1)
        dev = torch.empty(n, dtype=torch.uint8, device="cuda")
        out[f"{gb}GB"] = {f"{c}x{s}": rate(host, dev, c, s) for c, s in ((1, 1), (4, 1), (4, 2), (8, 4), (16, 4))}
        del host, dev
    print(json.dumps({"h2d_GBps_best_of_4": out}), flush=True)


if __name__ == "__main__":
    main()
