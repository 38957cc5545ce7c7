#!/usr/bin/env python3
"""A/B of cross-stream issue orders for the headline (configs[3] shard: 12,500 x 20 MHz TM1 MCS-28, 4 workspaces on
4 streams).  Each step is split into its front end (OFDM, channel estimation, fused demap + rate de-matching) and its
back end (turbo decoder + TB CRC) with mi_dl_batch_run_stages, and HIP events between streams impose an order:
  base       one run per step, streams round-robin (bench.py's form)
  split      front + back on the step's stream, no cross-stream order (must equal base)
  ser_back   the back end of step i waits for the back end of step i - 1 (one decoder launch at a time)
  ser_front  the front end of step i waits for the front end of step i - 1
  ser_both   both
  stagger    the first S steps start staggered (front end of step i after that of step i - 1), then free-running
  stagger_b  the first S steps' back ends staggered the same way, then free-running
  two        front ends and back ends on separate streams per workspace (2 S streams): the back end of step i waits for
             its front end, the front end of step i + S for the back end of step i (the workspace is reused)
  prio_f     the same with the front-end streams at high priority
  prio_b     the same with the back-end streams at high priority
Usage: python tools/sched_ab.py [steps] [reps] [schedules...]  -> one line per (schedule, rep): ms/step, Gbps, CRC-OK
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from srsue_amd import abi  # noqa: E402

FRONT = (1 << 0) | (1 << 1) | (1 << 2) | (1 << 3)
BACK = (1 << 4) | (1 << 5)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    scheds = sys.argv[3:] or ["base", "split", "ser_back", "ser_front", "ser_both"]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    B, S = 12500, 4
    cfgs = bench.config_cfgs(4, B, 0)
    pool_iq, pool_tb = bench.make_pool(cfgs[:256], 30.0, 16, 0, None)
    batches = [abi.Batch(cfgs, max_its=4, profile=False, tdec_i16=True, compact_ce=True) for _ in range(S)]
    d_iq = torch.empty(2 * batches[0].iq_samples, dtype=torch.float32, device=dev)
    sfl = len(pool_iq[0])
    d_pool = torch.from_numpy(np.stack(pool_iq)).to(dev)
    d_iq.view(B, sfl).copy_(d_pool[torch.arange(B, device=dev) % len(pool_iq)])
    del d_pool
    streams = bench.bench_streams(dev, S)
    sp = [s.cuda_stream for s in streams]
    bits = sum(c.tbs for c in cfgs)

    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    two = {"two": ([torch.cuda.Stream(dev) for _ in range(S)], [torch.cuda.Stream(dev) for _ in range(S)]),
           "prio_f": ([torch.cuda.Stream(dev, priority=hi) for _ in range(S)], [torch.cuda.Stream(dev) for _ in range(S)]),
           "prio_b": ([torch.cuda.Stream(dev) for _ in range(S)], [torch.cuda.Stream(dev, priority=hi) for _ in range(S)])}

    def run(sched, n):
        fe = [None] * n   # front-end done events
        be = [None] * n   # back-end done events
        if sched in two:
            fs, bs = two[sched]
            for i in range(n):
                k = i % S
                b = batches[k]
                if i >= S:
                    fs[k].wait_event(be[i - S])
                b.run_stages(FRONT, d_iq.data_ptr(), fs[k].cuda_stream)
                fe[i] = torch.cuda.Event()
                fe[i].record(fs[k])
                bs[k].wait_event(fe[i])
                b.run_stages(BACK, d_iq.data_ptr(), bs[k].cuda_stream)
                be[i] = torch.cuda.Event()
                be[i].record(bs[k])
            return
        for i in range(n):
            k = i % S
            b, st = batches[k], streams[k]
            if sched == "base":
                b.run(d_iq.data_ptr(), sp[k])
                continue
            if (sched in ("ser_front", "ser_both") or (sched == "stagger" and i < S)) and i:
                st.wait_event(fe[i - 1])
            b.run_stages(FRONT, d_iq.data_ptr(), sp[k])
            fe[i] = torch.cuda.Event()
            fe[i].record(st)
            if (sched in ("ser_back", "ser_both") or (sched == "stagger_b" and i < S)) and i:
                st.wait_event(be[i - 1])
            b.run_stages(BACK, d_iq.data_ptr(), sp[k])
            be[i] = torch.cuda.Event()
            be[i].record(st)

    # each schedule's warmup runs alone: the schedules use different streams for the same workspaces, and two of them
    # in flight at once would run two steps of one workspace concurrently (an earlier version of this script did, and
    # the continuation lists of the concurrent steps overran their buffers)
    for sched in scheds:
        run(sched, 2 * S)
        torch.cuda.synchronize()
    for r in range(reps):
        for sched in scheds:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(sched, steps)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            ok = int(sum(int(b.download(abi.BUF_TB_CRC, np.uint32)[:B].sum()) for b in batches)) / S
            print(f"{sched:10s} rep {r}: {el / steps * 1e3:.3f} ms/step  {bits * steps / el / 1e9:.1f} Gbps  "
                  f"crc_ok {ok:.0f}/{B}", flush=True)
    for b in batches:
        b.close()


if __name__ == "__main__":
    main()
