#!/usr/bin/env python3
"""A/B of CU-masked streams for the headline (configs[3] shard: 12,500 x 20 MHz TM1 MCS-28, 4 workspaces).  The front
end (OFDM, channel estimation, fused demap + rate de-matching) and the back end (turbo decoder + TB CRC) of each step run
on separate streams (sched_ab.py's "two" schedule: the back end of step i waits for its front end, the front end of step
i + S for the back end of step i), and the streams are created with hipExtStreamCreateWithCUMask, so that rate
de-matching and the decoder can be kept on disjoint CUs (or the front end confined to a share of them):
  base           one stream per workspace (plain non-blocking HIP streams), whole steps
  tbase          the same on bench.py's streams (torch's current stream + S - 1 torch streams)
  two            both stream sets on all CUs (equals sched_ab.py "two")
  split<F>       the product's mi_dl_batch_run_split on mi_stream_create_cu_share(0, F) / (F, 8 - F) streams
  fF_bB          front-end streams on CU set F, back-end streams on B; a set is "all", "lo<n>" (the CUs whose index mod
                 8 is < n), "hi<n>" (index mod 8 >= 8 - n), "blk<n>" (the first n / 8 of the CU indices)
Usage: python tools/cumask_ab.py [steps] [reps] [variants...]  -> one line per (variant, rep): ms/step, Gbps, CRC-OK
"""
import ctypes as C
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


def hip_lib():
    """The HIP runtime this process already loaded (through torch and libsrsue_amd), by its path in /proc/self/maps."""
    with open("/proc/self/maps") as f:
        for line in f:
            p = line.split()[-1]
            if "libamdhip64.so" in p:
                return C.CDLL(p)
    raise RuntimeError("libamdhip64 not loaded")


def cu_mask(spec, n_cu):
    bits = []
    for i in range(n_cu):
        if spec == "all":
            on = True
        elif spec.startswith("lo"):
            on = i % 8 < int(spec[2:])
        elif spec.startswith("hi"):
            on = i % 8 >= 8 - int(spec[2:])
        elif spec.startswith("blk"):
            on = i < n_cu * int(spec[3:]) // 8
        else:
            raise ValueError(spec)
        bits.append(on)
    words = [0] * ((n_cu + 31) // 32)
    for i, on in enumerate(bits):
        if on:
            words[i // 32] |= 1 << (i % 32)
    return words


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    variants = sys.argv[3:] or ["two", "flo3_ball", "flo3_bhi5", "flo2_ball"]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    hip = hip_lib()
    B, S = 12500, 4
    cfgs = bench.config_cfgs(4, B, 0)
    pool_iq, _ = bench.make_pool(cfgs[:256], 30.0, 16, 0, None)
    # MI_AB_PROFILE=1: the batches record their per-stage HIP events as bench.py's do
    prof = os.environ.get("MI_AB_PROFILE", "0") == "1"
    batches = [abi.Batch(cfgs, max_its=4, profile=prof, tdec_i16=True, compact_ce=True) for _ in range(S)]
    d_iq = torch.empty(2 * batches[0].iq_samples, dtype=torch.float32, device=dev)
    sfl = len(pool_iq[0])
    d_pool = torch.from_numpy(np.stack(pool_iq)).to(dev)
    d_iq.view(B, sfl).copy_(d_pool[torch.arange(B, device=dev) % len(pool_iq)])
    del d_pool
    torch.cuda.synchronize()
    bits = sum(c.tbs for c in cfgs)

    def stream(spec):
        h = C.c_void_p()
        if spec == "all":
            rc = hip.hipStreamCreateWithFlags(C.byref(h), C.c_uint(1))   # hipStreamNonBlocking
        else:
            w = cu_mask(spec, n_cu)
            arr = (C.c_uint32 * len(w))(*w)
            rc = hip.hipExtStreamCreateWithCUMask(C.byref(h), C.c_uint32(len(w)), arr)
        if rc:
            raise RuntimeError(f"stream create ({spec}): hip error {rc}")
        return h.value

    ev_n = 2 * (steps + 2 * S)
    evs = []
    for _ in range(ev_n):
        e = C.c_void_p()
        if hip.hipEventCreateWithFlags(C.byref(e), C.c_uint(2)):   # hipEventDisableTiming
            raise RuntimeError("event create")
        evs.append(e.value)

    sets = {}
    for v in variants:
        if v == "base":
            sets[v] = ([stream("all") for _ in range(S)], None)
            continue
        if v == "tbase":   # bench.py's streams: torch's current stream + S - 1 torch streams
            sets[v] = ([st.cuda_stream for st in bench.bench_streams(dev, S)], None)
            continue
        if v.startswith("split"):   # the product's split run (mi_dl_batch_run_split) on mi_stream_create_cu_share streams
            F = int(v[5:])
            sets[v] = ([abi.stream_cu_share(0, F) for _ in range(S)], [abi.stream_cu_share(F, 8 - F) for _ in range(S)],
                       "split")
            continue
        if v == "two":
            fspec, bspec = "all", "all"
        else:
            f, b = v.split("_")
            fspec, bspec = f[1:], b[1:]
        sets[v] = ([stream(fspec) for _ in range(S)], [stream(bspec) for _ in range(S)])

    def run(v, n):
        fs, bs = sets[v][:2]
        if len(sets[v]) == 3:
            for i in range(n):
                batches[i % S].run_split(d_iq.data_ptr(), fs[i % S], bs[i % S])
            return
        if bs is None:
            for i in range(n):
                batches[i % S].run(d_iq.data_ptr(), fs[i % S])
            return
        fe = evs[:n]
        be = evs[n:2 * n]
        for i in range(n):
            k = i % S
            b = batches[k]
            if i >= S:
                hip.hipStreamWaitEvent(C.c_void_p(fs[k]), C.c_void_p(be[i - S]), C.c_uint(0))
            b.run_stages(FRONT, d_iq.data_ptr(), fs[k])
            hip.hipEventRecord(C.c_void_p(fe[i]), C.c_void_p(fs[k]))
            hip.hipStreamWaitEvent(C.c_void_p(bs[k]), C.c_void_p(fe[i]), C.c_uint(0))
            b.run_stages(BACK, d_iq.data_ptr(), bs[k])
            hip.hipEventRecord(C.c_void_p(be[i]), C.c_void_p(bs[k]))

    def sync():
        if hip.hipDeviceSynchronize():
            raise RuntimeError("hipDeviceSynchronize")

    # each variant's warmup runs alone (the variants share the workspaces)
    for v in variants:
        run(v, 2 * S)
        sync()
    print(f"cus {n_cu}; masks: " + ", ".join(f"{v}" for v in variants), flush=True)
    for r in range(reps):
        for v in variants:
            for b in batches:
                if prof:
                    b.profile_reset()
            sync()
            t0 = time.perf_counter()
            run(v, steps)
            sync()
            el = time.perf_counter() - t0
            ok = int(sum(int(b.download(abi.BUF_TB_CRC, np.uint32)[:B].sum()) for b in batches)) / S
            print(f"{v:12s} rep {r}: {el / steps * 1e3:.3f} ms/step  {bits * steps / el / 1e9:.1f} Gbps  "
                  f"crc_ok {ok:.0f}/{B}", flush=True)
    for b in batches:
        b.close()


if __name__ == "__main__":
    main()
