"""bench.py -- PDSCH decoded Mbps + turbo code blocks/s for 20 MHz MCS-28 on 1..8 MI355X.

A step = one pass of the whole DL PDSCH receive chain (OFDM RX -> CRS chest -> equalise -> demap ->
descramble -> rate de-match + HARQ combine -> max-log-MAP turbo -> TB CRC -> payload) over one
batch of synthetic 20 MHz TM1 MCS-28 subframes per GPU (BASELINE configs[1]'s subframe; the batch
is configs[3]'s per-GPU shard, 100k / 8 = 12,500 subframes).  IQ is resident in HBM before timing.

Multi-GPU (torchrun, one process per GPU): every rank decodes its own shard; there is no collective
on the data path (subframes are independent); the only cross-rank traffic is the barrier and the
max-over-ranks of the elapsed time.  value = total decoded bits of CRC-OK TBs on all ranks / max
elapsed -> scaling "weak".

Prints ONE JSON line on rank 0 (driver contract), including the dominant kernel's roofline (HIP
events on the stream the kernels run on, averaged over the timed steps) and the CPU baseline
(the oracle, i.e. this repo's CPU restatement of the chain, timed on a bounded sample on rank 0).
"""
import argparse
import concurrent.futures as cf
import json
import os
import sys
import time

import numpy as np


def hw_queues_arg(argv, env=None):
    """--hw-queues N / --hw-queues=N (0 keeps the environment's value), checked to 0..32.  Default 8, or 16 when this
    process brings up the nccl (RCCL) process group (WORLD_SIZE > 1 without --share-gpu, or --pg): RCCL's own
    streams take hardware queues too, and at 8 the bench's streams then share queues (profiles/r5/rccl_queues: one
    rank under RCCL, 8 queues -1.7 % headline and -2 % waterfall, 16 queues level with the plain run)."""
    env = os.environ if env is None else env
    rccl = "--pg" in argv or (int(env.get("WORLD_SIZE", "1") or 1) > 1 and "--share-gpu" not in argv)
    # the low-occupancy configs (1: configs[0], 3: configs[2], 5: configs[4]) keep 8-16 batches in flight (main(): their
    # default streams), each on its own queue
    cfg = next((argv[i + 1] for i, a in enumerate(argv[:-1]) if a == "--config"), None)
    cfg = cfg or next((a.split("=", 1)[1] for a in argv if a.startswith("--config=")), "4")
    v = "16" if rccl or cfg in ("1", "3", "5") else "8"
    for i, a in enumerate(argv):
        if a == "--hw-queues" and i + 1 < len(argv):
            v = argv[i + 1]
        elif a.startswith("--hw-queues="):
            v = a.split("=", 1)[1]
    if not v.isdigit() or not 0 <= int(v) <= 32:
        raise SystemExit(f"bench.py: --hw-queues must be an integer in 0..32, got {v!r}")
    return v


# HIP hardware queues per process (--hw-queues, default 8, 16 under RCCL; 0 keeps the environment's value): the
# bench keeps 4 batches in flight on as many HIP streams, and with HIP's default of 4 queues per process the streams'
# kernels share them with the runtime's own copies; 8 queues measured +0.7 % at the headline, 16 no better
# (profiles/r4/ab_queues) -- except beside RCCL's streams (hw_queues_arg).  Set only when bench.py runs as the program (not when tests import it), before torch and
# the HIP runtime start (the runtime reads it once); the ranks bench.py spawns inherit it.
if __name__ == "__main__":
    HW_QUEUES = hw_queues_arg(sys.argv[1:])
    if HW_QUEUES != "0":
        os.environ["GPU_MAX_HW_QUEUES"] = HW_QUEUES

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from srsue_amd import abi  # noqa: E402

METRIC = "PDSCH decoded Mbps + turbo codeblocks/s, 20 MHz MCS-28, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
TBS_MCS28_100PRB = 75376
SF_CYCLE = (1, 2, 3, 4, 6, 7, 8, 9)   # headline runs avoid PSS/SSS/PBCH subframes
# 36.213 Table 7.1.7.2.1-1 columns (I_TBS 0..26) used by the mixed-bandwidth config
TBS_6 = (152, 208, 256, 328, 408, 504, 600, 712, 808, 936, 1032, 1192, 1352, 1544, 1736, 1800, 1928, 2152, 2344,
         2600, 2792, 2984, 3240, 3496, 3624, 3752, 4392)
TBS_25 = (680, 904, 1096, 1416, 1800, 2216, 2600, 3112, 3496, 4008, 4392, 4968, 5736, 6456, 7224, 7736, 7992, 9144,
          9912, 10680, 11448, 12576, 13536, 14112, 15264, 15840, 18336)
TBS_50 = (1384, 1800, 2216, 2856, 3624, 4392, 5160, 6200, 6968, 7992, 8760, 9912, 11448, 12960, 14112, 15264, 16416,
          18336, 19848, 21384, 22920, 25456, 27376, 28336, 30576, 31704, 36696)
TBS_100 = (2792, 3624, 4584, 5736, 7224, 8760, 10296, 12216, 14112, 15840, 17568, 19848, 22920, 25456, 28336, 30576,
           32856, 36696, 39232, 43816, 46888, 51024, 55056, 57336, 61664, 63776, 75376)


def tb_payload(seed, nbytes):
    """TB bytes from splitmix64(0x5EED0000 + index)."""
    out = np.zeros(((nbytes + 7) // 8) * 8, np.uint8)
    M = 0xFFFFFFFFFFFFFFFF
    s = (0x5EED0000 + seed) & M
    for i in range(0, len(out), 8):
        s = (s + 0x9E3779B97F4A7C15) & M
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        out[i:i + 8] = np.frombuffer(z.to_bytes(8, "little"), np.uint8)
    return out[:nbytes]


def kernel_src_hash():
    """Content hash of the sources that define the measured PDSCH path (its kernels, their layouts and
    the planner): a committed PMC traffic figure is only reported when it was measured on exactly these
    (profiles/traffic.json, written by tools/profile.sh).  Other rows (control, sync, per-TTI glue)
    do not enter the default bench."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(ROOT, "srsue_amd", "csrc")
    for f in PATH_SOURCES:
        h.update(f.encode())
        h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


PATH_SOURCES = ("cbscatter.hip", "chest.hip", "demap.hip", "demap_body.h", "dl_common.h", "engine.cpp", "engine.h",
                "kernels.h", "kernels_consts.h", "ofdm.hip", "p2.h", "plan.cpp", "plan.h", "rm.hip", "rm_body.h",
                "tables.cpp", "tables.h", "tb.hip", "tb_body.h", "tdec.hip", "tdec_body.h", "tdec_p2_body.h")


def pmc_traffic(sf_per_gpu, tdec, kernel):
    """The turbo kernel's PMC figures of the profiled build (tools/profile.sh -> profiles/traffic.json): HBM
    traffic per launch and VALU busy; only when the kernel sources, the shard size, the arithmetic and the
    kernel that ran all match the profiled run."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        t = json.load(open(p))
    except (OSError, ValueError):
        return None, None, None
    if (t.get("src_hash") != kernel_src_hash() or t.get("sf_per_gpu") != sf_per_gpu or t.get("tdec", "gen") != tdec
            or t.get("tdec_kernel", kernel) != kernel):
        return None, None, None
    return t["tdec_traffic_bytes_per_launch"], t.get("tdec_valu_busy_pct"), "profiles/traffic.json: " + t["source"]


def make_cfg(i, new_tb=1):
    return abi.sf_cfg(cell_id=1, nof_prb=100, nof_ports=1, sf_idx=SF_CYCLE[i % len(SF_CYCLE)], cfi=1, tm=1,
                      rnti=0x46, rv=0, tbs=TBS_MCS28_100PRB, Qm=6, new_tb=new_tb)


def shard_range(total, rank, world):
    """Contiguous subframe range of one rank (no exchange step, contiguous shards)."""
    per, rem = divmod(total, world)
    start = rank * per + min(rank, rem)
    return start, per + (1 if rank < rem else 0)


_LINE_FD = None   # the process's original stdout once native libraries' prints are sent to stderr (keep_stdout_clean)


def keep_stdout_clean():
    """RCCL prints a version banner on stdout when its communicator comes up (seen on the GPU box: 'RCCL version :
    ...'); the driver reads rank 0's stdout as ONE JSON line.  Before the nccl process group starts, file descriptor
    1 is pointed at stderr for the rest of the process, and emit() writes the line to the original stdout."""
    global _LINE_FD
    if _LINE_FD is None:
        sys.stdout.flush()
        _LINE_FD = os.dup(1)
        os.dup2(2, 1)


def emit(out):
    """Rank 0's one JSON line, on the process's original stdout."""
    line = (json.dumps(out) + "\n").encode()
    if _LINE_FD is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        sys.stdout.flush()
        os.write(_LINE_FD, line)


_STREAMS = []


def bench_streams(dev, S):
    """The S streams a block of the line runs its workspaces on: the current stream and S - 1 more, created once
    and shared by every block (headline, waterfall, h2d, planning).  HIP binds each stream to one of the
    process's GPU_MAX_HW_QUEUES hardware queues when it is created; fresh streams per block, created after RCCL's own
    streams under the nccl process group, landed on shared queues and serialised the waterfall block (16 %)."""
    while len(_STREAMS) < S - 1:
        _STREAMS.append(torch.cuda.Stream(dev))
    return [torch.cuda.current_stream(dev)] + _STREAMS[:S - 1]


_SPLIT = {}


AUTO_SPLIT = 2          # the front end's CU eighths of an auto-tuned split (profiles/r6/cumask: 1-3 measured alike)
SPLIT_MARGIN = 0.015    # auto: split runs are kept only when faster than whole runs by more than this


def split_share(args, S):
    """Eighths of the CUs the front end of a split run gets; 0 = whole runs on one stream per workspace; -1 = decide on
    the box (tune_split): --split F, or by default -1 for the headline shard on several streams (split runs are level
    with whole runs on the median box, -1 %, but 4-5 % ahead where whole runs co-schedule rate de-matching beside the
    decoder; profiles/r6/cumask) and 0 otherwise.  One stream: 0 (a lone workspace's front end waits for its own back
    end, nothing overlaps)."""
    if S < 2:
        return 0
    if args.split >= 0:
        return args.split
    return -1 if args.config == 4 else 0


def tune_split(whole, split, S, dev, reps=2):
    """The stream layout for this box, chosen after the warmup and before the timed region (untimed): `reps` rounds of
    3 S steps of whole runs and of split runs (each bracketed by device synchronisation, so the two layouts never
    overlap on a workspace), best ms per step of each; split runs are kept when faster by more than SPLIT_MARGIN.
    Returns (front-end eighths or 0, the record reported in the line)."""
    n = 3 * S

    def per_step(fn):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(n):
            fn(i)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / n * 1e3

    tw, ts = [], []
    for _ in range(reps):
        tw.append(per_step(whole))
        ts.append(per_step(split))
    F = AUTO_SPLIT if min(ts) < min(tw) * (1 - SPLIT_MARGIN) else 0
    return F, {"whole_ms_per_step": [round(x, 3) for x in tw], "split_ms_per_step": [round(x, 3) for x in ts],
               "steps_each": n, "split_front_cu_eighths": AUTO_SPLIT, "chosen": "split" if F else "whole",
               "rule": f"split runs when faster than whole runs by more than {SPLIT_MARGIN:.1%} (untimed, after the "
                       "warmup)"}


def split_streams(S, F):
    """S front-end streams on the CUs i mod 8 < F and S back-end streams on the others (mi_stream_create_cu_share),
    created once per share and kept for the process (like bench_streams)."""
    have = _SPLIT.setdefault(F, ([], []))
    while len(have[0]) < S:
        have[0].append(abi.stream_cu_share(0, F))
        have[1].append(abi.stream_cu_share(F, 8 - F))
    return have[0][:S], have[1][:S]


def release_split_streams(F):
    """Destroy the split streams of share F (after the device is idle): each CU-masked stream holds a hardware queue of
    its own."""
    have = _SPLIT.pop(F, None)
    if have:
        torch.cuda.synchronize()
        for h in have[0] + have[1]:
            abi.stream_destroy(h)


def dist_on():
    """A process group is up: N > 1 ranks, or one rank with --pg (the RCCL path rehearsed on a one-GPU box)."""
    return dist.is_available() and dist.is_initialized()


def reduce_over_ranks(elapsed, sums, world, device="cpu"):
    """The only cross-rank traffic, after the timed region: every rank's elapsed time (all-gathered: the max is
    the job's time, the list goes into the JSON) and the sums of this rank's end-of-run counters (`sums`: CRC-OK
    bits, code blocks, CRC-OK TBs, iteration sums, payload mismatches ...).  Returns (max elapsed, [sums],
    [elapsed per rank])."""
    sums = [float(x) for x in sums]
    if not dist_on():
        return elapsed, sums, [elapsed]
    if dist.get_backend() == "gloo":   # CPU rehearsal, or --share-gpu
        device = "cpu"
    t = torch.zeros(world, dtype=torch.float64, device=device)
    t[dist.get_rank()] = elapsed
    dist.all_reduce(t, op=dist.ReduceOp.SUM)          # = all-gather of one scalar per rank
    s = torch.tensor(sums, dtype=torch.float64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    per = [float(x) for x in t.cpu()]
    return max(per), [float(x) for x in s.cpu()], per


def rank_devices(world, dev):
    """Every rank's device identity (name, gfx arch, PCI domain:bus:device, UUID), gathered over the run's process
    group after the timed region: a multi-GPU line shows that its N ranks ran on N distinct cards (the driver's
    SCALE runs), a --share-gpu rehearsal that they shared one.  dev None = the CPU rehearsal (no GPU)."""
    if dev is None:
        me = {"device": "cpu (test-only host emulation)"}
    else:
        p = torch.cuda.get_device_properties(dev)
        me = {"device": p.name, "arch": getattr(p, "gcnArchName", ""), "cuda_index": dev.index,
              "pci_bus_id": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}", "uuid": str(p.uuid)}
    me = {"rank": dist.get_rank() if dist_on() else 0, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), **me}
    if not dist_on():
        return [me]
    allr = [None] * world
    dist.all_gather_object(allr, me)
    return allr


def make_pool(cfgs, snr_db, threads, first=0, h=None):
    """Distinct synthetic subframes from the product's transmitter (mi_tx_subframe), CPU threads.
    Subframe g (global index) carries TB splitmix64(0x5EED0000 + g) and noise seed 0xA5A5 + g."""
    def one(i):
        g = first + i
        c = cfgs[i]
        tb = tb_payload(g, c.tbs // 8)
        return abi.tx_subframe(c, tb, h=h, snr_db=snr_db, seed=0xA5A5 + g), tb
    with cf.ThreadPoolExecutor(max_workers=threads) as ex:
        res = list(ex.map(one, range(len(cfgs))))
    return [r[0] for r in res], [r[1] for r in res]


HOST_CPU_SHARE = 16   # CPUs a one-GPU job is granted on the GPU pool (nproc shows the whole machine's)


def host_threads():
    """CPU threads the baseline may use: this process's affinity, capped at the one-GPU box share: the box runs
    one GPU's job on a 16-CPU share of a larger machine (OMP_NUM_THREADS / MAX_JOBS are set to 16 there), so
    `nproc` overstates what this job may use; SURVEY 8d (ii)'s "all cores" is that share."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(HOST_CPU_SHARE, n))


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo), for the baseline line (core count and model)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def run_for(seconds, nthreads, work):
    """Calls work(thread_id, i) in nthreads threads until the deadline (ctypes releases the GIL, so the
    oracle's C code runs in parallel); returns (sum of work() results, elapsed s)."""
    deadline = time.perf_counter() + seconds

    def loop(t):
        acc, i = [0, 0, 0], 0
        while time.perf_counter() < deadline:
            r = work(t, i)
            acc = [a + b for a, b in zip(acc, r)]
            i += nthreads
        return acc
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(max_workers=nthreads) as ex:
        res = list(ex.map(loop, range(nthreads)))
    return [sum(r[j] for r in res) for j in range(3)], time.perf_counter() - t0


def cpu_baseline(seconds, pool_cfgs, pool_iq, pool_tb, what, i16):
    """The oracle chain (this repo's C restatement) on a bounded sample of the same workload, on one
    thread and on all host threads; the turbo decoder is the int16 one of the srsLTE SSE design in int16 mode -- AVX2
    with two code blocks per __m256i (oracle/o_avx2.c) where the host has AVX2, else SSE4.1 (oracle/o_simd.c) -- and
    the float srsLTE-gen restatement otherwise."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    import oracle_lib as O
    L = O.lib()
    avx2 = i16 and L.or_avx2_available() == 1
    L.or_set_tdec_mode((O.TDEC_AVX2 if avx2 else O.TDEC_SIMD) if i16 else O.TDEC_GEN)

    def one(t, i):
        i %= len(pool_iq)
        c = pool_cfgs[i]
        s = O.cbsegm(c.tbs)
        ncb = L.or_ncb(s.Kp)
        sb = np.zeros(s.C * ncb, np.float32)
        pay = np.zeros(c.tbs // 8, np.uint8)
        noi = C.c_uint32()
        cell = O.make_cell(c.cell_id, c.nof_prb, c.nof_ports)
        rc = L.or_decode_subframe(C.byref(cell), c.sf_idx, c.cfi, np.array(list(c.prb_mask), np.uint8), c.tbs, c.Qm,
                                  c.rv, c.rnti, c.tm, 2, pool_iq[i], sb, ncb, 1, 4, pay, C.byref(noi))
        good = rc == 0 and np.array_equal(pay, pool_tb[i])
        return (c.tbs if good else 0, s.C, 1)
    T = host_threads()
    (b1, c1, n1), dt1 = run_for(seconds / 3, 1, one)
    (bT, cT, nT), dtT = run_for(2 * seconds / 3, T, one)
    L.or_set_tdec_mode(O.TDEC_GEN)
    dec = ("AVX2 int16 turbo, code blocks in pairs (oracle/o_avx2.c)" if avx2 else
           "SSE4.1 int16 turbo (oracle/o_simd.c)") if i16 else "float srsLTE-gen turbo restatement"
    return {"value": round(bT / dtT / 1e6, 3), "unit": "Mbps", "cores": T, "kind": "port",
            "value_1core": round(b1 / dt1 / 1e6, 3), "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
            "cores_note": f"all of the job's {HOST_CPU_SHARE}-CPU share of the host (the pool's per-GPU grant; "
                          f"os.cpu_count() reports the whole machine)",
            "sample": f"{nT} subframes ({what}) through the oracle's full chain with the {dec}, {T} threads in "
                      f"{dtT:.1f} s; 1 thread: {n1} subframes in {dt1:.1f} s",
            "codeblocks_per_s": round(cT / dtT, 1)}


def config_cfgs(config, B, first):
    """Subframe configurations of BASELINE configs[1..4] (2/4: TM1 MCS-28; 3: TM2 64QAM MCS-28;
    5: mixed 1.4/5/10/20 MHz cells with variable allocation and MCS, seeded)."""
    if config in (2, 4):
        return [make_cfg(first + i) for i in range(B)]
    if config == 3:
        return [abi.sf_cfg(cell_id=1, nof_prb=100, nof_ports=2, sf_idx=SF_CYCLE[(first + i) % 8], cfi=1, tm=2,
                           rnti=0x46, rv=0, tbs=TBS_MCS28_100PRB, Qm=6) for i in range(B)]
    rng = np.random.default_rng(0x5EED + first)
    cols = {6: TBS_6, 25: TBS_25, 50: TBS_50, 100: TBS_100}
    cfgs = []
    for i in range(B):
        nprb = (6, 25, 50, 100)[(first + i) % 4]
        lprb = int(rng.choice([x for x in (6, 25, 50, 100) if x <= nprb]))
        start = int(rng.integers(0, nprb - lprb + 1))
        mcs = int(rng.integers(0, 29))
        prb = [start <= p < start + lprb for p in range(nprb)]
        while True:   # an eNB never schedules a code rate above ~0.93: step the MCS down until it fits
            qm, itbs = (2, mcs) if mcs <= 9 else (4, mcs - 1) if mcs <= 16 else (6, mcs - 2)
            c = abi.sf_cfg(cell_id=1 + (first + i) % 4, nof_prb=nprb, nof_ports=1, sf_idx=SF_CYCLE[(first + i) % 8],
                           cfi=1 if nprb > 10 else 2, tm=1, rnti=0x46, rv=0, tbs=cols[lprb][itbs], Qm=qm, prb=prb)
            ncb = -(-(c.tbs + 24) // 6120)
            if (c.tbs + 24 * (ncb + 1)) <= 0.93 * abi.pdsch_G(c) or mcs == 0:
                break
            mcs -= 1
        cfgs.append(c)
    return cfgs


SCHED_DESC = {"win": "latency form", "lanex": "lane per code block, crossed (2 wavefronts per group)",
              "lanexr": "lane per code block, crossed, recompute form (2 wavefronts per group, 5 per SIMD)",
              "lane": "lane per code block",
              "p2": "two code blocks per lane (packed int16), crossed (2 wavefronts per group pair, 3 per SIMD)"}


def tdec_kernel_name(sched):
    return {"win": "tdec_win_kernel (max-log-MAP turbo, one workgroup per code block)",
            "lanex": "tdec_kernel_*x (max-log-MAP turbo, one code block per lane, crossed schedule)",
            "lanexr": "tdec_kernel_i16xr (max-log-MAP turbo, one code block per lane, crossed, recompute form)",
            "p2": "tdec_kernel_p2x (max-log-MAP turbo, two code blocks per lane in packed int16, crossed)"}.get(
        sched, "tdec_kernel (max-log-MAP turbo, one code block per lane)")


def dtype_of(args):
    """f32 everywhere (front end, softbuffer); in i16 mode the turbo metrics are int16-exact integers."""
    return "f32+i16" if args.tdec == "i16" else "f32"


def bench_codeblocks(args, world, rank, dev):
    """configs[0]: turbodecoder_test -- K = 6144, 8 fixed iterations, BPSK/AWGN LLRs."""
    K, n = 6144, args.cb_per_gpu
    rng = np.random.default_rng(1 + rank)
    pool = min(args.pool, n)
    bits = rng.integers(0, 2, (pool, K)).astype(np.uint8)
    sigma2 = 1.0 / (2 * (K / (3.0 * K + 12)) * 10 ** (args.ebno / 10))
    llr = np.stack([(-2.0 * ((1.0 - 2.0 * abi.turbo_encode(b, K)) + rng.normal(0, np.sqrt(sigma2), 3 * K + 12))
                     / sigma2).astype(np.float32) for b in bits])
    # S workspaces on S streams, steps round-robin (measure()'s --streams): 65,536 code blocks give the packed
    # decoder one wavefront per SIMD, so consecutive steps overlap
    S = max(1, args.streams)
    tbs = [abi.TdecBatch(K, n, max_its=8, early_stop=False, profile=True, tdec_i16=args.tdec == "i16", sched=args.sched)
           for _ in range(S)]
    tb = tbs[0]
    d = torch.from_numpy(llr).to(dev)[torch.arange(n, device=dev) % pool].contiguous()
    streams = bench_streams(dev, S)
    sptr = [st.cuda_stream for st in streams]
    torch.cuda.synchronize(dev)
    for w in range(args.warmup * S):
        tbs[w % S].run(d.data_ptr(), sptr[w % S])
    torch.cuda.synchronize(dev)
    for t in tbs:
        t.profile_reset()
    if dist_on():
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        tbs[i % S].run(d.data_ptr(), sptr[i % S])
    torch.cuda.synchronize(dev)
    if dist_on():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per = [t.stage_ms() for t in tbs[:min(S, args.steps)]]
    nprof = sum(k for _, k in per)
    stage = {key: sum(st[key] * k for st, k in per) / nprof for key in per[0][0]}
    iso = isolated_stages(tb, lambda: tb.run(d.data_ptr(), sptr[0]), dev, S, args.steps)
    dec, its, _ = tb.results()
    for k, t in enumerate(tbs[1:min(S, args.steps)], 1):
        assert np.array_equal(t.results()[0][:pool], dec[:pool]), f"stream {k} decoded differently"
    ber = float(np.mean(dec[:pool] != bits))
    elapsed, (n_all,), _ = reduce_over_ranks(elapsed, [n], world, dev)
    devices = rank_devices(world, dev)
    if rank:
        return None
    cbps = n_all * args.steps / elapsed
    ab = tb.algo_bytes()
    tdec_ms = iso[0]["tdec"] if iso else stage["tdec"]
    ach = ab / (tdec_ms * 1e-3) / 1e9
    out = {"metric": METRIC, "value": round(cbps * K / 1e6, 2), "unit": "Mbps", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": dtype_of(args), "data": "synthetic",
           "config": {"workload": f"configs[0] turbodecoder_test: K=6144, 8 iterations, no early stop, BPSK/AWGN "
                                  f"Eb/N0 {args.ebno:g} dB, {n} code blocks per GPU per step", "K": K, "iterations": 8,
                      "codeblocks_per_gpu": n, "turbo_arithmetic": args.tdec, "streams": S,
                      "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                      "turbo_schedule": SCHED_DESC[tb.turbo_sched]},
           "turbo_codeblocks_per_s": round(cbps, 1), "ber": ber, "stage_ms_per_step": {k: round(v, 4) for k, v in stage.items()},
           "roofline": {"kernel": tdec_kernel_name(tb.turbo_sched), "bound": "hbm", "achieved": round(ach, 2),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
                        "algorithmic_bytes_per_launch": ab, **roofline_timing(stage, nprof, iso)},
           "rank_devices": devices}
    # the CPU baseline: rank 0, after the reduction (outside the timed region), at every N
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O
        L, T, i16 = O.lib(), host_threads(), args.tdec == "i16"
        avx2 = i16 and L.or_avx2_available() == 1

        def work_its(its_n, fn):
            # the int16 decoder (AVX2: two code blocks per __m256i; else SSE4.1), 4 code blocks per call and thread
            def work(t, i):
                m = 4
                out_b = np.zeros((m, K), np.uint8)
                its_ = np.zeros(m, np.uint32)
                ok_ = np.zeros(m, np.uint8)
                j = (i * m) % (pool - m + 1)
                fn(llr[j:j + m], llr.shape[1], m, K, its_n, 0, 0, out_b, its_, ok_, 1)
                return (m, 0, 0)
            return work
        if i16:
            fn = L.or_avx2_decode_batch if avx2 else L.or_simd_decode_batch
            work = work_its(8, fn)
        else:
            tds = [O.Tdec() for _ in range(T)]

            def work(t, i):
                tds[t].decode_cb(llr[i % pool], K, max_its=8, early_stop=False)
                return (1, 0, 0)
        (m1, _, _), dt1 = run_for(args.cpu_seconds / 3, 1, work)
        (mT, _, _), dtT = run_for(2 * args.cpu_seconds / 3, T, work)
        dec = ("AVX2 int16 max-log-MAP, two code blocks per __m256i (oracle/o_avx2.c)" if avx2 else
               "SSE4.1 int16 max-log-MAP (oracle/o_simd.c)") if i16 else "float max-log-MAP restatement (oracle/o_fec.c)"
        out["cpu_baseline"] = {"value": round(mT * K / dtT / 1e6, 4), "unit": "Mbps", "cores": T, "kind": "port",
                               "value_1core": round(m1 * K / dt1 / 1e6, 4),
                               "sample": f"{mT} code blocks K=6144 x 8 iterations through the {dec}, {T} threads "
                                         f"in {dtT:.1f} s; 1 thread: {m1} in {dt1:.1f} s",
                               "codeblocks_per_s": round(mT / dtT, 2), "cpu_model": cpu_model(),
                               "host_cpus_visible": os.cpu_count()}
        if i16:
            # per-core figures beside the reference README's "+100 Mbps" SSE decoder (README.md:18, iteration count
            # unstated): 8 and 4 iterations, the AVX2 and the SSE4.1 decoder, one thread, ~1/6 of the budget each
            per_core = {}
            for name, f in (("avx2", L.or_avx2_decode_batch if avx2 else None), ("sse41", L.or_simd_decode_batch)):
                for its_n in (8, 4):
                    if f is None:
                        continue
                    (mm, _, _), dd = run_for(args.cpu_seconds / 8, 1, work_its(its_n, f))
                    per_core[f"{name}_{its_n}its_Mbps"] = round(mm * K / dd / 1e6, 3)
            out["cpu_baseline"]["per_core"] = per_core
    tb.close()
    return out


def bench_ctrl(args, batch, dev):
    """PCFICH + PDCCH soft bits + DCI blind search (UE-specific + common space, formats 1A / 1) of every
    subframe of the batch, on the grid / channel estimates the timed steps left in HBM."""
    ctl = abi.Ctrl(batch, phich_ng=2)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(max(1, args.warmup)):
        ctl.run(sptr)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctl.run(sptr)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / args.steps
    B = len(batch.cfgs)
    cfi = [ctl.result(i)[0] for i in range(0, B, max(1, B // 16))]
    ctl.close()
    return {"ms_per_step": round(dt * 1e3, 3), "subframes_per_s": round(B / dt, 1),
            "cfi_ok": all(c == batch.cfgs[0].cfi for c in cfi),
            "what": "PCFICH + PDCCH soft bits + blind search (38 candidate x size decodes per subframe) for "
                    f"{B} subframes per step"}


def bench_ul(args, B, dev):
    """UL PUSCH transmitter (include/mi_ul.h): B subframes of 20 MHz full-band PUSCH,
    16QAM MCS 20 (I_TBS 19, TBS 43,816, 8 code blocks), TB payloads resident in HBM, SC-FDMA IQ written
    to HBM.  Roofline: pusch_mod_kernel (coded symbols read + IQ write per subframe)."""
    T = 43816
    cfgs = [abi.ul_cfg(cell_id=1, nof_prb=100, sf_idx=i % 10, rnti=0x46, n_prb=0, L_prb=100, tbs=T, Qm=4)
            for i in range(B)]
    b = abi.UlBatch(cfgs, profile=True)
    rng = np.random.default_rng(77)
    pay = rng.integers(0, 256, b.payload_bytes, dtype=np.uint8)
    d_pay = torch.from_numpy(pay).to(dev)
    d_iq = torch.empty(2 * b.iq_samples, dtype=torch.float32, device=dev)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(args.warmup):
        b.run(d_pay.data_ptr(), d_iq.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    b.profile_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.run(d_pay.data_ptr(), d_iq.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / args.steps
    st, n = b.stage_ms()
    mod_bytes = B * (12 * 1200 + 15 * 2048 * 8)
    out = {"workload": f"{B} x 20 MHz PUSCH, 100 PRB 16QAM MCS 20 (TBS {T}, 8 code blocks)",
           "ms_per_step": round(el * 1e3, 3), "Mbps": round(B * T / el / 1e6, 1),
           "subframes_per_s": round(B / el, 1), "stage_ms_per_step": {k: round(v, 4) for k, v in st.items()},
           "roofline": {"kernel": "pusch_mod_kernel", "bound": "hbm",
                        "achieved": round(mod_bytes / (st["mod"] * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(mod_bytes / (st["mod"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import ctypes
        import oracle_lib as O
        oc = O.ul_cfg(cell_id=1, nof_prb=100, sf_idx=1, rnti=0x46, n_prb=0, L_prb=100, tbs=T, Qm=4)
        iq = np.zeros(2 * 15 * 2048, np.float32)
        k, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < min(10.0, args.cpu_seconds):
            O.lib().or_pusch_encode(ctypes.byref(oc), pay[:T // 8], iq)
            k += 1
        dt = time.perf_counter() - t1
        out["cpu_baseline"] = {"value": round(k * T / dt / 1e6, 3), "unit": "Mbps", "cores": 1, "kind": "port",
                               "sample": f"{k} subframes through the oracle's UL chain (oracle/o_ul.c, direct "
                                         f"O(M^2) transform precoding, double precision) in {dt:.1f} s"}
    b.close()
    return out


def bench_sync(args, batch, dev):
    """Sync front end over the batch: every subframe arrives in a raw slot of
    15 N + 64 samples at an unknown offset (1..63) with a CFO (+-0.4 subcarriers); per step the PSS of
    every subframe 0 / 5 is tracked (+-31 lags around the expected position, mi_sync_pss) and every
    subframe is realigned + CFO-corrected into the batch's IQ buffer (mi_sync_correct), i.e. exactly
    what the DL chain then consumes.  Roofline: the correction kernel (one read + one write of each
    sample)."""
    B = len(batch.cfgs)
    N = 2048
    L, M, slot = 15 * N, 31, 15 * N + 64
    rng = np.random.default_rng(123)
    npool = 20
    raw = np.zeros((npool, 2 * slot), np.float32)
    taus = rng.integers(1, 64, npool)
    cfos = rng.uniform(-0.4, 0.4, npool).astype(np.float32)
    for k in range(npool):
        c = abi.sf_cfg(cell_id=1, nof_prb=100, sf_idx=k % 10, tbs=61664 if k % 10 in (0, 5) else 75376, Qm=6)
        iq = abi.tx_subframe(c, tb_payload(900 + k, c.tbs // 8), snr_db=30.0, seed=900 + k)
        abi.tx_sync(1, 100, k % 10, iq)
        z = iq[0::2] + 1j * iq[1::2]
        z = z * np.exp(2j * np.pi * cfos[k] * np.arange(L) / N)
        raw[k, 2 * taus[k]:2 * (taus[k] + L):2], raw[k, 2 * taus[k] + 1:2 * (taus[k] + L):2] = z.real, z.imag
    d_pool = torch.from_numpy(raw).to(dev)
    d_raw = d_pool[torch.arange(B, device=dev) % npool].contiguous()   # [B][2 slot]
    d_iq = torch.zeros(2 * batch.iq_samples, dtype=torch.float32, device=dev)
    s = abi.Sync(100)
    sym6 = (160 + N) + 5 * (144 + N) + 144                            # useful part of symbol 6 (N = 2048)
    idx = np.arange(B)
    pss_idx = idx[(idx % npool) % 10 % 5 == 0]                        # subframes 0 / 5
    pss_off = pss_idx.astype(np.uint64) * slot + 32 + sym6 - M        # receiver expects offset 32
    half = idx - (idx % npool) % 5                                    # the subframe carrying each one's PSS
    dst = np.array([batch.iq_offset(i) for i in range(B)], np.uint64)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    tmr = {"pss": 0.0}

    def step():
        t = time.perf_counter()
        res = np.array(s.pss(d_raw.data_ptr(), pss_off, 2 * M + 1, 1 << 1, sptr), np.float64)
        tmr["pss"] += time.perf_counter() - t
        tau = np.full(B, 32.0)
        cf = np.zeros(B, np.float32)
        tau[pss_idx] = 32 + res[:, 1] - M
        cf[pss_idx] = res[:, 3]
        # the other subframes take the timing / CFO of their half frame's PSS (the pool's per-subframe
        # offsets stand in for a drifting stream)
        src = idx.astype(np.uint64) * slot + tau[half].astype(np.uint64)
        s.correct(d_raw.data_ptr(), src, d_iq.data_ptr(), dst, cf[half], L, sptr)
        return res

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize(dev)
    tmr["pss"] = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / args.steps
    # correction kernel alone (HIP events on the launch stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    src = idx.astype(np.uint64) * slot + 32
    cf1 = np.full(B, 0.1, np.float32)
    e0.record()
    for _ in range(args.steps):
        s.correct(d_raw.data_ptr(), src, d_iq.data_ptr(), dst, cf1, L, sptr)
    e1.record()
    torch.cuda.synchronize(dev)
    cms = e0.elapsed_time(e1) / args.steps
    k = pss_idx % npool
    ok = bool(np.all(np.abs(32 + res[:, 1] - M - taus[k]) <= 1) and np.all(np.abs(res[:, 3] - cfos[k]) < 0.05))
    s.close()
    gbs = 2 * 8 * L * B / (cms * 1e-3) / 1e9
    return {"ms_per_step": round(dt * 1e3, 3), "subframes_per_s": round(B / dt, 1), "timing_cfo_ok": ok,
            "pss_tracks_per_step": int(len(pss_idx)), "pss_ms": round(tmr["pss"] / args.steps * 1e3, 3),
            "correct_kernel_ms": round(cms, 3),
            "correct_roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                                 "frac": round(gbs / 8000.0, 4)},
            "what": f"PSS tracking (+-{M} lags) of the {len(pss_idx)} subframes 0/5 + realignment and CFO "
                    f"correction of all {B} subframes into the batch IQ buffer, per step"}


def bench_h2d(args, cfgs, pool_iq, batch, bits_ok, iq=None, steps=None):
    """IQ resident in page-locked host memory, each step copied H2D and decoded through the
    double-buffered pipeline (copy of step i+1 overlaps the decode of step i): the deployable (PCIe-inclusive)
    rate, reported beside value and never as value."""
    B = len(cfgs)
    iq_fmt = iq or args.iq
    steps = steps or args.steps
    sc16 = iq_fmt == "sc16"
    pipe = abi.Pipe(cfgs, max_its=args.max_its, tdec_i16=args.tdec == "i16", iq_sc16=sc16)
    nfl = 2 * batch.iq_samples
    esz = 2 if sc16 else 4
    hb = abi.HostBuffer(nfl * esz, np.int16 if sc16 else np.float32)
    pool = [abi.to_sc16(x) for x in pool_iq] if sc16 else pool_iq
    for i in range(B):
        o = 2 * batch.iq_offset(i)
        iq = pool[i % len(pool)]
        hb.array[o:o + len(iq)] = iq
    for _ in range(max(2, args.warmup)):
        pipe.wait(pipe.submit(hb.ptr))
    t0 = time.perf_counter()
    last = [pipe.submit(hb.ptr) for _ in range(steps)]
    pipe.wait(last[-1] ^ 1)
    pipe.wait(last[-1])
    dt = time.perf_counter() - t0
    ok = pipe.batch(last[-1]).download(abi.BUF_TB_CRC, np.uint32)[:B]
    pipe.close()
    hb.close()
    # the pipe's own CRC-OK bits (quantised sc16 IQ can fail a TB the device-resident fc32 run decoded: ADVICE r5);
    # bits_ok (the fc32 run's) is kept beside it for comparison
    pipe_bits = float(sum(c.tbs for c, o in zip(cfgs, ok) if o))
    return {"value": round(pipe_bits * steps / dt / 1e6, 2), "resident_bits_ok": bits_ok, "pipe_bits_ok": pipe_bits, "unit": "Mbps", "ms_per_step": round(dt / steps * 1e3, 3),
            "steps": steps, "iq_bytes_per_subframe": round(nfl * esz / B),
            "pcie_GBps": round(nfl * esz * steps / dt / 1e9, 2), "crc_ok_rate": round(float(ok.mean()), 6),
            "what": f"IQ ({iq_fmt}, batch layout) from page-locked host memory via mi_dl_pipe: H2D on a copy "
                    "stream overlapped with the previous batch's decode"}


def measure(args, cfgs, pool_iq, pool_tb, world, dev, steps, warmup):
    """Plan the batch, stage the pool in HBM (replicated on device into the batch IQ layout), run `warmup` untimed
    and `steps` timed passes (barrier + synchronize on both sides), then check the last step's outputs: every TB's
    CRC verdict and, for every CRC-OK TB, its payload against the transmitted bytes.

    --streams S > 1: S workspaces (abi.Batch) of the same batch on S HIP streams, consecutive steps issued
    round-robin -- a streaming receiver's double (triple) buffering: step i + 1's front end (OFDM, channel
    estimation, rate de-matching) runs while step i's turbo decoder occupies the GPU.  Every step still decodes
    the whole batch; the timed region covers all `steps` steps."""
    B = len(cfgs)
    S = max(1, args.streams)
    compact = args.ce == "compact" and not args.ctrl   # --ctrl reads the batch's full channel estimates
    batches = [abi.Batch(cfgs, max_its=args.max_its, profile=True, tdec_i16=args.tdec == "i16", sched=args.sched,
                         compact_ce=compact, keep_llr=args.llr_stream) for _ in range(S)]
    batch = batches[0]
    d_iq = torch.empty(2 * batch.iq_samples, dtype=torch.float32, device=dev)
    if len(pool_iq) == B and len({len(x) for x in pool_iq}) > 1:
        flat = np.zeros(2 * batch.iq_samples, np.float32)
        for i, iq in enumerate(pool_iq):
            o = 2 * batch.iq_offset(i)
            flat[o:o + len(iq)] = iq
        d_iq.copy_(torch.from_numpy(flat))
    else:
        sfl = len(pool_iq[0])   # floats per subframe (one bandwidth)
        d_pool = torch.from_numpy(np.stack(pool_iq)).to(dev)
        idx = torch.arange(B, device=dev) % len(pool_iq)
        d_iq.view(B, sfl).copy_(d_pool[idx])
        del d_pool
    streams = bench_streams(dev, S)
    sptr = [st.cuda_stream for st in streams]

    def whole(i):
        batches[i % S].run(d_iq.data_ptr(), sptr[i % S])

    def split_runs(F):
        # split runs (mi_dl_batch_run_split): each workspace's front end on a stream of the CUs i mod 8 < F, its turbo
        # decoder + TB CRC on a stream of the others
        fr, bk = split_streams(S, F)
        return lambda i: batches[i % S].run_split(d_iq.data_ptr(), fr[i % S], bk[i % S])

    torch.cuda.synchronize(dev)
    for w in range(warmup * S):
        whole(w)
    torch.cuda.synchronize(dev)
    F, tune = split_share(args, S), None
    if F < 0:
        # tuned on one-process runs only: beside RCCL's streams (N ranks, --pg) the masked streams' extra hardware queues
        # are not worth the risk of oversubscribing the queue slots, and whole runs are the measured default there
        F, tune = (0, None) if dist_on() else tune_split(whole, split_runs(AUTO_SPLIT), S, dev)
        if not F:
            release_split_streams(AUTO_SPLIT)   # whole runs: the timed region sees the queue set it always had
    step = split_runs(F) if F else whole
    for b in batches:
        b.profile_reset()
    if dist_on():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize(dev)
    if dist_on():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # stage times: HIP events on each workspace's stream, averaged over every timed step
    per = [(b.stage_ms(), b) for b in batches[:min(S, steps)]]
    nprof = sum(n for (_, n), _ in per)
    stage = {k: sum(st[k] * n for (st, n), _ in per) / nprof for k in per[0][0][0]}
    iso = isolated_stages(batch, lambda: batch.run(d_iq.data_ptr(), sptr[0]), dev, S, steps)
    del d_iq
    bad, n_ok, its, bits_ok = 0, 0, None, 0.0
    for k, b in enumerate(batches[:min(S, steps)]):
        crc = b.download(abi.BUF_TB_CRC, np.uint32)[:B]
        pay = b.download(abi.BUF_PAYLOAD, np.uint8)
        bad += sum(int(not np.array_equal(b.payload(i, pay), pool_tb[i % len(pool_tb)])) for i in range(B) if crc[i])
        if k == 0:
            its = b.download(abi.BUF_TB_ITS, np.uint32)[:B]
            n_ok = int(crc.sum())
            bits_ok = float(sum(c.tbs for c, o in zip(cfgs, crc) if o))
            cb_its = b.download(abi.BUF_CB_ITS, np.uint32)
    for b in batches[1:]:
        b.close()
    return {"batch": batch, "stage": stage, "nprof": nprof, "elapsed": elapsed, "n_ok": n_ok, "its": its,
            "bad": bad, "bits_ok": bits_ok, "cb_its": cb_its, "iso": iso, "split": F, "split_tune": tune}


def varied_cfgs(P, first):
    """A pool of P distinct 20 MHz TM1 grants as a multi-UE receiver sees them (srsUE re-derives
    the grant every TTI, phch_worker.cc:297 -> :337): per subframe an RNTI from a seeded set of 64, MCS 20-28 (64QAM,
    36.213 Table 7.1.7.1-1) and rv 0 or (one in four) 2, all new transmissions."""
    rng = np.random.default_rng(0x5EED5 + first)
    rntis = [int(x) for x in rng.integers(0x003D, 0xFFF4, 64)]
    out = []
    for i in range(P):
        mcs = int(rng.integers(20, 29))
        out.append(abi.sf_cfg(cell_id=1, nof_prb=100, nof_ports=1, sf_idx=SF_CYCLE[(first + i) % 8], cfi=1, tm=1,
                              rnti=rntis[int(rng.integers(0, 64))], rv=2 if rng.integers(0, 4) == 3 else 0,
                              tbs=TBS_100[mcs - 2], Qm=6))
    return out


def static_workspaces(S, J):
    """Workspaces of the static planning replay over J lists on S streams: each keeps one list (workspace k: list
    k % J, stream k % S), so the count is a multiple of J -- S rounded up to one (J for S = 1).  Not lcm(S, J): that is
    2 S for odd S, and a 12,500-subframe workspace holds ~45 GB (S = 5 would need 10 of them)."""
    return J * -(-max(1, S) // J)


def replan_steps(args, lists, iqs, dev, steps, warmup, threads, replan=True):
    """The streaming receiver with the grant re-derived every step: step i decodes list i % J (a 12,500-subframe
    configuration, IQ buffer iqs[i % J] laid out for it).  With replan, every step's plan is BUILT from scratch on a
    pool of `threads` host planner threads (mi_dl_plan_build, no GPU call) while earlier steps decode, then swapped
    into the step's workspace (mi_dl_batch_replan: table upload on the step's stream) before its run; without, each
    workspace keeps one list's plan (the static replay the headline measures).  S workspaces on S streams as in
    measure().  Returns (elapsed, CRC-OK bits per list, replan ms on the main thread, payload mismatches)."""
    import collections
    S = max(1, args.streams)
    J = len(lists)
    # re-planned: one workspace per stream.  Static: each workspace keeps one list (static_workspaces)
    W = S if replan else static_workspaces(S, J)
    batches = [abi.Batch(lists[k % J], max_its=args.max_its, profile=False, tdec_i16=args.tdec == "i16",
                         sched=args.sched, compact_ce=True) for k in range(W)]
    streams = bench_streams(dev, S)
    sptr = [st.cuda_stream for st in streams]
    D = max(1, threads)
    plans = [abi.Plan() for _ in range(D + 1)]   # D building + one ready ahead of the step that takes it
    ex = cf.ThreadPoolExecutor(max_workers=D)
    queue = collections.deque()                  # FIFO of (build future, plan object, list index): step i gets list i % J
    nxt = [0]

    def submit(p):
        j = nxt[0] % J
        nxt[0] += 1
        queue.append((ex.submit(p.build, lists[j]), p, j))

    rep_t = [0.0, 0]
    last_list = [None] * W

    def step(i):
        b = batches[i % W]
        if replan:
            fut, p, j = queue.popleft()
            fut.result()
            t = time.perf_counter()
            b.replan(p, sptr[i % S])
            rep_t[0] += time.perf_counter() - t
            rep_t[1] += 1
            submit(p)            # the plan object now holds the previous data: rebuild it for a later step
        else:
            j = i % W % J
        b.run(iqs[j].data_ptr(), sptr[i % W % S])
        last_list[i % W] = j
    try:
        if replan:
            for p in plans:
                submit(p)
        for i in range(warmup * W):
            step(i)
        torch.cuda.synchronize(dev)
        rep_t[:] = [0.0, 0]
        t0 = time.perf_counter()
        for i in range(warmup * W, warmup * W + steps):
            step(i)
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
    finally:
        for fut, _, _ in queue:
            fut.cancel()
        ex.shutdown(wait=True)
    bits = [0.0] * J
    bad = 0
    seen = set()

    def check(b, j):
        nonlocal bad
        crc = b.download(abi.BUF_TB_CRC, np.uint32)[:len(b.cfgs)]
        bits[j] = float(sum(b.cfgs[i].tbs for i in range(len(crc)) if crc[i]))
        pay = b.download(abi.BUF_PAYLOAD, np.uint8)
        bad += sum(int(not np.array_equal(b.payload(i, pay), args._pool_tb[j][i % len(args._pool_tb[j])]))
                   for i in range(len(crc)) if crc[i])
    for k, b in enumerate(batches):
        j = last_list[k]
        if j is None or j in seen:
            continue
        seen.add(j)
        check(b, j)
    # a list no workspace ran last (fewer streams than lists, re-planned): one more run of it after the timed region,
    # so every list's CRC-OK bits and payloads come from a run of that list
    for j in range(J):
        if j in seen:
            continue
        p = abi.Plan()
        p.build(lists[j])
        batches[0].replan(p, sptr[0])
        batches[0].run(iqs[j].data_ptr(), sptr[0])
        torch.cuda.synchronize(dev)
        p.close()
        check(batches[0], j)
    if not all(bits):
        raise RuntimeError(f"replan_steps: a list decoded no CRC-OK TB ({bits})")
    for b in batches:
        b.close()
    for p in plans:
        p.close()
    nsteps_per_list = [sum(1 for i in range(warmup * W, warmup * W + steps) if (i % J if replan else i % W % J) == j)
                       for j in range(J)]
    total_bits = sum(bits[j] * nsteps_per_list[j] for j in range(J))
    return elapsed, total_bits, (rep_t[0] / max(1, rep_t[1])) * 1e3, bad, bits


def bench_planning(args, cfgs, pool_iq, pool_tb, dev, threads, value_mbps):
    """what planning per-TTI grants costs the batched throughput.
    plan_ms: host build time of mi_dl_plan_build (one thread, warm caches = the lookup tables srslte_ue_dl_set_rnti
    pregenerates; cold = the first build of a new planner) for (a) a fresh shard of varied grants (varied_cfgs) and
    (b) configs[4]'s mixed cells, plus the default shard; then the pipelined mode (every step re-planned on host
    threads while earlier steps decode) on the default shard -- comparable to `value` -- and on the varied grants,
    beside the same varied workload replayed with static plans.  Reported beside value, never as value."""
    B = len(cfgs)
    P = len(pool_iq)
    out = {}

    def tbuild(cl, reps=3):
        p = abi.Plan()
        arr = abi.cfg_array(cl)
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            p.build(arr)
            t.append((time.perf_counter() - t0) * 1e3)
        p.close()
        return round(t[0], 2), round(min(t[1:]), 2)
    vpool = varied_cfgs(P, 0)
    varied = [vpool[i % P] for i in range(B)]
    c_head = tbuild(cfgs)
    c_var = tbuild(varied)
    c_mix = tbuild(config_cfgs(5, B, 0))
    out["plan_ms"] = {"default_shard": {"cold": c_head[0], "warm": c_head[1]},
                      "varied_grants": {"cold": c_var[0], "warm": c_var[1]},
                      "configs4_mixed": {"cold": c_mix[0], "warm": c_mix[1]},
                      "what": f"mi_dl_plan_build of {B} subframes on one host thread (cold: a new planner; warm: its "
                              "caches of scrambling words / RE lists / per-K tables filled)"}
    steps = max(4, min(args.steps, args.plan_steps))
    D = max(1, min(args.plan_threads, threads))
    sfl = len(pool_iq[0])
    d_pool = torch.from_numpy(np.stack(pool_iq)).to(dev)
    iq_head = torch.empty(B * sfl, dtype=torch.float32, device=dev)
    iq_head.view(B, sfl).copy_(d_pool[torch.arange(B, device=dev) % P])
    del d_pool
    args._pool_tb = [pool_tb]
    el, bits, rep_ms, bad, _ = replan_steps(args, [abi.cfg_array(cfgs)], [iq_head], dev, steps, 1, D)
    out["pipelined_default"] = {"Mbps": round(bits / el / 1e6, 2), "ms_per_step": round(el / steps * 1e3, 3),
                                "vs_value": round(bits / el / 1e6 / value_mbps, 4) if value_mbps else None,
                                "replan_ms_main_thread": round(rep_ms, 3), "payload_mismatches_crc_ok": bad,
                                "steps": steps, "planner_threads": D,
                                "what": "the default shard with its plan rebuilt from scratch for every step on host "
                                        "planner threads (mi_dl_plan_build) while earlier steps decode, swapped in by "
                                        "mi_dl_batch_replan before the step's run"}
    del iq_head
    # varied grants: two assignments of the varied pool to the shard's positions, each with its own IQ buffer
    vq, vt = make_pool(vpool, args.snr, threads, 0)
    lists, iqs = [], []
    d_pool = torch.from_numpy(np.stack(vq)).to(dev)
    for j in range(2):
        idx = (np.arange(B) + 37 * j) % P
        lists.append(abi.cfg_array([vpool[i] for i in idx]))
        buf = torch.empty(B * sfl, dtype=torch.float32, device=dev)
        buf.view(B, sfl).copy_(d_pool[torch.from_numpy(idx).to(dev)])
        iqs.append(buf)
    del d_pool
    args._pool_tb = [[vt[i] for i in (np.arange(B) + 37 * j) % P] for j in range(2)]
    el_s, bits_s, _, bad_s, per_s = replan_steps(args, lists, iqs, dev, steps, 1, D, replan=False)
    el_p, bits_p, rep_p, bad_p, per_p = replan_steps(args, lists, iqs, dev, steps, 1, D, replan=True)
    out["varied_static"] = {"Mbps": round(bits_s / el_s / 1e6, 2), "ms_per_step": round(el_s / steps * 1e3, 3),
                            "crc_ok_bits_per_list": per_s, "payload_mismatches_crc_ok": bad_s}
    out["pipelined_varied"] = {"Mbps": round(bits_p / el_p / 1e6, 2), "ms_per_step": round(el_p / steps * 1e3, 3),
                               "vs_static": round((bits_p / el_p) / (bits_s / el_s), 4) if bits_s else None,
                               "replan_ms_main_thread": round(rep_p, 3), "payload_mismatches_crc_ok": bad_p,
                               "crc_ok_bits_per_list": per_p, "steps": steps, "planner_threads": D,
                               "what": f"{B} subframes of varied grants (varied_cfgs: 64 RNTIs, MCS 20-28, rv 0/2), two "
                                       "alternating assignments, every step re-planned on host threads"}
    del iqs
    return out


TTI_BUDGET_US = 3000.0   # srsUE: subframe n's DL decode and the UL it acknowledges go out at n + 4 (phch_recv.cc:330-337)


def bench_tti(args):
    """configs[1] as SURVEY 8d defines it: one 20 MHz TM1 MCS-28 subframe per call through the
    per-TTI srsLTE ABI, as srsUE's phch_worker drives it -- host IQ in -> srslte_ue_dl_decode_fft_estimate (:254) ->
    srslte_ue_dl_cfg_grant (:337) -> srslte_pdsch_decode_rnti (:347) -> payload out, then the UL PUSCH encode -- with
    1 and with 4 concurrent worker instances (srsUE runs 1-4 phch_workers, phy.h:118-119), each in its own thread
    (tests/c/tti_latency, plain C against include/srslte/srslte.h).  Latencies per TTI, pooled over the workers."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "c", "tti_latency")
    if not os.path.exists(exe):
        return {"error": "tests/c/tti_latency not built (__graft_entry__.build)"}
    out = {}
    for w in (1, 4):
        r = subprocess.run([exe, "100", str(args.tti_ttis), str(w)], capture_output=True, text=True, timeout=300)
        if r.returncode:
            out[f"workers_{w}"] = {"error": f"rc {r.returncode}: {r.stderr[-300:]}"}
            continue
        d = json.loads(r.stdout.strip().splitlines()[-1])
        dl, ul = d["dl_total"], d["ul_pusch_encode"]
        out[f"workers_{w}"] = {
            "ttis": d["ttis"], "crc_ok_and_payload_match": d["crc_ok_and_payload_match"],
            "dl_p50_us": dl["p50_us"], "dl_p99_us": dl["p99_us"], "dl_max_us": dl["max_us"],
            "decode_fft_estimate_p50_us": d["decode_fft_estimate"]["p50_us"],
            "pdsch_decode_rnti_p50_us": d["pdsch_decode_rnti"]["p50_us"],
            "ul_pusch_encode_p50_us": ul["p50_us"], "ul_pusch_encode_p99_us": ul["p99_us"],
            "dl_plus_ul_p99_us": round(dl["p99_us"] + ul["p99_us"], 1),
            "within_tti4_budget": dl["p99_us"] + ul["p99_us"] < TTI_BUDGET_US,
            "subframes_per_s": round(d["ttis"] / (d["wall_us"] * 1e-6), 1)}
    out["budget_us"] = TTI_BUDGET_US
    out["what"] = ("configs[1] through the per-TTI srsLTE ABI (tests/c/tti_latency): host IQ (30,720 cf32) -> "
                   "decode_fft_estimate -> cfg_grant -> pdsch_decode_rnti -> 9,422 payload bytes, then cfg_grant + "
                   "pusch_encode (UL 16QAM MCS 20) per TTI; p99 of DL + UL against the TTI+4 budget "
                   "(phch_recv.cc:330-337); 1 and 4 concurrent srsLTE worker instances (phy.h:118-119)")
    return out


def isolated_stages(runner, run_once, dev, S, steps):
    """With --streams S > 1 the timed steps overlap, so the per-stage HIP-event durations of the timed region
    include other streams' kernels sharing the GPU and are not per-kernel figures.  After the
    timed region (outside it), re-run one workspace alone on its stream -- each step synchronised before the
    next starts -- and return its per-stage averages and the number of runs; the roofline divides by these.
    None for S == 1 (the timed region's own events are already isolated)."""
    if S <= 1:
        return None
    n = max(1, min(steps, 10))
    torch.cuda.synchronize(dev)
    runner.profile_reset()
    for _ in range(n):
        run_once()
        torch.cuda.synchronize(dev)
    st, k = runner.stage_ms()
    return st, k


def roofline_timing(stage, nprof, iso):
    """The roofline's launch-duration fields: isolated runs when the timed steps overlapped (isolated_stages),
    with the overlapped average kept beside them; otherwise the timed region's own average."""
    if iso is None:
        return {"avg_launch_ms": round(stage["tdec"], 4), "launches_averaged": nprof}
    return {"avg_launch_ms": round(iso[0]["tdec"], 4), "launches_averaged": iso[1],
            "launch_timing": "isolated: one workspace alone on its stream after the timed region, each run synchronised",
            "avg_launch_ms_overlapped": round(stage["tdec"], 4), "launches_averaged_overlapped": nprof}


def wave_iterations(batch, cb_its):
    """Where the turbo iterations go: per code block, and per packed-decoder wavefront pair
    (a group pair = 128 code blocks: lanes 128 j .. 128 j + 127; without compaction a pair runs until its slowest
    code block stops).  Histograms of iteration counts, from the decoder's own per-code-block output."""
    n = batch.n_codeblocks
    cb = np.asarray(cb_its[:(batch.n_groups * 64)], np.int64)
    valid = cb > 0
    out = {"cb_its_hist": {int(v): int(c) for v, c in zip(*np.unique(cb[valid], return_counts=True))},
           "cb_mean_its": round(float(cb[valid].mean()), 4), "codeblocks": int(n),
           "codeblocks_past_iteration_0": int((cb > 1).sum())}
    if batch.turbo_sched == "p2":
        npair = len(cb) // 128
        pm = cb[:npair * 128].reshape(npair, 128).max(axis=1)
        out["pair_max_its_hist"] = {int(v): int(c) for v, c in zip(*np.unique(pm, return_counts=True))}
        out["pair_iterations_without_compaction"] = int(pm.sum())
        out["compaction"] = batch.turbo_compact
        if batch.turbo_compact:
            # iteration 0 over every pair, then dense pairs of the continuing code blocks
            out["continuation_pairs"] = int(-(-int((cb > 1).sum()) // 128))
    return out


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N copies of this command, one rank per GPU, BEFORE this
    process touches the GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in each child's environment, rendezvous on
    127.0.0.1).  Only rank 0 prints the JSON line; the exit code is the first failing rank's."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc), 0)


def dry_run(args, world, rank):
    """CPU rehearsal of the N-rank launch (tests/test_dist.py): gloo instead of RCCL, each rank decodes its
    contiguous shard of a small synthetic batch with the TEST-ONLY host emulation of the decoder kernels, from
    the LLR streams the test wrote to --dry-run-llr; reports n_gpus / shards / CRC-OK count exactly like the GPU
    path.  Never a measurement (no "value")."""
    import ctypes as C
    d = np.load(args.dry_run_llr)
    total = int(d["total"])
    first, n = shard_range(total, rank, world)
    cfgs = [abi.sf_cfg(cell_id=1, nof_prb=6, nof_ports=1, sf_idx=SF_CYCLE[g % 8], tbs=4392, Qm=6)
            for g in range(first, first + n)]
    llr = np.concatenate([d[f"llr{g}"] for g in range(first, first + n)]).astype(np.float32)
    pay = np.zeros(n * 549, np.uint8)
    ok = np.zeros(n, np.uint32)
    its = np.zeros(n, np.uint32)
    t0 = time.perf_counter()
    abi.emu().emu_decode_llr(C.cast(abi.cfg_array(cfgs), C.c_void_p), n, llr.ctypes.data, 4, pay.ctypes.data,
                             ok.ctypes.data, its.ctypes.data, None)
    elapsed = time.perf_counter() - t0
    good = sum(int(np.array_equal(pay[i * 549:(i + 1) * 549], tb_payload(first + i, 549))) for i in range(n))
    shards = [None] * world
    dist.all_gather_object(shards, [first, n, good])
    elapsed, (n_ok, n_cb, its_sum, n_bad), per = reduce_over_ranks(
        elapsed, [int(ok.sum()), n, int(its.sum()), n - good], world)
    devices = rank_devices(world, None)
    if rank == 0:
        out = {"dry_run": True, "n_gpus": world, "shards": shards, "crc_ok": n_ok, "subframes": n_cb,
               "crc_ok_rate": n_ok / n_cb, "mean_turbo_iterations": its_sum / n_cb, "payload_mismatches": n_bad,
               "elapsed_max_s": elapsed, "elapsed_per_rank_s": per, "rank_devices": devices}
        if not args.no_cpu_baseline:   # the same rank-0 baseline leg as the GPU line, on this rank's subframes
            iq = [abi.tx_subframe(c, tb_payload(first + i, c.tbs // 8), snr_db=30.0, seed=0xA5A5 + first + i)
                  for i, c in enumerate(cfgs)]
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, cfgs, iq,
                                               [tb_payload(first + i, c.tbs // 8) for i, c in enumerate(cfgs)],
                                               "6-PRB rehearsal subframes", True)
        emit(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 steps (~2.4 s of decoding at the headline): long enough for an outside GPU-activity sampler to see
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sf-per-gpu", type=int, default=12500, help="subframes per GPU per step")
    ap.add_argument("--pool", type=int, default=256, help="distinct synthetic subframes per rank")
    ap.add_argument("--snr", type=float, default=30.0)
    ap.add_argument("--max-its", type=int, default=4)
    ap.add_argument("--iterating-snr", type=float, default=21.5,
                    help="default config: also run the shard at this SNR (turbo waterfall, ~3 iterations at max_its 4) "
                         "and report it as the `iterating` block; 0 = skip")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--ce", choices=("compact", "full"), default="compact",
                    help="channel estimates of the batch: compact = the 4 pilot rows per port, interpolated in time "
                         "inside the fused demap (MI_DL_FLAG_CE_COMPACT, identical LLRs); full = all 14 symbols")
    ap.add_argument("--streams", type=int, default=0,
                    help="workspaces / HIP streams the steps rotate over (consecutive batches overlap); 1 = serial; "
                         "0 = auto: 4 for the headline shard (+13-15 %%: one batch's front end and rate de-matching run "
                         "beside the previous batch's turbo decoder; profiles/r3/ab_streams*), 16 for the low-occupancy "
                         "configs[2] / configs[4] batches and 8 for configs[0], at 16 hardware queues (profiles/r6/lowocc)")
    ap.add_argument("--iterating-streams", type=int, default=0,
                    help="--streams of the waterfall block; 0 = auto (= --streams: its continuation holds 0.74 "
                         "wavefronts per SIMD, so the next batches' iteration 0 fills the rest: 35 -> 56 Gbps with 4; "
                         "profiles/r3/ab_streams*)")
    ap.add_argument("--split", type=int, default=-1, choices=range(-1, 8), metavar="-1..7",
                    help="split runs (mi_dl_batch_run_split): each step's front end (OFDM, channel estimation, demap + "
                         "rate de-matching) on a stream of the CUs whose index mod 8 is < SPLIT, its turbo decoder and "
                         "TB CRC on a stream of the other CUs, so rate de-matching never shares a CU with the decoder; "
                         "0 = whole runs on one stream per workspace; -1 (default) = the headline shard on several "
                         "streams times both layouts after the warmup and keeps split runs (--split 2) only when they "
                         "are >1.5 %% faster, other configs whole runs.  Headline, 4 streams, --split 2: 7.96-8.08 ms "
                         "per step on every box sampled, whole runs 7.86-8.14 on most boxes and 8.2-8.35 on the boxes "
                         "where they co-schedule rate de-matching beside the decoder (profiles/r6/cumask)")
    ap.add_argument("--hw-queues", type=int, default=8, choices=range(0, 33), metavar="0..32",
                    help="GPU_MAX_HW_QUEUES for this process and its ranks (set before the HIP runtime starts, see "
                         "HW_QUEUES above); 0 = keep the environment's value")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--plan-steps", type=int, default=40,
                    help="default config: steps of the planning block (per-step re-planning on host threads, VERDICT r3 "
                         "item 3); 0 = skip the block")
    ap.add_argument("--plan-threads", type=int, default=4, help="host planner threads of the pipelined mode")
    ap.add_argument("--llr-stream", action="store_true",
                    help="A/B: demap writes the LLR stream and rate de-matching reads it (MI_DL_FLAG_KEEP_LLR; full "
                         "channel estimates) instead of the fused demap")
    ap.add_argument("--share-gpu", action="store_true",
                    help="N-rank rehearsal on one GPU: every rank on GPU 0, gloo collectives (not a scaling number)")
    ap.add_argument("--config", type=int, default=4, choices=(1, 2, 3, 4, 5),
                    help="BASELINE.json configs[n-1]; 4 (default) = 20 MHz TM1 MCS-28 shard per GPU")
    ap.add_argument("--cb-per-gpu", type=int, default=65536, help="config 1: code blocks per GPU per step")
    ap.add_argument("--ebno", type=float, default=1.5, help="config 1: Eb/N0 in dB")
    ap.add_argument("--h2d-steps", type=int, default=20,
                    help="steps of the PCIe-inclusive (h2d) block of the default line (0 = off)")
    ap.add_argument("--tti-ttis", type=int, default=200,
                    help="TTIs per worker of the per-TTI latency block (configs[1] through the srsLTE ABI at 1 and 4 "
                         "concurrent instances, tests/c/tti_latency); 0 = off")
    ap.add_argument("--h2d", action="store_true",
                    help="also measure the PCIe-inclusive rate: IQ from page-locked host memory through the "
                         "double-buffered mi_dl_pipe (SURVEY 8f-3); reported beside value, never as value")
    ap.add_argument("--sync", action="store_true",
                    help="also time the sync front end (PSS tracking + CFO correction, SURVEY 8f-2) on the batch")
    ap.add_argument("--ctrl", action="store_true",
                    help="also time the DL control stage (SURVEY 8f-1: PCFICH + PDCCH soft bits + DCI blind search "
                         "for each subframe's RNTI) on the batch's grid; reported beside value")
    ap.add_argument("--ul", action="store_true",
                    help="also time the UL PUSCH transmitter (SURVEY 8f-4) on as many subframes; reported beside value")
    ap.add_argument("--iq", choices=("fc32", "sc16"), default="fc32",
                    help="wire format of the host IQ in the --h2d measurement (sc16 = UHD int16, half the bytes)")
    ap.add_argument("--sched", choices=("auto", "win", "lane", "lanex", "lanexr", "p2"), default="auto",
                    help="int16 turbo schedule: latency form (one workgroup per code block, exact trellis segments), "
                         "one code block per lane, or auto (latency form up to 1024 code blocks)")
    ap.add_argument("--tdec", choices=("gen", "i16"), default="i16",
                    help="turbo arithmetic: gen = srsLTE-gen float, i16 = srsLTE SSE-design int16 (MI_DL_FLAG_TDEC_I16)")
    ap.add_argument("--pg", action="store_true",
                    help="one rank: still bring up the nccl (RCCL) process group, so the timing barrier, the reductions "
                         "and the device gather run over RCCL as in the N-GPU line (launch with WORLD_SIZE=1, MASTER_*)")
    ap.add_argument("--dry-run-llr", default=None, help=argparse.SUPPRESS)   # CPU launch rehearsal (tests only)
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))                     # before anything touches the GPU
    if args.streams <= 0:
        # one batch of the low-occupancy configs holds well under one turbo wavefront per SIMD (configs[2]: 1,000
        # subframes), so more batches in flight fill the GPU: configs[2] 39 Gbps on 4 streams -> 84 on 16 (with the
        # packed decoder), configs[4] 27 -> 32, configs[0] 20 -> 21 on 8 (profiles/r6/lowocc); the headline keeps 4 (5
        # measured slower, and 6 workspaces of its 12,500-subframe shard do not fit in HBM)
        args.streams = {1: 8, 3: 16, 4: 4, 5: 16}.get(args.config, 1)
    if args.config == 3 and args.sched == "auto" and args.streams >= 8:
        # with 8+ batches in flight the streams, not one batch's pairs, fill the SIMDs: the packed decoder's half VALU per
        # code block wins although one batch alone would pick the crossed lanes (16 streams: 84 vs 65 Gbps)
        args.sched = "p2"
    if args.config == 2:
        args.sf_per_gpu = 1
    elif args.config == 3 and args.sf_per_gpu == 12500:
        args.sf_per_gpu = 1000

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run_llr:
        dist.init_process_group("gloo")
        dry_run(args, world, rank)
        dist.destroy_process_group()
        return
    if world > 1 and args.share_gpu:
        # rehearsal of the N-rank path on a one-GPU box: every rank decodes its shard on GPU 0, the
        # timing barrier and the three-scalar reduction go over gloo (the ranks' kernels share the card,
        # so the aggregate is not a scaling measurement)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
    elif world > 1 or args.pg:
        keep_stdout_clean()
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    threads = max(1, min(16, (os.cpu_count() or 8) // max(1, world)))
    if args.config == 1:
        out = bench_codeblocks(args, world, rank, dev)
        if out:
            emit(out)
        if dist_on():
            dist.destroy_process_group()
        return

    B = args.sf_per_gpu
    first, _ = shard_range(B * world, rank, world)          # this rank's global subframe indices
    P = min(args.pool, B)
    P -= P % 8 if P >= 8 else 0                             # keep the sf_idx cycle aligned
    cfgs = config_cfgs(args.config, B, first)
    # the pool: subframes 0..P-1 of this shard; subframe i of the batch reuses pool entry i % P
    if args.config == 5:
        P = B                                               # every mixed subframe is distinct
    h = [0.8 + 0.3j, -0.4 + 0.5j] if args.config == 3 else None
    pool_iq, pool_tb = make_pool(cfgs[:P], args.snr, threads, first, h)
    m = measure(args, cfgs, pool_iq, pool_tb, world, dev, args.steps, args.warmup)
    batch, stage, nprof, elapsed = m["batch"], m["stage"], m["nprof"], m["elapsed"]
    n_ok, its, bad, bits_ok = m["n_ok"], m["its"], m["bad"], m["bits_ok"]
    # global counters: CRC-OK bits, code blocks, CRC-OK TBs, TB iterations, TBs, payload mismatches (every rank)
    elapsed, (bits_all, ncb_all, ok_all, its_all, tb_all, bad_all), per_rank = reduce_over_ranks(
        elapsed, [bits_ok, batch.n_codeblocks, n_ok, int(its.sum()), B, bad], world, dev)
    devices = rank_devices(world, dev)
    # the same shard in the turbo decoder's waterfall region (every code block iterates): reported beside value
    itr = None
    if args.config == 4 and args.iterating_snr > 0:
        ipool_iq, ipool_tb = make_pool(cfgs[:P], args.iterating_snr, threads, first, h)
        isteps = max(1, min(args.steps, 40))
        iargs = argparse.Namespace(**{**vars(args), "streams": args.iterating_streams or args.streams})
        im = measure(iargs, cfgs, ipool_iq, ipool_tb, world, dev, isteps, 1)
        iel, (ibits, incb, iok, iits, itb, ibad), _ = reduce_over_ranks(
            im["elapsed"], [im["bits_ok"], im["batch"].n_codeblocks, im["n_ok"], int(im["its"].sum()), B, im["bad"]],
            world, dev)
        if rank == 0:
            ib = im["batch"]
            ims = im["iso"][0]["tdec"] if im["iso"] else im["stage"]["tdec"]
            iach = ib.algo_bytes(4) / (ims * 1e-3) / 1e9
            itr = {"snr_db": args.iterating_snr, "steps": isteps, "streams": iargs.streams,
                   "split_front_cu_eighths": im["split"],
                   **({"stream_layout_autotune": im["split_tune"]} if im["split_tune"] else {}),
                   "ms_per_step": round(iel / isteps * 1e3, 3),
                   "Mbps": round(ibits * isteps / iel / 1e6, 2),
                   "turbo_codeblocks_per_s": round(incb * isteps / iel, 1),
                   "crc_ok_rate": round(iok / itb, 6), "mean_turbo_iterations": round(iits / itb, 4),
                   "payload_mismatches_crc_ok": int(ibad),
                   "turbo_waves": wave_iterations(ib, im["cb_its"]),
                   "stage_ms_per_step": {k: round(v, 4) for k, v in im["stage"].items()},
                   "tdec_roofline": {"kernel": tdec_kernel_name(ib.turbo_sched), "bound": "hbm",
                                     "achieved": round(iach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": round(iach / HBM_PEAK_GBS, 5),
                                     **roofline_timing(im["stage"], im["nprof"], im["iso"])},
                   "what": f"the same {B}-subframe shard at {args.iterating_snr:g} dB AWGN (turbo waterfall region, "
                           f"max_its {args.max_its}): Mbps counts CRC-OK TBs only"}
        im["batch"].close()

    what = {2: "configs[1] 20 MHz TM1 SISO PDSCH MCS-28 (TBS 75376, 13 x K=5824), single subframe",
            3: "configs[2] 20 MHz TM2 (2-port SFBC) 64QAM MCS-28 (TBS 75376)",
            4: "configs[3] shard: 20 MHz TM1 SISO PDSCH MCS-28 (TBS 75376, 13 x K=5824) subframes of configs[1]",
            5: "configs[4] mixed 1.4/5/10/20 MHz cells, random allocation 6-100 PRB and MCS 0-28"}[args.config]
    if rank == 0:
        K = args.steps
        mbps = bits_all * K / elapsed / 1e6
        cbps = ncb_all * K / elapsed
        tdec_ms = m["iso"][0]["tdec"] if m["iso"] else stage["tdec"]
        tdec_bytes = batch.algo_bytes(4)
        achieved = tdec_bytes / (tdec_ms * 1e-3) / 1e9
        traffic, valu_busy, traffic_src = pmc_traffic(B, args.tdec, tdec_kernel_name(batch.turbo_sched))
        out = {
            "metric": METRIC, "value": round(mbps, 2), "unit": "Mbps", "n_gpus": world, "steps": K,
            "warmup": args.warmup, "ms_per_step": round(elapsed / K * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": dtype_of(args), "data": "synthetic",
            "config": {"workload": f"{what}: {B} subframes per GPU per step, {args.snr:g} dB AWGN",
                       **({"share_gpu_rehearsal": True} if args.share_gpu and world > 1 else {}),
                       **({"process_group": dist.get_backend()} if dist_on() else {}),
                       "baseline_config": args.config, "subframes_per_gpu": B, "turbo_arithmetic": args.tdec,
                       "max_its": args.max_its, "turbo_schedule": SCHED_DESC[batch.turbo_sched],
                       "streams": max(1, args.streams),
                       "split_front_cu_eighths": m["split"],
                       **({"stream_layout_autotune": m["split_tune"]} if m["split_tune"] else {}),
                       "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "channel_estimates": "full" if (args.ce == "full" or args.ctrl or args.llr_stream) else "compact",
                       **({"llr_stream": True} if args.llr_stream else {}),
                       "parallelism": f"replicas x{world} (no collective on the data path)"},
            "turbo_codeblocks_per_s": round(cbps, 1),
            "crc_ok_rate": round(ok_all / tb_all, 6), "mean_turbo_iterations": round(its_all / tb_all, 4),
            "payload_mismatches_crc_ok": int(bad_all), "subframes_all_ranks": int(tb_all),
            "elapsed_per_rank_s": [round(x, 6) for x in per_rank], "rank_devices": devices,
            "stage_ms_per_step": {k: round(v, 4) for k, v in stage.items()},
            "roofline": {"kernel": tdec_kernel_name(batch.turbo_sched), "bound": "hbm", "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic, "valu_busy_pct": valu_busy, "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": tdec_bytes, **roofline_timing(stage, nprof, m["iso"])},
        }
        if args.h2d:
            out["h2d"] = bench_h2d(args, cfgs, pool_iq, batch, bits_ok)
        elif args.config == 4 and args.h2d_steps > 0 and world == 1:
            # the deployable rate of this build: UHD's sc16 wire format and srsLTE's fc32, IQ
            # from page-locked host memory, beside value
            out["h2d"] = {f: bench_h2d(args, cfgs, pool_iq, batch, bits_ok, iq=f, steps=args.h2d_steps)
                          for f in ("sc16", "fc32")}
        if itr:
            out["iterating"] = itr
        if args.config == 4 and args.plan_steps > 0 and world == 1:
            out["planning"] = bench_planning(args, cfgs, pool_iq, pool_tb, dev, threads, mbps)
        if args.config == 4 and args.tti_ttis > 0 and world == 1:
            out["tti"] = bench_tti(args)
        if args.ctrl:
            out["ctrl"] = bench_ctrl(args, batch, dev)
        if args.ul:
            out["ul"] = bench_ul(args, B, dev)
        if args.sync:
            out["sync"] = bench_sync(args, batch, dev)
        if not args.no_cpu_baseline:   # rank 0 at every N, after the reduction (outside the timed region)
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, cfgs[:len(pool_iq)], pool_iq, pool_tb, what,
                                               args.tdec == "i16")
        emit(out)
    batch.close()
    if dist_on():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
