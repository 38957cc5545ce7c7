"""CPU, world_size 2 over gloo: the multi-GPU structure of bench.py (one process per GPU, contiguous
subframe shards, no collective on the data path, max-over-ranks timing + sums) exercised with the
test-only host emulation of the decoder kernels standing in for the GPU."""
import ctypes as C
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from helpers import oracle_front
    from srsue_amd import abi
    total = 6
    first, n = bench.shard_range(total, rank, world)
    cfgs, llrs, tbs = [], [], []
    for g in range(first, first + n):
        c = abi.sf_cfg(cell_id=1, nof_prb=6, nof_ports=1, sf_idx=bench.SF_CYCLE[g % 8], tbs=4392, Qm=6)
        tb = bench.tb_payload(g, c.tbs // 8)
        iq = abi.tx_subframe(c, tb, snr_db=30.0, seed=0xA5A5 + g)
        cfgs.append(c); llrs.append(oracle_front(c, iq)[3]); tbs.append(tb)
    arr = abi.cfg_array(cfgs)
    flat = np.concatenate(llrs).astype(np.float32)
    pe = np.zeros(sum(c.tbs // 8 for c in cfgs), np.uint8)
    ok = np.zeros(n, np.uint32)
    its = np.zeros(n, np.uint32)
    abi.emu().emu_decode_llr(C.cast(arr, C.c_void_p), n, flat.ctypes.data, 4, pe.ctypes.data, ok.ctypes.data,
                             its.ctypes.data, None)
    good = all(np.array_equal(pe[i * 549:(i + 1) * 549], tbs[i]) for i in range(n))
    elapsed = 0.5 + rank       # stand-in timings: the max must win
    t, (n_ok, n_cb, its_sum), per = bench.reduce_over_ranks(elapsed, [int(ok.sum()), n, int(its.sum())], world)
    q.put((rank, first, n, good, t, n_ok, n_cb, its_sum, per))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_shards_without_data_path_collective(built):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert [(r[1], r[2]) for r in res] == [(0, 3), (3, 3)]          # contiguous shards cover 0..5
    assert all(r[3] for r in res)                                     # each rank decoded its own TBs
    assert all(r[4] == 1.5 for r in res)                              # max over ranks
    assert all(r[5] == 6 and r[6] == 6 for r in res)                  # sums over ranks
    assert all(r[7] == 6 for r in res)                                # iteration sums: 1 per TB at 30 dB
    assert all(r[8] == [0.5, 1.5] for r in res)                       # every rank's elapsed time, in rank order


def test_shard_range_covers_everything():
    import bench
    for total in (1, 7, 100000):
        for world in (1, 2, 4, 8):
            spans = [bench.shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and sum(n for _, n in spans) == total
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))


@pytest.mark.timeout(300)
def test_bench_spawns_its_own_ranks(built, tmp_path):
    """`bench.py --gpus 2` with no launcher starts 2 ranks itself (the driver's N-GPU command); the CPU
    rehearsal decodes each rank's contiguous shard with the emulated decoder over gloo and rank 0 prints one
    line with n_gpus == 2."""
    import json
    import subprocess
    import sys

    import bench
    from helpers import oracle_front
    from srsue_amd import abi
    total = 6
    llrs = {"total": np.array(total)}
    for g in range(total):
        c = abi.sf_cfg(cell_id=1, nof_prb=6, nof_ports=1, sf_idx=bench.SF_CYCLE[g % 8], tbs=4392, Qm=6)
        iq = abi.tx_subframe(c, bench.tb_payload(g, c.tbs // 8), snr_db=30.0, seed=0xA5A5 + g)
        llrs[f"llr{g}"] = oracle_front(c, iq)[3]
    path = tmp_path / "llr.npz"
    np.savez(path, **llrs)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run-llr", str(path),
                          "--cpu-seconds", "1.5"], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1                                   # only rank 0 prints
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["subframes"] == total and r["crc_ok"] == total
    # the line's statistics are global (both ranks' TBs), with each rank's elapsed time
    assert r["crc_ok_rate"] == 1.0 and r["mean_turbo_iterations"] == 1.0 and r["payload_mismatches"] == 0
    assert len(r["elapsed_per_rank_s"]) == 2 and r["elapsed_max_s"] == max(r["elapsed_per_rank_s"])
    assert [s[:2] for s in r["shards"]] == [[0, 3], [3, 3]]  # contiguous shards
    assert all(s[2] == s[1] for s in r["shards"])           # every TB equals the transmitted bytes
    # the N-rank line is complete: rank 0's CPU baseline and every rank's device identity
    assert r["cpu_baseline"]["value"] > 0 and r["cpu_baseline"]["cores"] >= 1 and r["cpu_baseline"]["kind"] == "port"
    assert [d["rank"] for d in r["rank_devices"]] == [0, 1]


def test_bench_rejects_world_mismatch(built):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu(built):
    """The N-rank launch on real hardware: `bench.py --gpus 2 --share-gpu` spawns two ranks that each decode
    their contiguous shard with the HIP kernels on GPU 0, synchronise and reduce over gloo (the one-GPU box has
    no second card for RCCL); rank 0 prints one line with n_gpus 2, the two shards' total and every TB
    decoded (crc_ok_rate 1.0, no payload mismatch).  The rate is not a scaling figure (the ranks share a card)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--share-gpu", "--sf-per-gpu",
                        "256", "--steps", "2", "--warmup", "1", "--cpu-seconds", "1.5", "--iterating-snr", "0"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["share_gpu_rehearsal"] is True
    assert d["config"]["subframes_per_gpu"] == 256
    assert d["crc_ok_rate"] == 1.0 and d["payload_mismatches_crc_ok"] == 0
    # global statistics: both ranks' subframes, each rank's elapsed time, value from the max of them
    assert d["subframes_all_ranks"] == 512 and d["mean_turbo_iterations"] == 1.0
    per = d["elapsed_per_rank_s"]
    assert len(per) == 2 and abs(d["ms_per_step"] - max(per) / 2 * 1e3) < 1e-2
    assert abs(d["value"] - 512 * 75376 * 2 / max(per) / 1e6) < 1e-3 * d["value"]
    # the N-rank line carries rank 0's CPU baseline and each rank's device identity (here: both on the one card)
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["kind"] == "port"
    devs = d["rank_devices"]
    assert [x["rank"] for x in devs] == [0, 1] and all(x["pci_bus_id"] and x["device"] for x in devs)
    assert len({x["pci_bus_id"] for x in devs}) == 1       # --share-gpu: one card


@pytest.mark.gpu
def test_bench_rccl_process_group_one_rank(built):
    """The RCCL side of the N-GPU line on a one-GPU box: one rank launched as torch.distributed.run launches each
    of the driver's ranks (WORLD_SIZE / RANK / LOCAL_RANK / MASTER_* in its environment), `--pg` bringing up the
    `nccl` process group with device_id; the timing barriers, the float64 all-reduces of elapsed time and counters on
    the card, and the device gather (all_gather_object) then run over RCCL exactly as at N = 8."""
    import json
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--pg", "--sf-per-gpu", "256", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline", "--iterating-snr", "0", "--plan-steps", "0",
                        "--h2d-steps", "0"], cwd=root, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.splitlines()   # RCCL's version banner goes to stderr (bench.py keep_stdout_clean)
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[:500]
    d = json.loads(lines[0])
    assert d["config"]["process_group"] == "nccl" and d["n_gpus"] == 1
    assert d["crc_ok_rate"] == 1.0 and d["payload_mismatches_crc_ok"] == 0 and d["subframes_all_ranks"] == 256
    per = d["elapsed_per_rank_s"]
    assert len(per) == 1 and abs(d["ms_per_step"] - per[0] / 2 * 1e3) < 1e-2
    devs = d["rank_devices"]
    assert len(devs) == 1 and devs[0]["rank"] == 0 and devs[0]["pci_bus_id"]


@pytest.mark.gpu
def test_bench_one_stream_full_line(built):
    """`bench.py --streams 1` (serial, the profiling runs' setting) prints the whole line: the planning block's
    static replay of two grant lists needs one workspace per list even on one stream (bench.py replan_steps), and
    the PCIe-inclusive h2d block runs beside it.  A small shard keeps it short."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--sf-per-gpu", "256", "--steps", "4",
                        "--warmup", "1", "--streams", "1", "--no-cpu-baseline", "--iterating-snr", "0",
                        "--plan-steps", "4", "--h2d-steps", "2"],
                       cwd=root, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["config"]["streams"] == 1 and d["crc_ok_rate"] == 1.0 and d["payload_mismatches_crc_ok"] == 0
    pl = d["planning"]
    for k in ("pipelined_default", "varied_static", "pipelined_varied"):
        assert pl[k]["payload_mismatches_crc_ok"] == 0 and pl[k]["Mbps"] > 0, k
    assert all(b > 0 for b in pl["varied_static"]["crc_ok_bits_per_list"])
    assert set(d["h2d"]) >= {"sc16", "fc32"}


def test_native_stdout_prints_kept_off_the_line():
    """bench.py keep_stdout_clean / emit: once the nccl process group is about to start, whatever native code
    writes to file descriptor 1 (RCCL's version banner) lands on stderr, and stdout carries only the JSON line."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import os, sys; sys.path.insert(0, %r); import bench; print('before'); bench.keep_stdout_clean(); "
            "os.write(1, b'RCCL version : x\\n'); print('python noise'); bench.emit({'metric': 'm', 'value': 1.5})"
            % root)
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.splitlines() == ["before", json.dumps({"metric": "m", "value": 1.5})]
    assert "RCCL version" in r.stderr and "python noise" in r.stderr


def _dry_worker(rank, world, port, q):
    """One rank of the N-GPU line's host side over gloo: its shard of configs[3]'s 100,000
    subframes, the reduce of its counters, the hardware-queue setting it would run with under RCCL, and its place in
    the gathered device list."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    first, n = bench.shard_range(100000, rank, world)
    # counters: the shard's subframes, its CRC-OK bits at MCS 28, code blocks (13 per subframe), a rank tag
    t, sums, per = bench.reduce_over_ranks(0.25 * (rank + 1), [n, n * 75376, 13 * n, rank + 1], world)
    env = {"WORLD_SIZE": str(world), "RANK": str(rank), "LOCAL_RANK": str(rank)}
    queues = (bench.hw_queues_arg([], env), bench.hw_queues_arg(["--share-gpu"], env))
    devs = bench.rank_devices(world, None)
    q.put((rank, first, n, t, sums, per, queues, [d["rank"] for d in devs]))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [4, 8])
def test_n_rank_dry_run(world):
    """The host side of `bench.py --gpus N` at the driver's rank counts over gloo (no GPU): contiguous shards of
    100,000 subframes cover every subframe once; reduce_over_ranks sums every counter and returns the max and every
    rank's elapsed time; each rank would run 16 HIP hardware queues under RCCL (8 sharing a GPU), within gpurun's
    32; rank_devices is gathered in rank order."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dry_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    spans = [(r[1], r[2]) for r in res]
    assert spans[0][0] == 0 and sum(n for _, n in spans) == 100000
    assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    assert all(n == 100000 // world for _, n in spans)           # 12,500 per GPU at N = 8
    for r in res:
        assert r[3] == 0.25 * world                               # max over ranks
        assert r[4] == [100000.0, 100000.0 * 75376, 1300000.0, world * (world + 1) / 2]
        assert r[5] == [0.25 * (k + 1) for k in range(world)]     # in rank order
        assert r[6] == ("16", "8") and int(r[6][0]) <= 32
        assert r[7] == list(range(world))


def test_rank_hbm_budget_configs3():
    """Each rank's HBM at configs[3]'s per-GPU shard: the bench keeps 4 workspaces of 12,500 subframes
    (one per stream) plus the IQ buffer; mi_dl_plan_device_bytes (host only) sizes a workspace.  They fit the
    MI355X's 288 GB with room, and the LLR stream is not allocated on the default fused path."""
    import bench
    from srsue_amd import abi
    first, n = bench.shard_range(100000, 7, 8)
    p = abi.Plan().build([bench.make_cfg(first + i) for i in range(n)])
    ws = p.device_bytes()
    assert p.device_bytes(keep_llr=True) - ws == n * 90000 * 4   # the LLR stream: 360 KB per subframe
    iq = n * 30720 * 8
    total = 4 * ws + iq
    assert total < 0.75 * 288e9, total / 1e9
    p.close()
