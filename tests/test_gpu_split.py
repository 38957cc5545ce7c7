"""Split runs (mi_dl_batch_run_split) against whole runs: the bench's split stream layout -- each workspace's front end
(OFDM, channel estimation, fused demap + rate de-matching) on a stream of a quarter of the CUs, its turbo decoder and TB
CRC on a stream of the other three quarters (mi_stream_create_cu_share) -- must give every run exactly the results of a
whole run (mi_dl_batch_run) of the same IQ: TB CRC, TB and per-code-block iterations, payload.

Two workspaces run three steps each, issued round-robin with no host synchronisation, on two alternating IQ sets, in
the turbo waterfall (16-25 dB: continuation rounds run): each run's outputs are copied to host memory on its back-end
stream right behind it, so a run whose back end overlapped the next front end of its workspace (the ordering the batch's
events impose) would show as a mismatch in that run's copy, not just in the last one.  Then each workspace's next front
end runs on a third stream without synchronisation (mi_dl_batch_run_stages): it must wait for the last split back end
too, and its back end must complete the step like a whole run.

Anchor: srsUE's srslte_pdsch_decode_rnti (reference ue/src/phy/phch_worker.cc:347-348) per subframe, as every batch run.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from helpers import tb_bytes
from srsue_amd import abi

pytestmark = pytest.mark.gpu

SF_CYCLE = (1, 2, 3, 4, 6, 7, 8, 9)
TBS, NCB = 75376, 13
FRONT = (1 << 0) | (1 << 1) | (1 << 2) | (1 << 3)   # OFDM, CHEST, DEMAP, RM (MI_DL_STAGE_*)
BACK = (1 << 4) | (1 << 5)                          # TDEC, TB


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert torch.cuda.is_available()


def hip_lib():
    """The HIP runtime this process loaded (torch, libsrsue_amd), found by its path in /proc/self/maps."""
    with open("/proc/self/maps") as f:
        for line in f:
            p = line.split()[-1]
            if "libamdhip64.so" in p:
                return C.CDLL(p)
    raise RuntimeError("libamdhip64 not loaded")


def test_split_runs_match_whole_runs():
    hip = hip_lib()
    simds = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    pool = 40
    n = -(-(-(-simds * 64 // NCB)) // pool) * pool            # the packed decoder's schedule (bench config)
    pcfgs = [abi.sf_cfg(nof_prb=100, sf_idx=SF_CYCLE[j % 8], tbs=TBS, Qm=6, rnti=0x46) for j in range(pool)]
    iqs = [abi.tx_subframe(c, tb_bytes(9100 + j, TBS), snr_db=16.0 + 9.0 * j / (pool - 1), seed=0xE000 + j)
           for j, c in enumerate(pcfgs)]
    cfgs = [pcfgs[i % pool] for i in range(n)]
    L = 2 * abi.lib().mi_sf_len(100)
    d_pool = torch.from_numpy(np.stack(iqs)).cuda()
    # IQ set 0: subframe i carries pool entry i % pool; set 1: entry (i + 8) % pool -- another TB and SNR under the same
    # grant (the entries' sf_idx cycles with period 8, and the batch's cfgs are fixed)
    idx = torch.arange(n, device="cuda")
    d_iq = [torch.empty((n, L), dtype=torch.float32, device="cuda") for _ in range(2)]
    d_iq[0].copy_(d_pool[idx % pool])
    d_iq[1].copy_(d_pool[(idx + 8) % pool])
    del d_pool
    bufs = ((abi.BUF_TB_CRC, np.uint32), (abi.BUF_TB_ITS, np.uint32), (abi.BUF_CB_ITS, np.uint32),
            (abi.BUF_PAYLOAD, np.uint8))

    # whole runs, one at a time
    ref = []
    b = abi.Batch(cfgs, max_its=4, tdec_i16=True, compact_ce=True)
    assert b.turbo_sched == "p2", b.turbo_sched
    for s in range(2):
        b.run(d_iq[s].data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ref.append([b.download(w, t) for w, t in bufs])
    b.close()
    crc0 = ref[0][0][:n]
    assert 0 < crc0.sum() < n and ref[0][2][:NCB * n].max() >= 3, "the waterfall must be exercised"
    assert not all(np.array_equal(x, y) for x, y in zip(ref[0], ref[1]))

    # split runs: two workspaces, three steps each, round-robin, outputs copied behind each run on its back stream
    S, steps = 2, 6
    ws = [abi.Batch(cfgs, max_its=4, tdec_i16=True, compact_ce=True) for _ in range(S)]
    fr = [abi.stream_cu_share(0, 2) for _ in range(S)]
    bk = [abi.stream_cu_share(2, 6) for _ in range(S)]
    pinned, caps, sets = [], [], []
    hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    try:
        for j in range(steps):
            k, s = j % S, (j // S + j % S) % 2
            ws[k].run_split(d_iq[s].data_ptr(), fr[k], bk[k])
            cap = []
            for w, t in bufs:
                nb = abi.lib().mi_dl_batch_bytes(ws[k].h, w)
                h = abi.lib().mi_host_alloc(nb)
                assert h, "pinned allocation"
                pinned.append(h)
                dev = abi.lib().mi_dl_batch_device_ptr(ws[k].h, w)
                assert hip.hipMemcpyAsync(h, dev, nb, 2, bk[k]) == 0   # hipMemcpyDeviceToHost, on the back stream
                cap.append(np.ctypeslib.as_array((C.c_uint8 * nb).from_address(h)).view(t))
            caps.append(cap)
            sets.append(s)
        # then, without synchronisation, the front end of another step of each workspace on a third stream: it rewrites
        # the softbuffer its last split run's back end reads, so it must wait for that back end (the batch orders every
        # run after a pending split back end) -- or the captures of runs steps - S .. steps - 1 would not match
        other = abi.stream_cu_share(0, 8)
        fr.append(other)
        nxt = [1 - sets[steps - S + k] for k in range(S)]
        for k in range(S):
            ws[k].run_stages(FRONT, d_iq[nxt[k]].data_ptr(), other)
        assert hip.hipDeviceSynchronize() == 0
        for j in range(steps):
            for (w, _), got, exp in zip(bufs, caps[j], ref[sets[j]]):
                assert np.array_equal(got, exp), f"split run {j} (workspace {j % S}, IQ set {sets[j]}): buffer {w}"
        # and its back end completes that step like a whole run
        for k in range(S):
            ws[k].run_stages(BACK, None, other)
            for w, t in bufs:
                assert np.array_equal(ws[k].download(w, t), ref[nxt[k]][[x for x, _ in bufs].index(w)]), \
                    f"workspace {k}: the step after the split runs, buffer {w}"
    finally:
        hip.hipDeviceSynchronize()
        for h in pinned:
            abi.lib().mi_host_free(h)
        for st in fr + bk:
            abi.stream_destroy(st)
        for b in ws:
            b.close()
