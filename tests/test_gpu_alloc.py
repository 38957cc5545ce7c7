"""GPU parity for partial PDSCH allocations and the BASELINE configs[4] mix, and an at-scale property test.

1. One batch over 6/15/25/50/75/100-PRB cells (TM1 and TM2) with the allocations srsUE receives in DCIs
   (phch_worker.cc:297): type-0 RBG masks, 1A localized RIVs with L_PRB < N_PRB and distributed VRBs
   (different PRBs per slot, 36.211 6.2.3.2), MCS 0..28 (QPSK / 16QAM / 64QAM, TBS from 36.213 Table
   7.1.7.2.1-1), sync / PBCH subframes included.  The ORACLE transmitter (oracle/o_tx.c) generates the IQ.
   LLRs within 1e-4 (max abs error over the RMS of the oracle's), payload, TB CRC and turbo iterations
   bit-exact against the oracle's decode of the same IQ.
2. The headline shape at scale: 12,500 subframes of 20 MHz TM1 MCS-28 in ONE batch (13 code blocks each,
   5,080 wavefronts of the crossed recompute-form turbo kernel -- the schedule the bench runs), IQ tiled
   from a pool of distinct subframes; every TB must pass CRC and equal its transmitted bytes.
LLR/grid parity is against the oracle restatement (srsLTE is absent: parity unpinned); TB bits are
pinned by the transmitted ground truth."""
import ctypes as C
import random

import numpy as np
import pytest
import torch

import oracle_lib as O
from helpers import oracle_dlsch, oracle_front, rel_err, tb_bytes
from srsue_amd import abi

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert torch.cuda.is_available()


def _mcs(m):
    return (2, m) if m <= 9 else (4, m - 1) if m <= 16 else (6, m - 2)


def _mask(N, kind, rnd):
    """two-slot PRB mask (bit s = used in slot s) of one random allocation of the given kind"""
    m = np.zeros(110, np.uint8)
    if kind == "type0":
        P = O.lib().or_rbg_size(N)
        nrbg = -(-N // P)
        bits = rnd.randint(1, (1 << nrbg) - 1)
        for g in range(nrbg):
            if (bits >> (nrbg - 1 - g)) & 1:
                m[g * P:min(N, g * P + P)] = 3
    elif kind == "local":
        L = rnd.randint(1, N - 1)
        s = rnd.randint(0, N - L)
        m[s:s + L] = 3
    else:
        gap2 = int(N >= 50 and rnd.random() < 0.5)
        nv = O.lib().or_nvrb_dist(N, gap2)
        L = rnd.randint(1, min(nv, 16))
        s = rnd.randint(0, nv - L)
        for n in range(s, s + L):
            for slot in (0, 1):
                m[O.lib().or_vrb_to_prb(N, gap2, n, slot)] |= 1 << slot
    return m


def _mix(seed, n):
    rnd = random.Random(seed)
    out = []
    cells = [(6, 1, 301), (15, 2, 7), (25, 1, 11), (50, 2, 2), (75, 1, 5), (100, 1, 1), (100, 2, 3)]
    for i in range(n):
        N, ports, cid = cells[i % len(cells)]
        kind = ("type0", "local", "dist")[i % 3]
        m = _mask(N, kind, rnd)
        nprb = int(np.count_nonzero(m[:N] & 1))
        for _ in range(50):
            mcs = rnd.randint(0, 28)
            qm, itbs = _mcs(mcs)
            tbs = abi.lib().srslte_ra_tbs_from_idx(itbs, nprb)
            cfg = abi.sf_cfg(cell_id=cid, nof_prb=N, nof_ports=ports, sf_idx=rnd.randint(0, 9), cfi=rnd.randint(1, 3),
                             tbs=tbs, Qm=qm, rnti=0x46 + i, prb=m)
            G = abi.lib().mi_pdsch_G(C.byref(cfg))
            if G > 0 and tbs + 24 < 0.85 * G:    # a decodable code rate at 30 dB
                break
        out.append(cfg)
    return out


def _oracle_tx(cfg, tb, seed):
    cell = O.make_cell(cfg.cell_id, cfg.nof_prb, cfg.nof_ports)
    tc = O.tx_cfg(cell, sf_idx=cfg.sf_idx, cfi=cfg.cfi, rnti=cfg.rnti, tm=cfg.tm, tbs=cfg.tbs, qm=cfg.Qm,
                  prb=np.array(list(cfg.prb_mask), np.uint8), snr_db=30.0, seed=seed)
    return O.tx_subframe(tc, tb)[0]


def _run(cfgs, iqs, **kw):
    b = abi.Batch(cfgs, **kw)
    flat = np.zeros(2 * b.iq_samples, np.float32)
    for i, iq in enumerate(iqs):
        o = 2 * b.iq_offset(i)
        flat[o:o + len(iq)] = iq
    d = torch.from_numpy(flat).cuda()
    b.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return b


@pytest.mark.parametrize("sched", [None, "win", "p2"])
def test_partial_allocations_mixed_cells_match_oracle(sched):
    cfgs = _mix(4, 42)
    tbs = [tb_bytes(700 + i, c.tbs) for i, c in enumerate(cfgs)]
    iqs = [_oracle_tx(c, tb, 0xB000 + i) for i, (c, tb) in enumerate(zip(cfgs, tbs))]
    b = _run(cfgs, iqs, tdec_i16=True, sched=sched, keep_llr=True)
    llr = b.download(abi.BUF_LLR, np.float32)
    pay = b.download(abi.BUF_PAYLOAD, np.uint8)
    crc = b.download(abi.BUF_TB_CRC, np.uint32)
    its = b.download(abi.BUF_TB_ITS, np.uint32)
    n_ok = 0
    for i, c in enumerate(cfgs):
        _, _, _, ollr = oracle_front(c, iqs[i])
        lo = b.offset(abi.BUF_LLR, i)
        assert len(ollr) == abi.lib().mi_pdsch_G(C.byref(c))
        assert rel_err(llr[lo:lo + len(ollr)], ollr) < TOL, f"llr case {i}"
        ok, opay, onoi, _ = oracle_dlsch(c, ollr, i16=True)
        p = b.payload(i, pay)
        assert bool(crc[i]) == ok, f"CRC case {i}"
        assert its[i] == onoi, f"iterations case {i}"
        if ok:
            n_ok += 1
            assert np.array_equal(p, tbs[i]) and np.array_equal(p, opay), f"payload case {i}"
    assert n_ok >= 0.9 * len(cfgs)
    b.close()


@pytest.mark.parametrize("sched", [None, "p2"])
def test_headline_shape_at_scale_every_tb(sched):
    """12,500 x (20 MHz TM1 MCS-28) in one batch: the schedule the bench times (5,080 wavefronts)."""
    n, pool = 12500, 64
    cfgs = [abi.sf_cfg(nof_prb=100, sf_idx=(1, 2, 3, 4, 6, 7, 8, 9)[i % 8], tbs=75376, Qm=6, rnti=0x46)
            for i in range(n)]
    b = abi.Batch(cfgs, max_its=4, tdec_i16=True, sched=sched)
    assert abi.lib().mi_dl_batch_n_codeblocks(b.h) == 13 * n
    assert b.turbo_sched == (sched or b.turbo_sched) and b.turbo_sched in ("lanex", "lanexr", "p2")
    L = 2 * abi.lib().mi_sf_len(100)
    assert b.iq_offset(1) * 2 == L and b.iq_samples * 2 == n * L
    # pool entry j is transmitted with sf_idx of subframe j (pool divides the 8-cycle)
    tbs = [tb_bytes(900 + j, 75376) for j in range(pool)]
    iq_pool = np.stack([abi.tx_subframe(cfgs[j], tbs[j], snr_db=30.0, seed=0xC000 + j) for j in range(pool)])
    d_pool = torch.from_numpy(iq_pool).cuda()
    d = torch.empty((n, L), dtype=torch.float32, device="cuda")
    idx = torch.arange(n, device="cuda") % pool
    d.copy_(d_pool[idx])
    b.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    crc = b.download(abi.BUF_TB_CRC, np.uint32)
    assert crc.all()
    pay = b.download(abi.BUF_PAYLOAD, np.uint8)
    offs = np.array([abi.lib().mi_dl_batch_payload_offset(b.h, i) for i in range(n)], np.int64)
    P = pay[offs[:, None] + np.arange(75376 // 8)[None, :]]
    want = np.stack(tbs)
    for j in range(pool):
        assert (P[j::pool] == want[j]).all(), f"pool entry {j}"
    b.close()
