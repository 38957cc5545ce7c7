"""GPU: the UL PUSCH transmitter (include/mi_ul.h, srsue_amd/csrc/ul.hip) against the
oracle's UL chain (oracle/o_ul.c): the multiplexed coded symbols (CQI + rate-matched data) bit-exact with
or_ulsch_encode, HARQ-ACK / RI / CQI on PUSCH (36.212 5.2.2.6-5.2.2.8) through the IQ check, and the
SC-FDMA IQ within 1e-4 (RMS-relative) of or_pusch_encode (double precision) -- over QPSK/16QAM/64QAM,
every redundancy version, K-/K+ segmentation with filler bits, single code blocks (CRC24A only), partial
allocations, group / sequence hopping, cyclic shifts, and 1.4-20 MHz cells in one batch."""
import ctypes as C

import numpy as np
import pytest
import torch

import oracle_lib as O
from srsue_amd import abi

pytestmark = pytest.mark.gpu
TOL = 1e-4

CASES = [  # nof_prb, n_prb, L_prb, tbs, Qm, rv, sf, cell, gh, sh, dss, cs, n2 [, ack_len, ack, I_offset_ack [, n_prb1]]
    (100, 0, 100, 39232, 4, 0, 1, 1, 0, 0, 0, 0, 0),     # 20 MHz full band, 16QAM (MCS 20)
    (100, 10, 75, 25456, 6, 2, 4, 7, 0, 1, 3, 2, 5),     # 64QAM, rv 2, sequence hopping
    (50, 5, 24, 5736, 2, 1, 7, 33, 1, 0, 0, 7, 3),       # group hopping, rv 1
    (25, 0, 3, 512, 2, 0, 0, 301, 0, 0, 0, 1, 1),        # L = 3 (smallest ZC DMRS), C = 1, 8 filler bits
    (25, 7, 1, 104, 2, 0, 3, 17, 0, 0, 0, 2, 1),         # L = 1: tabulated 12-point DMRS (36.211 5.5.1.2-1)
    (50, 12, 2, 256, 4, 1, 6, 88, 1, 0, 2, 5, 3),        # L = 2: tabulated 24-point DMRS, group hopping, rv 1
    (6, 0, 1, 56, 2, 0, 9, 29, 0, 0, 0, 0, 0, 1, 1, 5),  # L = 1 with HARQ-ACK (Msg3-sized grant)
    (6, 1, 5, 600, 4, 3, 9, 2, 1, 0, 29, 4, 6),          # 1.4 MHz, rv 3
    (75, 30, 45, 12216, 4, 0, 5, 11, 0, 1, 0, 3, 0),     # N = 1536
    (15, 0, 15, 4008, 6, 0, 2, 12, 0, 0, 0, 0, 2),       # 3 MHz, N = 256
    (100, 0, 100, 43816, 4, 0, 3, 1, 0, 0, 0, 0, 0, 1, 1, 5),    # HARQ-ACK on PUSCH: 1 bit (ACK)
    (25, 2, 20, 3000, 2, 1, 8, 4, 1, 0, 0, 2, 1, 2, 2, 12),      # 2 ACK bits, QPSK, rv 1, hopping
    (50, 0, 45, 9000, 6, 0, 6, 5, 0, 1, 0, 0, 4, 1, 0, 14),      # NACK, 64QAM, largest beta_offset
    (25, 0, 3, 104, 2, 0, 2, 9, 0, 0, 0, 0, 0, 2, 3, 14),        # Q'_ACK capped at 4 M (tiny TB), filler bits
    (100, 2, 48, 12216, 4, 0, 5, 3, 0, 0, 0, 1, 0, 0, 0, 0, 50),  # frequency hopping: slot 1 at PRB 50
    (50, 30, 20, 5736, 6, 1, 7, 8, 1, 0, 0, 2, 6, 1, 1, 9, 4),   # hopping down to PRB 4, ACK, group hopping
    # UCI on PUSCH (36.212 5.2.2.6): srsUE's 4-bit wideband CQI (phch_worker.cc:507-523) with and without ACK,
    # RI 1 / 2 bits, a long CQI report (CRC8 + convolutional code), CQI capped by the allocation, hopping
    (100, 0, 100, 39232, 4, 0, 1, 1, 0, 0, 0, 0, 0, dict(cqi=[1, 0, 1, 1], cqi_ioff=9)),
    (25, 2, 20, 3000, 2, 1, 8, 4, 1, 0, 0, 2, 1, 1, 1, 7, dict(cqi=[0, 1, 1, 0], cqi_ioff=15, ri_len=1, ri=1,
                                                                ri_ioff=12)),
    (50, 0, 45, 9000, 6, 0, 6, 5, 0, 1, 0, 0, 4, 2, 2, 14, dict(ri_len=2, ri=3, ri_ioff=6)),
    (100, 4, 90, 25456, 6, 2, 4, 7, 0, 1, 3, 2, 5, dict(cqi=[1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 1, 0, 1, 1, 0,
                                                            1, 0, 0, 1, 1, 1, 0], cqi_ioff=12, ri_len=1, ri=0)),
    (6, 0, 6, 1000, 4, 0, 3, 2, 0, 0, 0, 1, 2, 1, 0, 3, dict(cqi=[1] * 11, cqi_ioff=15, ri_len=2, ri=2,
                                                               ri_ioff=12)),
    (15, 0, 15, 328, 2, 0, 2, 12, 0, 0, 0, 0, 2, 0, 0, 0, dict(cqi=[1, 0, 0, 1, 1, 0, 1, 0, 0, 0, 1, 1, 1, 0] * 3,
                                                                 cqi_ioff=15)),   # Q'_CQI at its cap
    (100, 2, 48, 12216, 4, 0, 5, 3, 0, 0, 0, 1, 0, 1, 1, 5, 50, dict(cqi=[0, 0, 1, 1], cqi_ioff=7, ri_len=1, ri=1,
                                                                     ri_ioff=3)),
]


def mk(c):
    extra = c[-1] if isinstance(c[-1], dict) else {}
    c = c[:-1] if extra else c
    nof_prb, n_prb, L, tbs, Qm, rv, sf, cell, gh, sh, dss, cs, n2 = c[:13]
    ack_len, ack, ioff = c[13:16] if len(c) > 13 else (0, 0, 0)
    n1 = c[16] if len(c) > 16 else None      # slot-1 start PRB (frequency hopping)
    return dict(cell_id=cell, nof_prb=nof_prb, sf_idx=sf, rnti=0x46 + sf, n_prb=n_prb, L_prb=L, tbs=tbs, Qm=Qm, rv=rv,
                gh=gh, sh=sh, dss=dss, cs=cs, n2=n2, ack_len=ack_len, ack=ack, ioff=ioff, n_prb1=n1, **extra)


def tb_of(i, tbs):
    return np.random.default_rng(1000 + i).integers(0, 256, tbs // 8, dtype=np.uint8)


def oracle_symbols(oc, tb):
    """the multiplexed sequence g (CQI then data, 36.212 5.2.2.7) as Qm-bit symbols, then zeros for the
    Q'_RI cells (the layout of mi_ul_batch_symbols)"""
    G = O.lib().or_pusch_G(C.byref(oc))
    f = np.zeros(G, np.uint8)
    H = O.lib().or_ulsch_encode(C.byref(oc), tb, f)
    assert H == G - O.lib().or_ri_qprime(C.byref(oc)) * oc.Qm
    Qm = oc.Qm
    w = (1 << np.arange(Qm - 1, -1, -1)).astype(np.uint32)
    return (f.reshape(-1, Qm).astype(np.uint32) @ w).astype(np.uint8)


def oracle_iq(oc, tb):
    N = {6: 128, 15: 256, 25: 512, 50: 1024, 75: 1536, 100: 2048}[oc.nof_prb]
    iq = np.zeros(2 * 15 * N, np.float32)
    assert O.lib().or_pusch_encode(C.byref(oc), tb, iq) == 0
    return iq


def rel_err(a, b):
    return float(np.sqrt(np.mean((a - b) ** 2)) / np.sqrt(np.mean(b ** 2)))


@pytest.fixture(scope="module")
def encoded(built):
    cfgs = [abi.ul_cfg(**mk(c)) for c in CASES]
    b = abi.UlBatch(cfgs)
    pay = np.zeros(b.payload_bytes, np.uint8)
    tbs = []
    for i, c in enumerate(cfgs):
        tb = tb_of(i, c.tbs)
        o = b.payload_offset(i)
        pay[o:o + len(tb)] = tb
        tbs.append(tb)
    d_pay = torch.from_numpy(pay).cuda()
    d_iq = torch.zeros(2 * b.iq_samples, dtype=torch.float32, device="cuda")
    b.run(d_pay.data_ptr(), d_iq.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return b, cfgs, tbs, d_iq.cpu().numpy()


@pytest.mark.parametrize("i", range(len(CASES)))
def test_coded_symbols_bit_exact(encoded, i):
    b, cfgs, tbs, _ = encoded
    oc = O.ul_cfg(**mk(CASES[i]))
    assert np.array_equal(b.symbols(i), oracle_symbols(oc, tbs[i]))


@pytest.mark.parametrize("i", range(len(CASES)))
def test_scfdma_iq_matches_oracle(encoded, i):
    b, cfgs, tbs, iq = encoded
    oc = O.ul_cfg(**mk(CASES[i]))
    ref = oracle_iq(oc, tbs[i])
    o = 2 * b.iq_offset(i)
    got = iq[o:o + len(ref)]
    assert rel_err(got, ref) < TOL


def test_ul_batch_reuse_and_streams(built):
    """A second run with other payloads on a side stream overwrites every output sample."""
    cfgs = [abi.ul_cfg(**mk(CASES[0])), abi.ul_cfg(**mk(CASES[3]))]
    b = abi.UlBatch(cfgs)
    s = torch.cuda.Stream()
    d_iq = torch.full((2 * b.iq_samples,), 7.0, dtype=torch.float32, device="cuda")
    for seed in (5, 6):
        pay = np.zeros(b.payload_bytes, np.uint8)
        tbs = []
        for i, c in enumerate(cfgs):
            tb = tb_of(seed * 10 + i, c.tbs)
            pay[b.payload_offset(i):b.payload_offset(i) + len(tb)] = tb
            tbs.append(tb)
        d_pay = torch.from_numpy(pay).cuda()
        torch.cuda.synchronize()
        b.run(d_pay.data_ptr(), d_iq.data_ptr(), s.cuda_stream)
        s.synchronize()
        iq = d_iq.cpu().numpy()
        for i, c in enumerate(cfgs):
            oc = O.ul_cfg(**mk(CASES[[0, 3][i]]))
            ref = oracle_iq(oc, tbs[i])
            o = 2 * b.iq_offset(i)
            assert rel_err(iq[o:o + len(ref)], ref) < TOL
