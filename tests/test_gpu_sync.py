"""GPU: sync front end through the C ABI (mi_sync_*) against the oracle
(oracle/o_sync.c) and transmit-chain ground truth.

Bars: PSS lag and N_ID_2 exact vs the oracle (and vs the applied timing offset at >= 10 dB), rho and
the CFO estimate within 1e-3 of the oracle's (fp32 vs fp64 accumulation over N samples); SSS N_ID_1 /
half frame exact; CFO correction within 1e-4 relative of the oracle's; end to end, a subframe received
with a timing offset and a CFO of 0.3 subcarriers, realigned and corrected on the GPU, decodes (PDSCH CRC
and payload) through the DL chain."""
import ctypes as C

import numpy as np
import pytest
import torch

import oracle_lib as O
from helpers import rel_err, tb_bytes
from srsue_amd import abi
from test_oracle_sync import stream

pytestmark = pytest.mark.gpu

CASES = [(1, 100, 0, 37, 0.11, 10.0), (302, 25, 5, 5, -0.3, 0.0), (77, 6, 0, 0, 0.02, -3.0),
         (155, 50, 5, 120, 0.45, 5.0), (404, 75, 0, 64, -0.2, 12.0)]


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert torch.cuda.is_available()


@pytest.mark.parametrize("case", range(len(CASES)))
def test_pss_sss_cfo_parity(case):
    cell_id, nprb, sf, tau, cfo, snr = CASES[case]
    x, N = stream(cell_id, nprb, sf, tau, cfo, snr, seed=cell_id)
    l6 = O.lib().or_sync_sym_off(N, 6)
    lag0 = max(tau + l6 - 48, 0)
    nlag = 97
    s = abi.Sync(nprb)
    assert s.N == N
    d = torch.from_numpy(x).cuda()
    got = s.pss(d.data_ptr(), [lag0], nlag, 7)[0]
    want = O.pss_find(x[2 * lag0:], nprb, 7, nlag)
    assert got[0] == want[0] and got[1] == want[1], (got, want)
    assert abs(got[2] - want[2]) <= 1e-3 * want[2] and abs(got[3] - want[3]) <= 1e-3, (got, want)
    if snr >= 10:
        assert lag0 + got[1] == tau + l6
    start = lag0 + got[1] - l6
    gs = s.sss(d.data_ptr(), [start], [got[0]], [got[3]])[0]
    y = O.cfo_correct(x[2 * start:2 * (start + 15 * N)], got[3], N)
    ws = O.sss_detect(y, nprb, got[0])
    assert gs[:2] == ws[:2] == (cell_id // 3, int(sf == 5)), (gs, ws)
    out = torch.zeros(2 * 15 * N, dtype=torch.float32, device="cuda")
    s.correct(d.data_ptr(), [start], out.data_ptr(), [0], [got[3]], 15 * N)
    torch.cuda.synchronize()
    assert rel_err(out.cpu().numpy(), y) < 1e-4
    s.close()


def test_sync_then_pdsch_decode():
    """End to end: two subframes (sf 0 with PSS/SSS, then sf 1) of a 20 MHz cell arrive 211 samples late
    with a CFO of 0.3 subcarriers at 25 dB; the GPU finds the PSS, estimates the CFO, detects the cell's
    N_ID_1 / half frame, realigns and corrects both subframes into a batch's IQ buffer, and the DL chain
    decodes both TBs."""
    cfgs = [abi.sf_cfg(cell_id=9, nof_prb=100, sf_idx=0, tbs=61664, Qm=6),
            abi.sf_cfg(cell_id=9, nof_prb=100, sf_idx=1, tbs=75376, Qm=6)]
    tbs = [tb_bytes(300 + i, c.tbs) for i, c in enumerate(cfgs)]
    sig = []
    for i, c in enumerate(cfgs):
        iq = abi.tx_subframe(c, tbs[i], snr_db=300.0, seed=i)
        abi.tx_sync(9, 100, c.sf_idx, iq)
        sig.append(iq)
    sig = np.concatenate(sig)
    N, tau, cfo = 2048, 211, 0.3
    z = np.zeros(len(sig) // 2 + 2 * tau, np.complex64)
    z[tau:tau + len(sig) // 2] = sig[0::2] + 1j * sig[1::2]
    n = np.arange(len(z))
    rng = np.random.default_rng(5)
    z = z * np.exp(2j * np.pi * cfo * n / N) + (rng.normal(0, 1, z.shape) + 1j * rng.normal(0, 1, z.shape)) * np.sqrt(
        10 ** -2.5 / 2)
    x = np.zeros(2 * len(z), np.float32)
    x[0::2], x[1::2] = z.real, z.imag
    d = torch.from_numpy(x).cuda()
    s = abi.Sync(100)
    l6 = O.lib().or_sync_sym_off(N, 6)
    nid2, lag, rho, est = s.pss(d.data_ptr(), [0], 2 * tau + l6 + 64, 7)[0]
    assert nid2 == 9 % 3 and lag == tau + l6 and abs(est - cfo) < 0.05
    start = lag - l6
    nid1, sf5, _ = s.sss(d.data_ptr(), [start], [nid2], [est])[0]
    assert (nid1, sf5) == (9 // 3, 0)
    b = abi.Batch(cfgs, max_its=4)
    dst = torch.zeros(2 * b.iq_samples, dtype=torch.float32, device="cuda")
    L = 15 * N
    # each subframe is corrected with its own phase origin (the receiver's per-subframe convention)
    s.correct(d.data_ptr(), [start, start + L], dst.data_ptr(), [b.iq_offset(0), b.iq_offset(1)], [est, est], L)
    b.run(dst.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    crc = b.download(abi.BUF_TB_CRC, np.uint32)
    pay = b.download(abi.BUF_PAYLOAD, np.uint8)
    for i in range(2):
        assert crc[i] == 1 and np.array_equal(b.payload(i, pay), tbs[i])
    s.close()


class SrsCell(C.Structure):
    _fields_ = [("nof_prb", C.c_uint32), ("nof_ports", C.c_uint32), ("bw_idx", C.c_uint32), ("id", C.c_uint32),
                ("cp", C.c_int), ("phich_length", C.c_int), ("phich_resources", C.c_int)]


class Timestamp(C.Structure):
    _fields_ = [("full_secs", C.c_long), ("frac_secs", C.c_double)]


RECV = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(Timestamp))


def test_srslte_ue_sync_tracking_srsue_call_order():
    """srslte_ue_sync_* as srsUE's sync thread calls it (phch_recv.cc:108-120, 236, 321-330): a
    receive callback streams 24 subframes (sf 0..9 cycling, PSS/SSS on 0 and 5, a PDSCH TB in each)
    that arrive 1,111 samples late with a CFO of 0.2 subcarriers (3 kHz) at 25 dB.  The first zerocopy
    finds the cell (returns 0); every later one delivers the next subframe with the right subframe
    index, the CFO estimate converges to 3 kHz and each delivered subframe decodes through the DL chain."""
    L = abi.lib()
    L.srslte_ue_sync_init.restype = C.c_int
    L.srslte_ue_sync_init.argtypes = [C.c_void_p, SrsCell, RECV, C.c_void_p]
    L.srslte_ue_sync_zerocopy.argtypes = [C.c_void_p, C.c_void_p]
    L.srslte_ue_sync_get_sfidx.argtypes = [C.c_void_p]
    L.srslte_ue_sync_get_sfidx.restype = C.c_uint32
    L.srslte_ue_sync_get_cfo.argtypes = [C.c_void_p]
    L.srslte_ue_sync_get_cfo.restype = C.c_float
    L.srslte_ue_sync_get_last_timestamp.argtypes = [C.c_void_p, C.POINTER(Timestamp)]
    L.srslte_ue_sync_free.argtypes = [C.c_void_p]
    cell_id, N, tau, cfo = 9, 2048, 1111, 0.2
    cfgs, tbs, sig = [], [], []
    for i in range(24):
        c = abi.sf_cfg(cell_id=cell_id, nof_prb=100, sf_idx=i % 10, tbs=61664 if i % 10 in (0, 5) else 75376, Qm=6)
        tb = tb_bytes(400 + i, c.tbs)
        iq = abi.tx_subframe(c, tb, snr_db=300.0, seed=i)
        abi.tx_sync(cell_id, 100, c.sf_idx, iq)
        cfgs.append(c)
        tbs.append(tb)
        sig.append(iq)
    sig = np.concatenate(sig)
    z = np.zeros(len(sig) // 2 + tau, np.complex64)
    z[tau:] = sig[0::2] + 1j * sig[1::2]
    n = np.arange(len(z))
    rng = np.random.default_rng(17)
    z = z * np.exp(2j * np.pi * cfo * n / N) + (rng.normal(0, 1, z.shape) + 1j * rng.normal(0, 1, z.shape)) * np.sqrt(
        10 ** -2.5 / 2)
    stream_iq = np.zeros(2 * len(z), np.float32)
    stream_iq[0::2], stream_iq[1::2] = z.real, z.imag
    state = {"pos": 0}

    def recv(h, data, nsamples, ts):
        p = state["pos"]
        if p + nsamples > len(z):
            return -1
        C.memmove(data, stream_iq[2 * p:].ctypes.data, nsamples * 8)
        ts.contents.full_secs, ts.contents.frac_secs = 0, p / 30.72e6
        state["pos"] = p + nsamples
        return nsamples

    cb = RECV(recv)
    q = C.create_string_buffer(512)
    assert L.srslte_ue_sync_init(q, SrsCell(100, 1, 0, cell_id, 0, 0, 2), cb, None) == 0
    buf = np.zeros(2 * 15 * N, np.float32)
    assert L.srslte_ue_sync_zerocopy(q, buf.ctypes.data) == 0          # FIND
    got = []
    for k in range(12):
        assert L.srslte_ue_sync_zerocopy(q, buf.ctypes.data) == 1
        sf = L.srslte_ue_sync_get_sfidx(q)
        ts = Timestamp()
        L.srslte_ue_sync_get_last_timestamp(q, C.byref(ts))
        got.append((sf, buf.copy(), ts.frac_secs))
    # the stream starts with subframe 0 after tau samples: FIND aligns to the first PSS it sees
    first = round((got[0][2] * 30.72e6 - tau) / (15 * N))
    for k, (sf, _, t) in enumerate(got):
        assert sf == (first + k) % 10
        assert abs(t * 30.72e6 - (tau + (first + k) * 15 * N)) <= 2     # delivered at the true boundary
    assert abs(L.srslte_ue_sync_get_cfo(q) - 15000 * cfo) < 750
    dec = [(first + k, g[1]) for k, g in enumerate(got)][-6:]
    b = abi.Batch([cfgs[i] for i, _ in dec], max_its=4)
    dst = np.zeros(2 * b.iq_samples, np.float32)
    for j, (_, x) in enumerate(dec):
        dst[2 * b.iq_offset(j):2 * b.iq_offset(j) + len(x)] = x
    d = torch.from_numpy(dst).cuda()
    b.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    crc = b.download(abi.BUF_TB_CRC, np.uint32)
    pay = b.download(abi.BUF_PAYLOAD, np.uint8)
    for j, (i, _) in enumerate(dec):
        assert crc[j] == 1 and np.array_equal(b.payload(j, pay), tbs[i]), j
    L.srslte_ue_sync_free(q)
