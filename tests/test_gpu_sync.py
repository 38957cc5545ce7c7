"""GPU: sync front end through the C ABI (mi_sync_*) against the oracle
(oracle/o_sync.c) and transmit-chain ground truth.

Bars: PSS lag and N_ID_2 exact vs the oracle (and vs the applied timing offset at >= 10 dB), rho and
the CFO estimate within 1e-3 of the oracle's (fp32 vs fp64 accumulation over N samples); SSS N_ID_1 /
half frame exact; CFO correction within 1e-4 relative of the oracle's; end to end, a subframe received
with a timing offset and a CFO of 0.3 subcarriers, realigned and corrected on the GPU, decodes (PDSCH CRC
and payload) through the DL chain."""
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
