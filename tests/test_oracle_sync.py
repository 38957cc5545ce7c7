"""CPU: the sync-front-end oracle (oracle/o_sync.c) against 36.211 6.11 properties
and transmit-chain ground truth: a PSS / SSS put on the air at a known timing offset and carrier
frequency offset is found at that lag, with that N_ID_2 / N_ID_1 / half frame, and the CFO estimate
is within 0.05 (10 dB) / 0.12 (<= 5 dB) subcarrier spacings of the applied one."""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
from srsue_amd import abi


def pss(u):
    d = np.zeros(124, np.float32)
    O.lib().or_pss_seq(u, d)
    return d[0::2] + 1j * d[1::2]


def sss(nid1, nid2, sf5):
    d = np.zeros(62, np.float32)
    O.lib().or_sss_seq(nid1, nid2, sf5, d)
    return d


def test_pss_zadoff_chu_properties():
    """|d_u| = 1; roots 29 and 34 are complex conjugates (u + u' = 63); d_25(0) = exp(0)."""
    d = [pss(u) for u in range(3)]
    for x in d:
        assert np.allclose(np.abs(x), 1.0, atol=1e-6)
    assert np.allclose(d[1], np.conj(d[2]), atol=1e-6)
    assert abs(d[0][0] - 1.0) < 1e-6
    # the roots are told apart by time-domain correlation over all lags: test_sync_round_trip


def test_sss_m0_m1_table():
    """36.211 Table 6.11.2.1-1 rows: N_ID_1 0..29 -> (n, n+1), 30 -> (0, 2), 59 -> (0, 3); all 168
    pairs distinct with m0 < m1."""
    def mm(n):
        a, b = C.c_uint32(), C.c_uint32()
        O.lib().or_sss_m(n, C.byref(a), C.byref(b))
        return a.value, b.value
    for n in range(30):
        assert mm(n) == (n, n + 1)
    assert mm(30) == (0, 2) and mm(31) == (1, 3) and mm(59) == (0, 3)
    pairs = [mm(n) for n in range(168)]
    assert len(set(pairs)) == 168 and all(a < b for a, b in pairs)


def test_sss_sequences_distinct():
    seqs = {tuple(sss(n1, n2, h)) for n1 in range(168) for n2 in range(3) for h in range(2)}
    assert len(seqs) == 168 * 3 * 2
    assert set(np.unique(sss(17, 2, 1))) == {-1.0, 1.0}


def stream(cell_id, nof_prb, sf, tau, cfo, snr_db, seed):
    """a subframe (product DL TX + oracle PSS/SSS) delayed by tau samples inside a longer buffer, CFO
    applied as exp(+j 2 pi cfo n / N), AWGN"""
    cfg = abi.sf_cfg(cell_id=cell_id, nof_prb=nof_prb, sf_idx=sf, tbs=1000, Qm=2)
    iq = abi.tx_subframe(cfg, np.zeros(cfg.tbs // 8, np.uint8), snr_db=300.0, seed=seed)
    assert O.lib().or_tx_sync(cell_id, nof_prb, sf, 1.0, iq) == 1
    N = O.lib().or_symbol_sz(nof_prb)
    L = len(iq) // 2
    x = np.zeros(2 * (L + 2 * tau + 64), np.float32)
    x[2 * tau:2 * tau + len(iq)] = iq
    n = np.arange(len(x) // 2)
    z = (x[0::2] + 1j * x[1::2]) * np.exp(2j * np.pi * cfo * n / N)
    rng = np.random.default_rng(seed)
    z = z + (rng.normal(0, 1, z.shape) + 1j * rng.normal(0, 1, z.shape)) * np.sqrt(10 ** (-snr_db / 10) / 2)
    out = np.zeros(2 * len(z), np.float32)
    out[0::2], out[1::2] = z.real, z.imag
    return out, N


@pytest.mark.parametrize("cell_id,nof_prb,sf,tau,cfo,snr", [(1, 100, 0, 37, 0.11, 10.0), (302, 25, 5, 5, -0.3, 0.0),
                                                          (77, 6, 0, 0, 0.02, -3.0), (155, 50, 5, 120, 0.45, 5.0)])
def test_sync_round_trip(cell_id, nof_prb, sf, tau, cfo, snr):
    x, N = stream(cell_id, nof_prb, sf, tau, cfo, snr, seed=cell_id)
    l6 = O.lib().or_sync_sym_off(N, 6)
    lag0 = tau + l6 - 48 if tau + l6 >= 48 else 0
    nid2, lag, rho, est = O.pss_find(x[2 * lag0:], nof_prb, 7, 97)
    # the PSS occupies 62 of N subcarriers: its correlation main lobe is ~N / 62 samples wide, so at low
    # SNR the peak may land a sample or two off -- far inside the cyclic prefix
    assert nid2 == cell_id % 3 and abs(int(lag0 + lag) - (tau + l6)) <= (0 if snr >= 10 else 2), (lag0 + lag, tau + l6)
    # the half-window estimator (noise-free bias < 0.004) also sees the PDSCH of the PSS symbol's outer
    # subcarriers, orthogonal to the template over N samples but not over N/2: a few hundredths of a
    # subcarrier at 10 dB, ~0.1 at 5 dB and below (tracking averages it over time)
    assert abs(est - cfo) < (0.05 if snr >= 10 else 0.12) and 0 < rho <= 1.0
    sf_start = lag0 + lag - l6
    y = O.cfo_correct(x[2 * sf_start:2 * (sf_start + 15 * N)], est, N)
    nid1, sf5, score = O.sss_detect(y, nof_prb, nid2)
    assert (nid1, sf5) == (cell_id // 3, int(sf == 5)) and score > 0


@pytest.mark.parametrize("cell_id,nof_prb,sf", [(1, 100, 0), (302, 25, 5), (503, 6, 5), (77, 75, 0)])
def test_product_tx_sync_matches_oracle(cell_id, nof_prb, sf):
    """mi_tx_sync (the product's synthetic transmitter, host code) puts the same PSS / SSS samples on
    the air as the oracle's or_tx_sync; other subframes get nothing."""
    n = 2 * 15 * O.lib().or_symbol_sz(nof_prb)
    a = np.zeros(n, np.float32)
    b = np.zeros(n, np.float32)
    assert abi.tx_sync(cell_id, nof_prb, sf, a) == 1
    assert O.lib().or_tx_sync(cell_id, nof_prb, sf, 1.0, b) == 1
    assert np.max(np.abs(a - b)) < 1e-5 and np.max(np.abs(b)) > 0.01
    c = np.zeros(n, np.float32)
    assert abi.tx_sync(cell_id, nof_prb, 3, c) == 0 and not c.any()
