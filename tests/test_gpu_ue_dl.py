"""Per-TTI srsLTE API on the GPU (include/srslte/srslte.h), driven by tests/c/ue_dl_harness.c in the
call order of srsUE's phch_worker.  Checked against the oracle on the same IQ: PCFICH CFI, TB CRC,
payload bytes (bit-exact), turbo iterations (srslte_pdsch_last_noi), and HARQ soft combining across
two redundancy versions through one srslte_softbuffer_rx_t (dl_harq.cc:230-233)."""
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

from helpers import oracle_dlsch, oracle_front, tb_bytes
from srsue_amd import abi

pytestmark = pytest.mark.gpu
HARNESS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "ue_dl_harness")


def run_harness(cell_id, nof_prb, nof_ports, subframes):
    """subframes: list of (cfg, iq, reset_tbs, max_its, own_buffers)"""
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(fin, "wb") as f:
            f.write(struct.pack("8i", cell_id, nof_prb, nof_ports, len(subframes), 0, 0, 0, 0))
            for cfg, iq, reset, max_its, own in subframes:
                f.write(struct.pack("8i", cfg.sf_idx, cfg.tbs, cfg.Qm, cfg.rv, int(reset), cfg.rnti, max_its,
                                    int(own)))
                f.write(np.ascontiguousarray(iq, np.float32).tobytes())
        subprocess.check_call([HARNESS, fin, fout], timeout=300)
        out, raw = [], open(fout, "rb").read()
        pos = 0
        for cfg, *_ in subframes:
            r = struct.unpack_from("8i", raw, pos); pos += 32
            m = struct.unpack_from("5f", raw, pos); pos += 20
            pay = np.frombuffer(raw[pos:pos + cfg.tbs // 8], np.uint8); pos += cfg.tbs // 8
            out.append((r[0], r[1], r[2], m, pay))
        return out


@pytest.fixture(scope="module", autouse=True)
def _built(built):
    assert os.path.exists(HARNESS)


@pytest.mark.parametrize("ports,cfi,own", [(1, 1, True), (2, 2, True), (1, 3, False)])
def test_ue_dl_tti_matches_oracle(ports, cfi, own):
    cfgs = [abi.sf_cfg(nof_prb=100, nof_ports=ports, sf_idx=sf, cfi=cfi, tbs=75376 if cfi == 1 else 61664, Qm=6)
            for sf in (1, 0, 5)]
    iqs = [abi.tx_subframe(c, tb_bytes(i, c.tbs), snr_db=30.0, seed=i) for i, c in enumerate(cfgs)]
    res = run_harness(1, 100, ports, [(c, iq, True, 0, own) for c, iq in zip(cfgs, iqs)])
    for i, (c, (ret, cf, noi, met, pay)) in enumerate(zip(cfgs, res)):
        _, _, omet, ollr = oracle_front(c, iqs[i])
        ok, opay, onoi, _ = oracle_dlsch(c, ollr, i16=True)   # the library default arithmetic
        assert cf == cfi
        assert ret == 0 and ok
        assert np.array_equal(pay, tb_bytes(i, c.tbs)) and np.array_equal(pay, opay)
        assert noi == onoi
        np.testing.assert_allclose(met, omet, rtol=2e-3)


def test_ue_dl_harq_soft_combining():
    tb = tb_bytes(99, 75376)
    c0 = abi.sf_cfg(nof_prb=100, sf_idx=2, tbs=75376, Qm=6, rv=0)
    c1 = abi.sf_cfg(nof_prb=100, sf_idx=3, tbs=75376, Qm=6, rv=2)
    iq0 = abi.tx_subframe(c0, tb, snr_db=16.0, seed=11)
    iq1 = abi.tx_subframe(c1, tb, snr_db=16.0, seed=12)
    res = run_harness(1, 100, 1, [(c0, iq0, True, 4, True), (c1, iq1, False, 4, True)])
    l0, l1 = oracle_front(c0, iq0)[3], oracle_front(c1, iq1)[3]
    ok0, pay0, noi0, sb = oracle_dlsch(c0, l0, i16=True)
    ok1, pay1, noi1, _ = oracle_dlsch(c1, l1, sb=sb, new_tb=False, i16=True)
    assert (res[0][0] == 0) == ok0 and not ok0, "rv0 alone is expected to fail at 16 dB"
    # a failing decode is compared on CRC verdict and iterations only: the per-TTI path computes its own
    # LLRs (within 1e-4 of the oracle's, not bit-identical) and the int16 quantiser turns a few of those
    # last-bit differences into one-step input differences, which a non-converging decode does not hide.
    # Decoder bit-exactness on identical LLRs, failing decodes included: test_gpu_parity.py.
    assert res[0][2] == noi0
    assert res[1][0] == 0 and ok1
    assert np.array_equal(res[1][4], tb) and np.array_equal(res[1][4], pay1) and res[1][2] == noi1
