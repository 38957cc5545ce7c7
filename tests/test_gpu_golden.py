"""GPU: the HIP chain pinned to COMMITTED fixtures, not only to the live oracle.

tests/golden/sf_1p4mhz.npz and sf_20mhz_tm1.npz (BASELINE configs[1]: 20 MHz TM1 MCS-28, 21.5 dB, code blocks
iterating up to 4 times) hold the IQ, the transmitted TB and the oracle's grid, channel estimates, LLRs, payload
and iteration counts at the time they were generated (tests/golden/make_golden.py).  The GPU decodes the stored
IQ and is compared with the stored arrays: grid / ce / LLR within 1e-4 relative (max abs error over the RMS of the
stored array), payload byte-exact, TB CRC, and the iteration count of each turbo arithmetic.  Nothing here calls
the oracle, so a change that moved the oracle and the kernels together would fail this file; a change to the
oracle alone fails the CPU fixture tests (test_oracle.py test_golden_*_subframe_chain, exact equality).
"""
import os

import numpy as np
import pytest
import torch

from helpers import rel_err
from srsue_amd import abi

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TOL = 1e-4


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert torch.cuda.is_available()


def fixture(name):
    g = np.load(os.path.join(GOLDEN, name))
    cid, nprb, ports, sf, cfi, tbs, qm = g["cfg"].tolist()
    return g, abi.sf_cfg(cell_id=cid, nof_prb=nprb, nof_ports=ports, sf_idx=sf, cfi=cfi, tbs=tbs, Qm=qm)


def decode(cfg, iq, i16, sched=None):
    b = abi.Batch([cfg], max_its=4, tdec_i16=i16, sched=sched, keep_llr=True)
    flat = np.zeros(2 * b.iq_samples, np.float32)
    flat[2 * b.iq_offset(0):2 * b.iq_offset(0) + len(iq)] = iq
    d = torch.from_numpy(flat).cuda()
    b.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = dict(grid=b.download(abi.BUF_GRID, np.float32), ce=b.download(abi.BUF_CE, np.float32),
               llr=b.download(abi.BUF_LLR, np.float32), payload=b.payload(0),
               crc=int(b.download(abi.BUF_TB_CRC, np.uint32)[0]), its=int(b.download(abi.BUF_TB_ITS, np.uint32)[0]),
               go=2 * b.offset(abi.BUF_GRID, 0), co=2 * b.offset(abi.BUF_CE, 0), lo=b.offset(abi.BUF_LLR, 0))
    b.close()
    return out


def check_front(o, g):
    for k, off in (("grid", "go"), ("ce", "co"), ("llr", "lo")):
        ref = g[k]
        assert rel_err(o[k][o[off]:o[off] + len(ref)], ref) < TOL, k


@pytest.mark.parametrize("i16,sched", [(False, None), (True, None), (True, "p2"), (True, "lanex")])
def test_golden_20mhz_tm1_subframe(i16, sched):
    g, cfg = fixture("sf_20mhz_tm1.npz")
    o = decode(cfg, g["iq"], i16, sched)
    check_front(o, g)
    name = "i16" if i16 else "gen"
    assert o["crc"] == 1
    assert np.array_equal(o["payload"], g["payload_" + name]) and np.array_equal(o["payload"], g["tb"])
    assert o["its"] == int(g["noi_" + name][0]) == 4


@pytest.mark.parametrize("i16", [False, True])
def test_golden_1p4mhz_subframe(i16):
    g, cfg = fixture("sf_1p4mhz.npz")
    o = decode(cfg, g["iq"], i16)
    check_front(o, g)
    assert o["crc"] == 1
    assert np.array_equal(o["payload"], g["payload"]) and np.array_equal(o["payload"], g["tb"])
    if not i16:   # the fixture's iteration count is the float (srsLTE-gen) decoder's
        assert o["its"] == int(g["noi"][0])


MET_TOL = 2e-3   # channel-estimate metrics (RSRP, RSSI, RSRQ, noise, SNR): float reductions in another order


@pytest.mark.parametrize("name,sched", [("otx_1p4mhz.npz", None), ("otx_20mhz_tm1.npz", None),
                                        ("otx_20mhz_tm1.npz", "p2"), ("otx_20mhz_tm2.npz", None),
                                        ("otx_mixed.npz", None)])
def test_golden_oracle_transmitter(name, sched):
    """fixtures whose IQ the ORACLE's transmitter made (oracle/o_tx.c, not the product's
    csrc/tx.cpp), so a change to the product transmitter alone cannot move them -- configs[1] TM1 (20.5 dB, 4
    iterations), configs[2] TM2 SFBC through a 2-port channel, a configs[4] mixed 1.4 / 5 / 10 / 20 MHz batch (one
    batch, every subframe its own allocation and MCS) and 1.4 MHz.  The HIP chain decodes the stored IQ: grid / ce /
    LLR within 1e-4 of the stored oracle arrays, the channel metrics (RSRP, RSSI, RSRQ, noise, SNR; srsUE reads them
    at phch_worker.cc:799-848) within 2e-3, payload = the stored payload = the transmitted TB, and the int16
    iteration count of each TB."""
    from helpers import otx_fixture
    g, cfgs, part = otx_fixture(os.path.join(GOLDEN, name))
    b = abi.Batch(cfgs, max_its=4, tdec_i16=True, sched=sched, keep_llr=True)
    flat = np.zeros(2 * b.iq_samples, np.float32)
    for i in range(len(cfgs)):
        iq = part("iq", i)
        flat[2 * b.iq_offset(i):2 * b.iq_offset(i) + len(iq)] = iq
    d = torch.from_numpy(flat).cuda()
    b.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    grid, ce, llr = (b.download(k, np.float32) for k in (abi.BUF_GRID, abi.BUF_CE, abi.BUF_LLR))
    met = b.download(abi.BUF_METRICS, np.float32).reshape(-1, 5)
    crc = b.download(abi.BUF_TB_CRC, np.uint32)
    its = b.download(abi.BUF_TB_ITS, np.uint32)
    pay = b.download(abi.BUF_PAYLOAD, np.uint8)
    for i in range(len(cfgs)):
        for key, buf, scale in (("grid", grid, 2), ("ce", ce, 2), ("llr", llr, 1)):
            ref = part(key, i)
            o = scale * b.offset({"grid": abi.BUF_GRID, "ce": abi.BUF_CE, "llr": abi.BUF_LLR}[key], i)
            assert rel_err(buf[o:o + len(ref)], ref) < TOL, (key, i)
        ref = g["metrics"][i]
        assert np.all(np.abs(met[i] - ref) <= MET_TOL * np.abs(ref)), (i, met[i].tolist(), ref.tolist())
        assert crc[i] == 1, i
        assert np.array_equal(b.payload(i, pay), part("payload", i)) and np.array_equal(b.payload(i, pay), part("tb", i))
        assert its[i] == g["noi_i16"][i], (i, int(its[i]), int(g["noi_i16"][i]))
    b.close()
