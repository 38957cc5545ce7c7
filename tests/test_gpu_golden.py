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
