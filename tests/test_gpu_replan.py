"""Streaming re-planning on the GPU (include/mi_dl.h mi_dl_plan_build / mi_dl_batch_replan):
a workspace re-planned between different grant configurations decodes exactly what a freshly created batch of the
same configuration decodes -- payload bytes, TB CRC verdicts, TB and per-code-block iterations bit-identical -- and
every CRC-OK TB equals its transmitted bytes.  Configurations: the varied multi-UE grants the bench re-plans
(bench.varied_cfgs: per-subframe RNTI, MCS 20-28, rv 0 / 2) in two assignments, and configs[4]'s mixed cells, in
the bench's batch flags (compact estimates, fused demap, automatic turbo schedule).  Anchor: srsUE re-derives the
grant every TTI (reference ue/src/phy/phch_worker.cc:297 -> :337) and decodes it (:347-348)."""
import numpy as np
import pytest
import torch

import bench
from srsue_amd import abi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert torch.cuda.is_available()


def _config(cfgs, snr=30.0):
    iq, tb = bench.make_pool(cfgs, snr, 8, 0)
    probe = abi.Batch(cfgs, compact_ce=True)
    flat = np.zeros(2 * probe.iq_samples, np.float32)
    for i, x in enumerate(iq):
        o = 2 * probe.iq_offset(i)
        flat[o:o + len(x)] = x
    probe.close()
    return cfgs, torch.from_numpy(flat).cuda(), tb


def _results(b):
    return (b.download(abi.BUF_PAYLOAD, np.uint8), b.download(abi.BUF_TB_CRC, np.uint32)[:len(b.cfgs)],
            b.download(abi.BUF_TB_ITS, np.uint32)[:len(b.cfgs)], b.download(abi.BUF_CB_ITS, np.uint32))


def test_replan_matches_fresh_batches():
    vp = bench.varied_cfgs(96, 0)
    A = _config(vp)
    B = _config([vp[(i + 37) % 96] for i in range(96)], snr=24.0)   # waterfall-ish: some code blocks iterate
    M = _config(bench.config_cfgs(5, 64, 0))
    st = torch.cuda.current_stream().cuda_stream
    ref = {}
    for name, (cfgs, d, _) in (("A", A), ("B", B), ("M", M)):
        f = abi.Batch(cfgs, compact_ce=True)
        f.run(d.data_ptr(), st)
        ref[name] = _results(f)
        f.close()
    w = abi.Batch(A[0], compact_ce=True)
    p = abi.Plan()
    for name, (cfgs, d, tbs) in (("A", A), ("B", B), ("M", M), ("A", A), ("B", B)):
        p.build(cfgs)
        w.replan(p, st)
        w.run(d.data_ptr(), st)
        pay, crc, its, cbits = _results(w)
        rp, rc, ri, rcb = ref[name]
        assert np.array_equal(crc, rc) and np.array_equal(its, ri), name
        assert np.array_equal(cbits[:len(rcb)], rcb), name
        for i in range(len(cfgs)):
            if crc[i]:
                assert np.array_equal(w.payload(i, pay), tbs[i]), (name, i)
        assert crc.sum() >= len(cfgs) // 2, (name, int(crc.sum()))
    w.close()
    p.close()
