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
    """cfgs, their IQ laid out for a batch (in HBM) and their TBs; snr: one value, or one per subframe"""
    if np.ndim(snr):
        iq, tb = [], []
        for i, c in enumerate(cfgs):
            t = bench.tb_payload(i, c.tbs // 8)
            iq.append(abi.tx_subframe(c, t, snr_db=float(snr[i]), seed=0xA5A5 + i))
            tb.append(t)
    else:
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


def test_retransmission_after_replan():
    """HARQ continuity across mi_dl_batch_replan (include/mi_dl.h): a retransmission (new_tb = 0, rv 2) combines with
    the rows of its first transmission only when the softbuffer layout is the same; after a replan to a different
    layout the softbuffer is cleared, so the retransmission decodes exactly as in a fresh batch (RX_NULL history) --
    never against another plan's rows."""
    n = 32
    first = [abi.sf_cfg(nof_prb=100, sf_idx=bench.SF_CYCLE[i % 8], tbs=75376, Qm=6, rv=0) for i in range(n)]
    retx = [abi.sf_cfg(nof_prb=100, sf_idx=bench.SF_CYCLE[i % 8], tbs=75376, Qm=6, rv=2, new_tb=0) for i in range(n)]
    snrs = np.linspace(19.5, 23.0, n)         # through the waterfall: some TBs fail their first transmission
    X0 = _config(first, snr=snrs)
    X2 = (retx, _config(retx, snr=snrs)[1], X0[2])
    Y = _config(bench.config_cfgs(5, 48, 0))  # another layout (mixed cells)
    st = torch.cuda.current_stream().cuda_stream
    # reference: the retransmission alone, from a cleared softbuffer
    f = abi.Batch(retx, compact_ce=True)
    f.run(X2[1].data_ptr(), st)
    alone = _results(f)
    f.close()
    w = abi.Batch(first, compact_ce=True)
    p = abi.Plan()
    w.run(X0[1].data_ptr(), st)
    crc0 = _results(w)[1]
    assert 0 < crc0.sum() < n
    # same layout: rv 0 + rv 2 combine -- at least every TB rv 0 or rv 2 alone decoded
    p.build(retx)
    w.replan(p, st)
    w.run(X2[1].data_ptr(), st)
    comb = _results(w)
    assert comb[1].sum() >= max(crc0.sum(), alone[1].sum()) and comb[1].sum() > alone[1].sum()
    # another layout in between: the retransmission then combines with nothing
    w2 = abi.Batch(first, compact_ce=True)
    w2.run(X0[1].data_ptr(), st)
    for cfgs, d in ((Y[0], Y[1]), (retx, X2[1])):
        p.build(cfgs)
        w2.replan(p, st)
        w2.run(d.data_ptr(), st)
    got = _results(w2)
    for a, b in zip(got, alone):
        assert np.array_equal(a[:len(b)], b)
    for i in range(n):
        if got[1][i]:
            assert np.array_equal(w2.payload(i, got[0]), X0[2][i])
    for b in (w, w2):
        b.close()
    p.close()


def test_retransmission_survives_unrelated_replan():
    """HARQ continuity is per 64-lane group (include/mi_dl.h): when only another subframe's grant changes
    -- here the last subframe becomes a new TB of another code-block size (K = 6144, sorted after K = 5,824) -- every
    group whose layout is unchanged keeps combining its retransmissions, and only the group whose lanes changed is
    cleared.  Per code block: lanes of the unchanged groups decode exactly as the same-layout retransmission, the
    changed group's retransmission lanes exactly as from a cleared softbuffer.  (srsLTE keeps one softbuffer per HARQ
    process: dl_harq.h:88, reset only by its own new grant, dl_harq.cc:232.)"""
    n = 32
    first = [abi.sf_cfg(nof_prb=100, sf_idx=bench.SF_CYCLE[i % 8], tbs=75376, Qm=6, rv=0) for i in range(n)]
    retx = [abi.sf_cfg(nof_prb=100, sf_idx=bench.SF_CYCLE[i % 8], tbs=75376, Qm=6, rv=2, new_tb=0) for i in range(n)]
    # the unrelated change: subframe n - 1 a new TB of 6 code blocks of K = 6144 (B' = 36,864)
    mixed = retx[:n - 1] + [abi.sf_cfg(nof_prb=100, sf_idx=bench.SF_CYCLE[(n - 1) % 8], tbs=36696, Qm=6, rv=0)]
    snrs = np.linspace(19.5, 23.0, n)
    X0 = _config(first, snr=snrs)
    X2 = _config(retx, snr=snrs)
    XM = _config(mixed, snr=snrs)
    st = torch.cuda.current_stream().cuda_stream
    f = abi.Batch(retx, compact_ce=True)
    f.run(X2[1].data_ptr(), st)
    alone = _results(f)
    f.close()
    runs = {}
    for name, cfgs, d in (("same", retx, X2[1]), ("mixed", mixed, XM[1])):
        w = abi.Batch(first, compact_ce=True)
        p = abi.Plan()
        w.run(X0[1].data_ptr(), st)
        p.build(cfgs)
        w.replan(p, st)
        w.run(d.data_ptr(), st)
        runs[name] = (_results(w), w.n_groups)
        if name == "mixed":
            for i in range(n):
                if runs[name][0][1][i]:
                    assert np.array_equal(w.payload(i, runs[name][0][0]), (X0[2] if i < n - 1 else XM[2])[i])
        w.close()
        p.close()
    same, mix = runs["same"][0], runs["mixed"][0]
    cb_its = lambda r: r[3]
    kept = 6 * 64                                  # groups 0..5: the lanes of code blocks 0 .. 383, unchanged
    cleared = (n - 1) * 13 - kept                  # group 6: the remaining K = 5,824 code blocks
    assert np.array_equal(cb_its(mix)[:kept], cb_its(same)[:kept])
    assert np.array_equal(cb_its(mix)[kept:kept + cleared], cb_its(alone)[kept:kept + cleared])
    # combining happened where it was kept: the same-layout run beats the cleared one on those code blocks
    assert cb_its(same)[:kept].sum() < cb_its(alone)[:kept].sum()
    # the TBs whose code blocks all lie in the kept groups decode exactly as with the same layout
    full = kept // 13
    for k in (1, 2):
        assert np.array_equal(mix[k][:full], same[k][:full])
