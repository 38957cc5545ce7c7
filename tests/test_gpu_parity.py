"""GPU parity tests: the HIP chain (through the C ABI) against the CPU oracle on identical inputs.

Tolerances (BASELINE.json north_star): grid / channel estimates / LLRs within 1e-4 relative (max abs
error over the RMS of the oracle array); decoded TB bits, TB CRC and turbo iteration counts
bit-exact.  The turbo decoder itself is compared on identical LLRs (uploaded into the batch), where
even CRC-failing decodes must match the oracle bit for bit.
"""
import numpy as np
import pytest
import torch

import oracle_lib as O
from helpers import make_subframes, oracle_dlsch, oracle_front, rel_err, tb_bytes
from srsue_amd import abi

pytestmark = pytest.mark.gpu

TOL = 1e-4
S_RM_TDEC_TB = (1 << 3) | (1 << 4) | (1 << 5)


# turbo decoders: float (lane per code block), int16 lane per code block, int16 latency form
DECODERS = [(False, "lane"), (True, "lane"), (True, "win"), (False, "lanex"), (True, "lanex"), (True, "lanexr"),
            (True, "p2")]


def run_batch(cfgs, iqs, max_its=4, profile=False, tdec_i16=False, sched=None, keep_llr=False, compact_ce=False):
    b = abi.Batch(cfgs, max_its=max_its, profile=profile, tdec_i16=tdec_i16, sched=sched, keep_llr=keep_llr,
                  compact_ce=compact_ce)
    flat = np.zeros(2 * b.iq_samples, np.float32)
    for i, iq in enumerate(iqs):
        o = 2 * b.iq_offset(i)
        flat[o:o + len(iq)] = iq
    d = torch.from_numpy(flat).cuda()
    b.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return b


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert torch.cuda.is_available()


CASES = [
    dict(nof_prb=100, nof_ports=1, sf_idx=1, tbs=75376, Qm=6),                 # configs[1]: 20 MHz TM1 MCS-28
    dict(nof_prb=100, nof_ports=2, sf_idx=2, tbs=75376, Qm=6),                 # configs[2]: TM2 64QAM
    dict(nof_prb=100, nof_ports=1, sf_idx=0, tbs=75376, Qm=6),                 # PBCH / sync holes
    dict(nof_prb=100, nof_ports=2, sf_idx=5, tbs=40000, Qm=4, cfi=2),
    dict(nof_prb=6, nof_ports=1, sf_idx=1, tbs=4392, Qm=6, cell_id=301),       # 1.4 MHz
    dict(nof_prb=15, nof_ports=2, sf_idx=3, tbs=2856, Qm=4, cell_id=7),        # 3 MHz, N = 256
    dict(nof_prb=25, nof_ports=1, sf_idx=4, tbs=7000, Qm=4, cell_id=11, rv=2), # filler bits, K-/K+
    dict(nof_prb=50, nof_ports=1, sf_idx=6, tbs=36696, Qm=6, cell_id=2),
    dict(nof_prb=75, nof_ports=1, sf_idx=9, tbs=40000, Qm=6, cell_id=5, cfi=3),  # N = 1536
]


@pytest.mark.parametrize("i16,sched", DECODERS)
def test_mixed_batch_front_end_and_decode(i16, sched):
    cfgs = [abi.sf_cfg(**c) for c in CASES]
    iqs, tbs = make_subframes(cfgs, snr_db=30.0)
    b = run_batch(cfgs, iqs, tdec_i16=i16, sched=sched, keep_llr=True)
    grid = b.download(abi.BUF_GRID, np.float32)
    ce = b.download(abi.BUF_CE, np.float32)
    llr = b.download(abi.BUF_LLR, np.float32)
    pay = b.download(abi.BUF_PAYLOAD, np.uint8)
    crc = b.download(abi.BUF_TB_CRC, np.uint32)
    its = b.download(abi.BUF_TB_ITS, np.uint32)
    for i, c in enumerate(cfgs):
        og, oce, _, ollr = oracle_front(c, iqs[i])
        go = 2 * b.offset(abi.BUF_GRID, i)
        co = 2 * b.offset(abi.BUF_CE, i)
        lo = b.offset(abi.BUF_LLR, i)
        assert rel_err(grid[go:go + len(og)], og) < TOL, f"grid case {i}"
        assert rel_err(ce[co:co + len(oce)], oce) < TOL, f"ce case {i}"
        assert rel_err(llr[lo:lo + len(ollr)], ollr) < TOL, f"llr case {i}"
        with O.tdec_mode(O.TDEC_I16 if i16 else O.TDEC_GEN):
            ok, opay, onoi, _ = oracle_dlsch(c, ollr)
        p = b.payload(i, pay)
        assert crc[i] == 1 and ok, f"CRC case {i}"
        assert np.array_equal(p, tbs[i]), f"payload vs transmitted TB, case {i}"
        assert np.array_equal(p, opay), f"payload vs oracle, case {i}"
        assert its[i] == onoi


@pytest.mark.parametrize("snr", [30.0, 19.0])
def test_fused_demap_rate_dematching_matches_unfused(snr):
    """The default full run fuses demap into rate de-matching (LLRs computed from grid + ce inside the rm
    staging, demap_body.h); it must give the same softbuffer input as the unfused stages: payload, TB CRC
    and per-code-block iteration counts identical over every configuration of CASES (TM1/TM2, 1.4-20
    MHz, sync holes, filler bits, rv 2), in the waterfall too."""
    cfgs = [abi.sf_cfg(**c) for c in CASES]
    iqs, tbs = make_subframes(cfgs, snr_db=snr, seed0=int(snr))
    res = []
    for keep in (True, False):
        b = run_batch(cfgs, iqs, tdec_i16=True, keep_llr=keep)
        res.append((b.download(abi.BUF_PAYLOAD, np.uint8), b.download(abi.BUF_TB_CRC, np.uint32),
                    b.download(abi.BUF_CB_ITS, np.uint32)))
        b.close()
    for a, f in zip(res[0], res[1]):
        assert np.array_equal(a, f)
    if snr >= 30.0:
        assert res[1][1].all()


@pytest.mark.parametrize("snr", [30.0, 19.0])
def test_compact_channel_estimates_identical_softbuffer(snr):
    """MI_DL_FLAG_CE_COMPACT: channel estimation writes only the 4 pilot rows per port and the fused demap
    interpolates each RE's estimate in time with the chest kernel's own expression.  The rate-de-matched
    softbuffer must be bit-identical to the full-estimate run (every float of the arena), and so payload,
    TB CRC and per-code-block iterations, over every configuration of CASES (TM1/TM2, 1.4-20 MHz, sync
    holes, filler bits, rv 2)."""
    cfgs = [abi.sf_cfg(**c) for c in CASES]
    iqs, _ = make_subframes(cfgs, snr_db=snr, seed0=int(snr) + 7)
    res = []
    for compact in (False, True):
        b = run_batch(cfgs, iqs, tdec_i16=True, compact_ce=compact)
        res.append((b.download(abi.BUF_SB, np.uint32), b.download(abi.BUF_PAYLOAD, np.uint8),
                    b.download(abi.BUF_TB_CRC, np.uint32), b.download(abi.BUF_CB_ITS, np.uint32)))
        b.close()
    for a, c in zip(res[0], res[1]):
        assert np.array_equal(a, c)
    assert res[0][0].any()


@pytest.mark.parametrize("snr", [30.0, 19.0])
def test_direct_rate_dematching_identical_softbuffer(snr, monkeypatch):
    """Direct groups of rate de-matching (Plan::rm_direct, rm.hip): groups whose lanes are all new TBs with one
    rank table, one k0 rank, one modulation and E <= N_v store their staged LLRs rank by rank through the rank ->
    row table, with row maps from rm_direct_map_kernel.  The softbuffer arena (every float, row-map byte and zero row) must be bit-identical to
    the per-position gather of rm_combine_kernel (MI_RM_DIRECT=0), after one run and after a second run over
    the first run's rows, and so payload, TB CRC and per-code-block iterations.  The batch mixes direct TM1
    and TM2 groups (a partial one with padding lanes) with gather groups (mixed modulation, filler bits, rv 2)."""
    cfgs = [abi.sf_cfg(**c) for c in CASES] + [abi.sf_cfg(**CASES[0]) for _ in range(8)] + \
        [abi.sf_cfg(**CASES[1]) for _ in range(8)]
    iqs, _ = make_subframes(cfgs, snr_db=snr, seed0=int(snr) + 11)
    res, ndirect = [], []
    for direct in ("1", "0"):
        monkeypatch.setenv("MI_RM_DIRECT", direct)
        b = abi.Batch(cfgs, max_its=4, tdec_i16=True, compact_ce=True)
        ndirect.append(b.rm_direct_groups)
        flat = np.zeros(2 * b.iq_samples, np.float32)
        for i, iq in enumerate(iqs):
            flat[2 * b.iq_offset(i):2 * b.iq_offset(i) + len(iq)] = iq
        d = torch.from_numpy(flat).cuda()
        out = []
        for _ in range(2):
            b.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            out += [b.download(abi.BUF_SB, np.uint32), b.download(abi.BUF_PAYLOAD, np.uint8),
                    b.download(abi.BUF_TB_CRC, np.uint32), b.download(abi.BUF_CB_ITS, np.uint32)]
        res.append(out)
        b.close()
    assert ndirect[0] >= 2 and ndirect[1] == 0, ndirect
    for a, c in zip(res[0], res[1]):
        assert np.array_equal(a, c)
    assert res[0][0].any()
    if snr >= 30.0:
        assert res[0][2].all()


@pytest.mark.parametrize("i16,sched", DECODERS)
@pytest.mark.parametrize("snr", [15.0, 17.5, 18.5, 19.5, 21.0])
def test_turbo_bit_exact_on_identical_llrs(snr, i16, sched):
    """Waterfall region: CRC passes and fails; GPU == oracle bit for bit either way."""
    cfgs = [abi.sf_cfg(nof_prb=100, sf_idx=1 + (i % 4), tbs=75376, Qm=6) for i in range(4)]
    iqs, _ = make_subframes(cfgs, snr_db=snr, seed0=int(snr * 10))
    b = abi.Batch(cfgs, max_its=4, tdec_i16=i16, sched=sched)
    llrs = [oracle_front(c, iq)[3] for c, iq in zip(cfgs, iqs)]
    flat = np.zeros(b.download(abi.BUF_LLR, np.float32).shape, np.float32)
    for i, l in enumerate(llrs):
        o = b.offset(abi.BUF_LLR, i)
        flat[o:o + len(l)] = l
    b.upload(abi.BUF_LLR, flat)
    b.run_stages(S_RM_TDEC_TB)
    pay = b.download(abi.BUF_PAYLOAD, np.uint8)
    crc = b.download(abi.BUF_TB_CRC, np.uint32)
    its = b.download(abi.BUF_TB_ITS, np.uint32)
    for i, c in enumerate(cfgs):
        with O.tdec_mode(O.TDEC_I16 if i16 else O.TDEC_GEN):
            ok, opay, onoi, _ = oracle_dlsch(c, llrs[i])
        assert bool(crc[i]) == ok
        assert its[i] == onoi
        assert np.array_equal(b.payload(i, pay), opay)


@pytest.mark.parametrize("sched", ["p2", "lanexr"])
def test_turbo_bit_exact_paired_groups_waterfall(sched):
    """Identical LLRs through a batch whose code blocks fill PAIRED groups (11 subframes of 20 MHz MCS-28:
    143 code blocks of K = 5824 = one pair + one unpaired group for the two-code-blocks-per-lane decoder),
    per-subframe SNRs across the waterfall so the two code blocks of a lane stop at different iterations:
    payload, TB CRC and iterations == the oracle's int16 decoder, per code block iterations as well."""
    cfgs = [abi.sf_cfg(nof_prb=100, sf_idx=1 + (i % 4), tbs=75376, Qm=6, rnti=0x46 + i) for i in range(11)]
    snrs = [18.4 + 0.4 * (i % 6) for i in range(11)]
    iqs = [abi.tx_subframe(c, tb_bytes(i, c.tbs), snr_db=snrs[i], seed=300 + i) for i, c in enumerate(cfgs)]
    b = abi.Batch(cfgs, max_its=6, tdec_i16=True, sched=sched)
    assert b.turbo_sched == sched
    llrs = [oracle_front(c, iq)[3] for c, iq in zip(cfgs, iqs)]
    flat = np.zeros(b.download(abi.BUF_LLR, np.float32).shape, np.float32)
    for i, l in enumerate(llrs):
        o = b.offset(abi.BUF_LLR, i)
        flat[o:o + len(l)] = l
    b.upload(abi.BUF_LLR, flat)
    b.run_stages(S_RM_TDEC_TB)
    pay = b.download(abi.BUF_PAYLOAD, np.uint8)
    crc = b.download(abi.BUF_TB_CRC, np.uint32)
    its = b.download(abi.BUF_TB_ITS, np.uint32)
    cbits = b.download(abi.BUF_CB_ITS, np.uint32)
    for i, c in enumerate(cfgs):
        with O.tdec_mode(O.TDEC_I16):
            ok, opay, onoi, _ = oracle_dlsch(c, llrs[i], max_its=6)
        assert bool(crc[i]) == ok, i
        assert its[i] == onoi, i
        assert np.array_equal(b.payload(i, pay), opay), i
    assert len(set(cbits[cbits > 0].tolist())) >= 3
    b.close()


def test_host_iq_pipeline_matches_batch():
    """mi_dl_pipe_* (SURVEY 8f-3): host IQ in page-locked memory, double-buffered H2D + decode on two
    streams; each slot's outputs equal a plain batch run on the same IQ, across slot reuse."""
    cfgs = [abi.sf_cfg(nof_prb=100, sf_idx=1 + (i % 4), tbs=75376, Qm=6) for i in range(6)]
    iqs, tbs = make_subframes(cfgs, snr_db=30.0, seed0=40)
    ref = run_batch(cfgs, iqs)
    want = ref.download(abi.BUF_PAYLOAD, np.uint8)
    p = abi.Pipe(cfgs)
    nfl = 2 * ref.iq_samples
    hb = abi.HostBuffer(nfl * 4)
    for i, iq in enumerate(iqs):
        o = 2 * ref.iq_offset(i)
        hb.array[o:o + len(iq)] = iq
    slots = [p.submit(hb.ptr) for _ in range(3)]      # slot 0, 1, 0 again (reuse behind its decode)
    assert slots == [0, 1, 0]
    for s in (1, 0):
        p.wait(s)
        b = p.batch(s)
        assert np.array_equal(b.download(abi.BUF_PAYLOAD, np.uint8), want)
        assert np.all(b.download(abi.BUF_TB_CRC, np.uint32)[:len(cfgs)] == 1)
    p.close()
    hb.close()


def test_sc16_wire_format_is_exact():
    """FLAG_IQ_SC16: the OFDM stage converts sc16 on load (x / 32768, exact in fp32), so a batch fed
    sc16 IQ produces the same grid bit for bit, and the same payloads, as a batch fed the fc32 values
    of those same samples."""
    cfgs = [abi.sf_cfg(nof_prb=100, sf_idx=3, tbs=75376, Qm=6), abi.sf_cfg(nof_prb=25, nof_ports=2, sf_idx=5,
                                                                            tbs=7000, Qm=4, cell_id=7)]
    iqs, tbs = make_subframes(cfgs, snr_db=30.0, seed0=70)
    q = [abi.to_sc16(iq) for iq in iqs]
    ref = run_batch(cfgs, [x.astype(np.float32) / 32768.0 for x in q])
    b = abi.Batch(cfgs, max_its=4, iq_sc16=True)
    flat = np.zeros(2 * b.iq_samples, np.int16)
    for i, x in enumerate(q):
        o = 2 * b.iq_offset(i)
        flat[o:o + len(x)] = x
    d = torch.from_numpy(flat).cuda()
    b.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(b.download(abi.BUF_GRID, np.float32), ref.download(abi.BUF_GRID, np.float32))
    pay = b.download(abi.BUF_PAYLOAD, np.uint8)
    for i in range(len(cfgs)):
        assert np.array_equal(b.payload(i, pay), tbs[i])


@pytest.mark.parametrize("i16,sched", DECODERS)
def test_batch_harq_combining_sparse_rows(i16, sched):
    """HARQ in the batch path with the sparse softbuffer rows (dl_common.h sb_group_floats): one
    64-lane group mixes first transmissions (rv 0, overwrite) and retransmissions (rv 2 / rv 3,
    combine).  Two launches with different LLRs: combining lanes must equal the oracle's dense float
    softbuffer after both, the fresh lanes the oracle's single decode -- rows that only one lane
    materialises, rows dropped by a fresh lane and the zero row all take part."""
    spec = [(0, 1), (2, 0), (0, 1), (3, 0)]
    cfgs = [abi.sf_cfg(nof_prb=100, sf_idx=1 + i, tbs=75376, Qm=6, rv=rv, new_tb=nt) for i, (rv, nt) in enumerate(spec)]
    b = abi.Batch(cfgs, max_its=4, tdec_i16=i16, sched=sched)
    flat_len = b.download(abi.BUF_LLR, np.float32).shape
    osb = [None] * len(cfgs)
    for run, snr in enumerate((14.0, 16.0)):
        iqs, _ = make_subframes(cfgs, snr_db=snr, seed0=90 + 10 * run)
        llrs = [oracle_front(c, iq)[3] for c, iq in zip(cfgs, iqs)]
        flat = np.zeros(flat_len, np.float32)
        for i, l in enumerate(llrs):
            flat[b.offset(abi.BUF_LLR, i):b.offset(abi.BUF_LLR, i) + len(l)] = l
        b.upload(abi.BUF_LLR, flat)
        b.run_stages(S_RM_TDEC_TB)
        pay = b.download(abi.BUF_PAYLOAD, np.uint8)
        crc = b.download(abi.BUF_TB_CRC, np.uint32)
        its = b.download(abi.BUF_TB_ITS, np.uint32)
        for i, c in enumerate(cfgs):
            ok, opay, onoi, osb[i] = oracle_dlsch(c, llrs[i], sb=None if c.new_tb else osb[i], new_tb=bool(c.new_tb),
                                                  i16=i16)
            assert bool(crc[i]) == ok, (run, i)
            assert its[i] == onoi, (run, i)
            assert np.array_equal(b.payload(i, pay), opay), (run, i)
