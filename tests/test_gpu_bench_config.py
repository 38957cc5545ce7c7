"""The bench's own configuration against the oracle (VERDICT r2 "next round" item 1).

`bench.py` times `abi.Batch(..., compact_ce=True)` with the automatic turbo schedule: demap fused into rate
de-matching, compact channel estimates (4 pilot rows per port), and -- because the batch is large enough for the
group pairs to cover every SIMD (`Engine::tdec_crossed`) -- the packed two-code-blocks-per-lane int16 decoder
`tdec_kernel_p2x`.  These tests run exactly that configuration at batch sizes where the automatic choice IS p2x
and compare it with the oracle in the turbo waterfall, where the two code blocks of a lane stop at different
iterations (the lane-pair early-stop logic of `tdec_p2_body.h`):

* the expected decode of a subframe is the oracle's int16 decoder (`or_dlsch_decode_cbits`, o_rx.c /
  o_fec.c `or_decode_cb16`) on the GPU front end's own LLRs (a small unfused, full-estimate batch of the same IQ,
  `MI_DL_FLAG_KEEP_LLR`): payload, TB CRC, TB iterations and every code block's iterations must be identical in
  every copy of the subframe, wherever its code blocks land in the big batch (lane, group, pair half);
* those GPU LLRs are within 1e-4 of the oracle front end's (`or_ofdm_rx` + `or_chest` + `or_pdsch_llr`), and the
  oracle decode of the oracle's own LLRs gives the same TB CRC and payload (iterations are compared on the GPU's
  LLRs only: the int16 quantiser q(x) = rint(32 x) can turn a 1e-7 LLR difference into a one-step input
  difference, which may move a code block's stopping iteration without changing its decisions).

Anchor: srsUE's `srslte_pdsch_decode_rnti` call (reference ue/src/phy/phch_worker.cc:347-348), iteration cap
srslte_sch_set_max_noi (phch_worker.cc:87-89, 4 = ue.conf.example's default, the bench's max_its).
"""
import numpy as np
import pytest
import torch

from helpers import oracle_dlsch_cbits, oracle_front, rel_err, tb_bytes
from srsue_amd import abi

pytestmark = pytest.mark.gpu

SF_CYCLE = (1, 2, 3, 4, 6, 7, 8, 9)
TBS, C = 75376, 13


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert torch.cuda.is_available()


def min_subframes_for_p2():
    """Smallest 20 MHz MCS-28 batch for which the automatic schedule picks the packed decoder: 2 wavefronts per
    group pair must cover every SIMD (4 per CU), pairs of 64-code-block groups, 13 code blocks per subframe."""
    simds = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    # Engine::tdec_crossed: 2 x (group pairs) >= SIMDs, i.e. >= `simds` groups of 64 code blocks
    return -(-simds * 64 // C)


def run_bench_config(n, pool_iq, max_its=4, seg_rounds=False):
    """n subframes (subframe i carries pool entry i % pool, sf_idx cycling as the bench does) through the bench's
    batch flags; returns the batch after one run."""
    pool = len(pool_iq)
    cfgs = [abi.sf_cfg(nof_prb=100, sf_idx=SF_CYCLE[i % 8], tbs=TBS, Qm=6, rnti=0x46) for i in range(n)]
    b = abi.Batch(cfgs, max_its=max_its, tdec_i16=True, compact_ce=True, seg_rounds=seg_rounds)
    L = 2 * abi.lib().mi_sf_len(100)
    assert b.iq_offset(1) * 2 == L and b.iq_samples * 2 == n * L
    d_pool = torch.from_numpy(np.stack(pool_iq)).cuda()
    d = torch.empty((n, L), dtype=torch.float32, device="cuda")
    d.copy_(d_pool[torch.arange(n, device="cuda") % pool])
    b.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    del d, d_pool
    return b, cfgs


def expected_from_gpu_llrs(cfgs, iqs, max_its):
    """The pool through a small unfused, full-estimate batch (its LLR stream kept): per entry the GPU LLRs and
    the oracle int16 decode of them; plus the oracle front end's LLRs and their decode."""
    b = abi.Batch(cfgs, max_its=max_its, tdec_i16=True, keep_llr=True)
    flat = np.zeros(2 * b.iq_samples, np.float32)
    for i, iq in enumerate(iqs):
        flat[2 * b.iq_offset(i):2 * b.iq_offset(i) + len(iq)] = iq
    dflat = torch.from_numpy(flat).cuda()
    b.run(dflat.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    llr = b.download(abi.BUF_LLR, np.float32)
    exp, oracle = [], []
    for i, c in enumerate(cfgs):
        _, _, _, ollr = oracle_front(c, iqs[i])
        g = llr[b.offset(abi.BUF_LLR, i):b.offset(abi.BUF_LLR, i) + len(ollr)]
        assert rel_err(g, ollr) < 1e-4, f"LLR pool entry {i}"
        exp.append(oracle_dlsch_cbits(c, g, max_its=max_its))
        oracle.append(oracle_dlsch_cbits(c, ollr, max_its=max_its))
    b.close()
    return exp, oracle


def check_against(b, n, pool, exp, tbs_pool, check_entries):
    crc = b.download(abi.BUF_TB_CRC, np.uint32)
    its = b.download(abi.BUF_TB_ITS, np.uint32)
    cbits = b.download(abi.BUF_CB_ITS, np.uint32)
    pay = b.download(abi.BUF_PAYLOAD, np.uint8)
    offs = np.array([abi.lib().mi_dl_batch_payload_offset(b.h, i) for i in range(n)], np.int64)
    P = pay[offs[:, None] + np.arange(TBS // 8)[None, :]]
    # one K: code block r of subframe s is lane 13 s + r (plan.cpp: lanes in CB order, padding only at the end)
    CB = cbits[:C * n].reshape(n, C)
    for i in range(n):
        if crc[i]:
            assert np.array_equal(P[i], tbs_pool[i % pool]), f"CRC-OK TB {i} differs from its transmitted bytes"
    for j in check_entries:
        ok, opay, onoi, ocb = exp[j]
        sl = slice(j, n, pool)
        assert (crc[sl] == int(ok)).all(), f"pool entry {j}: TB CRC"
        assert (its[sl] == onoi).all(), f"pool entry {j}: TB iterations {np.unique(its[sl])} vs {onoi}"
        assert (CB[sl] == ocb[None, :]).all(), f"pool entry {j}: per-code-block iterations"
        assert (P[sl] == opay[None, :]).all(), f"pool entry {j}: payload"
    return crc, CB


def test_bench_config_p2_waterfall_mix_vs_oracle():
    """Test A: the bench's flags at the smallest batch that auto-selects p2x, a pool of 48 distinct subframes at
    18-22 dB (CRC failing to one-iteration decodes), each copied ~100 times across lanes, groups and pair halves."""
    pool = 48
    n = -(-min_subframes_for_p2() // pool) * pool
    snrs = [18.0 + 4.0 * j / (pool - 1) for j in range(pool)]
    pcfgs = [abi.sf_cfg(nof_prb=100, sf_idx=SF_CYCLE[j % 8], tbs=TBS, Qm=6, rnti=0x46) for j in range(pool)]
    tbs_pool = [tb_bytes(4000 + j, TBS) for j in range(pool)]
    iqs = [abi.tx_subframe(c, tbs_pool[j], snr_db=snrs[j], seed=0xB000 + j) for j, c in enumerate(pcfgs)]
    exp, orc = expected_from_gpu_llrs(pcfgs, iqs, 4)
    b, cfgs = run_bench_config(n, iqs)
    assert b.turbo_sched == "p2", b.turbo_sched
    crc, CB = check_against(b, n, pool, exp, tbs_pool, range(pool))
    # the waterfall is really exercised: failing and passing TBs, code blocks stopping after 1..4 iterations, and
    # lanes whose pair partner stopped at a different iteration (pairs are groups 2p, 2p+1 of one K)
    assert 0 < crc.sum() < n
    assert set(np.unique(CB).tolist()) >= {1, 2, 3, 4}
    lane_its = CB.reshape(-1)[:(C * n // 128) * 128].reshape(-1, 2, 64)
    assert (lane_its[:, 0, :] != lane_its[:, 1, :]).mean() > 0.2
    # the oracle front end's own LLRs decode to the same TB verdicts and payloads
    for j in range(pool):
        assert orc[j][0] == exp[j][0], f"pool entry {j}: oracle-front CRC"
        assert np.array_equal(orc[j][1], exp[j][1]), f"pool entry {j}: oracle-front payload"
    b.close()


def test_bench_iterating_shape_compact_vs_oracle():
    """Test B: the bench's `iterating` block shape -- 12,500 x 20 MHz MCS-28 at 21.5 dB, max_its 4, compact
    estimates, auto schedule (p2x) -- every CRC-OK TB equals its transmitted bytes and 32 of the 64 pool entries
    (every one of their ~195 copies) equal the oracle decode: CRC, TB and per-code-block iterations, payload."""
    n, pool = 12500, 64
    pcfgs = [abi.sf_cfg(nof_prb=100, sf_idx=SF_CYCLE[j % 8], tbs=TBS, Qm=6, rnti=0x46) for j in range(pool)]
    tbs_pool = [tb_bytes(5000 + j, TBS) for j in range(pool)]
    iqs = [abi.tx_subframe(c, tbs_pool[j], snr_db=21.5, seed=0xB100 + j) for j, c in enumerate(pcfgs)]
    sample = list(range(0, pool, 2))
    exp, orc = expected_from_gpu_llrs([pcfgs[j] for j in sample], [iqs[j] for j in sample], 4)
    exp_full = [None] * pool
    for k, j in enumerate(sample):
        exp_full[j] = exp[k]
    b, cfgs = run_bench_config(n, iqs)
    assert b.turbo_sched == "p2", b.turbo_sched
    crc, CB = check_against(b, n, pool, exp_full, tbs_pool, sample)
    # the waterfall: a few failing TBs, most code blocks stop early while their TB's slowest one iterates on
    assert 0.8 < crc.mean() < 1.0 and 1.1 < CB.mean() < CB.max(axis=1).mean()
    for k, j in enumerate(sample):
        assert orc[k][0] == exp[k][0] and np.array_equal(orc[k][1], exp[k][1]), f"pool entry {j}: oracle front"
    b.close()


def test_waterfall_compaction_matches_uncompacted(monkeypatch):
    """Test C: the waterfall compaction (tdec.hip launch_tdec_cont: iteration 0 over the group pairs, the code
    blocks whose CRC failed gathered into dense continuation pairs for iterations 1..) against the packed
    decoder running every iteration in place (MI_TDEC_COMPACT=0): identical TB CRCs, TB and per-code-block
    iterations and payload on a 16-25 dB mix -- continuation partners differ between runs (slot order is
    atomic), so this also checks that a lane's two halves never interact.  The last two runs decode the rounds after
    the first as exact trellis segments (tdec.hip tdec_kernel_p2s): 8 per pair through the batch flag
    MI_DL_FLAG_TDEC_SEG, 4 per pair through MI_TDEC_SEG -- bit-identical too."""
    pool = 40
    n = -(-min_subframes_for_p2() // pool) * pool
    pcfgs = [abi.sf_cfg(nof_prb=100, sf_idx=SF_CYCLE[j % 8], tbs=TBS, Qm=6, rnti=0x46) for j in range(pool)]
    iqs = [abi.tx_subframe(c, tb_bytes(7000 + j, TBS), snr_db=16.0 + 9.0 * j / (pool - 1), seed=0xC000 + j)
           for j, c in enumerate(pcfgs)]
    outs = []
    # compacted with the first launch's extrinsic rows dropped (re-formed by the continuation), uncompacted,
    # compacted with them stored and gathered, and that with one iteration per round and the failing code blocks
    # re-compacted between rounds (engine.cpp: the waterfall's choice)
    # re-compacted between rounds (engine.cpp: the waterfall's choice); then segmented late rounds (flag; env)
    for compact, store_w, rounds, seg in (("1", "0", "0", None), ("0", "0", "0", None), ("1", "1", "0", None),
                                          ("1", "1", "1", None), ("1", "1", "1", "flag"), ("1", "1", "1", "4")):
        monkeypatch.setenv("MI_TDEC_COMPACT", compact)
        monkeypatch.setenv("MI_TDEC_STORE_W", store_w)
        monkeypatch.setenv("MI_TDEC_ROUNDS", rounds)
        if seg not in (None, "flag"):
            monkeypatch.setenv("MI_TDEC_SEG", seg)
        b, _ = run_bench_config(n, iqs, seg_rounds=seg == "flag")
        monkeypatch.delenv("MI_TDEC_SEG", raising=False)
        assert b.turbo_sched == "p2", b.turbo_sched
        outs.append([b.download(k, np.uint32 if k != abi.BUF_PAYLOAD else np.uint8)
                     for k in (abi.BUF_TB_CRC, abi.BUF_TB_ITS, abi.BUF_CB_ITS, abi.BUF_PAYLOAD)])
        b.close()
    for k, name in enumerate(("TB CRC", "TB its", "CB its", "payload")):
        for o in (0, 2, 3, 4, 5):
            assert np.array_equal(outs[o][k], outs[1][k]), (o, name)
    crc, cbits = outs[0][0], outs[0][2][:C * n]
    assert 0 < crc.sum() < n and set(np.unique(cbits).tolist()) >= {1, 2, 3, 4}


def test_configs2_tm2_at_size_vs_oracle():
    """Test D: BASELINE configs[2] at its stated size in the bench's configuration -- 1,000 x
    20 MHz TM2 (2-port SFBC, Alamouti) 64QAM MCS-28 subframes through the bench's channel (h = 0.8+0.3j,
    -0.4+0.5j), compact estimates, fused demap, automatic turbo schedule (crossed lanes at this size) -- on a
    24-29 dB pool of 40 distinct subframes (TM2's waterfall through this channel) so that code blocks iterate.  Every CRC-OK TB equals its transmitted
    bytes; 16 pool entries (all 25 copies of each) equal the oracle int16 decode of the GPU front end's LLRs: TB
    CRC, TB and per-code-block iterations, payload; those LLRs are within 1e-4 of the oracle front end's."""
    n, pool = 1000, 40
    H = [0.8 + 0.3j, -0.4 + 0.5j]
    snrs = [24.0 + 5.0 * j / (pool - 1) for j in range(pool)]   # TM2's waterfall through this channel: 24-29 dB
    pcfgs = [abi.sf_cfg(nof_prb=100, nof_ports=2, tm=2, sf_idx=SF_CYCLE[j % 8], tbs=TBS, Qm=6, rnti=0x46)
             for j in range(pool)]
    tbs_pool = [tb_bytes(8000 + j, TBS) for j in range(pool)]
    iqs = [abi.tx_subframe(c, tbs_pool[j], h=H, snr_db=snrs[j], seed=0xD000 + j) for j, c in enumerate(pcfgs)]
    sample = list(range(0, pool, pool // 16))[:16]
    exp, orc = expected_from_gpu_llrs([pcfgs[j] for j in sample], [iqs[j] for j in sample], 4)
    exp_full = [None] * pool
    for k, j in enumerate(sample):
        exp_full[j] = exp[k]
    cfgs = [pcfgs[i % pool] for i in range(n)]
    b = abi.Batch(cfgs, max_its=4, tdec_i16=True, compact_ce=True)
    assert b.turbo_sched in ("lanex", "lanexr"), b.turbo_sched
    L = 2 * abi.lib().mi_sf_len(100)
    d_pool = torch.from_numpy(np.stack(iqs)).cuda()
    d = torch.empty((n, L), dtype=torch.float32, device="cuda")
    d.copy_(d_pool[torch.arange(n, device="cuda") % pool])
    b.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    crc, CB = check_against(b, n, pool, exp_full, tbs_pool, sample)
    assert n // 2 < crc.sum() < n and CB.max() >= 2 and (CB > 1).mean() > 0.01
    for k, j in enumerate(sample):
        assert orc[k][0] == exp[k][0] and np.array_equal(orc[k][1], exp[k][1]), f"pool entry {j}: oracle front"
    b.close()
