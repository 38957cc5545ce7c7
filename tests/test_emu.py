"""CPU: the gfx950 kernel bodies of rate de-matching, turbo decoding and TB assembly (rm_body.h,
tdec_body.h, tb_body.h), driven by the real planner and compiled for the host (-DMI_EMU, test-only
library srsue_amd/libsrsue_amd_emu.so), against the oracle on identical LLRs: payload bytes, TB CRC
and iteration counts must be bit-identical -- including CRC-failing decodes, filler bits, K-/K+
segmentation, every redundancy version and SFBC (N_L = 2) rate-matching splits.  The GPU runs the
same per-lane code (tests/test_gpu_parity.py checks it there)."""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
from helpers import oracle_dlsch, oracle_dlsch_cbits, oracle_front, tb_bytes
from srsue_amd import abi

CASES = [  # nof_prb, ports, tbs, Qm, snr, sf, rv, cell
    (100, 1, 75376, 6, 30.0, 1, 0, 1),     # headline, 1 iteration
    (100, 1, 75376, 6, 18.5, 2, 0, 1),     # waterfall: CRC fails, 4 iterations
    (6, 1, 512, 2, 10.0, 3, 0, 3),         # C = 1 (CRC24A early stop), F = 8 filler bits
    (25, 1, 7000, 4, 12.0, 1, 2, 3),       # K- / K+, F = 32, rv 2, 2 iterations
    (50, 2, 7000, 2, 3.0, 4, 1, 3),        # TM2, rv 1, failing
    (100, 1, 40000, 6, 19.0, 0, 3, 3),     # sf 0 (PBCH holes), rv 3
    (6, 1, 16, 2, 0.0, 1, 0, 3),           # smallest TB (K = 40)
    (100, 2, 61664, 6, 30.0, 6, 0, 9),     # TM2 64QAM
]


@pytest.mark.parametrize("sched", ["lane", "x", "xr", "p2"])
@pytest.mark.parametrize("mode", ["gen", "i16"])
@pytest.mark.parametrize("nprb,ports,tbs,qm,snr,sf,rv,cid", CASES)
def test_emulated_kernels_bit_exact_vs_oracle(built, nprb, ports, tbs, qm, snr, sf, rv, cid, mode, sched):
    """Planner + rate de-matching + turbo (float gen or int16 SSE arithmetic) + TB assembly, emulated
    lane by lane on the host, against the oracle decoder of the same arithmetic.  sched "x": the
    crossed schedule (two wavefronts per group meeting in the middle of each half-iteration, phases
    of both waves run in turn as the kernel's barriers order them); "xr": its recompute form; "p2": two code
    blocks per lane in packed int16 (int16 arithmetic only; a single subframe leaves its groups unpaired)."""
    if sched == "p2" and mode == "gen":
        pytest.skip("the packed decoder is the int16 arithmetic")
    cfg = abi.sf_cfg(cell_id=cid, nof_prb=nprb, nof_ports=ports, sf_idx=sf, tbs=tbs, Qm=qm, rv=rv)
    tb = tb_bytes(sf, tbs)
    iq = abi.tx_subframe(cfg, tb, snr_db=snr, seed=sf + 7)
    llr = oracle_front(cfg, iq)[3]
    q16 = mode == "i16"
    with O.tdec_mode(O.TDEC_I16 if q16 else O.TDEC_GEN):
        ok, opay, onoi, _ = oracle_dlsch(cfg, llr)
    arr = abi.cfg_array([cfg])
    pe = np.zeros(tbs // 8, np.uint8)
    eok = np.zeros(1, np.uint32)
    eits = np.zeros(1, np.uint32)
    abi.emu().emu_set_tdec_i16(int(q16))
    abi.emu().emu_set_tdec_x({"lane": 0, "x": 1, "xr": 2, "p2": 3}[sched])
    try:
        rc = abi.emu().emu_decode_llr(C.cast(arr, C.c_void_p), 1, np.ascontiguousarray(llr).ctypes.data, 4,
                                      pe.ctypes.data, eok.ctypes.data, eits.ctypes.data, None)
    finally:
        abi.emu().emu_set_tdec_i16(0)
        abi.emu().emu_set_tdec_x(0)
    assert rc == 0
    assert bool(eok[0]) == ok
    assert eits[0] == onoi
    assert np.array_equal(pe, opay)
    if ok:
        assert np.array_equal(pe, tb)


def test_emulated_batch_of_mixed_subframes(built):
    """Several TBs of different K share 64-lane groups: the planner's grouping, lane offsets and TB
    lane lists are exercised together."""
    specs = [(100, 1, 75376, 6, 1), (25, 1, 7000, 4, 2), (6, 1, 512, 2, 3), (100, 1, 40000, 6, 4),
             (50, 1, 36696, 6, 6), (100, 1, 75376, 6, 7)]
    cfgs, llrs, truth = [], [], []
    for i, (nprb, ports, tbs, qm, sf) in enumerate(specs):
        c = abi.sf_cfg(cell_id=5, nof_prb=nprb, nof_ports=ports, sf_idx=sf, tbs=tbs, Qm=qm)
        tb = tb_bytes(100 + i, tbs)
        iq = abi.tx_subframe(c, tb, snr_db=25.0, seed=i)
        cfgs.append(c); llrs.append(oracle_front(c, iq)[3]); truth.append(tb)
    arr = abi.cfg_array(cfgs)
    flat = np.concatenate(llrs).astype(np.float32)
    tot = sum(c.tbs // 8 for c in cfgs)
    pe = np.zeros(tot, np.uint8)
    ok = np.zeros(len(cfgs), np.uint32)
    its = np.zeros(len(cfgs), np.uint32)
    assert abi.emu().emu_decode_llr(C.cast(arr, C.c_void_p), len(cfgs), flat.ctypes.data, 4, pe.ctypes.data,
                                    ok.ctypes.data, its.ctypes.data, None) == 0
    for i, c in enumerate(cfgs):
        off = abi.emu().emu_payload_offset(C.cast(arr, C.c_void_p), len(cfgs), i)
        assert ok[i] == 1
        assert np.array_equal(pe[off:off + c.tbs // 8], truth[i])


@pytest.mark.parametrize("threads", [64, 256])
@pytest.mark.parametrize("nprb,ports,tbs,qm,snr,sf,rv,cid", CASES)
def test_emulated_segment_parallel_turbo_bit_exact(built, nprb, ports, tbs, qm, snr, sf, rv, cid, threads):
    """The latency-form int16 decoder (one workgroup per code block, trellis segments with exact
    boundary fix-up, tdec_win_body.h), emulated phase by phase, against the oracle's int16 decoder:
    payload, TB CRC and iteration counts identical -- incl. CRC-failing waterfall decodes, where
    paths merge late and fix-up rounds cascade over several segments."""
    cfg = abi.sf_cfg(cell_id=cid, nof_prb=nprb, nof_ports=ports, sf_idx=sf, tbs=tbs, Qm=qm, rv=rv)
    tb = tb_bytes(sf, tbs)
    iq = abi.tx_subframe(cfg, tb, snr_db=snr, seed=sf + 7)
    llr = oracle_front(cfg, iq)[3]
    with O.tdec_mode(O.TDEC_I16):
        ok, opay, onoi, _ = oracle_dlsch(cfg, llr)
    arr = abi.cfg_array([cfg])
    pe = np.zeros(tbs // 8, np.uint8)
    eok = np.zeros(1, np.uint32)
    eits = np.zeros(1, np.uint32)
    E = abi.emu()
    E.emu_set_tdec_i16(1)
    E.emu_set_tdec_win(threads)
    try:
        rc = E.emu_decode_llr(C.cast(arr, C.c_void_p), 1, np.ascontiguousarray(llr).ctypes.data, 4,
                              pe.ctypes.data, eok.ctypes.data, eits.ctypes.data, None)
    finally:
        E.emu_set_tdec_i16(0)
        E.emu_set_tdec_win(0)
    assert rc == 0
    assert bool(eok[0]) == ok
    assert eits[0] == onoi
    assert np.array_equal(pe, opay)


@pytest.mark.parametrize("compact", [False, True, "store_w", "rounds", "segments8", "segments3"])
@pytest.mark.parametrize("snr0", [18.6, 30.0])
def test_emulated_packed_pairs_bit_exact_vs_oracle(built, snr0, compact):
    """The packed decoder (two code blocks per lane, tdec_p2_body.h) on a batch whose code blocks fill
    PAIRED groups: 11 subframes of 20 MHz MCS-28 (143 code blocks of K = 5824: one pair + one unpaired
    group) at per-subframe SNRs across the waterfall (code blocks of one lane stop at different
    iterations, some never), plus a 1.4 MHz subframe (another K, unpaired); every TB against the
    oracle's int16 decoder: payload, CRC verdict, iterations, and every code block's iterations.
    compact: the waterfall compaction (iteration 0 over the pairs, then the CRC-failing code blocks
    gathered -- in reverse lane order, so with new partners -- into continuation pairs, tdec_p2_lane<true>);
    "store_w": the same with the first launch storing its extrinsic rows and the continuation gathering them
    instead of re-running iteration 0's DEC2 (engine.cpp: the waterfall's choice); "rounds": that, with one iteration
    per continuation round and the code blocks still failing re-compacted (in reverse slot order, new partners again)
    between rounds (tdec.hip launch_tdec_cont); "segments<S>": those rounds after the first decoded by S trellis
    segments per pair made exact by fix-up rounds (tdec_p2_body.h p2s_*, tdec.hip tdec_kernel_p2s; 3 segments: the
    last one shorter)."""
    cfgs = [abi.sf_cfg(nof_prb=100, sf_idx=1 + i % 4, tbs=75376, Qm=6, rnti=0x46 + i) for i in range(11)]
    cfgs.append(abi.sf_cfg(cell_id=301, nof_prb=6, sf_idx=2, tbs=4392, Qm=6))
    snrs = [snr0 + 0.35 * (i % 5) for i in range(len(cfgs))]
    iqs = [abi.tx_subframe(c, tb_bytes(60 + i, c.tbs), snr_db=snrs[i], seed=90 + i) for i, c in enumerate(cfgs)]
    llrs = [oracle_front(c, iq)[3] for c, iq in zip(cfgs, iqs)]
    arr = abi.cfg_array(cfgs)
    n = len(cfgs)
    offs = [abi.emu().emu_payload_offset(C.cast(arr, C.c_void_p), n, i) for i in range(n)]
    pe = np.zeros(offs[-1] + cfgs[-1].tbs // 8, np.uint8)
    eok = np.zeros(n, np.uint32)
    eits = np.zeros(n, np.uint32)
    cbits = np.zeros(64 * 4, np.uint32)   # 4 groups: 1 of K = 4416 (1.4 MHz), 3 of K = 5824
    flat = np.concatenate(llrs).astype(np.float32)
    E = abi.emu()
    E.emu_set_tdec_i16(1)
    E.emu_set_tdec_x(3)
    E.emu_set_tdec_compact(int(bool(compact)))
    E.emu_set_tdec_store_w(int(compact in ("store_w", "rounds")))
    rounds = compact in ("rounds", "segments8", "segments3")
    E.emu_set_tdec_store_w(int(compact in ("store_w",) or rounds))
    E.emu_set_tdec_rounds(int(rounds))
    E.emu_set_tdec_seg(int(compact[8:]) if isinstance(compact, str) and compact.startswith("segments") else 0)
    E.emu_round_codeblocks.restype = C.c_uint64
    E.emu_cont_codeblocks.restype = C.c_uint64
    try:
        rc = E.emu_decode_llr(C.cast(arr, C.c_void_p), n, flat.ctypes.data, 4, pe.ctypes.data,
                              eok.ctypes.data, eits.ctypes.data, cbits.ctypes.data)
        n_cont = E.emu_cont_codeblocks()
        n_round = E.emu_round_codeblocks()
    finally:
        E.emu_set_tdec_i16(0)
        E.emu_set_tdec_x(0)
        E.emu_set_tdec_compact(0)
        E.emu_set_tdec_store_w(0)
        E.emu_set_tdec_rounds(0)
        E.emu_set_tdec_seg(0)
    assert rc == 0
    # lanes sorted by K (plan.cpp), each K's groups padded to 64 lanes: the 1.4 MHz code block is group 0
    lane = 64
    for i, c in enumerate(cfgs):
        with O.tdec_mode(O.TDEC_I16):
            ok, opay, onoi, ocb = oracle_dlsch_cbits(c, llrs[i])
        assert bool(eok[i]) == ok, i
        assert eits[i] == onoi, i
        assert np.array_equal(pe[offs[i]:offs[i] + c.tbs // 8], opay), i
        if i < 11:
            assert np.array_equal(cbits[lane:lane + len(ocb)], ocb), i
            lane += len(ocb)
    if snr0 < 20:
        assert len(set(cbits[64:64 + 143].tolist())) >= 3   # code blocks of one lane stopped at different its
        assert not compact or n_cont > 20
        assert not rounds or n_round > 0   # some code blocks went through a re-compaction


@pytest.mark.parametrize("base", [1, 2, 3])
def test_emulated_packed_payload_at_misaligned_base(built, base):
    """The packed decoder's check pass writes each code block's payload run as aligned dwords (tdec_p2_body.h
    tdec_p2_check_range, MI_TDEC_P2_PAY32): the dword a chunk completes is the previous chunk's last m bytes and its
    first 4 - m, m = the run's misalignment, and only the run's edges go byte by byte.  With the payload buffer at
    base offsets 1-3 every code block's m changes; the bytes must equal the oracle's, and the bytes in front of the
    buffer and behind it must stay untouched (no write outside any run)."""
    cfgs = [abi.sf_cfg(nof_prb=100, sf_idx=1 + i % 4, tbs=75376, Qm=6, rnti=0x46 + i) for i in range(10)]
    cfgs.append(abi.sf_cfg(cell_id=301, nof_prb=6, sf_idx=2, tbs=4392, Qm=6))
    iqs = [abi.tx_subframe(c, tb_bytes(300 + i, c.tbs), snr_db=30.0, seed=700 + i) for i, c in enumerate(cfgs)]
    llrs = [oracle_front(c, iq)[3] for c, iq in zip(cfgs, iqs)]
    arr = abi.cfg_array(cfgs)
    n = len(cfgs)
    E = abi.emu()
    offs = [E.emu_payload_offset(C.cast(arr, C.c_void_p), n, i) for i in range(n)]
    total = offs[-1] + cfgs[-1].tbs // 8
    raw = np.full(total + 16, 0xA5, np.uint8)   # guard bytes before and after the payload
    pe = raw[base:base + total]
    eok = np.zeros(n, np.uint32)
    eits = np.zeros(n, np.uint32)
    flat = np.concatenate(llrs).astype(np.float32)
    E.emu_set_tdec_i16(1)
    E.emu_set_tdec_x(3)
    try:
        rc = E.emu_decode_llr(C.cast(arr, C.c_void_p), n, flat.ctypes.data, 4, pe.ctypes.data,
                              eok.ctypes.data, eits.ctypes.data, None)
    finally:
        E.emu_set_tdec_i16(0)
        E.emu_set_tdec_x(0)
    assert rc == 0
    assert np.all(raw[:base] == 0xA5) and np.all(raw[base + total:] == 0xA5)
    for i, c in enumerate(cfgs):
        with O.tdec_mode(O.TDEC_I16):
            ok, opay, onoi, _ = oracle_dlsch(c, llrs[i])
        assert ok and bool(eok[i]), i
        assert np.array_equal(pe[offs[i]:offs[i] + c.tbs // 8], opay), i


def test_packed_start_state_llrs_without_masking():
    """The packed decoder drops the REACH-masked LLR copies of window 0 (tdec_p2_body.h header): the unreachable alpha
    start states hold -32768 and every add that takes an alpha metric saturates (p2.h tadd_a), so they lose every LLR
    maximum of steps 0..2 by themselves.  200,000 adversarial draws (inputs at the quantiser clamps half of the time,
    beta vectors from recursions over such inputs) of llr_step and alpha_step against the float recursion with -inf,
    both halves: no difference.  A start value of -4096 differs in many draws, so the draws do reach the margin (the
    bound, -32768 + 9 R with R = 2046, is what makes -32768 safe for every input the decoder can form)."""
    f = abi.emu().emu_p2_start_llr_check
    f.restype = C.c_uint64
    f.argtypes = [C.c_uint64, C.c_uint32, C.c_int]
    assert f(0x5EED, 200000, -32768) == 0
    assert f(0x5EED, 20000, -4096) > 0


def test_emulated_packed_pairs_at_clamp_magnitudes(built):
    """The packed decoder on channel LLRs scaled so that most quantised inputs sit at the clamp (+-511) -- the largest
    branch metrics and metric spreads the int16 design admits, where the saturating alpha adds and the unmasked start
    window would first show a difference -- against the oracle's int16 decoder: payload, CRC, iterations, per code
    block."""
    cfgs = [abi.sf_cfg(nof_prb=100, sf_idx=1 + i % 4, tbs=75376, Qm=6, rnti=0x46 + i) for i in range(6)]   # 78 CBs: a pair
    iqs = [abi.tx_subframe(c, tb_bytes(80 + i, c.tbs), snr_db=17.0 + 0.5 * (i % 4), seed=40 + i)
           for i, c in enumerate(cfgs)]
    llrs = [(oracle_front(c, iq)[3] * 60.0).astype(np.float32) for c, iq in zip(cfgs, iqs)]
    arr = abi.cfg_array(cfgs)
    n = len(cfgs)
    offs = [abi.emu().emu_payload_offset(C.cast(arr, C.c_void_p), n, i) for i in range(n)]
    pe = np.zeros(offs[-1] + cfgs[-1].tbs // 8, np.uint8)
    eok = np.zeros(n, np.uint32)
    eits = np.zeros(n, np.uint32)
    cbits = np.zeros(64 * 2, np.uint32)
    flat = np.concatenate(llrs)   # held: ctypes.data of a temporary would dangle
    E = abi.emu()
    E.emu_set_tdec_i16(1)
    E.emu_set_tdec_x(3)
    try:
        rc = E.emu_decode_llr(C.cast(arr, C.c_void_p), n, flat.ctypes.data, 4, pe.ctypes.data,
                              eok.ctypes.data, eits.ctypes.data, cbits.ctypes.data)
    finally:
        E.emu_set_tdec_i16(0)
        E.emu_set_tdec_x(0)
    assert rc == 0
    lane = 0
    for i, c in enumerate(cfgs):
        with O.tdec_mode(O.TDEC_I16):
            ok, opay, onoi, ocb = oracle_dlsch_cbits(c, llrs[i])
        assert bool(eok[i]) == ok, i
        assert eits[i] == onoi, i
        assert np.array_equal(pe[offs[i]:offs[i] + c.tbs // 8], opay), i
        assert np.array_equal(cbits[lane:lane + len(ocb)], ocb), i
        lane += len(ocb)
    assert len(set(cbits[:78].tolist())) >= 2
