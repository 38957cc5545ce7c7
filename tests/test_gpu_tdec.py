"""GPU: raw code-block turbo decoding (mi_tdec_*, the srslte_tdec_* contract of BASELINE configs[0],
srsLTE's turbodecoder_test): K = 6144, 8 fixed iterations, no early stop, BPSK/AWGN LLRs across the
waterfall -- decisions bit-identical to the oracle and to the committed golden fixture, for both the
float (srsLTE-gen) and the int16 (srsLTE SSE design) arithmetic, and for the int16 decoder in both
schedules: one code block per lane, and the latency form (one workgroup per code block, exact
trellis segments; at 0.6-0.8 dB paths merge late, so fix-up rounds cascade)."""
import os

import numpy as np
import pytest
import torch

import oracle_lib as O
from srsue_amd import abi

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def llr_bpsk(d, K, ebno_db, rng):
    x = 1.0 - 2.0 * d
    sigma2 = 1.0 / (2 * (K / (3.0 * K + 12)) * 10 ** (ebno_db / 10))
    y = x + rng.normal(0, np.sqrt(sigma2), x.shape)
    return (-2.0 * y / sigma2).astype(np.float32)


# turbo schedules: float decoder (lane per code block), int16 lane per code block, int16 latency form
MODES = [(False, "lane"), (True, "lane"), (True, "win"), (False, "lanex"), (True, "lanex"), (True, "lanexr"),
         (True, "p2")]   # p2: two code blocks per lane (the 70 code blocks fill one group pair)


@pytest.mark.parametrize("i16,sched", MODES)
def test_golden_config1_on_gpu(built, i16, sched):
    g = np.load(os.path.join(GOLDEN, "tdec_K6144_ebno.npz"))
    ref = np.load(os.path.join(GOLDEN, "tdec16_K6144.npz"))["dec"] if i16 else g["dec"]
    n = len(g["ebno"])
    tb = abi.TdecBatch(6144, n, max_its=8, early_stop=False, tdec_i16=i16, sched=sched)
    d = torch.from_numpy(np.ascontiguousarray(g["llr"])).cuda()
    tb.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    bits, its, _ = tb.results()
    assert np.all(its == 8)
    assert np.array_equal(bits, ref)


@pytest.mark.parametrize("i16,sched", MODES)
@pytest.mark.parametrize("K,ebno", [(6144, 0.6), (6144, 0.8), (5824, 1.0), (40, 2.0), (512, 1.5), (1024, 1.0)])
def test_codeblocks_bit_exact_vs_oracle(built, K, ebno, i16, sched):
    rng = np.random.default_rng(K + int(ebno * 10))
    n = 70                                      # two 64-lane groups, the second partial
    bits = rng.integers(0, 2, (n, K)).astype(np.uint8)
    llr = np.stack([llr_bpsk(abi.turbo_encode(b, K), K, ebno, rng) for b in bits])
    if i16:
        llr *= np.float32(rng.uniform(0.5, 8.0))   # exercise the quantiser range too
    tb = abi.TdecBatch(K, n, max_its=8, early_stop=False, tdec_i16=i16, sched=sched)
    d = torch.from_numpy(llr).cuda()
    tb.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    got, its, _ = tb.results()
    td = O.Tdec(O.TDEC_I16 if i16 else O.TDEC_GEN)
    for i in range(n):
        dec, oits, _ = td.decode_cb(llr[i], K, max_its=8, early_stop=False)
        assert np.array_equal(got[i], dec), f"cb {i}"
    assert np.all(its == 8)


@pytest.mark.parametrize("threads", ["64", "128", "256"])
def test_latency_form_thread_counts(built, threads, monkeypatch):
    """Segment count does not change results: 64/128/256 segments per code block (MI_TDEC_WIN_THREADS)
    with CRC early stop, against the oracle's int16 decoder."""
    monkeypatch.setenv("MI_TDEC_WIN_THREADS", threads)
    rng = np.random.default_rng(int(threads))
    K, n = 6144, 24
    bits = rng.integers(0, 2, (n, K)).astype(np.uint8)
    llr = np.stack([llr_bpsk(abi.turbo_encode(b, K), K, e, rng) for b, e in zip(bits, np.linspace(0.4, 1.6, n))])
    tb = abi.TdecBatch(K, n, max_its=6, early_stop=True, tdec_i16=True, sched="win")
    d = torch.from_numpy(llr).cuda()
    tb.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    got, its, ok = tb.results()
    td = O.Tdec(O.TDEC_I16)
    for i in range(n):
        dec, oits, ook = td.decode_cb(llr[i], K, max_its=6, early_stop=True)
        assert its[i] == oits and bool(ok[i]) == bool(ook), f"cb {i}"
        assert np.array_equal(got[i], dec), f"cb {i}"


@pytest.mark.parametrize("n", [70, 150])
@pytest.mark.parametrize("K,ebno", [(6144, 0.8), (512, 1.5)])
def test_packed_one_iteration_launch(built, n, K, ebno):
    """The one-iteration packed launch (tdec.hip tdec_kernel_p2x<true>: iteration 0 only, the 30-row LDS stash of the
    16-step spans) is what the headline and the waterfall's first launch run; here on its own through the raw
    code-block contract (max_its 1): decisions, CRC verdicts and iteration counts equal the oracle's int16 decoder
    for a partial second group (70 code blocks: one pair) and an unpaired third group (150: two pairs, the second
    with no high half)."""
    rng = np.random.default_rng(K + n)
    bits = rng.integers(0, 2, (n, K)).astype(np.uint8)
    llr = np.stack([llr_bpsk(abi.turbo_encode(b, K), K, ebno, rng) for b in bits])
    llr *= np.float32(rng.uniform(0.5, 8.0))
    tb = abi.TdecBatch(K, n, max_its=1, early_stop=True, tdec_i16=True, sched="p2")
    d = torch.from_numpy(llr).cuda()
    tb.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    got, its, ok = tb.results()
    td = O.Tdec(O.TDEC_I16)
    for i in range(n):
        dec, oits, ook = td.decode_cb(llr[i], K, max_its=1, early_stop=True)
        assert its[i] == oits == 1 and bool(ok[i]) == bool(ook), f"cb {i}"
        assert np.array_equal(got[i], dec), f"cb {i}"


def crc24a_attach(payload):
    """payload bits + their CRC24A parity bits (36.212 5.1.1, g = 0x864CFB, MSB first)"""
    reg = 0
    for b in payload:
        fb = ((reg >> 23) & 1) ^ int(b)
        reg = (reg << 1) & 0xFFFFFF
        if fb:
            reg ^= 0x864CFB
    par = [(reg >> (23 - i)) & 1 for i in range(24)]
    return np.concatenate([payload, np.array(par, np.uint8)])


@pytest.mark.parametrize("seg", ["8", "4"])
def test_segmented_rounds_short_last_segment(built, seg, monkeypatch):
    """the waterfall's segmented late rounds (tdec.hip tdec_kernel_p2s) at a K whose segments do not
    divide evenly -- K = 328: 8 wavefronts get L = 48-step segments, so nseg = 7 (one idle wavefront) and a 40-step last
    segment; 4 wavefronts: L = 96, a 40-step last segment -- equal the packed decoder running every iteration in place
    (MI_TDEC_COMPACT=0): decisions, iterations, CRC verdicts.  65,536 code blocks (the compaction needs the packed
    schedule, i.e. group pairs covering every SIMD) of 128 distinct CRC24A-carrying blocks across 0.5-3.5 dB, early
    stop on the CRC; a sample is checked against the oracle's int16 decoder too."""
    K, n, distinct = 328, 65536, 128
    rng = np.random.default_rng(328)
    blocks = [crc24a_attach(rng.integers(0, 2, K - 24).astype(np.uint8)) for _ in range(distinct)]
    ebnos = np.linspace(0.5, 3.5, distinct)
    llr = np.stack([llr_bpsk(abi.turbo_encode(b, K), K, e, rng) for b, e in zip(blocks, ebnos)])
    d = torch.from_numpy(llr).cuda()[torch.arange(n, device="cuda") % distinct].contiguous()
    outs = []
    for env in ({"MI_TDEC_COMPACT": "0"}, {"MI_TDEC_STORE_W": "1", "MI_TDEC_ROUNDS": "1", "MI_TDEC_SEG": seg}):
        for k in ("MI_TDEC_COMPACT", "MI_TDEC_STORE_W", "MI_TDEC_ROUNDS", "MI_TDEC_SEG"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        tb = abi.TdecBatch(K, n, max_its=6, early_stop=True, crc24a=True, tdec_i16=True)
        assert lib_sched(tb) == 4, "the packed schedule (compaction needs it)"
        tb.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
        outs.append(tb.results())
        tb.close()
    for a, b, name in zip(outs[0], outs[1], ("decisions", "iterations", "crc")):
        assert np.array_equal(a, b), name
    its, ok = outs[0][1], outs[0][2]
    # the waterfall reaches the late (segmented) rounds: code blocks stopping at iterations 1 .. >= 3
    assert 0 < ok.mean() < 1 and its.max() >= 3 and (its >= 3).sum() > 0
    td = O.Tdec(O.TDEC_I16)
    bits = outs[1][0]
    for i in range(0, distinct, 9):
        dec, oits, ook = td.decode_cb(llr[i], K, max_its=6, early_stop=True, crc24a=True)
        assert outs[1][1][i] == oits and bool(outs[1][2][i]) == bool(ook), f"cb {i}"
        assert np.array_equal(bits[i], dec), f"cb {i}"


def lib_sched(tb):
    return abi.lib().mi_tdec_turbo_win(tb.h)


@pytest.mark.parametrize("max_its", [1, 8])
@pytest.mark.parametrize("K", [6144, 40])
def test_packed_at_clamp_magnitudes(built, K, max_its):
    """The packed decoder's trellis start without masked copies (tdec_p2_body.h header: unreachable alpha states at
    -32768, saturating alpha adds) on the GPU at the inputs that stress it most: channel LLRs far beyond the quantiser
    clamp (+-511 after q), a third of them with the wrong sign, so every branch metric and metric spread sits at its
    int16 design bound -- decisions, iterations and CRC verdicts equal the oracle's int16 decoder.  K = 40: window 0
    is a fifth of the trellis."""
    rng = np.random.default_rng(K + max_its)
    n = 70
    bits = rng.integers(0, 2, (n, K)).astype(np.uint8)
    x = np.stack([1.0 - 2.0 * abi.turbo_encode(b, K) for b in bits])
    flip = rng.random(x.shape) < 0.33
    llr = (np.where(flip, x, -x) * rng.uniform(20.0, 200.0, x.shape)).astype(np.float32)
    tb = abi.TdecBatch(K, n, max_its=max_its, early_stop=max_its == 1, tdec_i16=True, sched="p2")
    d = torch.from_numpy(np.ascontiguousarray(llr)).cuda()
    tb.run(d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    got, its, ok = tb.results()
    td = O.Tdec(O.TDEC_I16)
    for i in range(n):
        dec, oits, ook = td.decode_cb(llr[i], K, max_its=max_its, early_stop=max_its == 1)
        assert its[i] == oits and bool(ok[i]) == bool(ook), f"cb {i}"
        assert np.array_equal(got[i], dec), f"cb {i}"
