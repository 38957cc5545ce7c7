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

import oracle_lib as O
from helpers import oracle_dlsch, oracle_front, tb_bytes
from srsue_amd import abi

pytestmark = pytest.mark.gpu
HARNESS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "ue_dl_harness")


def run_harness(cell_id, nof_prb, nof_ports, subframes, phich_ng=0, pdcch=False, full=False, phich=None):
    """subframes: list of (cfg, iq, reset_tbs, max_its, own_buffers); phich = (I_lowest, n_dmrs) asks
    srslte_ue_dl_decode_phich every subframe (full: its result is the last entry of the extras)"""
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(fin, "wb") as f:
            q = 0 if phich is None else phich[0] | (phich[1] << 16)
            f.write(struct.pack("8i", cell_id, nof_prb, nof_ports, len(subframes), phich_ng, int(pdcch),
                                int(phich is not None), q))
            for cfg, iq, reset, max_its, own, *rtype in subframes:
                rt = rtype[0] if rtype else 0      # srslte_rnti_type_t of the PDCCH search (0 = C-RNTI)
                f.write(struct.pack("8i", cfg.sf_idx, cfg.tbs, cfg.Qm, cfg.rv, int(reset), cfg.rnti | (rt << 16),
                                    max_its, int(own)))
                f.write(np.ascontiguousarray(iq, np.float32).tobytes())
        subprocess.check_call([HARNESS, fin, fout], timeout=300)
        out, raw = [], open(fout, "rb").read()
        pos = 0
        for cfg, *_ in subframes:
            r = struct.unpack_from("8i", raw, pos); pos += 32
            m = struct.unpack_from("5f", raw, pos); pos += 20
            ph, = struct.unpack_from("i", raw, pos); pos += 4
            pay = np.frombuffer(raw[pos:pos + cfg.tbs // 8], np.uint8); pos += cfg.tbs // 8
            out.append((r[0], r[1], r[2], m, pay) + ((r[3:] + (ph,),) if full else ()))
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


def test_ue_dl_new_tb_after_retransmission_drops_stale_rows():
    """One softbuffer, three TTIs in srsUE's order: TB A at rv 0, its rv 2 retransmission (combining:
    the rv 0 rows stay materialised while rate de-matching only works on rv 2's chunks), then a new TB B
    at rv 0 after the MAC's srslte_softbuffer_rx_reset_tbs.  Nothing of TB A may leak into TB B's
    decoder input: TB B decodes exactly as the oracle's fresh decode (4 iterations at 21 dB, where
    stale parity would show).  (Rate de-matching only visits chunks with received LLRs; rows left in
    the other chunks by an earlier plan are settled by rm_idle_kernel -- unreachable through the
    public APIs, which reset or keep the plan, so a safety net.)"""
    ta, tb = tb_bytes(71, 75376), tb_bytes(72, 75376)
    c0 = abi.sf_cfg(nof_prb=100, sf_idx=2, tbs=75376, Qm=6, rv=0)
    c1 = abi.sf_cfg(nof_prb=100, sf_idx=3, tbs=75376, Qm=6, rv=2)
    c2 = abi.sf_cfg(nof_prb=100, sf_idx=4, tbs=75376, Qm=6, rv=0)
    iq0 = abi.tx_subframe(c0, ta, snr_db=16.0, seed=21)
    iq1 = abi.tx_subframe(c1, ta, snr_db=16.0, seed=22)
    iq2 = abi.tx_subframe(c2, tb, snr_db=21.0, seed=23)
    res = run_harness(1, 100, 1, [(c0, iq0, True, 4, True), (c1, iq1, False, 4, True), (c2, iq2, True, 8, True)])
    ok2, pay2, noi2, _ = oracle_dlsch(c2, oracle_front(c2, iq2)[3], max_its=8, i16=True)
    assert res[1][0] == 0 and np.array_equal(res[1][4], ta)
    assert ok2 and res[2][0] == 0
    assert np.array_equal(res[2][4], tb) and np.array_equal(res[2][4], pay2) and res[2][2] == noi2


def test_ue_dl_pdcch_to_pdsch_srsue_call_order():
    """SURVEY 8f-1 end to end through the per-TTI ABI in srsUE's order: the grant is NOT given to the
    harness -- it blind-decodes the DCI 1A the transmitter put on the PDCCH (GPU PCFICH, PDCCH soft
    bits, blind search), converts it with srslte_dci_msg_to_dl_grant and decodes the PDSCH with it."""
    import ctypes as C
    import oracle_lib as O
    from test_oracle_ctrl import tx_with_dci
    rnti, ng = 0x3D, 2      # the first C-RNTI (36.321 7.1: 0x0001-0x003C are RA-RNTIs)
    subs, truth = [], []
    for i, (ports, cfi, sf, mcs) in enumerate([(1, 1, 1, 28), (2, 2, 3, 20), (1, 3, 6, 9)]):
        qm, itbs = (2, mcs) if mcs <= 9 else (4, mcs - 1) if mcs <= 16 else (6, mcs - 2)
        tbs = O.lib().or_tbs(itbs, 100)
        cfg = abi.sf_cfg(cell_id=11, nof_prb=100, nof_ports=ports, sf_idx=sf, cfi=cfi, tbs=tbs, Qm=qm, rnti=rnti,
                         rv=i % 2 * 2)
        tb = tb_bytes(50 + i, tbs)
        q = O.ctrl_cfg(11, 100, ports, ng, cfi, sf)
        n = C.c_uint32()
        O.lib().or_pdcch_regs(C.byref(q), None, C.byref(n))
        Ls = np.zeros(32, np.uint32)
        nc = np.zeros(32, np.uint32)
        k = O.lib().or_search_space(n.value, sf, rnti, 0, Ls, nc)
        bits = np.zeros(64, np.uint8)
        A = O.lib().or_dci1a_pack(100, C.byref(O.Dci1a(0, 100, mcs, i + 1, 1, cfg.rv, 1)), bits)
        h = [0.8 + 0.3j, -0.4 + 0.5j] if ports == 2 else None
        iq = abi.tx_subframe(cfg, tb, h=h, snr_db=300.0, seed=i)
        qq = O.ctrl_cfg(11, 100, ports, ng, cfi, sf)
        hh = None if h is None else np.array([v for z in h for v in (z.real, z.imag)], np.float32)
        assert O.lib().or_tx_pdcch(C.byref(qq), rnti, int(Ls[k - 1]), int(nc[k - 1]), bits[:A], A,
                                   None if hh is None else hh.ctypes.data, iq) == 0
        iq = (iq + np.random.default_rng(i).normal(0, np.sqrt(10 ** -3.0 / 2), iq.shape)).astype(np.float32)
        subs.append((cfg, iq, True, 4, True))
        truth.append((tb, int(nc[k - 1]), i + 1, cfg.rv, tbs))
    res = run_harness(11, 100, 1, subs[:1], phich_ng=ng, pdcch=True, full=True)
    res += run_harness(11, 100, 2, subs[1:2], phich_ng=ng, pdcch=True, full=True)
    res += run_harness(11, 100, 1, subs[2:], phich_ng=ng, pdcch=True, full=True)
    for (cfg, *_), (ret, cf, noi, met, pay, extra), (tb, ncce, harq, rv, tbs) in zip(subs, res, truth):
        found, gncce, gtbs, gharq, grv, _ = extra
        assert cf == cfg.cfi and found == 1 and gncce == ncce
        assert (gtbs, gharq, grv) == (tbs, harq, rv)
        assert ret == 0 and np.array_equal(pay, tb)


def test_ue_dl_decode_phich_srsue_call_order():
    """srslte_ue_dl_decode_phich (phch_worker.cc:381) after the PDSCH of the same TTI: the HI the
    oracle's transmitter put on the UL grant's PHICH (36.213 9.1.2) is returned, alternating ACK /
    NACK over subframes; the PDSCH of those subframes still decodes."""
    from test_oracle_ctrl import tx_with_phich
    ng, il, nd = 2, 17, 3
    g, sq = O.phich_calc(100, ng, il, nd)
    subs, tbs = [], []
    for i, sf in enumerate((1, 2, 3, 4)):
        c = abi.sf_cfg(nof_prb=100, sf_idx=sf, tbs=75376, Qm=6)
        ack = i % 2
        iq, _ = tx_with_phich(c, ng, [(g, sq, ack)], snr_db=None, seed=i)
        tb = tb_bytes(200 + i, c.tbs)
        iq = iq + abi.tx_subframe(c, tb, snr_db=30.0, seed=i) - abi.tx_subframe(c, np.zeros(c.tbs // 8, np.uint8),
                                                                               snr_db=300.0, seed=i)
        subs.append((c, iq.astype(np.float32), True, 0, True))
        tbs.append((tb, ack))
    res = run_harness(1, 100, 1, subs, phich_ng=ng, full=True, phich=(il, nd))
    for (ret, cf, noi, met, pay, extra), (tb, ack) in zip(res, tbs):
        assert ret == 0 and np.array_equal(pay, tb)
        assert extra[-1] == ack


RNTI_USER, RNTI_SI, RNTI_RAR, RNTI_PCH = 0, 1, 2, 5


def _clog2(x):
    n = 0
    while (1 << n) < x:
        n += 1
    return n


def _riv(N, start, L):
    return N * (L - 1) + start if L - 1 <= N // 2 else N * (N - L + 1) + (N - 1 - start)


def _put(bits, v, n):
    bits.extend((v >> (n - 1 - i)) & 1 for i in range(n))


def _dci_bits(N, kind, **f):
    """36.212 5.3.3.1 field layouts (see tests/test_dl_grant.py for the field-by-field checks)"""
    b = []
    if kind == "1a":
        common, dist, gap = f.get("common", False), f.get("dist", 0), f.get("gap", 0)
        b += [1, dist]
        rba = _clog2(N * (N + 1) // 2)
        if dist and N >= 50 and not common:
            _put(b, gap, 1); _put(b, _riv(N, f["start"], f["L"]), rba - 1)
        else:
            _put(b, _riv(N, f["start"], f["L"]), rba)
        _put(b, f["mcs"], 5); _put(b, f.get("harq", 0), 3)
        _put(b, gap if (common and dist and N >= 50) else f.get("ndi", 1), 1)
        _put(b, f.get("rv", 0), 2); _put(b, f.get("tpc", 0), 2)
        n = O.lib().or_dci_size(O.DCI_1A, N)
    elif kind == "1c":
        step = 2 if N < 50 else 4
        Np = O.lib().or_nvrb_dist(N, 0) // step
        if N >= 50:
            _put(b, f.get("gap", 0), 1)
        _put(b, _riv(Np, f["start"] // step, f["L"] // step), _clog2(Np * (Np + 1) // 2)); _put(b, f["itbs"], 5)
        n = O.lib().or_dci1c_size(N)
    else:   # format 1, type 1
        P = O.lib().or_rbg_size(N)
        nrbg = -(-N // P)
        pb = _clog2(P)
        b += [1]
        _put(b, f["subset"], pb); _put(b, f["shift"], 1); _put(b, f["bitmap"], nrbg - pb - 1)
        _put(b, f["mcs"], 5); _put(b, f.get("harq", 0), 3); _put(b, 1, 1); _put(b, f.get("rv", 0), 2); _put(b, 0, 2)
        n = O.lib().or_dci_size(O.DCI_1, N)
    return np.array(b + [0] * (n - len(b)), np.uint8)


def _tx_grant_subframe(cell_id, N, ng, cfi, sf, rnti, common, bits, tb_seed, seed, snr_db=30.0):
    """The ORACLE transmitter (o_tx.c) puts the PDSCH on the grant's per-slot PRBs (oracle/o_ra.c decode of
    the same DCI) and the DCI on a PDCCH candidate of the right search space; then AWGN."""
    import ctypes as C
    g = O.dl_grant(bits, rnti, N)
    assert g is not None
    tbs = g.tbs if g.tbs > 0 else abi.lib().srslte_ra_tbs_from_idx(g.i_tbs, g.n_prb_tbs)
    tb = tb_bytes(tb_seed, tbs)
    cell = O.make_cell(cell_id, N, 1)
    tc = O.tx_cfg(cell, sf_idx=sf, cfi=cfi, rnti=rnti, tbs=tbs, qm=g.Qm, prb=np.array(g.prb, np.uint8),
                  snr_db=300.0, seed=seed)
    iq, _ = O.tx_subframe(tc, tb)
    q = O.ctrl_cfg(cell_id, N, 1, ng, cfi, sf)
    n = C.c_uint32()
    O.lib().or_pdcch_regs(C.byref(q), None, C.byref(n))
    Ls, nc = np.zeros(32, np.uint32), np.zeros(32, np.uint32)
    k = O.lib().or_search_space(n.value, sf, 0 if common else rnti, int(common), Ls, nc)
    assert k > 0
    assert O.lib().or_tx_pdcch(C.byref(q), rnti, int(Ls[k - 1]), int(nc[k - 1]), bits, len(bits), None, iq) == 0
    iq = (iq + np.random.default_rng(seed).normal(0, np.sqrt(10 ** (-snr_db / 10) / 2), iq.shape)).astype(np.float32)
    cfg = abi.sf_cfg(cell_id=cell_id, nof_prb=N, nof_ports=1, sf_idx=sf, cfi=cfi, tbs=tbs, Qm=g.Qm, rnti=rnti,
                     rv=g.rv, prb=np.array(g.prb, np.uint8))
    return cfg, iq, tb, g, int(nc[k - 1])


@pytest.mark.parametrize("N", [100, 25])
def test_ue_dl_common_and_partial_grants_srsue_call_order(N):
    """SURVEY 8a a5.1 / 8f-1 through the per-TTI ABI in srsUE's order (phch_worker.cc:286-305, :337-348):
    the harness blind-decodes each DCI with srslte_ue_dl_find_dl_dci_type for the RNTI type srsUE asks
    for, converts it with srslte_dci_msg_to_dl_grant and decodes the PDSCH on the grant's per-slot PRBs:
    a format-1C SI grant (distributed VRB, sf 5 with PSS/SSS holes), a 13-PRB localized 1A, a distributed
    1A (gap in the RBA for N_RB >= 50), an RA-RNTI 1A (N_PRB^1A = 3, the NDI bit as gap), a P-RNTI 1C and
    a format-1 type-1 allocation.  The oracle transmitter puts PDSCH and PDCCH on the air; checked: the
    decoded grant (TBS, PRB count) against the oracle's DCI decode, payload == transmitted TB (bit-exact)
    and == the oracle's decode of the same IQ, iterations == the oracle's."""
    step = 2 if N < 50 else 4
    big = N >= 50
    cases = [   # (rnti, rnti type, sf, cfi, dci)
        (0xFFFF, RNTI_SI, 5, 2, _dci_bits(N, "1c", start=2 * step, L=2 * step, itbs=12, gap=int(big))),
        (0x4601, RNTI_USER, 2, 1, _dci_bits(N, "1a", start=3, L=13, mcs=17, harq=5, rv=0)),
        (0x4601, RNTI_USER, 3, 3, _dci_bits(N, "1a", start=4, L=10, mcs=12, harq=2, dist=1, gap=0)),
        (0x0002, RNTI_RAR, 6, 3, _dci_bits(N, "1a", start=1, L=4, mcs=6, tpc=1, common=True, dist=1,
                                            gap=int(big))),
        (0xFFFE, RNTI_PCH, 7, 2, _dci_bits(N, "1c", start=0, L=3 * step, itbs=20)),
        (0x4601, RNTI_USER, 8, 1, _dci_bits(N, "t1", subset=1, shift=1, bitmap=0b1011011, mcs=20, harq=1)),
    ]
    subs, truth = [], []
    for i, (rnti, rt, sf, cfi, bits) in enumerate(cases):
        common = rt != RNTI_USER
        cfg, iq, tb, g, ncce = _tx_grant_subframe(21, N, 2, cfi, sf, rnti, common, bits, 300 + i, 40 + i)
        subs.append((cfg, iq, True, 4, True, rt))
        truth.append((tb, g, ncce))
    res = run_harness(21, N, 1, subs, phich_ng=2, pdcch=True, full=True)
    for (cfg, iq, *_), (ret, cf, noi, met, pay, extra), (tb, g, ncce) in zip(subs, res, truth):
        found, gncce, gtbs, gharq, grv, _ = extra
        assert cf == cfg.cfi and found == 1 and gncce == ncce
        assert gtbs == cfg.tbs and (gharq, grv) == ((g.harq, g.rv) if g.format != O.DCI_1C else (0, 0))
        _, _, _, ollr = oracle_front(cfg, iq)
        ok, opay, onoi, _ = oracle_dlsch(cfg, ollr, i16=True)
        assert ok and ret == 0, f"rnti {cfg.rnti:#x}: GPU ret {ret}"
        assert np.array_equal(pay, tb) and np.array_equal(pay, opay) and noi == onoi


def test_ue_dl_concurrent_worker_instances():
    """srsUE runs 1-4 phch_worker threads, each with its own srslte_ue_dl_t (phy.h:118-119): four instances
    decoding different TTIs at the same time (tests/c/ue_dl_mt.c) give exactly the results one instance
    gives sequentially -- return value, CFI, iteration count and payload per TTI -- and every CRC-OK payload
    is the transmitted TB.  20 TTIs per thread revisit every subframe index twice (memoised plans re-used)
    and half of them sit in the turbo waterfall (iterating, some failing)."""
    mt = os.path.join(os.path.dirname(HARNESS), "ue_dl_mt")
    r = subprocess.run([mt, "4", "20"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    import json
    d = json.loads(r.stdout)
    assert d["mismatches_vs_sequential"] == 0 and d["errors"] == 0 and d["crc_ok_payload_mismatches"] == 0
    # both outcomes occur (CFI 3 at MCS 28 and the waterfall half fail some TTIs), and decodes iterate
    assert d["crc_ok"] >= 20 and d["crc_failed"] > 0 and d["iterating_ttis"] > 0, d


def test_tti_latency_harness_four_workers():
    """bench.py's `tti` block (configs[1] through the per-TTI ABI): tests/c/tti_latency with 4
    concurrent worker instances decodes every TTI to its transmitted TB (30 dB) and reports the pooled latencies."""
    import json
    exe = os.path.join(os.path.dirname(HARNESS), "tti_latency")
    r = subprocess.run([exe, "100", "24", "4"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["workers"] == 4 and d["ttis"] == 96 and d["crc_ok_and_payload_match"] == 96, d
    for k in ("decode_fft_estimate", "pdsch_decode_rnti", "dl_total", "ul_pusch_encode"):
        assert 0 < d[k]["p50_us"] <= d[k]["p99_us"] <= d[k]["max_us"], k


def test_ue_dl_plan_memo_eviction_srsue_call_order():
    """The per-TTI plan memos evict least-recently-used entries (Engine::plan_memo: 32 PDSCH / front-end plans;
    ue_dl.cpp ctrl_plan: 64 control plans keyed by (sf_idx, CFI, RNTI, PHICH query)).  120 TTIs cycle 10 subframe
    indices x 8 RNTIs x 5 TBS values (MCS 24-28) -- 50 PDSCH configurations and 80 control plans, both far past
    their memo sizes -- in an order that revisits recently used, long-evicted and never-seen entries; every TTI
    must still decode exactly as a fresh decode: CFI, CRC, iterations and payload equal to the oracle's and to the
    transmitted TB."""
    tbs_list = [abi.lib().srslte_ra_tbs_from_idx(i, 100) for i in (22, 23, 24, 25, 26)]
    rntis = [0x46 + 17 * k for k in range(8)]
    subs, tbs_sent = [], []
    for t in range(120):
        sf = (t * 7) % 10
        cfg = abi.sf_cfg(nof_prb=100, sf_idx=sf, tbs=tbs_list[(t // 3) % 5], Qm=6, rnti=rntis[(t * 3 + t // 10) % 8])
        tb = tb_bytes(2000 + t, cfg.tbs)
        iq = abi.tx_subframe(cfg, tb, snr_db=30.0, seed=3000 + t)
        subs.append((cfg, iq, True, 0, True))
        tbs_sent.append(tb)
    keys_pdsch = {(c.sf_idx, c.tbs, c.rnti) for c, *_ in subs}
    keys_ctrl = {(c.sf_idx, c.rnti) for c, *_ in subs}
    assert len(keys_pdsch) > 32 and len(keys_ctrl) > 64
    res = run_harness(1, 100, 1, subs)
    for (c, iq, *_), tb, (ret, cf, noi, met, pay) in zip(subs, tbs_sent, res):
        _, _, _, ollr = oracle_front(c, iq)
        ok, opay, onoi, _ = oracle_dlsch(c, ollr, i16=True)
        assert cf == 1 and ret == 0 and ok, (c.sf_idx, c.tbs, hex(c.rnti))
        assert np.array_equal(pay, tb) and np.array_equal(pay, opay) and noi == onoi
