"""CPU: the DL control-channel oracle (oracle/o_ctrl.c) against 3GPP known answers,
independent re-derivations and transmit-chain ground truth: a DCI put on the air by the oracle's
transmitter is found by blind search with the same bits, format, aggregation level and CCE."""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
from helpers import oracle_front
from srsue_amd import abi


def crc16_ref(bits):
    reg = 0
    for b in bits:
        fb = ((reg >> 15) ^ b) & 1
        reg = ((reg << 1) & 0xFFFF) ^ (0x1021 if fb else 0)
    return reg


def test_crc16_known_answer():
    """CRC-16 g = D^16 + D^12 + D^5 + 1, zero init (36.212 5.1.1): '123456789' -> 0x31C3 (XMODEM)."""
    bits = np.unpackbits(np.frombuffer(b"123456789", np.uint8)).astype(np.uint8)
    assert O.lib().or_crc16(bits, len(bits)) == 0x31C3 == crc16_ref(bits)


@pytest.mark.parametrize("nprb,s1a,s1", [(6, 21, 19), (15, 22, 23), (25, 25, 27), (50, 27, 31), (75, 27, 33),
                                         (100, 28, 39)])
def test_dci_sizes_36212(nprb, s1a, s1):
    """Formats 0/1A (equal, ambiguous sizes padded) and 1 (RBG bitmap) payload sizes, FDD."""
    L = O.lib()
    assert L.or_dci_size(O.DCI_1A, nprb) == s1a == L.or_dci_size(O.DCI_0, nprb)
    assert L.or_dci_size(O.DCI_1, nprb) == s1


def test_cce_count_20mhz():
    """20 MHz, 2 ports, CFI 3, Ng = 1/6: 200 + 300 + 300 REGs - 4 PCFICH - 3 x 3 PHICH = 787 -> 87 CCEs."""
    n = C.c_uint32()
    q = O.ctrl_cfg(nof_prb=100, nof_ports=2, ng=0, cfi=3)
    assert O.lib().or_pdcch_regs(C.byref(q), None, C.byref(n)) == 787 and n.value == 87
    assert O.lib().or_phich_ngroups(100, 2) == 13 and O.lib().or_phich_ngroups(6, 0) == 1


def test_regs_disjoint_from_crs_pcfich_phich():
    for cid, nprb, ng, cfi in [(1, 100, 2, 1), (301, 6, 3, 2), (17, 25, 1, 3), (5, 50, 0, 2)]:
        q = O.ctrl_cfg(cell_id=cid, nof_prb=nprb, ng=ng, cfi=cfi)
        n = C.c_uint32()
        M = O.lib().or_pdcch_regs(C.byref(q), None, C.byref(n))
        re = np.zeros(4 * M, np.uint32)
        O.lib().or_pdcch_regs(C.byref(q), re.ctypes.data, C.byref(n))
        assert len(set(re.tolist())) == 4 * M                      # no RE twice
        kp = np.zeros(16, np.uint32)
        O.lib().or_pcfich_k(C.byref(O.Cell(cid, nprb, 1)), kp.ctypes.data_as(C.c_void_p))
        assert not set(kp.tolist()) & set(re.tolist())             # PCFICH excluded
        W = 12 * nprb
        sym0 = re[re < W]
        assert all((k % 3) != (cid % 6) % 3 for k in sym0)          # CRS (ports 0/1) excluded
        # the REGs left in symbol 0 = 2 N_RB - 4 - 3 N_group
        assert len(sym0) // 4 == 2 * nprb - 4 - 3 * O.lib().or_phich_ngroups(nprb, ng)


def test_quadruplet_permutation_is_a_permutation():
    for M in (23, 157, 787, 32, 64):
        p = np.zeros(M, np.uint32)
        O.lib().or_pdcch_quad_perm(M, 301, p)
        assert sorted(p.tolist()) == list(range(M))


@pytest.mark.parametrize("D", [36, 41, 44, 55, 60])
def test_tail_biting_code_round_trip(D):
    rng = np.random.default_rng(D)
    c = rng.integers(0, 2, D).astype(np.uint8)
    d = np.zeros(3 * D, np.uint8)
    O.lib().or_conv_encode_tb(c, D, d)
    # tail biting: a cyclic shift of the input shifts every output stream the same way
    d2 = np.zeros(3 * D, np.uint8)
    O.lib().or_conv_encode_tb(np.roll(c, 5), D, d2)
    assert all(np.array_equal(np.roll(d[i * D:(i + 1) * D], 5), d2[i * D:(i + 1) * D]) for i in range(3))
    for snr_scale, noise in ((4.0, 0.0), (2.0, 0.8)):
        soft = (2.0 * d - 1.0) * snr_scale + rng.normal(0, noise, 3 * D)
        out = np.zeros(D, np.uint8)
        O.lib().or_viterbi_tb(soft.astype(np.float32), D, out)
        assert np.array_equal(out, c)


@pytest.mark.parametrize("A,L", [(28, 1), (28, 2), (39, 4), (21, 8), (27, 1)])
def test_dci_coding_round_trip_and_rnti_mask(A, L):
    rng = np.random.default_rng(A * 10 + L)
    a = rng.integers(0, 2, A).astype(np.uint8)
    e = np.zeros(72 * L, np.uint8)
    O.lib().or_dci_encode(a, A, 0x1234, L, e)
    soft = ((2.0 * e - 1.0) * 3.0).astype(np.float32)
    out = np.zeros(A, np.uint8)
    assert O.lib().or_dci_decode(soft, L, A, 0x1234, out.ctypes.data) == 1 and np.array_equal(out, a)
    assert O.lib().or_dci_decode(soft, L, A, 0x1235, None) == 0


def test_search_space_36213_9_1_1():
    def ref(n_cce, sf, rnti, common):
        out = []
        Y = 0
        if not common:
            Y = rnti
            for _ in range(sf + 1):
                Y = (39827 * Y) % 65537
        for L, M in (((4, 4), (8, 2)) if common else ((1, 6), (2, 6), (4, 2), (8, 2))):
            nl = n_cce // L
            out += [(L, L * ((Y + m) % nl)) for m in range(M)] if nl else []
        return out
    for n_cce, sf, rnti, common in [(87, 3, 0x46, 0), (17, 0, 0xFFFF, 0), (20, 9, 0x1234, 1), (5, 4, 0x46, 0)]:
        Ls = np.zeros(32, np.uint32)
        nc = np.zeros(32, np.uint32)
        n = O.lib().or_search_space(n_cce, sf, rnti, common, Ls, nc)
        assert list(zip(Ls[:n].tolist(), nc[:n].tolist())) == ref(n_cce, sf, rnti, common)


def test_dci1a_pack_unpack_riv():
    for nprb, start, L in [(100, 0, 100), (100, 10, 37), (25, 3, 22), (6, 0, 6), (50, 49, 1), (50, 5, 26)]:
        g = O.Dci1a(start, L, 27, 5, 1, 2, 1)
        bits = np.zeros(64, np.uint8)
        n = O.lib().or_dci1a_pack(nprb, C.byref(g), bits)
        h = O.Dci1a()
        assert O.lib().or_dci1a_unpack(nprb, bits, n, C.byref(h)) == 0
        assert (h.rb_start, h.L_crb, h.mcs, h.harq, h.ndi, h.rv, h.tpc) == (start, L, 27, 5, 1, 2, 1)


def tx_with_dci(cfg, ng, rnti, L, ncce, a, h=None, snr_db=None, seed=0):
    """Product-TX subframe (noiseless) + the oracle's PDCCH, then AWGN (numpy) at snr_db per RE."""
    iq = abi.tx_subframe(cfg, np.zeros(cfg.tbs // 8, np.uint8), h=h, snr_db=300.0, seed=seed)
    q = O.ctrl_cfg(cfg.cell_id, cfg.nof_prb, cfg.nof_ports, ng, cfg.cfi, cfg.sf_idx)
    hh = None
    if h is not None:
        hh = np.array([v for z in h for v in (z.real, z.imag)], np.float32)
    assert O.lib().or_tx_pdcch(C.byref(q), rnti, L, ncce, np.ascontiguousarray(a, np.uint8), len(a),
                               None if hh is None else hh.ctypes.data, iq) == 0
    if snr_db is not None:
        rng = np.random.default_rng(seed)
        iq = iq + rng.normal(0, np.sqrt(10 ** (-snr_db / 10) / 2), iq.shape).astype(np.float32)
    return iq.astype(np.float32), q


@pytest.mark.parametrize("nprb,ports,cfi,ng,sf,snr", [(100, 1, 1, 2, 1, None), (100, 2, 3, 0, 4, 10.0),
                                                       (25, 1, 2, 1, 0, 8.0), (6, 2, 2, 3, 9, None),
                                                       (50, 1, 3, 2, 5, 6.0)])
def test_pdcch_round_trip_blind_search(nprb, ports, cfi, ng, sf, snr):
    """Transmit-chain ground truth: DCI 1A for C-RNTI 0x46 at a UE-specific candidate is found by the
    blind search with the same bits, format and first CCE; another RNTI finds nothing."""
    cfg = abi.sf_cfg(cell_id=7 + nprb, nof_prb=nprb, nof_ports=ports, sf_idx=sf, cfi=cfi, tbs=1000, Qm=2)
    rnti = 0x46
    q = O.ctrl_cfg(cfg.cell_id, nprb, ports, ng, cfi, sf)
    n = C.c_uint32()
    O.lib().or_pdcch_regs(C.byref(q), None, C.byref(n))
    Ls = np.zeros(32, np.uint32)
    nc = np.zeros(32, np.uint32)
    k = O.lib().or_search_space(n.value, sf, rnti, 0, Ls, nc)
    pick = [i for i in range(k) if Ls[i] == (2 if nprb > 6 else 1)][-1]
    bits = np.zeros(64, np.uint8)
    A = O.lib().or_dci1a_pack(nprb, C.byref(O.Dci1a(0, nprb, 9, 3, 1, 0, 1)), bits)
    h = [0.8 + 0.3j, -0.4 + 0.5j] if ports == 2 else None
    iq, _ = tx_with_dci(cfg, ng, rnti, int(Ls[pick]), int(nc[pick]), bits[:A], h=h, snr_db=snr, seed=sf)
    grid, ce, _, _ = oracle_front(cfg, iq)
    llr, n_cce = O.pdcch_llr(q, grid, ce)
    got = O.find_dci(llr, n_cce, nprb, sf, rnti)
    assert got is not None
    fmt, b, L, ncce = got
    # a DCI sent on L CCEs also decodes from a smaller candidate starting at the same CCE (the first
    # 72 L' bits of the circular buffer are the same): the search tries L = 1 first, the CCE matches
    assert fmt == O.DCI_1A and np.array_equal(b, bits[:A]) and L <= Ls[pick] and ncce == nc[pick]
    assert O.find_dci(llr, n_cce, nprb, sf, 0x47) is None
    assert O.find_dci(llr, n_cce, nprb, sf, rnti, ul=True) is None    # a 1A is not a format 0


# ---- PHICH (36.211 6.9, 36.213 9.1.2) -----------------------------------------------------------
@pytest.mark.parametrize("nprb,ng", [(100, 2), (25, 0), (6, 3), (50, 1)])
def test_phich_resource_36213(nprb, ng):
    """group = (I_lowest + n_dmrs) mod N_group, seq = (floor(I_lowest / N_group) + n_dmrs) mod 8."""
    N = O.lib().or_phich_ngroups(nprb, ng)
    for i_low in range(0, nprb, 3):
        for n_dmrs in range(8):
            assert O.phich_calc(nprb, ng, i_low, n_dmrs) == ((i_low + n_dmrs) % N, (i_low // N + n_dmrs) % 8)


@pytest.mark.parametrize("nprb,ports,ng,cid", [(100, 1, 2, 1), (25, 2, 3, 11), (6, 1, 0, 301), (50, 2, 1, 7)])
def test_phich_res_disjoint(nprb, ports, ng, cid):
    """The 3 REGs of every PHICH group: 12 symbol-0 REs, no CRS, disjoint across groups, from the
    PCFICH REs and from every PDCCH REG."""
    q = O.ctrl_cfg(cid, nprb, ports, ng, 1, 0)
    N = O.lib().or_phich_ngroups(nprb, ng)
    seen = set()
    for g in range(N):
        re = np.zeros(12, np.uint32)
        assert O.lib().or_phich_res(C.byref(q), g, re) == 0
        assert all(int(r) < 12 * nprb for r in re)                          # symbol 0
        assert all(int(r) % 3 != (cid % 6) % 3 for r in re)                 # not a CRS RE
        assert not (set(int(r) for r in re) & seen) and len(set(re)) == 12
        seen |= set(int(r) for r in re)
    assert O.lib().or_phich_res(C.byref(q), N, np.zeros(12, np.uint32)) == -1
    k16 = np.zeros(16, np.uint32)
    O.lib().or_pcfich_k(C.byref(O.Cell(cid, nprb, 1)), k16.ctypes.data_as(C.c_void_p))
    assert not (set(int(k) for k in k16) & seen)
    n = C.c_uint32()
    M = O.lib().or_pdcch_regs(C.byref(q), None, C.byref(n))
    re4 = np.zeros(4 * M, np.uint32)
    O.lib().or_pdcch_regs(C.byref(q), re4.ctypes.data, C.byref(n))
    assert not (set(int(r) for r in re4) & seen)


def tx_with_phich(cfg, ng, hs, h=None, snr_db=None, seed=0):
    """Product-TX subframe + the oracle's PHICHs hs = [(group, seq, ack)], then AWGN (numpy)."""
    iq = abi.tx_subframe(cfg, np.zeros(cfg.tbs // 8, np.uint8), h=h, snr_db=300.0, seed=seed)
    q = O.ctrl_cfg(cfg.cell_id, cfg.nof_prb, cfg.nof_ports, ng, cfg.cfi, cfg.sf_idx)
    hh = None if h is None else np.array([v for z in h for v in (z.real, z.imag)], np.float32)
    for g, sq, ack in hs:
        assert O.lib().or_tx_phich(C.byref(q), g, sq, int(ack), None if hh is None else hh.ctypes.data, iq) == 0
    if snr_db is not None:
        rng = np.random.default_rng(seed)
        iq = iq + rng.normal(0, np.sqrt(10 ** (-snr_db / 10) / 2), iq.shape).astype(np.float32)
    return iq.astype(np.float32), q


@pytest.mark.parametrize("nprb,ports,ng,sf,snr", [(100, 1, 2, 1, None), (100, 2, 1, 4, 5.0), (25, 1, 3, 0, 3.0),
                                                  (6, 2, 0, 9, None)])
def test_phich_round_trip(nprb, ports, ng, sf, snr):
    """Transmit-chain ground truth: ACK / NACK on two orthogonal sequences of one group (and a third
    PHICH in another group when there is one) decode to the transmitted HI; noiseless soft = +-12
    (12 despread chips); an unused sequence of the group reads ~0."""
    cfg = abi.sf_cfg(cell_id=3 + nprb, nof_prb=nprb, nof_ports=ports, sf_idx=sf, cfi=1, tbs=1000, Qm=2)
    N = O.lib().or_phich_ngroups(nprb, ng)
    hs = [(0, 1, 1), (0, 6, 0)] + ([(N - 1, 3, 1)] if N > 1 else [])
    h = [0.8 + 0.3j, -0.4 + 0.5j] if ports == 2 else None
    iq, q = tx_with_phich(cfg, ng, hs, h=h, snr_db=snr, seed=sf + 1)
    grid, ce, _, _ = oracle_front(cfg, iq)
    for g, sq, ack in hs:
        s = O.phich_soft(q, grid, ce, g, sq)
        assert (s > 0) == bool(ack), (g, sq, ack, s)
        if snr is None:
            assert abs(abs(s) - 12.0) < 1e-3
    if snr is None:
        assert abs(O.phich_soft(q, grid, ce, 0, 2)) < 1e-3
