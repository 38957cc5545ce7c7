"""CPU: srslte_dci_msg_to_dl_grant (phch_worker.cc:297) for every DL allocation srsUE can be given --
format 1 with resource allocation type 0 and type 1, format 1A localized and distributed (gap 1 / gap 2,
C-RNTI and SI/RA/P-RNTI field meanings), format 1C -- checked against the oracle's literal restatement
(oracle/o_ra.c: the 36.211 6.2.3.2 interleaver as a matrix with null cells, type-1 subsets as RBG lists)
on seeded random DCIs over N_RB = 6 .. 110.  Compared: per-slot PRB sets (prb_idx[0] / [1]), nof_prb,
Qm, MCS, HARQ process, NDI, RV and TBS (oracle columns where it carries them, otherwise the product's
Table 7.1.7.2.1-1 at the oracle's (I_TBS, N_PRB) -- that table is pinned by tests/test_tables.py).
Parity is against the oracle restatement of the specification (srsLTE is absent: parity unpinned)."""
import ctypes as C
import random

import numpy as np
import pytest

import oracle_lib as O
from srsue_amd import abi

NRBS = (6, 7, 11, 15, 25, 27, 33, 50, 64, 75, 100, 110)
SI_RNTI, P_RNTI, RA_RNTI, C_RNTI = 0xFFFF, 0xFFFE, 0x0003, 0x1234


class Mcs(C.Structure):
    _fields_ = [("mod", C.c_int), ("tbs", C.c_int), ("idx", C.c_uint32)]


class Grant(C.Structure):
    _fields_ = [("prb_idx", (C.c_bool * 110) * 2), ("nof_prb", C.c_uint32), ("Qm", C.c_uint32), ("mcs", Mcs)]


class Dci(C.Structure):
    _fields_ = [("alloc_type", C.c_int), ("type2_start", C.c_uint32), ("type2_len", C.c_uint32),
                ("type0_alloc", C.c_uint32), ("mcs_idx", C.c_uint32), ("harq_process", C.c_uint32),
                ("ndi", C.c_bool), ("rv_idx", C.c_uint32), ("tpc_pucch", C.c_uint32), ("dci_format", C.c_int),
                ("type1_subset", C.c_uint32), ("type1_shift", C.c_uint32), ("type1_bitmap", C.c_uint32),
                ("type2_distributed", C.c_bool), ("type2_gap", C.c_uint32)]


class Msg(C.Structure):
    _fields_ = [("data", C.c_uint8 * 64), ("nof_bits", C.c_uint32), ("format", C.c_int)]


def clog2(x):
    n = 0
    while (1 << n) < x:
        n += 1
    return n


def riv(N, start, L):
    return N * (L - 1) + start if L - 1 <= N // 2 else N * (N - L + 1) + (N - 1 - start)


class Bits(list):
    def put(self, v, n):
        self.extend((v >> (n - 1 - i)) & 1 for i in range(n))
        return self


def pad(bits, n):
    assert len(bits) <= n
    return list(bits) + [0] * (n - len(bits))


def pack_1a(N, start, L, mcs, harq, ndi, rv, tpc, dist=0, gap=0, common=False):
    """36.212 5.3.3.1.3"""
    rba = clog2(N * (N + 1) // 2)
    b = Bits([1, dist])
    if dist and N >= 50 and not common:
        b.put(gap, 1).put(riv(N, start, L), rba - 1)
    else:
        b.put(riv(N, start, L), rba)
    ndi_field = gap if (common and dist and N >= 50) else ndi
    b.put(mcs, 5).put(harq, 3).put(ndi_field, 1).put(rv, 2).put(tpc, 2)
    return pad(b, O.lib().or_dci_size(O.DCI_1A, N))


def pack_1c(N, start, L, itbs, gap=0):
    """36.212 5.3.3.1.4; start / L in PRBs (multiples of N_step)"""
    step = 2 if N < 50 else 4
    Np = O.lib().or_nvrb_dist(N, 0) // step
    b = Bits()
    if N >= 50:
        b.put(gap, 1)
    b.put(riv(Np, start // step, L // step), clog2(Np * (Np + 1) // 2)).put(itbs, 5)
    assert len(b) == O.lib().or_dci1c_size(N)
    return list(b)


def pack_1(N, alloc, mcs, harq, ndi, rv, tpc):
    """36.212 5.3.3.1.2; alloc = ('t0', rbg bitmap) | ('t1', subset, shift, bitmap)"""
    P = O.lib().or_rbg_size(N)
    nrbg = -(-N // P)
    b = Bits()
    if N > 10:
        b.put(0 if alloc[0] == "t0" else 1, 1)
    if alloc[0] == "t0":
        b.put(alloc[1], nrbg)
    else:
        pb = clog2(P)
        b.put(alloc[1], pb).put(alloc[2], 1).put(alloc[3], nrbg - pb - 1)
    b.put(mcs, 5).put(harq, 3).put(ndi, 1).put(rv, 2).put(tpc, 2)
    return pad(b, O.lib().or_dci_size(O.DCI_1, N))


def product_grant(bits, rnti, N):
    m, d, g = Msg(), Dci(), Grant()
    for i, v in enumerate(bits):
        m.data[i] = v
    m.nof_bits = len(bits)
    ret = abi.lib().srslte_dci_msg_to_dl_grant(C.byref(m), rnti, N, C.byref(d), C.byref(g))
    return ret, d, g


def check(bits, rnti, N):
    """product == oracle on one DCI; returns the oracle grant (None if both reject)"""
    og = O.dl_grant(bits, rnti, N)
    ret, d, g = product_grant(bits, rnti, N)
    if og is None:
        assert ret != 0, "product accepted a DCI the oracle rejects"
        return None
    tbs = og.tbs if og.tbs > 0 else abi.lib().srslte_ra_tbs_from_idx(og.i_tbs, og.n_prb_tbs)
    if tbs <= 0:
        assert ret != 0
        return None
    assert ret == 0, f"product rejected a valid DCI (N={N}, rnti={rnti:#x}, format={og.format})"
    s0 = [p for p in range(N) if g.prb_idx[0][p]]
    s1 = [p for p in range(N) if g.prb_idx[1][p]]
    assert s0 == [p for p in range(N) if og.prb[p] & 1]
    assert s1 == [p for p in range(N) if og.prb[p] & 2]
    assert not any(g.prb_idx[s][p] for s in (0, 1) for p in range(N, 110))
    assert (g.nof_prb, g.Qm, g.mcs.idx, g.mcs.tbs) == (og.nof_prb, og.Qm, og.mcs, tbs)
    assert (d.harq_process, int(d.ndi), d.rv_idx) == ((og.harq, og.ndi, og.rv) if og.format != O.DCI_1C
                                                       else (0, 0, 0))
    return og


def test_1c_sizes():
    """36.212 5.3.3.1.4 with 36.211 Table 6.2.3.2-1 gaps and the 36.213 7.1.6.3 N_step"""
    expect = {6: 8, 15: 10, 25: 12, 50: 13, 75: 14, 100: 15}
    for N, n in expect.items():
        assert O.lib().or_dci1c_size(N) == n


def test_distributed_mapping_properties():
    """36.211 6.2.3.2: per slot the mapping is injective into [0, N_RB); slot 1 uses the same PRB set as
    slot 0 for the whole N_VRB range; gap 1 leaves the PRBs [N_VRB/2, N_gap) of the band unused"""
    L = O.lib()
    for N in range(6, 111):
        for gap2 in (0, 1):
            nv = L.or_nvrb_dist(N, gap2)
            if nv == 0:
                assert gap2 == 1 and N < 50
                continue
            s = [[L.or_vrb_to_prb(N, gap2, n, slot) for n in range(nv)] for slot in (0, 1)]
            for slot in (0, 1):
                assert len(set(s[slot])) == nv and min(s[slot]) >= 0 and max(s[slot]) < N
            assert sorted(s[0]) == sorted(s[1])
            if not gap2:
                g = L.or_ngap(N, 0)
                assert set(s[0]) == set(range(nv // 2)) | set(range(g, g + nv // 2))


@pytest.mark.parametrize("N", NRBS)
def test_format1a_localized_and_distributed(built, N):
    rnd = random.Random(N)
    for _ in range(150):
        dist = rnd.random() < 0.6
        common = rnd.random() < 0.35
        rnti = rnd.choice((SI_RNTI, P_RNTI, RA_RNTI)) if common else C_RNTI
        gap = rnd.randint(0, 1) if (dist and N >= 50) else 0
        nv = O.lib().or_nvrb_dist(N, gap) if dist else N
        L = rnd.randint(1, nv)
        start = rnd.randint(0, nv - L)
        if dist and not common and N >= 50 and riv(N, start, L) >= 1 << (clog2(N * (N + 1) // 2) - 1):
            continue        # not expressible with one RBA bit taken by the gap
        mcs = rnd.randint(0, 26 if common else 28)
        bits = pack_1a(N, start, L, mcs, rnd.randint(0, 7), rnd.randint(0, 1), rnd.randint(0, 3),
                       rnd.randint(0, 3), dist=int(dist), gap=gap, common=common)
        og = check(bits, rnti, N)
        if og is not None:
            assert og.nof_prb == L and og.distributed == int(dist)
            if common:
                assert og.Qm == 2 and og.n_prb_tbs in (2, 3)


@pytest.mark.parametrize("N", NRBS)
def test_format1c(built, N):
    rnd = random.Random(1000 + N)
    step = 2 if N < 50 else 4
    for _ in range(80):
        gap = rnd.randint(0, 1) if N >= 50 else 0
        nv = O.lib().or_nvrb_dist(N, gap)
        Np = O.lib().or_nvrb_dist(N, 0) // step
        Lp = rnd.randint(1, Np)
        sp = rnd.randint(0, Np - Lp)
        if (sp + Lp) * step > nv:
            bits = pack_1c(N, sp * step, Lp * step, rnd.randint(0, 31), gap)
            assert check(bits, SI_RNTI, N) is None      # beyond N_VRB of the indicated gap: rejected
            continue
        bits = pack_1c(N, sp * step, Lp * step, rnd.randint(0, 31), gap)
        og = check(bits, rnd.choice((SI_RNTI, P_RNTI, RA_RNTI)), N)
        assert og is not None and og.format == O.DCI_1C and og.nof_prb == Lp * step


@pytest.mark.parametrize("N", NRBS)
def test_format1_type0_and_type1(built, N):
    rnd = random.Random(2000 + N)
    P = O.lib().or_rbg_size(N)
    nrbg = -(-N // P)
    for _ in range(120):
        if N <= 10 or rnd.random() < 0.5:
            alloc = ("t0", rnd.randint(1, (1 << nrbg) - 1))
        else:
            pb = clog2(P)
            alloc = ("t1", rnd.randint(0, P - 1), rnd.randint(0, 1), rnd.randint(1, (1 << (nrbg - pb - 1)) - 1))
        bits = pack_1(N, alloc, rnd.randint(0, 28), rnd.randint(0, 7), rnd.randint(0, 1), rnd.randint(0, 3),
                      rnd.randint(0, 3))
        og = check(bits, C_RNTI, N)
        if og is not None:
            assert og.alloc_type == (0 if alloc[0] == "t0" else 1)


def test_type1_known_answer(built):
    """36.213 7.1.6.2 worked by hand for N_RB = 25 (P = 2, 13 RBGs, N_TYPE1 = 11): subset 1 holds the
    RBGs 1, 3, .., 11 = PRBs {2,3, 6,7, 10,11, 14,15, 18,19, 22,23} (12 PRBs); without shift bit i maps
    to the i-th of them, with shift to the (i + 1)-th."""
    bits = pack_1(25, ("t1", 1, 0, 0b10000000001), 5, 0, 0, 0, 0)
    og = check(bits, C_RNTI, 25)
    assert [p for p in range(25) if og.prb[p]] == [2, 23 - 1]
    bits = pack_1(25, ("t1", 1, 1, 0b10000000001), 5, 0, 0, 0, 0)
    og = check(bits, C_RNTI, 25)
    assert [p for p in range(25) if og.prb[p]] == [3, 23]


def test_distributed_known_answer(built):
    """36.211 6.2.3.2 worked by hand for N_RB = 50, gap 1 (N_gap = 27, N~_VRB = 46, P = 3, N_row = 12,
    N_null = 2): VRB 0 -> slot-0 PRB 0 and slot-1 PRB (0 + 23) + 27 - 23 = 27; VRB 1 sits in column 1
    (row 0): slot-0 n~' = 12, slot-1 (12 + 23) mod 46 = 35 -> 35 + 4 = 39."""
    L = O.lib()
    assert (L.or_vrb_to_prb(50, 0, 0, 0), L.or_vrb_to_prb(50, 0, 0, 1)) == (0, 27)
    assert (L.or_vrb_to_prb(50, 0, 1, 0), L.or_vrb_to_prb(50, 0, 1, 1)) == (12, 39)
    bits = pack_1a(50, 0, 2, 10, 0, 1, 0, 0, dist=1, gap=0)
    og = check(bits, C_RNTI, 50)
    assert [p for p in range(50) if og.prb[p] & 1] == [0, 12]
    assert [p for p in range(50) if og.prb[p] & 2] == [27, 39]


def test_distributed_re_list_follows_both_slots(built):
    """the two-slot mask of the PDSCH RE list: slot 0 symbols take the bit-0 PRBs, slot 1 the bit-1 PRBs,
    in increasing k per symbol (36.211 6.3.5); identical for the oracle and the product's mi_pdsch_G"""
    cell = O.make_cell(1, 50, 1)
    mask = np.zeros(110, np.uint8)
    mask[[0, 12]] |= 1
    mask[[27, 39]] |= 2
    re = np.zeros(14 * 600, np.uint32)
    n = O.lib().or_pdsch_re_list(C.byref(cell), 1, 1, mask, re)
    W = 600
    for r in re[:n]:
        l, k = divmod(int(r), W)
        assert (k // 12) in ((0, 12) if l < 7 else (27, 39))
    cfg = abi.sf_cfg(nof_prb=50, sf_idx=1, cfi=1, tbs=1000, Qm=2)
    for p in range(110):
        cfg.prb_mask[p] = int(mask[p])
    assert abi.lib().mi_pdsch_G(C.byref(cfg)) == 2 * n
