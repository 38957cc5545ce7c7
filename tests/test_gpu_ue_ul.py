"""Per-TTI srsLTE UL API on the GPU (include/srslte/srslte.h, srsue_amd/csrc/ue_ul.cpp), driven by
tests/c/ue_ul_harness.c in the call order of srsUE's phch_worker (init / normalisation / CFO / RNTI /
set_cfg, then per TTI set_cfo, [dci_msg_to_ul_grant], cfg_grant, pusch_encode_rnti_softbuffer).
Checked against the oracle's PUSCH transmitter (oracle/o_ul.c) on the same TB: direct grants, a grant
decoded from DCI format 0 bits, a retransmission (rv 2) re-encoded from the HARQ softbuffer with a NULL
payload, the normalisation factor and the CFO rotation, and the rejection of a retransmission with nothing stored."""
import ctypes
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_lib as O
from test_ul_grant import format0

pytestmark = pytest.mark.gpu
HARNESS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "ue_ul_harness")
TOL = 1e-4
NFFT = {6: 128, 15: 256, 25: 512, 50: 1024, 75: 1536, 100: 2048}


def run(cell_id, nof_prb, txs, dmrs=(0, 0, 0, 0), flags=0, cfo=0.0):
    """txs: list of dict(tti, rnti, rv, dci (DciMsg or None), n_prb, L_prb, tbs, Qm, ncs, tb, pass_data)"""
    N = NFFT[nof_prb]
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(fin, "wb") as f:
            f.write(struct.pack("8i", cell_id, nof_prb, len(txs), *dmrs, flags))
            f.write(struct.pack("f", cfo))
            for t in txs:
                dci = t.get("dci")
                use = 2 if t.get("rar") else int(dci is not None)
                f.write(struct.pack("12i", t["tti"], t["rnti"], t["rv"] | (t.get("tx_nb", 0) << 8), use,
                                    t.get("n_prb", 0),
                                    t.get("L_prb", 0), t["tbs"], t.get("Qm", 0), t.get("ncs", 0),
                                    int(t.get("pass_data", True)), t.get("ack_len", 0), t.get("ack", 0)))
                if t.get("rar"):
                    bits = list(t["rar"])
                    f.write(struct.pack("i", 20))
                    f.write(bytes(bits + [0] * (64 - len(bits))))
                else:
                    f.write(struct.pack("i", dci.nof_bits if dci else 0))
                    f.write(bytes(dci.data) if dci else bytes(64))
                raw_cqi = list(t.get("cqi_bits", []))
                f.write(struct.pack("3i", t["cqi_wb"] + 1 if "cqi_wb" in t else -len(raw_cqi), t.get("ri_len", 0),
                                    t.get("ri", 0)))
                f.write(bytes(raw_cqi + [0] * (64 - len(raw_cqi))))
                f.write(np.ascontiguousarray(t["tb"], np.uint8).tobytes())
        subprocess.check_call([HARNESS, fin, fout], timeout=300)
        raw = open(fout, "rb").read()
    out, pos = [], 0
    for _ in txs:
        r = struct.unpack_from("7i", raw, pos)[:6] + (struct.unpack_from("7i", raw, pos)[6],)
        pos += 28
        iq = np.frombuffer(raw[pos:pos + 15 * N * 8], np.float32)
        pos += 15 * N * 8
        out.append((r, iq))
    return out


def oracle_iq(cell_id, nof_prb, t, sf, dmrs=(0, 0, 0, 0), n_prb=None, L=None, Qm=None, ncs=None, ioff=0, n_prb1=None,
              cqi_ioff=2, ri_ioff=0):
    # srsUE's wideband CQI: 4 bits, MSB first (36.212 Table 5.2.2.6.2-1 wideband CQI field)
    cqi = [(t["cqi_wb"] >> (3 - i)) & 1 for i in range(4)] if "cqi_wb" in t else list(t.get("cqi_bits", []))
    c = O.ul_cfg(n_prb1=n_prb1, cell_id=cell_id, nof_prb=nof_prb, sf_idx=sf, rnti=t["rnti"], n_prb=t.get("n_prb", 0) if n_prb is None else n_prb,
                 L_prb=t.get("L_prb") if L is None else L, tbs=t["tbs"], Qm=t.get("Qm") if Qm is None else Qm,
                 rv=t["rv"], gh=dmrs[0], sh=dmrs[1], dss=dmrs[2], cs=dmrs[3], n2=t.get("ncs", 0) if ncs is None else ncs,
                 ack_len=t.get("ack_len", 0), ack=t.get("ack", 0), ioff=ioff, cqi=cqi, cqi_ioff=cqi_ioff,
                 ri_len=t.get("ri_len", 0), ri=t.get("ri", 0), ri_ioff=ri_ioff)
    iq = np.zeros(2 * 15 * NFFT[nof_prb], np.float32)
    assert O.lib().or_pusch_encode(ctypes.byref(c), t["tb"], iq) == 0
    return iq


def rel_err(a, b):
    return float(np.sqrt(np.mean((a - b) ** 2)) / np.sqrt(np.mean(b ** 2)))


def tb(seed, tbs):
    return np.random.default_rng(seed).integers(0, 256, tbs // 8, dtype=np.uint8)


@pytest.fixture(scope="module", autouse=True)
def _built(built):
    assert os.path.exists(HARNESS)


def test_direct_grants_match_oracle():
    dmrs = (0, 1, 2, 3)
    txs = [dict(tti=14, rnti=0x46, rv=0, n_prb=0, L_prb=100, tbs=43816, Qm=4, ncs=2, tb=tb(1, 43816)),
           dict(tti=27, rnti=0x1234, rv=0, n_prb=20, L_prb=50, tbs=12216, Qm=6, ncs=5, tb=tb(2, 12216)),
           dict(tti=9, rnti=0x46, rv=1, n_prb=4, L_prb=3, tbs=256, Qm=2, ncs=0, tb=tb(3, 256))]
    res = run(7, 100, txs, dmrs=dmrs)
    for t, (r, iq) in zip(txs, res):
        assert r[0] == 0
        assert rel_err(iq, oracle_iq(7, 100, t, t["tti"] % 10, dmrs)) < TOL


def test_dci_format0_grant_and_harq_retransmission():
    """PDCCH-style grant (format 0 bits) -> cfg_grant -> encode; then rv 2 with payload NULL re-encodes the
    TB the softbuffer kept from the rv 0 transmission."""
    m = format0(100, 0, 100, 20, ncs=3)        # 16QAM, I_TBS 19
    T = 43816
    data = tb(9, T)
    txs = [dict(tti=33, rnti=0x46, rv=0, dci=m, tbs=T, tb=data),
           dict(tti=41, rnti=0x46, rv=2, dci=m, tbs=T, tb=np.zeros(T // 8, np.uint8), pass_data=False)]
    res = run(1, 100, txs)
    for t, (r, iq) in zip(txs, res):
        assert r[0] == 0 and r[1:6] == (0, 100, T, 4, 3) and r[6] == 0
        ref = oracle_iq(1, 100, dict(t, tb=data), t["tti"] % 10, n_prb=0, L=100, Qm=4, ncs=3)
        assert rel_err(iq, ref) < TOL


def test_normalisation_and_cfo():
    t = dict(tti=5, rnti=0x77, rv=0, n_prb=0, L_prb=25, tbs=5736, Qm=2, ncs=1, tb=tb(4, 5736))
    cfo = 0.37
    (r, iq), = run(3, 25, [t], flags=3, cfo=cfo)
    assert r[0] == 0
    ref = oracle_iq(3, 25, t, 5).reshape(-1, 2)
    N = NFFT[25]
    z = (ref[:, 0] + 1j * ref[:, 1]) * (25 / 15 / np.sqrt(25)) * np.exp(2j * np.pi * cfo * np.arange(len(ref)) / N)
    ref2 = np.stack([z.real, z.imag], 1).astype(np.float32).ravel()
    assert rel_err(iq, ref2) < 2e-4


def test_retransmission_without_stored_tb_is_rejected():
    T = 5736
    txs = [dict(tti=5, rnti=0x46, rv=0, n_prb=0, L_prb=25, tbs=T, Qm=2, ncs=0, tb=tb(5, T), pass_data=False)]
    (r, _), = run(3, 25, txs)       # nothing stored in the fresh softbuffer and no data: error
    assert r[0] == -3


@pytest.mark.parametrize("ack", [0, 1])
def test_harq_ack_on_pusch_srsue_call_order(ack):
    """srsUE multiplexes the DL HARQ-ACK into the PUSCH when both fall in one TTI (uci_ack_len = 1,
    phch_worker.cc:486-487, 555): the encoded subframe matches the oracle's ACK multiplexing (36.212
    5.2.2.6 / 5.2.2.8, beta_offset index 6 from set_cfg's uci_cfg)."""
    txs = [dict(tti=12, rnti=0x46, rv=0, n_prb=0, L_prb=25, tbs=5736, Qm=2, ncs=0, tb=tb(6, 5736), ack_len=1, ack=ack),
           dict(tti=16, rnti=0x46, rv=0, n_prb=0, L_prb=50, tbs=12216, Qm=4, ncs=1, tb=tb(7, 12216), ack_len=1,
                ack=1 - ack)]
    res = run(9, 50, txs, flags=6 << 8)
    for t, (r, iq) in zip(txs, res):
        assert r[0] == 0
        assert rel_err(iq, oracle_iq(9, 50, t, t["tti"] % 10, ioff=6)) < TOL


@pytest.mark.parametrize("intra", [True, False])
def test_type1_frequency_hopping_srsue_call_order(intra):
    """DCI format 0 with the hopping flag (type 1, 36.213 8.4.1 / Table 8.4-2) through
    srslte_dci_msg_to_ul_grant(.., n_rb_ho = pusch-HoppingOffset, ..) and cfg_grant: intra-subframe mode
    moves slot 1; inter-subframe mode moves the whole subframe when CURRENT_TX_NB is odd."""
    from test_ul_grant import hop_expect
    n_ho, start, L = 6, 4, 6                          # N_RB^PUSCH = 94, '10': hop by N / 2
    from srsue_amd import abi
    T = abi.lib().srslte_ra_tbs_from_idx(19, L)      # MCS 20: 16QAM, I_TBS 19
    m = format0(100, start, L, 20, ncs=1, hop=1, hbits=2)
    data = tb(31, T)
    flags = (n_ho << 12) | ((1 << 20) if intra else 0)
    txs = [dict(tti=12 + 8 * k, rnti=0x46, rv=0 if k == 0 else 2, tx_nb=k, dci=m, tbs=T, tb=data if k == 0 else
                np.zeros(T // 8, np.uint8), pass_data=k == 0) for k in range(2)]
    res = run(3, 100, txs, flags=flags)
    a = start + n_ho // 2
    b = hop_expect(100, n_ho, start, 2) + n_ho // 2
    for k, (t, (r, iq)) in enumerate(zip(txs, res)):
        s0, s1 = (a, b) if intra else ((b, b) if k % 2 else (a, a))
        assert r[0] == 0 and (r[1], r[6]) == (s0, s1), (k, r)
        ref = oracle_iq(3, 100, dict(t, tb=data), t["tti"] % 10, n_prb=s0, L=L, Qm=4, ncs=1,
                        n_prb1=s1 if s1 != s0 else None)
        assert rel_err(iq, ref) < TOL


def test_periodic_cqi_and_ri_on_pusch_srsue_call_order():
    """srsUE packs a periodic wideband CQI into uci_data (srslte_cqi_value_pack, phch_worker.cc:507-523) before
    srslte_ue_ul_pusch_encode_rnti_softbuffer (:555): the PUSCH carries it (36.212 5.2.2.6.4 (32, O) code,
    multiplexed ahead of the data), with and without the HARQ-ACK bit; RI (1 / 2 bits) and a long raw CQI
    report (CRC8 + convolutional code) through the same call.  beta_offset indices from set_cfg's uci_cfg
    (I_offset_cqi 9, I_offset_ri 6, I_offset_ack 6); every subframe matches the oracle within 1e-4."""
    long_cqi = list(np.random.default_rng(5).integers(0, 2, 30).astype(int))
    txs = [dict(tti=12, rnti=0x46, rv=0, n_prb=0, L_prb=25, tbs=5736, Qm=2, ncs=0, tb=tb(16, 5736), cqi_wb=11),
           dict(tti=16, rnti=0x46, rv=0, n_prb=5, L_prb=40, tbs=12216, Qm=4, ncs=1, tb=tb(17, 12216), cqi_wb=7,
                ack_len=1, ack=1),
           dict(tti=23, rnti=0x46, rv=0, n_prb=0, L_prb=50, tbs=21384, Qm=6, ncs=2, tb=tb(18, 21384), ri_len=1, ri=1,
                ack_len=1, ack=0),
           dict(tti=27, rnti=0x46, rv=0, n_prb=10, L_prb=30, tbs=7992, Qm=4, ncs=3, tb=tb(19, 7992),
                cqi_bits=long_cqi, ri_len=2, ri=2)]
    res = run(9, 50, txs, flags=(6 << 8) | (9 << 21) | (6 << 25))
    for t, (r, iq) in zip(txs, res):
        assert r[0] == 0
        assert rel_err(iq, oracle_iq(9, 50, t, t["tti"] % 10, ioff=6, cqi_ioff=9, ri_ioff=6)) < TOL


def rar_bits(hop, rba, tmcs, tpc=1, delay=0, cqi=0):
    """the 20 RAR UL-grant bits (36.213 6.2) as the MAC hands them to the PHY (phy.cc:248, phch_common.cc:122)"""
    return [int(b) for b in f"{hop:01b}{rba:010b}{tmcs:04b}{tpc:03b}{delay:01b}{cqi:01b}"]


@pytest.mark.parametrize("nof_prb,start,L,tmcs", [(25, 7, 1, 3), (50, 12, 2, 6), (6, 0, 1, 0), (100, 40, 2, 10)])
def test_msg3_rar_grant_small_allocation(nof_prb, start, L, tmcs):
    """srsUE's Msg3 path (phch_worker.cc:412-415 then :551-555): the RAR grant's 20 bits -> rar_grant_unpack ->
    rar_to_ul_grant -> cfg_grant -> pusch_encode, 1- and 2-PRB allocations (the tabulated DMRS base sequences of
    36.211 5.5.1.2), with group hopping on; the IQ matches the oracle's transmitter within 1e-4."""
    from test_ul_grant import riv, ul_mcs
    from srsue_amd import abi
    qm, itbs = ul_mcs(tmcs)
    T = abi.lib().srslte_ra_tbs_from_idx(itbs, L)
    t = dict(tti=21, rnti=0x3C, rv=0, rar=rar_bits(0, riv(nof_prb, start, L), tmcs), tbs=T, tb=tb(40 + L, T))
    (r, iq), = run(11, nof_prb, [t], dmrs=(1, 0, 2, 3))
    assert r[0] == 0 and (r[1], r[2], r[4], r[6]) == (start, L, qm, start)
    assert rel_err(iq, oracle_iq(11, nof_prb, t, t["tti"] % 10, dmrs=(1, 0, 2, 3), n_prb=start, L=L, Qm=qm,
                                 ncs=0)) < TOL


@pytest.mark.parametrize("n_sb,intra,via", [(1, True, "dci"), (2, False, "dci"), (3, True, "dci"), (4, True, "rar"),
                                            (2, True, "rar")])
def test_type2_subband_hopping_srsue_call_order(n_sb, intra, via):
    """PUSCH hopping type 2 (36.211 5.3.4): the all-ones hopping bits of a format-0 or RAR grant, the cell's
    pusch-HoppingSubbands / -Offset / hopping mode from set_cfg, several TTIs and CURRENT_TX_NB values; the slot
    PRBs cfg_grant chooses equal the oracle's restatement (or_pusch_hop_type2) and the IQ matches the oracle's
    transmitter on those PRBs within 1e-4."""
    import ctypes as C
    from test_ul_grant import riv, ul_mcs
    from srsue_amd import abi
    nof_prb, n_ho, start, L, mcs = 50, 4, 9, 2, 6
    qm, itbs = ul_mcs(mcs)
    T = abi.lib().srslte_ra_tbs_from_idx(itbs, L)
    data = tb(50 + n_sb, T)
    if via == "dci":
        grant = dict(dci=format0(nof_prb, start, L, mcs, ncs=2, hop=1, hbits=3))
    else:
        # N = 50 > 44: the RBA's 2 MSBs are the hopping bits ('11': type 2), its 8 LSBs the RIV's low bits
        grant = dict(rar=rar_bits(1, (3 << 8) | riv(nof_prb, start, L), mcs))
    flags = (n_ho << 12) | ((1 << 20) if intra else 0) | ((n_sb - 1) << 29)
    txs = [dict(tti=tt, rnti=0x46, rv=0, tx_nb=k, tbs=T, tb=data, **grant) for k, tt in enumerate((3, 8, 17, 26))]
    res = run(5, nof_prb, txs, flags=flags)
    O.lib().or_pusch_hop_type2.restype = C.c_int
    moved = 0
    for t, (r, iq) in zip(txs, res):
        sf = t["tti"] % 10
        s = []
        for sl in range(2):
            prb = (C.c_uint32 * L)()
            s.append(O.lib().or_pusch_hop_type2(nof_prb, n_ho, n_sb, int(intra), 5, start, L, 2 * sf + sl, t["tx_nb"], prb))
        assert min(s) >= 0
        assert r[0] == 0 and (r[1], r[6]) == tuple(s), (t, r, s)
        moved += s[0] != start or s[1] != start
        ncs = 0 if via == "rar" else 2
        ref = oracle_iq(5, nof_prb, t, sf, n_prb=s[0], L=L, Qm=qm, ncs=ncs, n_prb1=s[1] if s[1] != s[0] else None)
        assert rel_err(iq, ref) < TOL
    assert moved > 0
