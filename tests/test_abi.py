"""CPU: the C-ABI library builds, loads and exports every function declared in include/*.h; the
headers compile as plain C (what srsUE's build would see); the product's synthetic transmitter is
sample-identical to the oracle's transmitter (independent implementations of the same chain)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_lib as O
from srsue_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", "srslte", "srslte.h"), os.path.join(ROOT, "include", "mi_dl.h"),
           os.path.join(ROOT, "include", "mi_ul.h"), os.path.join(ROOT, "include", "srslte", "common", "timestamp.h"),
           os.path.join(ROOT, "include", "srslte", "utils", "debug.h"),
           os.path.join(ROOT, "include", "srslte", "utils", "bit.h")]
OOS_BEGIN = "OUT OF SCOPE (SURVEY.md 8"
OOS_END = "host utilities srsUE calls outside the worker"


def out_of_scope():
    """functions srslte.h declares between its OUT OF SCOPE marker and the host-utilities block: declared only
    so srsUE's PHY compiles unchanged (PUCCH / SRS / UL power control, PRACH, cell search, MIB)"""
    src = open(HEADERS[0]).read()
    a, b = src.index(OOS_BEGIN), src.index(OOS_END)
    seg = src[a - 8:b]
    names = set()
    for m in re.finditer(r"SRSLTE_API\s+[A-Za-z_][\w\s\*]*?\b(\w+)\s*\(", re.sub(r"/\*.*?\*/", "", seg, flags=re.S)):
        names.add(m.group(1))
    return names


OUT_OF_SCOPE = out_of_scope()


def declared_functions(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set()
    for m in re.finditer(r"(?:SRSLTE_API\s+)?[A-Za-z_][\w\s\*]*?\b(\w+)\s*\([^;{]*\)\s*;", src):
        n = m.group(1)
        if n.startswith(("srslte_", "mi_", "get_time_interval")):
            names.add(n)
    return names


def test_library_exports_every_declared_symbol(built):
    lib = abi.lib()
    missing = []
    for h in HEADERS:
        for n in sorted(declared_functions(h) - OUT_OF_SCOPE):
            if not hasattr(lib, n):
                missing.append(n)
    assert not missing, missing
    assert len(declared_functions(HEADERS[0])) >= 25
    assert OUT_OF_SCOPE <= declared_functions(HEADERS[0])
    # PUCCH / SRS / UL power control, PRACH, cell search and MIB decoding -- and nothing on the DL data path
    assert {"srslte_ue_ul_pucch_encode", "srslte_prach_gen", "srslte_ue_cellsearch_scan",
            "srslte_ue_mib_sync_decode"} <= OUT_OF_SCOPE
    assert not any(n.startswith(("srslte_ue_dl", "srslte_pdsch", "srslte_softbuffer", "srslte_chest")) for n in OUT_OF_SCOPE)
    lib = abi.lib()
    assert not [n for n in OUT_OF_SCOPE if hasattr(lib, n)], "an out-of-scope symbol is exported"


def test_headers_compile_as_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "srslte/srslte.h"\n#include "mi_dl.h"\n#include "mi_ul.h"\n'
                   "int main(void){srslte_ue_dl_t q; srslte_softbuffer_rx_t s; (void)q; (void)s;"
                   " return SRSLTE_VERSION_CHECK(1,0,0) ? 0 : 1;}\n")
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                           str(src)])


def test_version_and_helpers(built):
    lib = abi.lib()
    lib.srslte_check_version.restype = C.c_int
    assert lib.srslte_check_version(1, 0, 0) == 1
    assert lib.srslte_check_version(2, 0, 0) == 0
    assert lib.srslte_symbol_sz(100) == 2048 and lib.srslte_symbol_sz(75) == 1536 and lib.srslte_symbol_sz(6) == 128
    assert lib.srslte_ra_tbs_idx_from_mcs(28) == 26
    assert lib.srslte_ra_tbs_from_idx(26, 100) == 75376
    assert lib.mi_sf_len(100) == 30720


@pytest.mark.parametrize("nprb,ports,sf,cfi,tbs,qm", [(100, 1, 1, 1, 75376, 6), (100, 2, 0, 2, 61664, 6),
                                                      (75, 1, 5, 3, 40000, 6), (6, 2, 9, 2, 1000, 2),
                                                      (25, 1, 3, 1, 7000, 4)])
def test_product_tx_matches_oracle_tx(built, nprb, ports, sf, cfi, tbs, qm):
    cfg = abi.sf_cfg(cell_id=13, nof_prb=nprb, nof_ports=ports, sf_idx=sf, cfi=cfi, tbs=tbs, Qm=qm, rv=sf % 4)
    tb = O.splitmix_bytes(sf, tbs // 8)
    h = [0.9 + 0.2j, -0.3 + 0.6j]
    a = abi.tx_subframe(cfg, tb, h=h[:ports] if ports == 2 else [h[0]], snr_db=300.0)
    cell = O.make_cell(13, nprb, ports)
    oc = O.tx_cfg(cell, sf_idx=sf, cfi=cfi, tm=2 if ports == 2 else 1, tbs=tbs, qm=qm, rv=sf % 4, snr_db=300.0,
                  h=h if ports == 2 else [h[0], 0j])
    b, _ = O.tx_subframe(oc, tb)
    assert np.max(np.abs(a - b)) < 1e-5 * np.sqrt(np.mean(b * b))


def test_product_lib_fails_loudly_without_gpu(built):
    """No CPU fallback: planning a batch needs the HIP runtime and a device."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        abi.Batch([abi.sf_cfg()])


def test_srslte_reporting_helpers(built):
    """The srsLTE host helpers srsUE's worker calls (srslte_util.cpp): 36.213 reporting instants and the
    CQI packing used for UCI (phch_worker.cc:495-532)."""
    import ctypes as C
    from srsue_amd import abi
    L = abi.lib()
    L.srslte_cqi_send.restype = C.c_bool
    L.srslte_ue_ul_sr_send_tti.restype = C.c_bool
    L.srslte_cqi_from_snr.restype = C.c_uint8
    L.srslte_cqi_from_snr.argtypes = [C.c_float]
    # CQI: I = 2..6 -> N_pd 5, offset I - 2; I = 20 -> N_pd 20, offset 3
    assert [L.srslte_cqi_send(4, t) for t in range(10)] == [t % 5 == 2 for t in range(10)]
    assert [t for t in range(60) if L.srslte_cqi_send(20, t)] == [3, 23, 43]
    assert not L.srslte_cqi_send(317, 0)
    # SR: I = 7 -> period 10, offset 2; I = 157 -> every subframe
    assert [t for t in range(30) if L.srslte_ue_ul_sr_send_tti(7, t)] == [2, 12, 22]
    assert all(L.srslte_ue_ul_sr_send_tti(157, t) for t in range(12))
    # SRS: cell config 7 = subframes {0, 1} mod 5; UE I = 10 -> period 10, offset 3
    assert [L.srslte_refsignal_srs_send_cs(7, s) for s in range(10)] == [1, 1, 0, 0, 0, 1, 1, 0, 0, 0]
    assert [t for t in range(25) if L.srslte_refsignal_srs_send_ue(10, t) == 1] == [3, 13, 23]
    assert L.srslte_tti_interval(5, 10230) == 15 and L.srslte_tti_interval(20, 8) == 12
    assert L.srslte_cqi_from_snr(-3.0) == 0 and L.srslte_cqi_from_snr(30.0) == 15 and L.srslte_cqi_from_snr(10.5) == 5

    class Cqi(C.Structure):
        _fields_ = [("v0", C.c_uint8), ("v1", C.c_uint8), ("type", C.c_int)]
    buf = (C.c_uint8 * 64)()
    v = Cqi(11, 0, 0)
    assert L.srslte_cqi_value_pack(C.byref(v), buf) == 4 and list(buf[:4]) == [1, 0, 1, 1]
    v = Cqi(6, 1, 1)
    assert L.srslte_cqi_value_pack(C.byref(v), buf) == 5 and list(buf[:5]) == [0, 1, 1, 0, 1]


def test_host_utilities_outside_the_worker(built):
    """bit utilities, MIB unpacking, RAR grant unpacking and timing advance (srslte.h host-utilities block;
    phch_recv.cc:216,220,253, phch_common.cc:122, phy.cc:125-132, pdu.cc:776,791)"""
    lib = abi.lib()
    rng = np.random.default_rng(7)
    for nbits in (1, 7, 8, 13, 24, 32):
        bits = rng.integers(0, 2, nbits, dtype=np.uint8)
        packed = np.zeros((nbits + 7) // 8, np.uint8)
        lib.srslte_bit_pack_vector(bits.ctypes.data_as(C.c_void_p), packed.ctypes.data_as(C.c_void_p), nbits)
        assert np.array_equal(packed, np.packbits(bits)), nbits      # MSB first, trailing byte left-aligned
        back = np.zeros(nbits, np.uint8)
        lib.srslte_bit_unpack_vector(packed.ctypes.data_as(C.c_void_p), back.ctypes.data_as(C.c_void_p), nbits)
        assert np.array_equal(back, bits)
    # cursor form: pack / unpack advance the caller's pointer
    buf = (C.c_uint8 * 16)()
    cur = C.cast(buf, C.POINTER(C.c_uint8))
    lib.srslte_bit_unpack.argtypes = [C.c_uint32, C.POINTER(C.POINTER(C.c_uint8)), C.c_int]
    lib.srslte_bit_unpack(0x2D, C.byref(cur), 6)
    lib.srslte_bit_unpack(0x5, C.byref(cur), 3)
    assert list(buf[:9]) == [1, 0, 1, 1, 0, 1, 1, 0, 1]
    cur = C.cast(buf, C.POINTER(C.c_uint8))
    lib.srslte_bit_pack.argtypes = [C.POINTER(C.POINTER(C.c_uint8)), C.c_int]
    lib.srslte_bit_pack.restype = C.c_uint32
    assert lib.srslte_bit_pack(C.byref(cur), 6) == 0x2D and lib.srslte_bit_pack(C.byref(cur), 3) == 0x5

    class Cell(C.Structure):
        _fields_ = [("nof_prb", C.c_uint32), ("nof_ports", C.c_uint32), ("bw_idx", C.c_uint32), ("id", C.c_uint32),
                    ("cp", C.c_int), ("phich_length", C.c_int), ("phich_resources", C.c_int)]
    for bw, prb in enumerate((6, 15, 25, 50, 75, 100)):
        for sfn in (0, 4, 517, 1020):
            cell = Cell(prb, 2, 0, 1, 0, bw & 1, (bw + 1) & 3)
            mib = np.zeros(24, np.uint8)
            lib.srslte_pbch_mib_pack(C.byref(cell), sfn, mib.ctypes.data_as(C.c_void_p))
            # 36.331 MIB: 3 bandwidth bits, phich-Duration, 2 phich-Resource bits, 8 SFN MSBs, 10 spare
            want = [int(b) for b in f"{bw:03b}{bw & 1:01b}{(bw + 1) & 3:02b}{sfn >> 2:08b}"] + [0] * 10
            assert mib.tolist() == want
            out, osfn = Cell(), C.c_uint32()
            lib.srslte_pbch_mib_unpack(mib.ctypes.data_as(C.c_void_p), C.byref(out), C.byref(osfn))
            assert (out.nof_prb, out.phich_length, out.phich_resources, osfn.value) == (prb, bw & 1, (bw + 1) & 3,
                                                                                         sfn & ~3)

    class Rar(C.Structure):
        _fields_ = [("hopping_flag", C.c_bool), ("rba", C.c_uint32), ("trunc_mcs", C.c_uint32),
                    ("tpc_pusch", C.c_uint32), ("ul_delay", C.c_bool), ("cqi_request", C.c_bool)]
    for hop, rba, mcs, tpc, dly, cqi in [(1, 0x2A5, 9, 5, 0, 1), (0, 1023, 15, 7, 1, 0), (0, 0, 0, 0, 0, 0)]:
        g = np.array([int(b) for b in f"{hop:01b}{rba:010b}{mcs:04b}{tpc:03b}{dly:01b}{cqi:01b}"], np.uint8)
        r = Rar()
        lib.srslte_dci_rar_grant_unpack(C.byref(r), g.ctypes.data_as(C.c_void_p))
        assert (r.hopping_flag, r.rba, r.trunc_mcs, r.tpc_pusch, r.ul_delay, r.cqi_request) == (
            bool(hop), rba, mcs, tpc, bool(dly), bool(cqi))
    # 36.213 4.2.3 timing advance
    lib.srslte_N_ta_new_rar.restype = C.c_uint32
    lib.srslte_N_ta_new.restype = C.c_uint32
    assert lib.srslte_N_ta_new_rar(1282) == 20512
    assert lib.srslte_N_ta_new(20512, 31) == 20512 and lib.srslte_N_ta_new(20512, 63) == 20512 + 512
    assert lib.srslte_N_ta_new(100, 0) == 0
