"""ctypes bindings to oracle/liboracle.so -- the CPU restatement used as the parity checker.

Test infrastructure only (imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg).  Builds the library on first use if it is missing (gcc, oracle/Makefile).
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

NRB_MAX = 110
NSYMB = 14


class Cell(C.Structure):
    _fields_ = [("id", C.c_uint32), ("nof_prb", C.c_uint32), ("nof_ports", C.c_uint32)]


class CbSegm(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("C", "Cp", "Cm", "Kp", "Km", "F", "B")]


class CtrlCfg(C.Structure):
    _fields_ = [("cell", Cell), ("ng", C.c_uint32), ("cfi", C.c_uint32), ("sf", C.c_uint32)]


class Dci1a(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("rb_start", "L_crb", "mcs", "harq", "ndi", "rv", "tpc")]


class DciFound(C.Structure):
    _fields_ = [("format", C.c_uint32), ("nbits", C.c_uint32), ("L", C.c_uint32), ("ncce", C.c_uint32),
                ("bits", C.c_uint8 * 64)]


class DlGrant(C.Structure):
    _fields_ = [("prb", C.c_uint8 * NRB_MAX)] + [(n, C.c_uint32) for n in (
        "format", "alloc_type", "distributed", "gap2", "nof_prb", "mcs", "harq", "ndi", "rv", "tpc", "Qm", "i_tbs",
        "n_prb_tbs")] + [("tbs", C.c_int)]


DCI_0, DCI_1, DCI_1A, DCI_1C = 0, 1, 2, 3


class TxCfg(C.Structure):
    _fields_ = [
        ("cell", Cell),
        ("sf_idx", C.c_uint32), ("cfi", C.c_uint32), ("mcs", C.c_uint32), ("rv", C.c_uint32),
        ("rnti", C.c_uint32), ("tm", C.c_uint32),
        ("tbs", C.c_uint32), ("qm", C.c_uint32),
        ("prb_mask", C.c_uint8 * NRB_MAX),
        ("snr_db", C.c_float),
        ("h_re", C.c_float * 2), ("h_im", C.c_float * 2),
        ("noise_seed", C.c_uint64),
        ("nl_td", C.c_uint32),
    ]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = np.ctypeslib.ndpointer
        f32 = P(np.float32, flags="C_CONTIGUOUS")
        u8 = P(np.uint8, flags="C_CONTIGUOUS")
        u32 = P(np.uint32, flags="C_CONTIGUOUS")
        sig = {
            "or_symbol_sz": (C.c_int, [C.c_uint32]),
            "or_sf_len": (C.c_int, [C.c_uint32]),
            "or_gold": (None, [C.c_uint32, u8, C.c_uint32]),
            "or_crc": (C.c_uint32, [u8, C.c_uint32, C.c_uint32, C.c_int]),
            "or_crc24a": (C.c_uint32, [u8, C.c_uint32]),
            "or_crc24b": (C.c_uint32, [u8, C.c_uint32]),
            "or_crc16": (C.c_uint32, [u8, C.c_uint32]),
            "or_cb_size": (C.c_uint32, [C.c_uint32]),
            "or_cb_size_idx": (C.c_int, [C.c_uint32]),
            "or_qpp": (C.c_int, [C.c_uint32, u32]),
            "or_qpp_f": (C.c_int, [C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
            "or_cbsegm": (C.c_int, [C.c_uint32, C.POINTER(CbSegm)]),
            "or_tbs": (C.c_int, [C.c_uint32, C.c_uint32]),
            "or_mcs": (C.c_int, [C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
            "or_crs_seq": (None, [C.c_uint32, C.c_uint32, C.c_uint32, f32]),
            "or_pdsch_re_list": (C.c_int, [C.POINTER(Cell), C.c_uint32, C.c_uint32, u8, u32]),
            "or_rm_E": (C.c_int, [C.c_uint32] * 5),
            "or_ncb": (C.c_uint32, [C.c_uint32]),
            "or_tcod": (C.c_int, [u8, C.c_uint32, C.c_uint32, u8]),
            "or_rm_tx": (C.c_int, [u8, C.c_uint32, C.c_uint32, C.c_uint32, u8]),
            "or_rm_rx": (C.c_int, [f32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, f32, f32]),
            "or_decode_cb": (C.c_int, [C.c_void_p, f32, C.c_uint32, C.c_uint32, C.c_int, C.c_int, u8,
                                       C.POINTER(C.c_int)]),
            "or_decode_cb16": (C.c_int, [C.c_void_p, f32, C.c_uint32, C.c_uint32, C.c_int, C.c_int, u8,
                                         C.POINTER(C.c_int)]),
            "or_q16": (C.c_int32, [C.c_float]),
            "or_simd_tdec_size": (C.c_size_t, []),
            "or_simd_decode_cb": (C.c_int, [C.c_void_p, f32, C.c_uint32, C.c_uint32, C.c_int, C.c_int, u8,
                                            C.POINTER(C.c_int)]),
            "or_simd_decode_batch": (C.c_int, [f32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                               C.c_int, u8, u32, u8, C.c_uint32]),
            "or_avx2_available": (C.c_int, []),
            "or_avx2_tdec_size": (C.c_size_t, []),
            "or_avx2_decode_pair": (C.c_int, [C.c_void_p, f32, C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_int,
                                              u8, C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                              C.POINTER(C.c_int), C.POINTER(C.c_int)]),
            "or_avx2_decode_batch": (C.c_int, [f32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                               C.c_int, u8, u32, u8, C.c_uint32]),
            "or_set_tdec_mode": (None, [C.c_int]),
            "or_get_tdec_mode": (C.c_int, []),
            "or_phich_ngroups": (C.c_uint32, [C.c_uint32, C.c_uint32]),
            "or_pdcch_regs": (C.c_int, [C.POINTER(CtrlCfg), C.c_void_p, C.POINTER(C.c_uint32)]),
            "or_pdcch_quad_perm": (None, [C.c_uint32, C.c_uint32, u32]),
            "or_pdcch_llr": (C.c_int, [C.POINTER(CtrlCfg), f32, f32, C.c_float, f32, C.POINTER(C.c_uint32)]),
            "or_conv_encode_tb": (None, [u8, C.c_uint32, u8]),
            "or_conv_rm_tx": (C.c_int, [u8, C.c_uint32, C.c_uint32, u8]),
            "or_conv_rm_rx": (None, [f32, C.c_uint32, C.c_uint32, f32]),
            "or_viterbi_tb": (None, [f32, C.c_uint32, u8]),
            "or_dci_size": (C.c_uint32, [C.c_uint32, C.c_uint32]),
            "or_riv": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32]),
            "or_dci1a_pack": (C.c_int, [C.c_uint32, C.POINTER(Dci1a), u8]),
            "or_dci1a_unpack": (C.c_int, [C.c_uint32, u8, C.c_uint32, C.POINTER(Dci1a)]),
            "or_dci_encode": (C.c_int, [u8, C.c_uint32, C.c_uint16, C.c_uint32, u8]),
            "or_dci_decode": (C.c_int, [f32, C.c_uint32, C.c_uint32, C.c_uint16, C.c_void_p]),
            "or_search_space": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint16, C.c_int, u32, u32]),
            "or_find_dci": (C.c_int, [f32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint16, C.c_int,
                                      C.POINTER(DciFound)]),
            "or_find_dci_mode": (C.c_int, [f32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint16, C.c_int,
                                           C.POINTER(DciFound)]),
            "or_rbg_size": (C.c_uint32, [C.c_uint32]),
            "or_ngap": (C.c_uint32, [C.c_uint32, C.c_int]),
            "or_nvrb_dist": (C.c_uint32, [C.c_uint32, C.c_int]),
            "or_vrb_to_prb": (C.c_int, [C.c_uint32, C.c_int, C.c_uint32, C.c_uint32]),
            "or_dci1c_size": (C.c_uint32, [C.c_uint32]),
            "or_dl_dci_to_grant": (C.c_int, [u8, C.c_uint32, C.c_uint16, C.c_uint32, C.POINTER(DlGrant)]),
            "or_tx_pdcch": (C.c_int, [C.POINTER(CtrlCfg), C.c_uint16, C.c_uint32, C.c_uint32, u8, C.c_uint32,
                                      C.c_void_p, f32]),
            "or_phich_calc": (None, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_uint32)]),
            "or_phich_cinit": (C.c_uint32, [C.c_uint32, C.c_uint32]),
            "or_phich_res": (C.c_int, [C.POINTER(CtrlCfg), C.c_uint32, u32]),
            "or_phich_soft": (C.c_float, [C.POINTER(CtrlCfg), f32, f32, C.c_uint32, C.c_uint32]),
            "or_tx_phich": (C.c_int, [C.POINTER(CtrlCfg), C.c_uint32, C.c_uint32, C.c_int, C.c_void_p, f32]),
            "or_pss_seq": (None, [C.c_uint32, f32]),
            "or_sss_m": (None, [C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
            "or_sss_seq": (None, [C.c_uint32, C.c_uint32, C.c_uint32, f32]),
            "or_pss_time": (None, [C.c_uint32, C.c_uint32, f32]),
            "or_sync_sym_off": (C.c_uint32, [C.c_uint32, C.c_uint32]),
            "or_tx_sync": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_float, f32]),
            "or_pss_find": (C.c_int, [f32, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(PssRes)]),
            "or_cfo_correct": (None, [f32, C.c_uint32, C.c_float, C.c_uint32, f32]),
            "or_sss_detect": (C.c_int, [f32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_float)]),
            "or_pusch_G": (C.c_uint32, [C.POINTER(UlCfg)]),
            "or_ulsch_encode": (C.c_int, [C.POINTER(UlCfg), u8, u8]),
            "or_pusch_mod": (C.c_int, [C.POINTER(UlCfg), u8, f32]),
            "or_dft_m": (None, [f32, C.c_uint32, f32, C.c_int]),
            "or_dmrs_params": (C.c_int, [C.POINTER(UlCfg), C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_uint32)]),
            "or_dmrs_pusch": (C.c_int, [C.POINTER(UlCfg), C.c_uint32, f32]),
            "or_pusch_grid": (C.c_int, [C.POINTER(UlCfg), u8, f32]),
            "or_scfdma_tx": (C.c_int, [C.c_uint32, f32, f32]),
            "or_pusch_encode": (C.c_int, [C.POINTER(UlCfg), u8, f32]),
            "or_ack_qprime": (C.c_uint32, [C.POINTER(UlCfg)]),
            "or_ack_block": (C.c_uint32, [C.POINTER(UlCfg), u8]),
            "or_ri_qprime": (C.c_uint32, [C.POINTER(UlCfg)]),
            "or_cqi_qprime": (C.c_uint32, [C.POINTER(UlCfg)]),
            "or_ri_block": (C.c_uint32, [C.POINTER(UlCfg), u8]),
            "or_cqi_encode": (C.c_int, [C.POINTER(UlCfg), u8]),
            "or_cqi_rm32": (C.c_uint32, [u8, C.c_uint32]),
            "or_tx_subframe": (C.c_int, [C.POINTER(TxCfg), u8, f32, C.POINTER(C.c_uint32)]),
            "or_ofdm_rx": (C.c_int, [C.POINTER(Cell), f32, f32]),
            "or_chest": (C.c_int, [C.POINTER(Cell), C.c_uint32, f32, f32, f32]),
            "or_pdsch_llr": (C.c_int, [C.POINTER(Cell), C.c_uint32, C.c_uint32, u8, C.c_uint32, C.c_uint32,
                                       C.c_uint32, C.c_float, f32, f32, f32, C.POINTER(C.c_uint32), C.c_void_p]),
            "or_pcfich": (C.c_int, [C.POINTER(Cell), C.c_uint32, f32, f32]),
            "or_dlsch_decode": (C.c_int, [f32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.c_int, f32, C.c_uint32, C.c_uint32, u8, C.POINTER(C.c_uint32),
                                          C.POINTER(C.c_uint32)]),
            "or_dlsch_decode_cbits": (C.c_int, [f32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                                C.c_int, f32, C.c_uint32, C.c_uint32, u8, C.POINTER(C.c_uint32),
                                                C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
            "or_decode_subframe": (C.c_int, [C.POINTER(Cell), C.c_uint32, C.c_uint32, u8, C.c_uint32, C.c_uint32,
                                             C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, f32, f32, C.c_uint32,
                                             C.c_int, C.c_uint32, u8, C.POINTER(C.c_uint32)]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


# ------------------------------------------------------------------ convenience wrappers
TDEC_STATE_BYTES = 4 + 4 * 6144 * 2 + 4 * 6144 * 3 + 4 * 6147 * 2 + 4 * 6148 * 8
TDEC16_STATE_BYTES = TDEC_STATE_BYTES + 4 * (3 * 6144 + 12)
TDEC_GEN, TDEC_I16, TDEC_SIMD, TDEC_AVX2 = 0, 1, 2, 3


def avx2_decode_pair(llr_a, llr_b, K, max_its=8, early_stop=True, crc24a=False, state=None):
    """Two equal-K code blocks through the AVX2 decoder (o_avx2.c; llr_b None: A alone).
    Returns [(bits, its, ok)] per block."""
    L = lib()
    st = state if state is not None else C.create_string_buffer(L.or_avx2_tdec_size() + 64)
    ba, bb = np.zeros(K, np.uint8), np.zeros(K, np.uint8)
    oka, okb, ia, ib = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    a = np.ascontiguousarray(llr_a, np.float32)
    b = None if llr_b is None else np.ascontiguousarray(llr_b, np.float32)
    assert L.or_avx2_decode_pair(st, a, None if b is None else b.ctypes.data, K, max_its, int(early_stop), int(crc24a),
                                 ba, None if b is None else bb.ctypes.data, C.byref(oka), C.byref(okb), C.byref(ia),
                                 C.byref(ib)) == 0
    out = [(ba, ia.value, bool(oka.value))]
    if b is not None:
        out.append((bb, ib.value, bool(okb.value)))
    return out


class Tdec:
    """One oracle turbo decoder; mode TDEC_GEN (float, srsLTE gen) or TDEC_I16 (int16, SSE design)."""
    def __init__(self, mode=TDEC_GEN):
        self.mode = mode
        size = {TDEC_GEN: TDEC_STATE_BYTES, TDEC_I16: TDEC16_STATE_BYTES}.get(mode) or lib().or_simd_tdec_size()
        self.buf = C.create_string_buffer(size + 64)

    def decode_cb(self, llr, K, max_its=8, early_stop=True, crc24a=False):
        bits = np.zeros(K, np.uint8)
        ok = C.c_int(0)
        fn = {TDEC_GEN: lib().or_decode_cb, TDEC_I16: lib().or_decode_cb16,
              TDEC_SIMD: lib().or_simd_decode_cb}[self.mode]
        its = fn(self.buf, np.ascontiguousarray(llr, np.float32), K, max_its,
                                 int(early_stop), int(crc24a), bits, C.byref(ok))
        return bits, its, bool(ok.value)


class tdec_mode:
    """Context manager selecting the decoder or_dlsch_decode / or_decode_subframe use."""
    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        self.prev = lib().or_get_tdec_mode()
        lib().or_set_tdec_mode(self.mode)

    def __exit__(self, *a):
        lib().or_set_tdec_mode(self.prev)


class UlCfg(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("cell_id", "nof_prb", "sf_idx", "rnti", "n_prb", "L_prb", "tbs", "Qm", "rv",
                                          "group_hopping", "sequence_hopping", "delta_ss", "cyclic_shift", "n_dmrs2",
                                          "ack_len", "ack", "I_offset_ack", "hop", "n_prb1", "cqi_len",
                                          "I_offset_cqi")] + [("cqi", C.c_uint8 * 64)] + \
        [(n, C.c_uint32) for n in ("ri_len", "ri", "I_offset_ri")]


def ul_cfg(cell_id=1, nof_prb=100, sf_idx=1, rnti=0x46, n_prb=0, L_prb=100, tbs=0, Qm=4, rv=0, gh=0, sh=0, dss=0,
           cs=0, n2=0, ack_len=0, ack=0, ioff=0, n_prb1=None, cqi=(), cqi_ioff=2, ri_len=0, ri=0, ri_ioff=0):
    """n_prb1: start PRB of slot 1 (frequency hopping), None = no hopping; cqi: CQI bits o_0.. (36.212
    5.2.2.6.4) with beta_offset index cqi_ioff; ri_len / ri / ri_ioff: RI on PUSCH"""
    hop, n1 = (0, 0) if n_prb1 is None else (1, n_prb1)
    c = UlCfg(cell_id, nof_prb, sf_idx, rnti, n_prb, L_prb, tbs, Qm, rv, gh, sh, dss, cs, n2, ack_len, ack, ioff,
              hop, n1, len(cqi), cqi_ioff)
    for i, b in enumerate(cqi):
        c.cqi[i] = b
    c.ri_len, c.ri, c.I_offset_ri = ri_len, ri, ri_ioff
    return c


class PssRes(C.Structure):
    _fields_ = [("nid2", C.c_uint32), ("lag", C.c_uint32), ("rho", C.c_float), ("cfo", C.c_float)]


def pss_find(x, nof_prb, nid2_mask, nlag):
    r = PssRes()
    assert lib().or_pss_find(np.ascontiguousarray(x, np.float32), nof_prb, nid2_mask, nlag, C.byref(r)) == 0
    return r.nid2, r.lag, r.rho, r.cfo


def cfo_correct(x, cfo, N):
    x = np.ascontiguousarray(x, np.float32)
    y = np.zeros_like(x)
    lib().or_cfo_correct(x, len(x) // 2, cfo, N, y)
    return y


def sss_detect(sf_iq, nof_prb, nid2):
    a, b, s = C.c_uint32(), C.c_uint32(), C.c_float()
    lib().or_sss_detect(np.ascontiguousarray(sf_iq, np.float32), nof_prb, nid2, C.byref(a), C.byref(b), C.byref(s))
    return a.value, b.value, s.value


def ctrl_cfg(cell_id=1, nof_prb=100, nof_ports=1, ng=2, cfi=1, sf=1):
    return CtrlCfg(Cell(cell_id, nof_prb, nof_ports), ng, cfi, sf)


def pdcch_llr(q, grid, ce):
    """Oracle PDCCH soft bits (logical CCE order) of a subframe's grid / channel estimates."""
    n = C.c_uint32()
    M = lib().or_pdcch_regs(C.byref(q), None, C.byref(n))
    llr = np.zeros(8 * M, np.float32)
    lib().or_pdcch_llr(C.byref(q), np.ascontiguousarray(grid, np.float32), np.ascontiguousarray(ce, np.float32),
                       0.0, llr, C.byref(n))
    return llr, n.value


def phich_calc(nof_prb, ng, i_lowest, n_dmrs):
    g, q = C.c_uint32(), C.c_uint32()
    lib().or_phich_calc(nof_prb, ng, i_lowest, n_dmrs, C.byref(g), C.byref(q))
    return g.value, q.value


def phich_soft(q, grid, ce, group, seq):
    """Oracle soft HI of PHICH (group, seq): > 0 favours ACK."""
    return lib().or_phich_soft(C.byref(q), np.ascontiguousarray(grid, np.float32),
                               np.ascontiguousarray(ce, np.float32), group, seq)


def find_dci(llr, n_cce, nof_prb, sf, rnti, ul=False, mode=None):
    """mode: 0 = DL C-RNTI, 1 = UL, 2 = DL SI/RA/P-RNTI (common space, 1A then 1C); default from ul"""
    out = DciFound()
    m = (1 if ul else 0) if mode is None else mode
    ok = lib().or_find_dci_mode(np.ascontiguousarray(llr, np.float32), n_cce, nof_prb, sf, rnti, m, C.byref(out))
    return (out.format, np.array(out.bits[:out.nbits], np.uint8), out.L, out.ncce) if ok else None


def dl_grant(bits, rnti, nof_prb):
    """or_dl_dci_to_grant: DlGrant or None"""
    g = DlGrant()
    b = np.ascontiguousarray(bits, np.uint8)
    return g if lib().or_dl_dci_to_grant(b, len(b), rnti, nof_prb, C.byref(g)) == 0 else None


def cbsegm(tbs):
    s = CbSegm()
    assert lib().or_cbsegm(tbs, C.byref(s)) == 0
    return s


def make_cell(cell_id=1, nof_prb=100, nof_ports=1):
    return Cell(cell_id, nof_prb, nof_ports)


def tx_cfg(cell, sf_idx=1, cfi=1, mcs=28, rv=0, rnti=0x46, tm=1, tbs=0, qm=0, prb=None, snr_db=30.0,
           h=None, seed=0xA5A5, nl_td=2):
    cfg = TxCfg()
    cfg.cell = cell
    cfg.sf_idx, cfg.cfi, cfg.mcs, cfg.rv, cfg.rnti, cfg.tm = sf_idx, cfi, mcs, rv, rnti, tm
    cfg.tbs, cfg.qm = tbs, qm
    for p in range(NRB_MAX):
        # prb entries are kept as given: 0/1 (both slots) or the two-slot encoding (bit s = slot s)
        cfg.prb_mask[p] = (1 if prb is None else int(prb[p])) if p < cell.nof_prb else 0
    cfg.snr_db = snr_db
    h = h if h is not None else [1.0 + 0j, 0.0 + 0j] if cell.nof_ports == 1 else [0.8 + 0.3j, -0.4 + 0.5j]
    for p in range(2):
        cfg.h_re[p] = h[p].real
        cfg.h_im[p] = h[p].imag
    cfg.noise_seed = seed
    cfg.nl_td = nl_td
    return cfg


def tx_subframe(cfg, tb_bytes):
    n = lib().or_sf_len(cfg.cell.nof_prb)
    iq = np.zeros(2 * n, np.float32)
    G = C.c_uint32(0)
    assert lib().or_tx_subframe(C.byref(cfg), np.ascontiguousarray(tb_bytes, np.uint8), iq, C.byref(G)) == 0
    return iq, G.value


def splitmix_bytes(seed, n):
    """TB payload generator: splitmix64 stream, little-endian bytes."""
    out = np.zeros(((n + 7) // 8) * 8, np.uint8)
    s = seed & 0xFFFFFFFFFFFFFFFF
    M = 0xFFFFFFFFFFFFFFFF
    for i in range(0, len(out), 8):
        s = (s + 0x9E3779B97F4A7C15) & M
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        out[i:i + 8] = np.frombuffer(z.to_bytes(8, "little"), np.uint8)
    return out[:n]
