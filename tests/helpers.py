"""Shared test helpers: oracle decodes of product-generated subframes."""
import ctypes as C

import numpy as np

import oracle_lib as O
from srsue_amd import abi


def oracle_front(cfg, iq):
    """Oracle OFDM RX + chest + PDSCH LLRs of one subframe (mirrors srslte_ue_dl_decode_fft_estimate +
    the front half of srslte_pdsch_decode_rnti)."""
    L = O.lib()
    cell = O.Cell(cfg.cell_id, cfg.nof_prb, cfg.nof_ports)
    W = 12 * cfg.nof_prb
    grid = np.zeros(2 * 14 * W, np.float32)
    ce = np.zeros(2 * 14 * W * cfg.nof_ports, np.float32)
    met = np.zeros(5, np.float32)
    L.or_ofdm_rx(C.byref(cell), np.ascontiguousarray(iq, np.float32), grid)
    L.or_chest(C.byref(cell), cfg.sf_idx, grid, ce, met)
    llr = np.zeros(14 * W * 6, np.float32)
    G = C.c_uint32()
    mask = np.array(list(cfg.prb_mask), np.uint8)
    L.or_pdsch_llr(C.byref(cell), cfg.cfi, cfg.sf_idx, mask, cfg.Qm, cfg.rnti, cfg.tm, 0.01, grid, ce, llr,
                   C.byref(G), None)
    return grid, ce, met, llr[:G.value]


def oracle_dlsch(cfg, llr, max_its=4, sb=None, new_tb=True, i16=None):
    """Oracle rate de-matching + turbo decoding + TB CRC of one TB.  i16: True = int16 (SSE-design)
    decoder, False = float gen decoder, None = whatever O.tdec_mode currently selects."""
    if i16 is not None:
        with O.tdec_mode(O.TDEC_I16 if i16 else O.TDEC_GEN):
            return oracle_dlsch(cfg, llr, max_its, sb, new_tb)
    L = O.lib()
    s = O.cbsegm(cfg.tbs)
    ncb = L.or_ncb(s.Kp)
    if sb is None:
        sb = np.zeros(s.C * ncb, np.float32)
    pay = np.zeros(cfg.tbs // 8, np.uint8)
    noi = C.c_uint32()
    cbok = C.c_uint32()
    nl = (cfg.nl_td or 2) if cfg.tm == 2 else 1
    rc = L.or_dlsch_decode(np.ascontiguousarray(llr, np.float32), len(llr), cfg.tbs, cfg.Qm, nl, cfg.rv,
                           int(new_tb), sb, ncb, max_its, pay, C.byref(noi), C.byref(cbok))
    return rc == 0, pay, noi.value, sb


def oracle_dlsch_cbits(cfg, llr, max_its=4, i16=True):
    """oracle_dlsch of a new TB that also returns each code block's iteration count:
    (crc_ok, payload, tb_iterations, cb_iterations[C])"""
    with O.tdec_mode(O.TDEC_I16 if i16 else O.TDEC_GEN):
        L = O.lib()
        s = O.cbsegm(cfg.tbs)
        ncb = L.or_ncb(s.Kp)
        sb = np.zeros(s.C * ncb, np.float32)
        pay = np.zeros(cfg.tbs // 8, np.uint8)
        noi, cbok = C.c_uint32(), C.c_uint32()
        cbits = (C.c_uint32 * s.C)()
        nl = (cfg.nl_td or 2) if cfg.tm == 2 else 1
        rc = L.or_dlsch_decode_cbits(np.ascontiguousarray(llr, np.float32), len(llr), cfg.tbs, cfg.Qm, nl, cfg.rv,
                                     1, sb, ncb, max_its, pay, C.byref(noi), C.byref(cbok), cbits)
    return rc == 0, pay, noi.value, np.array(cbits[:], np.uint32)


def tb_bytes(seed, tbs):
    return O.splitmix_bytes(0x5EED0000 + seed, tbs // 8)


def make_subframes(cfgs, snr_db=30.0, h=None, seed0=0):
    iqs, tbs = [], []
    for i, c in enumerate(cfgs):
        tb = tb_bytes(seed0 + i, c.tbs)
        iqs.append(abi.tx_subframe(c, tb, h=h, snr_db=snr_db, seed=0xA5A5 + seed0 + i))
        tbs.append(tb)
    return iqs, tbs


def rel_err(a, b):
    """max |a - b| relative to the RMS of b (the tolerance metric of the parity tests)."""
    b = np.asarray(b, np.float64)
    a = np.asarray(a, np.float64)
    rms = np.sqrt(np.mean(b * b)) + 1e-30
    return float(np.max(np.abs(a - b)) / rms)


def otx_fixture(path):
    """An oracle-transmitter chain fixture (tests/golden/make_golden.py otx_fixture): (arrays, [abi.sf_cfg], accessor)
    where accessor(key, i) is subframe i's slice of a concatenated array (iq, tb, grid, ce, llr, payload)."""
    from srsue_amd import abi
    g = np.load(path)
    cfgs = []
    for row in g["cfg"]:
        cid, nprb, ports, sf, cfi, tbs, qm, tm, rnti = (int(x) for x in row[:9])
        cfgs.append(abi.sf_cfg(cell_id=cid, nof_prb=nprb, nof_ports=ports, sf_idx=sf, cfi=cfi, tm=tm, rnti=rnti,
                               tbs=tbs, Qm=qm, prb=[bool(x) for x in row[9:9 + nprb]]))

    def part(key, i):
        o = g[key + "_off"]
        return g[key][o[i]:o[i + 1]]
    return g, cfgs, part
