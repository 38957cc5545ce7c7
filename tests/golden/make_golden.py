"""Generates the committed golden fixtures under tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`).  Parity is unpinned against srsLTE itself (not in the
container), so the fixtures pin (a) 3GPP-derived known answers and transmit-chain
ground truth and (b) the oracle's own outputs, so any later change to the oracle is caught.

Fixtures
  tdec_K40.npz            info bits, noiseless LLRs (+-4), decoded bits           
  tdec_K6144_ebno.npz     config 1 (turbodecoder_test): K=6144, BPSK/AWGN at Eb/N0 {0.5,1,1.5,2,3} dB,
                          8 fixed iterations, early stop off: LLRs, decisions, bit errors
  rm_K5824.npz            rate-match -> de-match round trip, rv 0..3, E = 6924   
  sf_1p4mhz.npz           1.4 MHz TM1 subframe: IQ (product TX, 20 dB), TB, oracle grid/ce/LLR/payload
  tdec16_K6144.npz        the config-1 LLRs of tdec_K6144_ebno.npz through the int16 ("SSE") decoder:
                          decisions, bit errors, and the decisions after 1 and 2 iterations
  sf_20mhz_tm1.npz        BASELINE configs[1]: one 20 MHz TM1 MCS-28 subframe (product TX at 21.5 dB, where code
                          blocks need up to 4 iterations): IQ, TB, oracle grid / ce / metrics / LLR, and the payload and
                          iteration count of both turbo arithmetics (float srsLTE-gen, int16 SSE design)

  otx_*.npz               the same kind of chain fixtures with the IQ from the ORACLE's own transmitter
                          (oracle/o_tx.c or_tx_subframe, independent of the product's csrc/tx.cpp): a change to the
                          product transmitter alone cannot move them.  Each holds per subframe
                          the config (OTX_FIELDS + PRB mask), IQ, TB, the oracle's grid / ce / metrics / LLR and the
                          payload + iteration count of the int16 decoder:
    otx_1p4mhz.npz        1.4 MHz TM1 16QAM (cell 301, CFI 2), 20 dB
    otx_20mhz_tm1.npz     configs[1]: 20 MHz TM1 MCS 28, 20.5 dB (code blocks iterating: 4 iterations)
    otx_20mhz_tm2.npz     configs[2]: 20 MHz TM2 (2-port SFBC) 64QAM MCS 28 through h = (0.8+0.3j, -0.4+0.5j), 25 dB (2 iterations)
    otx_mixed.npz         configs[4]: one 1.4 / 5 / 10 / 20 MHz subframe each (bench.config_cfgs(5)), 30 dB

`python tests/golden/make_golden.py tdec16` regenerates only the int16 fixture, `... sf20` only the 20 MHz one,
`... otx` only the oracle-transmitter ones.
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.dirname(HERE)]
import oracle_lib as O  # noqa: E402
from helpers import oracle_dlsch, oracle_front  # noqa: E402
from srsue_amd import abi  # noqa: E402


def turbo_llr(bits, K, ebno_db, rng, amp=None):
    d = np.zeros(3 * (K + 4), np.uint8)
    assert O.lib().or_tcod(np.ascontiguousarray(bits, np.uint8), K, 0, d) == 0
    x = 1.0 - 2.0 * d                       # BPSK: 0 -> +1
    if amp is not None:
        return (-amp * x).astype(np.float32)
    rate = K / (3.0 * K + 12)
    sigma2 = 1.0 / (2 * rate * 10 ** (ebno_db / 10))
    y = x + rng.normal(0, np.sqrt(sigma2), x.shape)
    return (-2.0 * y / sigma2).astype(np.float32)   # LLR > 0 => bit 1


def make_tdec16():
    """int16 decoder on the committed config-1 LLRs (so the fixture is tied to tdec_K6144_ebno.npz)."""
    g = np.load(os.path.join(HERE, "tdec_K6144_ebno.npz"))
    td = O.Tdec(O.TDEC_I16)
    decs, d1, d2, errs = [], [], [], []
    for llr in g["llr"]:
        dec, its, ok = td.decode_cb(llr, 6144, max_its=8, early_stop=False)
        decs.append(dec); errs.append(int(np.sum(dec != g["bits"])))
        d1.append(td.decode_cb(llr, 6144, max_its=1, early_stop=False)[0])
        d2.append(td.decode_cb(llr, 6144, max_its=2, early_stop=False)[0])
    np.savez_compressed(os.path.join(HERE, "tdec16_K6144.npz"), ebno=g["ebno"], dec=np.stack(decs),
                        dec_it1=np.packbits(np.stack(d1), axis=1), dec_it2=np.packbits(np.stack(d2), axis=1),
                        errors=np.array(errs))
    print("int16 K=6144 bit errors per Eb/N0", dict(zip(g["ebno"].tolist(), errs)))


def make_sf20():
    """configs[1]'s subframe through the oracle chain, both turbo arithmetics (GPU tests compare against the arrays)."""
    cfg = abi.sf_cfg(cell_id=1, nof_prb=100, nof_ports=1, sf_idx=1, cfi=1, tbs=75376, Qm=6)
    tb = O.splitmix_bytes(0x5EED0000 + 20, cfg.tbs // 8)
    iq = abi.tx_subframe(cfg, tb, snr_db=21.5, seed=0xA5A5 + 20)
    grid, ce, met, llr = oracle_front(cfg, iq)
    out = {}
    for name, mode in (("gen", O.TDEC_GEN), ("i16", O.TDEC_I16)):
        with O.tdec_mode(mode):
            ok, pay, noi, _ = oracle_dlsch(cfg, llr)
        assert ok and np.array_equal(pay, tb), name
        out["payload_" + name], out["noi_" + name] = pay, np.array([noi])
    np.savez_compressed(os.path.join(HERE, "sf_20mhz_tm1.npz"), iq=iq, tb=tb, grid=grid, ce=ce, metrics=met, llr=llr,
                        cfg=np.array([cfg.cell_id, cfg.nof_prb, cfg.nof_ports, cfg.sf_idx, cfg.cfi, cfg.tbs, cfg.Qm]),
                        **out)
    print("sf_20mhz_tm1: iterations gen", out["noi_gen"][0], "i16", out["noi_i16"][0])


OTX_FIELDS = ("cell_id", "nof_prb", "nof_ports", "sf_idx", "cfi", "tbs", "Qm", "tm", "rnti")


def otx_cfg_row(c):
    return [int(getattr(c, f)) for f in OTX_FIELDS] + [int(c.prb_mask[p]) for p in range(110)]


def otx_fixture(name, cfgs, snr, h=None, seed0=0x07A0):
    """cfgs (abi.sf_cfg) through the ORACLE transmitter and the oracle receive chain; the int16 decode must pass."""
    rows, iqs, tbs, grids, ces, mets, llrs, pays, nois = [], [], [], [], [], [], [], [], []
    for i, c in enumerate(cfgs):
        tb = O.splitmix_bytes(0x5EED0000 + seed0 + i, c.tbs // 8)
        tc = O.tx_cfg(O.make_cell(c.cell_id, c.nof_prb, c.nof_ports), sf_idx=c.sf_idx, cfi=c.cfi, rv=0, rnti=c.rnti,
                      tm=c.tm, tbs=c.tbs, qm=c.Qm, prb=[c.prb_mask[p] for p in range(c.nof_prb)], snr_db=snr, h=h,
                      seed=0xA5A5 + seed0 + i)
        iq, G = O.tx_subframe(tc, tb)
        grid, ce, met, llr = oracle_front(c, iq)
        assert len(llr) == G, (name, i, len(llr), G)
        ok, pay, noi, _ = oracle_dlsch(c, llr, i16=True)
        assert ok and np.array_equal(pay, tb), (name, i)
        rows.append(otx_cfg_row(c)); iqs.append(iq); tbs.append(tb); grids.append(grid); ces.append(ce)
        mets.append(met); llrs.append(llr); pays.append(pay); nois.append(noi)
    cat = lambda v: (np.concatenate(v), np.cumsum([0] + [len(x) for x in v]))
    hh = h if h is not None else [1.0 + 0j, 0.0 + 0j]
    arrs = {"cfg": np.array(rows, np.int64), "noi_i16": np.array(nois, np.uint32), "metrics": np.stack(mets),
            "snr_db": np.array([snr]), "seed0": np.array([seed0]),
            "h": np.array([[x.real, x.imag] for x in hh], np.float64)}
    for k, v in (("iq", iqs), ("tb", tbs), ("grid", grids), ("ce", ces), ("llr", llrs), ("payload", pays)):
        arrs[k], arrs[k + "_off"] = cat(v)
    np.savez_compressed(os.path.join(HERE, name), **arrs)
    print(name, "int16 iterations", nois, os.path.getsize(os.path.join(HERE, name)), "B")


def make_otx():
    import bench
    otx_fixture("otx_1p4mhz.npz", [abi.sf_cfg(cell_id=301, nof_prb=6, nof_ports=1, sf_idx=1, cfi=2, tbs=2344, Qm=4)],
                20.0)
    otx_fixture("otx_20mhz_tm1.npz", [abi.sf_cfg(cell_id=1, nof_prb=100, nof_ports=1, sf_idx=1, cfi=1, tbs=75376,
                                                 Qm=6)], 20.5)
    otx_fixture("otx_20mhz_tm2.npz", [abi.sf_cfg(cell_id=1, nof_prb=100, nof_ports=2, sf_idx=2, cfi=1, tm=2,
                                                 tbs=75376, Qm=6)], 25.0, h=[0.8 + 0.3j, -0.4 + 0.5j])
    otx_fixture("otx_mixed.npz", bench.config_cfgs(5, 4, 0), 30.0)


def main():
    if sys.argv[1:] == ["otx"]:
        make_otx()
        return
    if sys.argv[1:] == ["tdec16"]:
        make_tdec16()
        return
    if sys.argv[1:] == ["sf20"]:
        make_sf20()
        return
    L = O.lib()
    rng = np.random.default_rng(1)
    # --- K = 40 noiseless
    b40 = rng.integers(0, 2, 40).astype(np.uint8)
    l40 = turbo_llr(b40, 40, None, rng, amp=4.0)
    dec40, its, ok = O.Tdec().decode_cb(l40, 40, max_its=8, early_stop=False)
    np.savez_compressed(os.path.join(HERE, "tdec_K40.npz"), bits=b40, llr=l40, dec=dec40)
    # --- K = 6144, config 1 sweep
    K = 6144
    ebnos = np.array([0.5, 1.0, 1.5, 2.0, 3.0])
    bits = rng.integers(0, 2, K).astype(np.uint8)
    llrs, decs, errs = [], [], []
    td = O.Tdec()
    for e in ebnos:
        llr = turbo_llr(bits, K, e, np.random.default_rng(int(e * 10) + 1))
        dec, its, ok = td.decode_cb(llr, K, max_its=8, early_stop=False)
        llrs.append(llr); decs.append(dec); errs.append(int(np.sum(dec != bits)))
    np.savez_compressed(os.path.join(HERE, "tdec_K6144_ebno.npz"), ebno=ebnos, bits=bits, llr=np.stack(llrs),
                        dec=np.stack(decs), errors=np.array(errs))
    print("K=6144 bit errors per Eb/N0", dict(zip(ebnos.tolist(), errs)))
    # --- rate matching round trip
    K, E = 5824, 6924
    bk = rng.integers(0, 2, K).astype(np.uint8)
    d = np.zeros(3 * (K + 4), np.uint8)
    L.or_tcod(bk, K, 0, d)
    ncb = L.or_ncb(K)
    es, outs = [], []
    for rv in range(4):
        e = np.zeros(E, np.uint8)
        L.or_rm_tx(d, K, E, rv, e)
        llr = (2.0 * e - 1.0).astype(np.float32)
        sb = np.zeros(ncb, np.float32)
        out = np.zeros(3 * (K + 4), np.float32)
        L.or_rm_rx(llr, E, K, 0, rv, 1, sb, out)
        es.append(e); outs.append(out)
    np.savez_compressed(os.path.join(HERE, "rm_K5824.npz"), d=d, e=np.stack(es), out=np.stack(outs))
    # --- 1.4 MHz subframe
    cfg = abi.sf_cfg(cell_id=301, nof_prb=6, nof_ports=1, sf_idx=1, cfi=2, tbs=2344, Qm=4)
    tb = O.splitmix_bytes(0x5EED0000 + 7, cfg.tbs // 8)
    iq = abi.tx_subframe(cfg, tb, snr_db=20.0, seed=0xA5A5 + 7)
    grid, ce, met, llr = oracle_front(cfg, iq)
    ok, pay, noi, _ = oracle_dlsch(cfg, llr)
    assert ok and np.array_equal(pay, tb)
    np.savez_compressed(os.path.join(HERE, "sf_1p4mhz.npz"), iq=iq, tb=tb, grid=grid, ce=ce, metrics=met, llr=llr,
                        payload=pay, noi=np.array([noi]),
                        cfg=np.array([cfg.cell_id, cfg.nof_prb, cfg.nof_ports, cfg.sf_idx, cfg.cfi, cfg.tbs, cfg.Qm]))
    make_tdec16()
    make_sf20()
    make_otx()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
