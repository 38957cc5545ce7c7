"""GPU: DL control channels through the C ABI (mi_dl_ctrl_*) against the oracle
(oracle/o_ctrl.c) and transmit-chain ground truth.

Bars: PCFICH CFI exact; PDCCH soft bits within 1e-4 relative (GPU fp32 vs oracle fp64 front end);
blind search on identical soft bits bit-exact (found / not found, DCI bits, format, L, CCE), also at
SNRs where decoding is marginal; a DCI put on the air is found with its bits and first CCE."""
import ctypes as C

import numpy as np
import pytest
import torch

import oracle_lib as O
from helpers import oracle_front, rel_err
from srsue_amd import abi
from test_oracle_ctrl import tx_with_dci

pytestmark = pytest.mark.gpu


def front_batch(cfgs, iqs):
    b = abi.Batch(cfgs, max_its=4)
    flat = np.zeros(2 * b.iq_samples, np.float32)
    for i, iq in enumerate(iqs):
        o = 2 * b.iq_offset(i)
        flat[o:o + len(iq)] = iq
    d = torch.from_numpy(flat).cuda()
    b.run_stages(3, d.data_ptr(), torch.cuda.current_stream().cuda_stream)   # OFDM + chest
    torch.cuda.synchronize()
    return b, d


CASES = [  # nof_prb, ports, cfi, ng, sf, snr (dB per RE; None = noiseless), L
    (100, 1, 1, 2, 1, None, 2), (100, 2, 3, 0, 4, 12.0, 4), (25, 1, 2, 1, 0, 10.0, 1), (6, 2, 2, 3, 9, None, 1),
    (50, 1, 3, 2, 5, 8.0, 8), (75, 1, 2, 2, 7, 15.0, 2),
]


def make_case(i, nprb, ports, cfi, ng, sf, snr, Lw, rnti):
    cfg = abi.sf_cfg(cell_id=3 + 7 * i, nof_prb=nprb, nof_ports=ports, sf_idx=sf, cfi=cfi, tbs=1000, Qm=2, rnti=rnti)
    q = O.ctrl_cfg(cfg.cell_id, nprb, ports, ng, cfi, sf)
    n = C.c_uint32()
    O.lib().or_pdcch_regs(C.byref(q), None, C.byref(n))
    Ls = np.zeros(32, np.uint32)
    nc = np.zeros(32, np.uint32)
    k = O.lib().or_search_space(n.value, sf, rnti, 0, Ls, nc)
    cand = [j for j in range(k) if Ls[j] == Lw] or [j for j in range(k) if Ls[j] <= Lw]
    pick = cand[-1]
    bits = np.zeros(64, np.uint8)
    A = O.lib().or_dci1a_pack(nprb, C.byref(O.Dci1a(0, nprb, 5 + i, i % 8, 1, i % 4, 1)), bits)
    h = [0.8 + 0.3j, -0.4 + 0.5j] if ports == 2 else None
    iq, _ = tx_with_dci(cfg, ng, rnti, int(Ls[pick]), int(nc[pick]), bits[:A], h=h, snr_db=snr, seed=17 + i)
    return cfg, q, iq, bits[:A], int(Ls[pick]), int(nc[pick])


@pytest.mark.parametrize("ng", [0, 2])
def test_ctrl_round_trip_and_oracle_parity(ng):
    cases = [c for c in CASES if c[3] == ng] or CASES[:2]
    built = [make_case(i, *c[:3], ng, *c[4:], rnti=0x46 + i) for i, c in enumerate(cases)]
    cfgs = [b[0] for b in built]
    b, d = front_batch(cfgs, [x[2] for x in built])
    ctl = abi.Ctrl(b, phich_ng=ng)
    ctl.run(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    gl = ctl.llr()
    for s, (cfg, q, iq, bits, L, ncce) in enumerate(built):
        cfi, got = ctl.result(s)
        assert cfi == cfg.cfi
        grid, ce, _, _ = oracle_front(cfg, iq)
        ollr, n_cce = O.pdcch_llr(q, grid, ce)
        assert ctl.n_cce(s) == n_cce
        off = ctl.llr_offset(s)
        assert rel_err(gl[off:off + len(ollr)], ollr) < 1e-4
        assert got is not None, f"subframe {s}: DCI not found"
        fmt, gb, gL, gncce = got
        assert fmt == O.DCI_1A and np.array_equal(gb, bits) and gncce == ncce and gL <= L
        assert ctl.result(s, ul=True)[1] is None
        ofind = O.find_dci(ollr, n_cce, cfg.nof_prb, cfg.sf_idx, cfg.rnti)
        assert ofind is not None and ofind[0] == fmt and np.array_equal(ofind[1], gb) and ofind[2:] == (gL, gncce)
    ctl.close()


@pytest.mark.parametrize("snr", [-2.0, 0.0, 2.0])
def test_blind_search_bit_exact_on_identical_soft_bits(snr):
    """The oracle's soft bits uploaded into the GPU buffer: the GPU search must reach the same verdicts
    as the oracle's for many RNTIs, including marginal SNRs where some decodes fail."""
    n_sf = 16
    base = [make_case(i, 25, 1 + (i % 2), 1 + (i % 3), 2, i % 10, snr, 1 << (i % 4), rnti=0x100 + i) for i in range(n_sf)]
    cfgs = [x[0] for x in base]
    b, d = front_batch(cfgs, [x[2] for x in base])
    ctl = abi.Ctrl(b, phich_ng=2)
    flat = np.zeros(abi.lib().mi_dl_ctrl_llr_floats(ctl.h), np.float32)
    oll = []
    for s, (cfg, q, iq, bits, L, ncce) in enumerate(base):
        grid, ce, _, _ = oracle_front(cfg, iq)
        ollr, n_cce = O.pdcch_llr(q, grid, ce)
        off = ctl.llr_offset(s)
        flat[off:off + len(ollr)] = ollr
        oll.append((ollr, n_cce))
    ctl.set_llr(flat)
    ctl.run(torch.cuda.current_stream().cuda_stream, mask=abi.Ctrl.SEARCH)
    torch.cuda.synchronize()
    nfound = 0
    for s, (cfg, q, iq, bits, L, ncce) in enumerate(base):
        for ul in (False, True):
            _, got = ctl.result(s, ul=ul)
            ref = O.find_dci(oll[s][0], oll[s][1], cfg.nof_prb, cfg.sf_idx, cfg.rnti, ul=ul)
            assert (got is None) == (ref is None), (s, ul)
            if got is not None:
                nfound += 1
                assert got[0] == ref[0] and np.array_equal(got[1], ref[1]) and got[2:] == ref[2:]
    assert 0 <= nfound <= 2 * n_sf
    ctl.close()


@pytest.mark.parametrize("ng", [0, 2, 3])
def test_phich_batch_round_trip_and_oracle_parity(ng):
    """PHICH (36.211 6.9) through mi_dl_ctrl_set_phich / _phich: per subframe an UL grant (I_lowest,
    n_dmrs) -> (group, seq); the oracle's transmitter puts ACK or NACK there (plus an interfering
    PHICH on another sequence of the same group); the GPU HI equals the transmitted one and its soft
    value the oracle's on the oracle's own front end within 1e-3 relative."""
    from test_oracle_ctrl import tx_with_phich
    cases = [(100, 1, 1, 7, 0, 1, None), (100, 2, 4, 33, 3, 0, 6.0), (25, 1, 0, 5, 1, 1, 4.0),
             (6, 2, 9, 2, 7, 0, None), (50, 1, 6, 49, 2, 1, 8.0)]   # nprb, ports, sf, I_lowest, n_dmrs, ack, snr
    cfgs, iqs, want = [], [], []
    for i, (nprb, ports, sf, il, nd, ack, snr) in enumerate(cases):
        cfg = abi.sf_cfg(cell_id=11 + 5 * i, nof_prb=nprb, nof_ports=ports, sf_idx=sf, cfi=1, tbs=1000, Qm=2)
        g, sq = O.phich_calc(nprb, ng, il, nd)
        h = [0.8 + 0.3j, -0.4 + 0.5j] if ports == 2 else None
        iq, q = tx_with_phich(cfg, ng, [(g, sq, ack), (g, (sq + 3) % 8, 1 - ack)], h=h, snr_db=snr, seed=i + 1)
        grid, ce, _, _ = oracle_front(cfg, iq)
        cfgs.append(cfg)
        iqs.append(iq)
        want.append((ack, O.phich_soft(q, grid, ce, g, sq)))
    b, d = front_batch(cfgs, iqs)
    c = abi.Ctrl(b, phich_ng=ng)
    c.set_phich([x[3] for x in cases], [x[4] for x in cases])
    c.run(torch.cuda.current_stream().cuda_stream, mask=abi.Ctrl.PHICH)
    for i, (ack, osoft) in enumerate(want):
        got, soft = c.phich(i)
        assert got == bool(ack) and (osoft > 0) == bool(ack), (i, got, soft, osoft)
        assert abs(soft - osoft) <= 1e-3 * max(1.0, abs(osoft)), (i, soft, osoft)
    c.close()
