"""ctypes bindings of the C ABI in include/mi_dl.h and include/srslte/srslte.h.

The product is the C-ABI shared library srsue_amd/libsrsue_amd.so (gfx950 kernels + host C++);
this module only binds it.  Loading fails loudly if the library has not been built -- there is no
CPU fallback for the receive path.
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SRSUE_AMD_LIB") or os.path.join(PKG_DIR, "libsrsue_amd.so")
EMU_PATH = os.path.join(PKG_DIR, "libsrsue_amd_emu.so")

MAX_PRB = 110
STAGES = ("ofdm", "chest", "demap", "rm", "tdec", "tb")
BUF_GRID, BUF_CE, BUF_LLR, BUF_PAYLOAD, BUF_TB_CRC, BUF_TB_ITS, BUF_METRICS, BUF_CB_ITS, BUF_CB_CRC, BUF_SB = range(10)
FLAG_PROFILE = 1
FLAG_TDEC_I16 = 2   # int16 ("SSE") turbo arithmetic (the default), see include/mi_dl.h
FLAG_TDEC_GEN = 4   # float srsLTE-gen turbo arithmetic
FLAG_IQ_SC16 = 8    # IQ input as UHD sc16 (int16 I/Q, fc32 = sc16 / 32768)
FLAG_TDEC_WIN = 16  # int16 turbo: force the latency form (one workgroup per code block)
FLAG_TDEC_LANE = 32  # int16 turbo: force one code block per lane of 64-lane wavefronts
FLAG_TDEC_X = 128  # lane-per-code-block decoder, crossed schedule (two wavefronts per group)
FLAG_TDEC_XR = 256  # crossed kernel, recompute form (5 waves per SIMD)
FLAG_TDEC_P2 = 512   # two code blocks per lane (packed int16), crossed
FLAG_CE_COMPACT = 1024  # compact channel estimates (4 pilot rows per port), interpolated in the fused demap
FLAG_TDEC_SEG = 2048  # packed turbo waterfall: late rounds as exact 8-step segments (one stream faster, see mi_dl.h)
SCHED_FLAGS = {None: 0, "auto": 0, "win": FLAG_TDEC_WIN, "lane": FLAG_TDEC_LANE, "lanex": FLAG_TDEC_LANE | FLAG_TDEC_X,
               "lanexr": FLAG_TDEC_LANE | FLAG_TDEC_X | FLAG_TDEC_XR, "p2": FLAG_TDEC_LANE | FLAG_TDEC_P2}
FLAG_KEEP_LLR = 64  # keep the LLR stream of a full run (else demap is fused into rate de-matching)


class SfCfg(C.Structure):
    """mi_dl_sf_cfg_t (include/mi_dl.h)."""
    _fields_ = [(n, C.c_uint32) for n in ("cell_id", "nof_prb", "nof_ports", "sf_idx", "cfi", "tm", "nl_td",
                                          "rnti", "rv", "tbs", "Qm", "new_tb")] + \
               [("prb_mask", C.c_uint8 * MAX_PRB)]


def sf_cfg(cell_id=1, nof_prb=100, nof_ports=1, sf_idx=1, cfi=1, tm=None, rnti=0x46, rv=0, tbs=75376, Qm=6,
           new_tb=1, prb=None, nl_td=2):
    c = SfCfg()
    c.cell_id, c.nof_prb, c.nof_ports, c.sf_idx, c.cfi = cell_id, nof_prb, nof_ports, sf_idx, cfi
    c.tm = tm if tm is not None else (2 if nof_ports == 2 else 1)
    c.nl_td, c.rnti, c.rv, c.tbs, c.Qm, c.new_tb = nl_td, rnti, rv, tbs, Qm, new_tb
    for p in range(MAX_PRB):
        # 0/1 entries (both slots) or the two-slot encoding of mi_dl_sf_cfg_t (bit s = used in slot s)
        c.prb_mask[p] = (1 if prb is None else int(prb[p])) if p < nof_prb else 0
    return c


def cfg_array(cfgs):
    arr = (SfCfg * len(cfgs))()
    for i, c in enumerate(cfgs):
        arr[i] = c
    return arr


_lib = None
_emu = None


def lib():
    """The product library; raises if it is missing (build with __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        vp, u32, sz = C.c_void_p, C.c_uint32, C.c_size_t
        sig = {
            "mi_dl_batch_create": (vp, [vp, u32, u32, u32]),
            "mi_dl_batch_destroy": (None, [vp]),
            "mi_dl_batch_iq_offset": (sz, [vp, u32]),
            "mi_dl_batch_iq_samples": (sz, [vp]),
            "mi_dl_batch_payload_offset": (sz, [vp, u32]),
            "mi_dl_batch_bytes": (sz, [vp, C.c_int]),
            "mi_dl_batch_offset": (sz, [vp, C.c_int, u32]),
            "mi_dl_batch_run": (C.c_int, [vp, vp, vp]),
            "mi_dl_batch_download": (C.c_int, [vp, C.c_int, vp, sz]),
            "mi_dl_batch_run_stages": (C.c_int, [vp, vp, vp, u32]),
            "mi_dl_batch_run_split": (C.c_int, [vp, vp, vp, vp]),
            "mi_dl_batch_upload": (C.c_int, [vp, C.c_int, vp, sz]),
            "mi_dl_batch_device_ptr": (vp, [vp, C.c_int]),
            "mi_dl_batch_stage_ms": (C.c_int, [vp, vp, vp]),
            "mi_dl_batch_profile_reset": (None, [vp]),
            "mi_dl_batch_algo_bytes": (C.c_double, [vp, C.c_int]),
            "mi_dl_batch_n_codeblocks": (u32, [vp]),
            "mi_dl_batch_turbo_win": (C.c_int, [vp]),
            "mi_dl_batch_turbo_compact": (C.c_int, [vp]),
            "mi_tdec_turbo_win": (C.c_int, [vp]),
            "mi_dl_batch_n_groups": (u32, [vp]),
            "mi_dl_batch_rm_direct_groups": (u32, [vp]),
            "mi_dl_batch_set_tdec_history": (C.c_int, [vp, C.c_int]),
            "mi_dl_batch_reset_history": (None, [vp]),
            "mi_dl_plan_create": (vp, []),
            "mi_dl_plan_destroy": (None, [vp]),
            "mi_dl_plan_build": (C.c_int, [vp, vp, u32]),
            "mi_dl_batch_replan": (C.c_int, [vp, vp, vp]),
            "mi_dl_batch_device_bytes": (sz, [vp]),
            "mi_dl_plan_device_bytes": (sz, [vp, u32, u32]),
            "mi_tx_subframe": (C.c_int, [vp, vp, vp, C.c_float, C.c_uint64, vp]),
            "mi_turbo_encode": (C.c_int, [vp, u32, u32, vp]),
            "mi_tdec_create": (vp, [u32, u32, u32, C.c_int, C.c_int, u32]),
            "mi_tdec_destroy": (None, [vp]),
            "mi_tdec_run": (C.c_int, [vp, vp, vp]),
            "mi_tdec_download": (C.c_int, [vp, vp, vp, vp]),
            "mi_tdec_stage_ms": (C.c_int, [vp, vp, vp]),
            "mi_tdec_profile_reset": (None, [vp]),
            "mi_tdec_algo_bytes": (C.c_double, [vp]),
            "mi_sf_len": (C.c_int, [u32]),
            "mi_pdsch_G": (C.c_int, [vp]),
            "mi_dl_ctrl_create": (vp, [vp, u32]),
            "mi_dl_ctrl_destroy": (None, [vp]),
            "mi_dl_ctrl_run": (C.c_int, [vp, vp]),
            "mi_dl_ctrl_run_stages": (C.c_int, [vp, u32, vp]),
            "mi_dl_ctrl_result": (C.c_int, [vp, u32, C.c_int, vp, vp, vp, vp, vp, vp]),
            "mi_dl_ctrl_llr_floats": (sz, [vp]),
            "mi_dl_ctrl_llr_offset": (sz, [vp, u32]),
            "mi_dl_ctrl_n_cce": (u32, [vp, u32]),
            "mi_dl_ctrl_llr": (C.c_int, [vp, vp, sz, C.c_int]),
            "mi_dl_ctrl_set_phich": (C.c_int, [vp, vp, vp]),
            "mi_dl_ctrl_phich": (C.c_int, [vp, u32, vp]),
            "mi_sync_create": (vp, [u32]),
            "mi_sync_destroy": (None, [vp]),
            "mi_sync_fft_size": (u32, [vp]),
            "mi_sync_pss": (C.c_int, [vp, vp, vp, u32, u32, u32, vp, vp]),
            "mi_sync_sss": (C.c_int, [vp, vp, vp, vp, vp, u32, vp, vp]),
            "mi_sync_correct": (C.c_int, [vp, vp, vp, vp, vp, vp, u32, u32, vp]),
            "mi_tx_sync": (C.c_int, [u32, u32, u32, C.c_float, vp]),
            "mi_dl_pipe_create": (vp, [vp, u32, u32, u32]),
            "mi_dl_pipe_destroy": (None, [vp]),
            "mi_dl_pipe_submit": (C.c_int, [vp, vp]),
            "mi_dl_pipe_wait": (C.c_int, [vp, C.c_int]),
            "mi_dl_pipe_batch": (vp, [vp, C.c_int]),
            "mi_host_alloc": (vp, [sz]),
            "mi_host_free": (None, [vp]),
            "mi_device_count": (C.c_int, []),
            "mi_set_device": (C.c_int, [C.c_int]),
            "mi_last_error": (C.c_char_p, []),
            "mi_stream_create_cu_share": (C.c_int, [u32, u32, vp]),
            "mi_stream_destroy": (C.c_int, [vp]),
            "mi_ul_batch_create": (vp, [vp, u32, u32]),
            "mi_ul_batch_destroy": (None, [vp]),
            "mi_ul_batch_payload_offset": (sz, [vp, u32]),
            "mi_ul_batch_payload_bytes": (sz, [vp]),
            "mi_ul_batch_iq_offset": (sz, [vp, u32]),
            "mi_ul_batch_iq_samples": (sz, [vp]),
            "mi_ul_batch_n_codeblocks": (u32, [vp]),
            "mi_ul_batch_run": (C.c_int, [vp, vp, vp, vp]),
            "mi_ul_batch_symbols": (C.c_int, [vp, u32, vp]),
            "mi_ul_batch_stage_ms": (C.c_int, [vp, vp, vp]),
            "mi_ul_batch_profile_reset": (None, [vp]),
            "mi_ul_batch_algo_bytes": (C.c_double, [vp]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _lib = L
    return _lib


def emu():
    """TEST-ONLY host emulation of the per-lane kernel bodies (never used by the product path)."""
    global _emu
    if _emu is None:
        E = C.CDLL(EMU_PATH)
        E.emu_decode_llr.restype = C.c_int
        E.emu_decode_llr.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p]
        E.emu_set_tdec_i16.restype = None
        E.emu_set_tdec_i16.argtypes = [C.c_int]
        E.emu_set_tdec_x.restype = None
        E.emu_set_tdec_x.argtypes = [C.c_int]
        E.emu_payload_offset.restype = C.c_size_t
        E.emu_payload_offset.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        _emu = E
    return _emu


def last_error():
    return lib().mi_last_error().decode()


def stream_cu_share(first, count):
    """A HIP stream (handle as int) on the CUs whose index mod 8 lies in [first, first + count) (mi_stream_create_cu_share);
    release with stream_destroy."""
    h = C.c_void_p()
    if lib().mi_stream_create_cu_share(first, count, C.byref(h)):
        raise RuntimeError("mi_stream_create_cu_share: " + last_error())
    return h.value


def stream_destroy(h):
    if lib().mi_stream_destroy(C.c_void_p(h)):
        raise RuntimeError("mi_stream_destroy: " + last_error())


def tx_subframe(cfg, tb_bytes, h=None, snr_db=30.0, seed=0xA5A5):
    """Synthetic subframe from the product transmitter (mi_tx_subframe)."""
    n = lib().mi_sf_len(cfg.nof_prb)
    iq = np.zeros(2 * n, np.float32)
    hh = None
    if h is not None:
        hh = np.zeros(4, np.float32)
        for p, v in enumerate(h[:2]):
            hh[2 * p], hh[2 * p + 1] = v.real, v.imag
    tb = np.ascontiguousarray(tb_bytes, np.uint8)
    rc = lib().mi_tx_subframe(C.byref(cfg), tb.ctypes.data, None if hh is None else hh.ctypes.data,
                              float(snr_db), seed, iq.ctypes.data)
    if rc:
        raise RuntimeError("mi_tx_subframe failed")
    return iq


class Batch:
    """Owns one mi_dl_batch_t (planned once; run() only enqueues kernels)."""

    def __init__(self, cfgs, max_its=4, profile=False, tdec_i16=True, iq_sc16=False, sched=None, keep_llr=False,
                 compact_ce=False, seg_rounds=False):
        self.cfgs = list(cfgs)
        self._arr = cfg_array(self.cfgs)
        flags = (FLAG_PROFILE if profile else 0) | (FLAG_TDEC_I16 if tdec_i16 else FLAG_TDEC_GEN) | \
            (FLAG_IQ_SC16 if iq_sc16 else 0) | SCHED_FLAGS[sched] | (FLAG_KEEP_LLR if keep_llr else 0) | \
            (FLAG_CE_COMPACT if compact_ce else 0) | (FLAG_TDEC_SEG if seg_rounds else 0)
        self.h = lib().mi_dl_batch_create(C.cast(self._arr, C.c_void_p), len(self.cfgs), max_its, flags)
        if not self.h:
            raise RuntimeError("mi_dl_batch_create: " + last_error())

    @classmethod
    def view(cls, handle, cfgs):
        """Non-owning wrapper of a batch owned elsewhere (a pipe slot)."""
        b = cls.__new__(cls)
        b.cfgs, b._arr, b.h, b._owned = list(cfgs), None, handle, False
        return b

    def close(self):
        if self.h and getattr(self, "_owned", True):
            lib().mi_dl_batch_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def iq_samples(self):
        return lib().mi_dl_batch_iq_samples(self.h)

    def iq_offset(self, sf):
        return lib().mi_dl_batch_iq_offset(self.h, sf)

    def run(self, d_iq_ptr, stream_ptr=None):
        rc = lib().mi_dl_batch_run(self.h, C.c_void_p(d_iq_ptr), C.c_void_p(stream_ptr or 0))
        if rc:
            raise RuntimeError("mi_dl_batch_run: " + last_error())

    def replan(self, plan, stream_ptr=None):
        """Swap plan's built configuration in (mi_dl_batch_replan): table upload enqueued on stream_ptr, the
        stream this batch runs on; plan then holds the previous configuration's data, ready for a rebuild."""
        cfgs = plan.cfgs
        if lib().mi_dl_batch_replan(self.h, plan.h, C.c_void_p(stream_ptr or 0)):
            raise RuntimeError("mi_dl_batch_replan: " + last_error())
        plan.cfgs, self.cfgs = self.cfgs, cfgs

    def run_split(self, d_iq_ptr, front_ptr, back_ptr):
        """mi_dl_batch_run_split: front end on front_ptr, turbo decoder + TB CRC on back_ptr (complete with it)."""
        rc = lib().mi_dl_batch_run_split(self.h, C.c_void_p(d_iq_ptr), C.c_void_p(front_ptr or 0),
                                         C.c_void_p(back_ptr or 0))
        if rc:
            raise RuntimeError("mi_dl_batch_run_split: " + last_error())

    def run_stages(self, mask, d_iq_ptr=None, stream_ptr=None):
        rc = lib().mi_dl_batch_run_stages(self.h, C.c_void_p(d_iq_ptr or 0), C.c_void_p(stream_ptr or 0), mask)
        if rc:
            raise RuntimeError("mi_dl_batch_run_stages: " + last_error())

    def upload(self, which, host_array):
        a = np.ascontiguousarray(host_array)
        if lib().mi_dl_batch_upload(self.h, which, a.ctypes.data, a.nbytes):
            raise RuntimeError("upload: " + last_error())

    def download(self, which, dtype):
        n = lib().mi_dl_batch_bytes(self.h, which)
        out = np.zeros(n // np.dtype(dtype).itemsize, dtype)
        if lib().mi_dl_batch_download(self.h, which, out.ctypes.data, n):
            raise RuntimeError("download: " + last_error())
        return out

    def offset(self, which, sf):
        return lib().mi_dl_batch_offset(self.h, which, sf)

    def stage_ms(self):
        """Per-stage device ms averaged over the profiled runs since profile_reset()."""
        ms = np.zeros(len(STAGES), np.float32)
        n = C.c_uint32(0)
        if lib().mi_dl_batch_stage_ms(self.h, ms.ctypes.data, C.byref(n)):
            raise RuntimeError("stage_ms: " + last_error())
        return dict(zip(STAGES, ms.tolist())), n.value

    def profile_reset(self):
        lib().mi_dl_batch_profile_reset(self.h)

    def algo_bytes(self, stage=-1):
        return lib().mi_dl_batch_algo_bytes(self.h, stage)

    @property
    def n_codeblocks(self):
        return lib().mi_dl_batch_n_codeblocks(self.h)

    @property
    def turbo_win(self):
        """True when the turbo stage runs the latency form (one workgroup per code block)."""
        return lib().mi_dl_batch_turbo_win(self.h) == 1

    @property
    def turbo_sched(self):
        """'win' (latency form), 'lanex' (lane per code block, two wavefronts per group) or 'lane'"""
        return {1: "win", 2: "lanex", 3: "lanexr", 4: "p2"}.get(lib().mi_dl_batch_turbo_win(self.h), "lane")

    @property
    def turbo_compact(self):
        """True when the packed decoder compacts the CRC-failing code blocks after iteration 0 (tdec.hip)."""
        return lib().mi_dl_batch_turbo_compact(self.h) == 1

    @property
    def n_groups(self):
        return lib().mi_dl_batch_n_groups(self.h)

    @property
    def rm_direct_groups(self):
        """groups rate-de-matched in the direct form (rm.hip rm_direct_kernel; MI_RM_DIRECT=0 disables)"""
        return lib().mi_dl_batch_rm_direct_groups(self.h)

    @property
    def device_bytes(self):
        """HBM this batch holds (mi_dl_batch_device_bytes)."""
        return lib().mi_dl_batch_device_bytes(self.h)

    def set_tdec_history(self, mode):
        """Waterfall compaction's schedule source (mi_dl_batch_set_tdec_history): -1 = this batch's history of
        continuation counts (default), 0 = fixed high-SNR schedule, 1 = fixed waterfall schedule (results identical)."""
        if lib().mi_dl_batch_set_tdec_history(self.h, int(mode)):
            raise RuntimeError("set_tdec_history: " + last_error())

    def reset_history(self):
        lib().mi_dl_batch_reset_history(self.h)

    def payload(self, sf, all_payload=None):
        p = all_payload if all_payload is not None else self.download(BUF_PAYLOAD, np.uint8)
        off = lib().mi_dl_batch_payload_offset(self.h, sf)
        return p[off:off + self.cfgs[sf].tbs // 8]


class Plan:
    """Owns one mi_dl_plan_t: host-only planning of a batch (no GPU call; ctypes releases the GIL, so worker
    threads plan while the main thread keeps the GPU busy), swapped into a Batch by Batch.replan()."""

    def __init__(self):
        self.h = lib().mi_dl_plan_create()
        self.cfgs = None

    def build(self, cfgs):
        """cfgs: a list of SfCfg, or a prebuilt cfg_array (no per-call Python conversion)."""
        arr = cfgs if isinstance(cfgs, C.Array) else cfg_array(list(cfgs))
        self.cfgs = arr
        if lib().mi_dl_plan_build(self.h, C.cast(arr, C.c_void_p), len(arr)):
            raise RuntimeError("mi_dl_plan_build: " + last_error())
        return self

    def device_bytes(self, max_its=4, compact_ce=True, keep_llr=False, tdec_i16=True):
        """HBM a batch of this plan would allocate for its work buffers and softbuffer (mi_dl_plan_device_bytes;
        host only)."""
        flags = (FLAG_TDEC_I16 if tdec_i16 else FLAG_TDEC_GEN) | (FLAG_CE_COMPACT if compact_ce else 0) | \
            (FLAG_KEEP_LLR if keep_llr else 0)
        n = lib().mi_dl_plan_device_bytes(self.h, max_its, flags)
        if not n:
            raise RuntimeError("mi_dl_plan_device_bytes: " + last_error())
        return n

    def close(self):
        if self.h:
            lib().mi_dl_plan_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Ctrl:
    """DL control channels over a batch's grid / channel estimates (mi_dl_ctrl_*)."""
    PCFICH, LLR, SEARCH, PHICH = 1, 2, 4, 8

    def __init__(self, batch, phich_ng=2):
        self.batch = batch
        self.h = lib().mi_dl_ctrl_create(batch.h, phich_ng)
        if not self.h:
            raise RuntimeError("mi_dl_ctrl_create: " + last_error())

    def set_phich(self, i_lowest, n_dmrs):
        """per-subframe PHICH queries: the UL grant's lowest PRB index and DMRS cyclic shift"""
        a = np.ascontiguousarray(i_lowest, np.uint32)
        b = np.ascontiguousarray(n_dmrs, np.uint32)
        if lib().mi_dl_ctrl_set_phich(self.h, a.ctypes.data, b.ctypes.data):
            raise RuntimeError("mi_dl_ctrl_set_phich: " + last_error())

    def phich(self, sf):
        """(ack, soft HI) of subframe sf after a run with the PHICH stage"""
        s = C.c_float()
        rc = lib().mi_dl_ctrl_phich(self.h, sf, C.byref(s))
        if rc < 0:
            raise RuntimeError("mi_dl_ctrl_phich: " + last_error())
        return rc == 1, s.value

    def run(self, stream_ptr=None, mask=15):
        if lib().mi_dl_ctrl_run_stages(self.h, mask, C.c_void_p(stream_ptr or 0)):
            raise RuntimeError("mi_dl_ctrl_run: " + last_error())

    def result(self, sf, ul=False):
        """(cfi, found DCI or None); DCI = (format, bits, L, ncce)"""
        v = [C.c_uint32() for _ in range(5)]
        bits = np.zeros(64, np.uint8)
        rc = lib().mi_dl_ctrl_result(self.h, sf, int(ul), C.byref(v[0]), C.byref(v[1]), C.byref(v[2]), C.byref(v[3]),
                                     bits.ctypes.data, C.byref(v[4]))
        if rc < 0:
            raise RuntimeError("mi_dl_ctrl_result: " + last_error())
        return v[0].value, ((v[1].value, bits[:v[4].value].copy(), v[2].value, v[3].value) if rc == 1 else None)

    def llr(self):
        n = lib().mi_dl_ctrl_llr_floats(self.h)
        out = np.zeros(n, np.float32)
        if lib().mi_dl_ctrl_llr(self.h, out.ctypes.data, n, 0):
            raise RuntimeError("mi_dl_ctrl_llr: " + last_error())
        return out

    def set_llr(self, host):
        a = np.ascontiguousarray(host, np.float32)
        if lib().mi_dl_ctrl_llr(self.h, a.ctypes.data, a.size, 1):
            raise RuntimeError("mi_dl_ctrl_llr: " + last_error())

    def llr_offset(self, sf):
        return lib().mi_dl_ctrl_llr_offset(self.h, sf)

    def n_cce(self, sf):
        return lib().mi_dl_ctrl_n_cce(self.h, sf)

    def close(self):
        if self.h:
            lib().mi_dl_ctrl_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PssResult(C.Structure):
    _fields_ = [("nid2", C.c_uint32), ("lag", C.c_uint32), ("rho", C.c_float), ("cfo", C.c_float)]


class SssResult(C.Structure):
    _fields_ = [("nid1", C.c_uint32), ("sf5", C.c_uint32), ("score", C.c_float)]


def tx_sync(cell_id, nof_prb, sf_idx, iq, amp=1.0):
    """add the PSS / SSS of subframe 0 / 5 to iq (float32 interleaved, in place)"""
    assert iq.dtype == np.float32 and iq.flags.c_contiguous
    rc = lib().mi_tx_sync(cell_id, nof_prb, sf_idx, amp, iq.ctypes.data)
    if rc < 0:
        raise RuntimeError("mi_tx_sync: " + last_error())
    return rc


class Sync:
    """Sync front end (mi_sync_*) over device-resident IQ (offsets in cf32 samples)."""

    def __init__(self, nof_prb):
        self.h = lib().mi_sync_create(nof_prb)
        if not self.h:
            raise RuntimeError("mi_sync_create: " + last_error())
        self.N = lib().mi_sync_fft_size(self.h)

    def pss(self, d_iq, offsets, nlag, nid2_mask=7, stream_ptr=None):
        off = np.ascontiguousarray(offsets, np.uint64)
        out = (PssResult * max(len(off), 1))()
        if lib().mi_sync_pss(self.h, C.c_void_p(d_iq), off.ctypes.data, len(off), nlag, nid2_mask, out,
                             C.c_void_p(stream_ptr or 0)):
            raise RuntimeError("mi_sync_pss: " + last_error())
        return [(r.nid2, r.lag, r.rho, r.cfo) for r in out[:len(off)]]

    def sss(self, d_iq, sf_offsets, nid2, cfo, stream_ptr=None):
        off = np.ascontiguousarray(sf_offsets, np.uint64)
        n2 = np.ascontiguousarray(nid2, np.uint32)
        cf = np.ascontiguousarray(cfo, np.float32)
        out = (SssResult * max(len(off), 1))()
        if lib().mi_sync_sss(self.h, C.c_void_p(d_iq), off.ctypes.data, n2.ctypes.data, cf.ctypes.data, len(off), out,
                             C.c_void_p(stream_ptr or 0)):
            raise RuntimeError("mi_sync_sss: " + last_error())
        return [(r.nid1, r.sf5, r.score) for r in out[:len(off)]]

    def correct(self, d_src, src_off, d_dst, dst_off, cfo, length, stream_ptr=None):
        a = np.ascontiguousarray(src_off, np.uint64)
        b = np.ascontiguousarray(dst_off, np.uint64)
        c = np.ascontiguousarray(cfo, np.float32)
        if lib().mi_sync_correct(self.h, C.c_void_p(d_src), a.ctypes.data, C.c_void_p(d_dst), b.ctypes.data,
                                 c.ctypes.data, len(a), length, C.c_void_p(stream_ptr or 0)):
            raise RuntimeError("mi_sync_correct: " + last_error())

    def close(self):
        if self.h:
            lib().mi_sync_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostBuffer:
    """Page-locked host memory (mi_host_alloc) viewed as a numpy array."""

    def __init__(self, nbytes, dtype=np.float32):
        self.ptr = lib().mi_host_alloc(nbytes)
        if not self.ptr:
            raise RuntimeError("mi_host_alloc: " + last_error())
        self.array = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(self.ptr)).view(dtype)

    def close(self):
        if self.ptr:
            self.array = None
            lib().mi_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Pipe:
    """Double-buffered host-IQ pipeline (mi_dl_pipe_*): submit() returns a slot without blocking."""

    def __init__(self, cfgs, max_its=4, profile=False, tdec_i16=True, iq_sc16=False):
        self.cfgs = list(cfgs)
        self._arr = cfg_array(self.cfgs)
        flags = (FLAG_PROFILE if profile else 0) | (FLAG_TDEC_I16 if tdec_i16 else FLAG_TDEC_GEN) | \
            (FLAG_IQ_SC16 if iq_sc16 else 0)
        self.h = lib().mi_dl_pipe_create(C.cast(self._arr, C.c_void_p), len(self.cfgs), max_its, flags)
        if not self.h:
            raise RuntimeError("mi_dl_pipe_create: " + last_error())

    def submit(self, host_ptr):
        s = lib().mi_dl_pipe_submit(self.h, C.c_void_p(host_ptr))
        if s < 0:
            raise RuntimeError("mi_dl_pipe_submit: " + last_error())
        return s

    def wait(self, slot):
        if lib().mi_dl_pipe_wait(self.h, slot):
            raise RuntimeError("mi_dl_pipe_wait: " + last_error())

    def batch(self, slot):
        return Batch.view(lib().mi_dl_pipe_batch(self.h, slot), self.cfgs)

    def close(self):
        if self.h:
            lib().mi_dl_pipe_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


SC16_GAIN = 0.25   # receive gain before sc16 quantisation: the synthetic TX peaks at ~2.5 (a radio's AGC
                   # keeps samples inside [-1, 1)); a power of two, so gain * x is exact


def to_sc16(iq_f32, gain=SC16_GAIN):
    """fc32 interleaved I/Q -> UHD sc16 (gain, round to nearest, saturate): FLAG_IQ_SC16's wire format."""
    return np.clip(np.rint(np.asarray(iq_f32, np.float32) * (gain * 32768.0)), -32768, 32767).astype(np.int16)


def turbo_encode(bits, K, F=0):
    """36.212 turbo encoder of the product (host): 3(K+4) values in triplet order, 2 = <NULL>."""
    d = np.zeros(3 * (K + 4), np.uint8)
    b = np.ascontiguousarray(bits, np.uint8)
    if lib().mi_turbo_encode(b.ctypes.data, K, F, d.ctypes.data):
        raise RuntimeError("mi_turbo_encode failed")
    return d


class TdecBatch:
    """Raw code-block turbo decoding (mi_tdec_*, the srslte_tdec_* / turbodecoder_test contract)."""

    def __init__(self, K, n_cb, max_its=8, early_stop=False, crc24a=False, profile=False, tdec_i16=True, sched=None):
        self.K, self.n_cb = K, n_cb
        flags = (FLAG_PROFILE if profile else 0) | (FLAG_TDEC_I16 if tdec_i16 else FLAG_TDEC_GEN) | SCHED_FLAGS[sched]
        self.h = lib().mi_tdec_create(K, n_cb, max_its, int(early_stop), int(crc24a), flags)
        if not self.h:
            raise RuntimeError("mi_tdec_create: " + last_error())

    def run(self, d_in_ptr, stream_ptr=None):
        if lib().mi_tdec_run(self.h, C.c_void_p(d_in_ptr), C.c_void_p(stream_ptr or 0)):
            raise RuntimeError("mi_tdec_run: " + last_error())

    def results(self):
        bits = np.zeros(self.n_cb * self.K // 8, np.uint8)
        its = np.zeros(self.n_cb, np.uint32)
        ok = np.zeros(self.n_cb, np.uint32)
        if lib().mi_tdec_download(self.h, bits.ctypes.data, its.ctypes.data, ok.ctypes.data):
            raise RuntimeError("mi_tdec_download: " + last_error())
        return np.unpackbits(bits).reshape(self.n_cb, self.K), its, ok

    def stage_ms(self):
        ms = np.zeros(len(STAGES), np.float32)
        n = C.c_uint32(0)
        if lib().mi_tdec_stage_ms(self.h, ms.ctypes.data, C.byref(n)):
            raise RuntimeError("stage_ms: " + last_error())
        return dict(zip(STAGES, ms.tolist())), n.value

    def profile_reset(self):
        lib().mi_tdec_profile_reset(self.h)

    def algo_bytes(self):
        return lib().mi_tdec_algo_bytes(self.h)

    @property
    def turbo_win(self):
        return lib().mi_tdec_turbo_win(self.h) == 1

    @property
    def turbo_sched(self):
        return {1: "win", 2: "lanex", 3: "lanexr", 4: "p2"}.get(lib().mi_tdec_turbo_win(self.h), "lane")

    def close(self):
        if self.h:
            lib().mi_tdec_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pdsch_G(cfg):
    return lib().mi_pdsch_G(C.byref(cfg))


# ---- UL PUSCH transmitter (include/mi_ul.h) ---------------------------------------
UL_STAGES = ("crc", "encode", "mod")


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


class UlBatch:
    """Owns one mi_ul_batch_t: N PUSCH transmissions planned once; run() enqueues the chain."""

    def __init__(self, cfgs, profile=False):
        self.cfgs = list(cfgs)
        self._arr = (UlCfg * len(self.cfgs))(*self.cfgs)
        self.h = lib().mi_ul_batch_create(C.cast(self._arr, C.c_void_p), len(self.cfgs), 1 if profile else 0)
        if not self.h:
            raise RuntimeError("mi_ul_batch_create: " + last_error())

    def close(self):
        if self.h:
            lib().mi_ul_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def payload_bytes(self):
        return lib().mi_ul_batch_payload_bytes(self.h)

    @property
    def iq_samples(self):
        return lib().mi_ul_batch_iq_samples(self.h)

    @property
    def n_codeblocks(self):
        return lib().mi_ul_batch_n_codeblocks(self.h)

    def payload_offset(self, i):
        return lib().mi_ul_batch_payload_offset(self.h, i)

    def iq_offset(self, i):
        return lib().mi_ul_batch_iq_offset(self.h, i)

    def run(self, d_payload_ptr, d_iq_ptr, stream_ptr=None):
        if lib().mi_ul_batch_run(self.h, C.c_void_p(d_payload_ptr), C.c_void_p(d_iq_ptr), C.c_void_p(stream_ptr or 0)):
            raise RuntimeError("mi_ul_batch_run: " + last_error())

    def symbols(self, i):
        M = 12 * self.cfgs[i].L_prb
        out = np.zeros(12 * M, np.uint8)
        if lib().mi_ul_batch_symbols(self.h, i, out.ctypes.data):
            raise RuntimeError("mi_ul_batch_symbols: " + last_error())
        return out

    def stage_ms(self):
        ms = np.zeros(len(UL_STAGES), np.float32)
        n = C.c_uint32(0)
        if lib().mi_ul_batch_stage_ms(self.h, ms.ctypes.data, C.byref(n)):
            raise RuntimeError("mi_ul_batch_stage_ms: " + last_error())
        return dict(zip(UL_STAGES, ms.tolist())), n.value

    def profile_reset(self):
        lib().mi_ul_batch_profile_reset(self.h)

    def algo_bytes(self):
        return lib().mi_ul_batch_algo_bytes(self.h)
