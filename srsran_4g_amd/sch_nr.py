"""Python mirror of the NR shared-channel receive API (include/srsran_sch_nr.h).

Binds LDPC code block segmentation, TB info (sch_nr.c:114-176), and the DL-SCH / UL-SCH decoders
(sch_nr.c:554-750) of the in-tree HIP library, the way the reference's pdsch_nr_test.c /
sch_nr_test.c drive srsran_dlsch_nr_decode.  No CPU fallback: every decode runs the HIP kernels.
"""
import ctypes

import numpy as np

from .sch import MOD_FROM_QM, SoftbufferRx, _memcpy_d2h, srsran_cbsegm_t, srsran_softbuffer_rx_t
from .tdec import load_library

u32 = ctypes.c_uint32
MAX_CB_SIZE = 384 * 66  # SRSRAN_LDPC_MAX_LEN_ENCODED_CB
SRSRAN_SCH_NR_MAX_NOF_CB_LDPC = (156 * 275 * 8 + 8447) // 8448
BG1, BG2 = 0, 1
srsran_mcs_table_64qam, srsran_mcs_table_256qam, srsran_mcs_table_qam64LowSE = range(3)


class srsran_carrier_nr_t(ctypes.Structure):
    _fields_ = [("pci", u32), ("dl_center_frequency_hz", ctypes.c_double), ("ul_center_frequency_hz", ctypes.c_double),
                ("ssb_center_freq_hz", ctypes.c_double), ("offset_to_carrier", u32), ("scs", ctypes.c_int),
                ("nof_prb", u32), ("start", u32), ("max_mimo_layers", u32)]


class srsran_sch_cfg_t(ctypes.Structure):
    _fields_ = [("mcs_table", ctypes.c_int), ("xoverhead", ctypes.c_int), ("limited_buffer_rm", ctypes.c_bool)]


class _sch_softbuffer(ctypes.Union):
    _fields_ = [("tx", ctypes.c_void_p), ("rx", ctypes.POINTER(srsran_softbuffer_rx_t))]


class srsran_sch_tb_t(ctypes.Structure):
    _fields_ = [("mod", ctypes.c_int), ("N_L", u32), ("mcs", u32), ("tbs", ctypes.c_int), ("R", ctypes.c_double),
                ("R_prime", ctypes.c_double), ("rv", ctypes.c_int), ("ndi", ctypes.c_int), ("nof_re", u32),
                ("nof_bits", u32), ("cw_idx", u32), ("enabled", ctypes.c_bool), ("softbuffer", _sch_softbuffer)]


class srsran_sch_tb_res_nr_t(ctypes.Structure):
    _fields_ = [("payload", ctypes.POINTER(ctypes.c_uint8)), ("crc", ctypes.c_bool), ("avg_iter", ctypes.c_float)]


class srsran_sch_nr_args_t(ctypes.Structure):
    _fields_ = [("disable_simd", ctypes.c_bool), ("decoder_use_flooded", ctypes.c_bool),
                ("decoder_scaling_factor", ctypes.c_float), ("max_nof_iter", u32)]


TB_INFO_FIELDS = ("bg", "Qm", "G", "A", "L_tb", "L_cb", "B", "Bp", "Kp", "Kr", "F", "Nref", "Z", "Nl")


class srsran_sch_nr_tb_info_t(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int if n == "bg" else u32) for n in TB_INFO_FIELDS] + [
        ("mask", ctypes.c_bool * SRSRAN_SCH_NR_MAX_NOF_CB_LDPC), ("C", u32), ("Cp", u32)]

    def as_dict(self):
        d = {n: int(getattr(self, n)) for n in TB_INFO_FIELDS}
        d["C"] = int(self.C)
        return d


class srsran_sch_nr_t(ctypes.Structure):
    _fields_ = [("carrier", srsran_carrier_nr_t), ("gpu", ctypes.c_void_p)]


class srsran_sch_nr_gpu_tb_t(ctypes.Structure):
    _fields_ = [("sch_cfg", ctypes.POINTER(srsran_sch_cfg_t)), ("tb", ctypes.POINTER(srsran_sch_tb_t)),
                ("d_e_bits", ctypes.c_void_p), ("d_payload", ctypes.c_void_p), ("new_data", u32)]


_bound = False


def lib():
    global _bound
    L = load_library()
    if _bound:
        return L
    Q = ctypes.POINTER(srsran_sch_nr_t)
    CFG = ctypes.POINTER(srsran_sch_cfg_t)
    TB = ctypes.POINTER(srsran_sch_tb_t)
    RES = ctypes.POINTER(srsran_sch_tb_res_nr_t)
    i8p = ctypes.POINTER(ctypes.c_int8)
    sig = {
        "srsran_cbsegm_ldpc_bg1": ([ctypes.POINTER(srsran_cbsegm_t), u32], ctypes.c_int),
        "srsran_cbsegm_ldpc_bg2": ([ctypes.POINTER(srsran_cbsegm_t), u32], ctypes.c_int),
        "srsran_sch_nr_select_basegraph": ([u32, ctypes.c_double], ctypes.c_int),
        "srsran_sch_nr_fill_tb_info": ([ctypes.POINTER(srsran_carrier_nr_t), CFG, TB,
                                        ctypes.POINTER(srsran_sch_nr_tb_info_t)], ctypes.c_int),
        "srsran_sch_nr_init_rx": ([Q, ctypes.POINTER(srsran_sch_nr_args_t)], ctypes.c_int),
        "srsran_sch_nr_set_carrier": ([Q, ctypes.POINTER(srsran_carrier_nr_t)], ctypes.c_int),
        "srsran_sch_nr_free": ([Q], None),
        "srsran_dlsch_nr_decode": ([Q, CFG, TB, i8p, RES], ctypes.c_int),
        "srsran_ulsch_nr_decode": ([Q, CFG, TB, i8p, RES], ctypes.c_int),
        "srsran_sch_nr_gpu_decode_batch": ([Q, u32, ctypes.POINTER(srsran_sch_nr_gpu_tb_t), ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _bound = True
    return L


def cbsegm_ldpc(bg, tbs):
    s = srsran_cbsegm_t()
    f = lib().srsran_cbsegm_ldpc_bg1 if bg == BG1 else lib().srsran_cbsegm_ldpc_bg2
    if f(ctypes.byref(s), tbs) != 0:
        raise ValueError(f"cbsegm_ldpc failed for TBS={tbs}")
    return {"tbs": s.tbs, "L_tb": s.L_tb, "L_cb": s.L_cb, "C": s.C, "K": s.K1, "Z": s.Z}


def select_basegraph(tbs, R):
    return lib().srsran_sch_nr_select_basegraph(tbs, R)


def make_carrier(nof_prb=52, max_mimo_layers=1):
    c = srsran_carrier_nr_t()
    c.nof_prb = nof_prb
    c.max_mimo_layers = max_mimo_layers
    return c


def make_cfg(lbrm=False, mcs256=False):
    cfg = srsran_sch_cfg_t()
    cfg.mcs_table = srsran_mcs_table_256qam if mcs256 else srsran_mcs_table_64qam
    cfg.limited_buffer_rm = bool(lbrm)
    return cfg


def make_tb(tbs, R, Qm, G, Nl, rv=0, softbuffer=None):
    tb = srsran_sch_tb_t()
    tb.mod = MOD_FROM_QM[Qm]
    tb.N_L = Nl
    tb.tbs = tbs
    tb.R = R
    tb.rv = rv
    tb.nof_bits = G
    tb.nof_re = G // (Qm * Nl)
    tb.enabled = True
    if softbuffer is not None:
        tb.softbuffer.rx = ctypes.pointer(softbuffer.s)
    return tb


def tb_info(tbs, R, Qm, G, Nl, lbrm=False, nof_prb=52, mcs256=False):
    """srsran_sch_nr_fill_tb_info -> srsran_sch_nr_tb_info_t."""
    t = srsran_sch_nr_tb_info_t()
    car = make_carrier(nof_prb)
    cfg = make_cfg(lbrm, mcs256)
    tb = make_tb(tbs, R, Qm, G, Nl)
    if lib().srsran_sch_nr_fill_tb_info(ctypes.byref(car), ctypes.byref(cfg), ctypes.byref(tb), ctypes.byref(t)) != 0:
        raise ValueError("srsran_sch_nr_fill_tb_info failed")
    return t


def nr_softbuffer(max_cb=SRSRAN_SCH_NR_MAX_NOF_CB_LDPC):
    """A soft buffer sized the way the reference's NR users size theirs (MAX_LEN_ENCODED_CB per block)."""
    sb = SoftbufferRx(max_cb=max_cb, max_cb_size=MAX_CB_SIZE)
    sb.reset()
    return sb


def read_cb8(sb, r, n):
    """n int8 soft bits of code block r (the NR path uses the buffers as int8, sch_nr.c:614)."""
    import torch
    out = torch.empty(n, dtype=torch.int8)
    _memcpy_d2h(out, sb.s.buffer_f[r], n)
    return out.numpy()


class SchNr:
    """srsran_sch_nr_t (receive side) owner."""

    def __init__(self, nof_prb=52, scaling=0.8, max_nof_iter=10, disable_simd=False, max_mimo_layers=1):
        self.q = srsran_sch_nr_t()
        a = srsran_sch_nr_args_t()
        a.disable_simd = disable_simd
        a.decoder_scaling_factor = scaling
        a.max_nof_iter = max_nof_iter
        if lib().srsran_sch_nr_init_rx(ctypes.byref(self.q), ctypes.byref(a)) != 0:
            raise RuntimeError("srsran_sch_nr_init_rx failed (no HIP device?)")
        self.carrier = make_carrier(nof_prb, max_mimo_layers)
        lib().srsran_sch_nr_set_carrier(ctypes.byref(self.q), ctypes.byref(self.carrier))

    def decode(self, sb, tbs, R, Qm, G, Nl, rv, e_bits, lbrm=False, mcs256=False, uplink=False):
        """srsran_dlsch_nr_decode -> (ret, crc, avg_iter, payload)."""
        cfg = make_cfg(lbrm, mcs256)
        tb = make_tb(tbs, R, Qm, G, Nl, rv, sb)
        e = np.ascontiguousarray(e_bits, np.int8)
        assert e.size == G
        payload = np.zeros(tbs // 8 + 8, np.uint8)
        res = srsran_sch_tb_res_nr_t()
        res.payload = payload.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        f = lib().srsran_ulsch_nr_decode if uplink else lib().srsran_dlsch_nr_decode
        ret = f(ctypes.byref(self.q), ctypes.byref(cfg), ctypes.byref(tb), e.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)),
                ctypes.byref(res))
        return ret, bool(res.crc), float(res.avg_iter), payload[:tbs // 8]

    def decode_batch(self, entries, d_crc, d_avg, stream=None):
        """srsran_sch_nr_gpu_decode_batch. entries: list of (cfg, tb, d_e_bits, d_payload[, new_data]); the
        caller keeps cfg / tb alive until the call returns (descriptors are read during the call)."""
        arr = (srsran_sch_nr_gpu_tb_t * max(len(entries), 1))()
        for i, ent in enumerate(entries):
            cfg, tb, de, dp = ent[:4]
            arr[i].sch_cfg = ctypes.pointer(cfg)
            arr[i].tb = ctypes.pointer(tb)
            arr[i].d_e_bits, arr[i].d_payload = de, dp
            arr[i].new_data = int(ent[4]) if len(ent) > 4 else 0
        return lib().srsran_sch_nr_gpu_decode_batch(ctypes.byref(self.q), len(entries), arr, d_crc, d_avg, stream)

    def free(self):
        if self.q.gpu:
            lib().srsran_sch_nr_free(ctypes.byref(self.q))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
