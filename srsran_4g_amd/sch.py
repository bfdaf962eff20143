"""Python mirror of the DL-SCH C API (include/srsran_sch.h).

Binds cbsegm, CRC, rate de-matching, HARQ soft buffers and the DL-SCH decoder
(sch.c:371-609) of the in-tree HIP library, the way the reference's pdsch_test.c
drives srsran_dlsch_decode.  No CPU fallback: every decode runs the HIP kernels.
"""
import ctypes

import numpy as np

from .tdec import SRSRAN_TCOD_MAX_LEN_CB, load_library, srsran_tdec_t  # noqa: F401

SRSRAN_MAX_PRB = 110
SRSRAN_MAX_CODEWORDS = 2
SRSRAN_MAX_CODEBLOCKS = 32
SOFTBUFFER_SIZE = 18600
SRSRAN_LTE_CRC24A = 0x1864CFB
SRSRAN_LTE_CRC24B = 0x1800063

SRSRAN_MOD_BPSK, SRSRAN_MOD_QPSK, SRSRAN_MOD_16QAM, SRSRAN_MOD_64QAM, SRSRAN_MOD_256QAM = range(5)
MOD_FROM_QM = {1: SRSRAN_MOD_BPSK, 2: SRSRAN_MOD_QPSK, 4: SRSRAN_MOD_16QAM, 6: SRSRAN_MOD_64QAM, 8: SRSRAN_MOD_256QAM}

u32 = ctypes.c_uint32


class srsran_tcod_t(ctypes.Structure):  # turbocoder.h:45-48 (+ the added device pointer)
    _fields_ = [("max_long_cb", ctypes.c_uint32), ("temp", ctypes.c_void_p), ("gpu", ctypes.c_void_p)]


class srsran_cbsegm_t(ctypes.Structure):
    _fields_ = [(n, u32) for n in ("F", "C", "K1", "K2", "K1_idx", "K2_idx", "C1", "C2", "tbs", "L_tb", "L_cb", "Z")]


class srsran_crc_t(ctypes.Structure):
    _fields_ = [("table", ctypes.c_uint64 * 256), ("polynom", ctypes.c_int), ("order", ctypes.c_int),
                ("crcinit", ctypes.c_uint64), ("crcmask", ctypes.c_uint64), ("crchighbit", ctypes.c_uint64),
                ("srsran_crc_out", u32)]


class srsran_softbuffer_rx_t(ctypes.Structure):
    _fields_ = [("max_cb", u32), ("max_cb_size", u32), ("buffer_f", ctypes.POINTER(ctypes.c_void_p)),
                ("data", ctypes.POINTER(ctypes.c_void_p)), ("cb_crc", ctypes.POINTER(ctypes.c_bool)),
                ("tb_crc", ctypes.c_bool), ("gpu", ctypes.c_void_p)]


class srsran_ra_tb_t(ctypes.Structure):
    _fields_ = [("mod", ctypes.c_int), ("tbs", ctypes.c_int), ("rv", ctypes.c_int), ("nof_bits", u32),
                ("cw_idx", u32), ("enabled", ctypes.c_bool), ("mcs_idx", u32)]


class srsran_pdsch_grant_t(ctypes.Structure):
    _fields_ = [("tx_scheme", ctypes.c_int), ("pmi", u32), ("prb_idx", (ctypes.c_bool * SRSRAN_MAX_PRB) * 2),
                ("nof_prb", u32), ("nof_re", u32), ("nof_symb_slot", u32 * 2),
                ("tb", srsran_ra_tb_t * SRSRAN_MAX_CODEWORDS), ("last_tbs", ctypes.c_int * SRSRAN_MAX_CODEWORDS),
                ("nof_tb", u32), ("nof_layers", u32)]


class _softbuffers(ctypes.Union):
    _fields_ = [("tx", ctypes.c_void_p * SRSRAN_MAX_CODEWORDS),
                ("rx", ctypes.POINTER(srsran_softbuffer_rx_t) * SRSRAN_MAX_CODEWORDS)]


class srsran_pdsch_cfg_t(ctypes.Structure):
    _fields_ = [("grant", srsran_pdsch_grant_t), ("rnti", ctypes.c_uint16), ("max_nof_iterations", u32),
                ("decoder_type", ctypes.c_int), ("p_a", ctypes.c_float), ("p_b", u32), ("rs_power", ctypes.c_float),
                ("power_scale", ctypes.c_bool), ("csi_enable", ctypes.c_bool), ("use_tbs_index_alt", ctypes.c_bool),
                ("softbuffers", _softbuffers), ("meas_evm_en", ctypes.c_bool), ("meas_time_en", ctypes.c_bool),
                ("meas_time_value", u32)]


class srsran_sch_t(ctypes.Structure):
    _fields_ = [("max_iterations", u32), ("avg_iterations", ctypes.c_float), ("llr_is_8bit", ctypes.c_bool),
                ("decoder", srsran_tdec_t), ("gpu", ctypes.c_void_p)]


class srsran_dlsch_gpu_tb_t(ctypes.Structure):
    _fields_ = [("tbs", u32), ("Qm", u32), ("rv", u32), ("nof_e_bits", u32), ("d_e_bits", ctypes.c_void_p),
                ("d_data", ctypes.c_void_p), ("softbuffer", ctypes.POINTER(srsran_softbuffer_rx_t)),
                ("new_data", u32)]


SRSRAN_MAX_CARRIERS = 5
SRSRAN_UCI_MAX_M = 9


class srsran_uci_cfg_ack_t(ctypes.Structure):
    _fields_ = [("pending_tb", ctypes.c_bool * SRSRAN_MAX_CODEWORDS), ("nof_acks", u32), ("ncce", u32 * SRSRAN_UCI_MAX_M),
                ("N_bundle", u32), ("tdd_ack_M", u32), ("tdd_ack_m", u32), ("tdd_is_multiplex", ctypes.c_bool),
                ("tpc_for_pucch", u32), ("grant_cc_idx", u32)]


class srsran_cqi_cfg_t(ctypes.Structure):
    _fields_ = [("data_enable", ctypes.c_bool), ("pmi_present", ctypes.c_bool), ("four_antenna_ports", ctypes.c_bool),
                ("rank_is_not_one", ctypes.c_bool), ("subband_label_2_bits", ctypes.c_bool), ("scell_index", u32),
                ("L", u32), ("N", u32), ("sb_idx", u32), ("type", ctypes.c_int), ("ri_len", u32)]


class srsran_uci_cfg_t(ctypes.Structure):
    _fields_ = [("ack", srsran_uci_cfg_ack_t * SRSRAN_MAX_CARRIERS), ("cqi", srsran_cqi_cfg_t),
                ("is_scheduling_request_tti", ctypes.c_bool)]


class srsran_uci_offset_cfg_t(ctypes.Structure):
    _fields_ = [("I_offset_cqi", u32), ("I_offset_ri", u32), ("I_offset_ack", u32)]


class srsran_pusch_grant_t(ctypes.Structure):
    _fields_ = [("L_prb", u32), ("n_prb", u32 * 2), ("n_prb_tilde", u32 * 2), ("freq_hopping", u32), ("nof_re", u32),
                ("nof_symb", u32), ("tb", srsran_ra_tb_t), ("last_tb", srsran_ra_tb_t), ("n_dmrs", u32),
                ("is_rar", ctypes.c_bool)]


class _pusch_softbuffers(ctypes.Union):
    _fields_ = [("tx", ctypes.c_void_p), ("rx", ctypes.POINTER(srsran_softbuffer_rx_t))]


class srsran_pusch_cfg_t(ctypes.Structure):
    _fields_ = [("rnti", ctypes.c_uint16), ("uci_cfg", srsran_uci_cfg_t), ("uci_offset", srsran_uci_offset_cfg_t),
                ("grant", srsran_pusch_grant_t), ("max_nof_iterations", u32), ("last_O_cqi", u32), ("K_segm", u32),
                ("current_tx_nb", u32), ("csi_enable", ctypes.c_bool), ("enable_64qam", ctypes.c_bool),
                ("softbuffers", _pusch_softbuffers), ("meas_time_en", ctypes.c_bool), ("meas_time_value", u32),
                ("meas_epre_en", ctypes.c_bool), ("meas_ta_en", ctypes.c_bool), ("use_cedron_alg", ctypes.c_bool),
                ("meas_evm_en", ctypes.c_bool)]


u8 = ctypes.c_uint8
SRSRAN_CQI_TYPE_WIDEBAND, SRSRAN_CQI_TYPE_SUBBAND_UE, SRSRAN_CQI_TYPE_SUBBAND_UE_DIFF, SRSRAN_CQI_TYPE_SUBBAND_HL = range(4)
SRSRAN_CQI_MAX_BITS = 64


class srsran_cqi_hl_subband_t(ctypes.Structure):
    _fields_ = [("wideband_cqi_cw0", u8), ("subband_diff_cqi_cw0", u32), ("wideband_cqi_cw1", u8),
                ("subband_diff_cqi_cw1", u32), ("pmi", u32)]


class srsran_cqi_ue_diff_subband_t(ctypes.Structure):
    _fields_ = [("wideband_cqi", u8), ("subband_diff_cqi", u8), ("position_subband", u32)]


class srsran_cqi_format2_wideband_t(ctypes.Structure):
    _fields_ = [("wideband_cqi", u8), ("spatial_diff_cqi", u8), ("pmi", u8)]


class srsran_cqi_ue_subband_t(ctypes.Structure):
    _fields_ = [("subband_cqi", u8), ("subband_label", u8)]


class _cqi_value_u(ctypes.Union):
    _fields_ = [("wideband", srsran_cqi_format2_wideband_t), ("subband_ue", srsran_cqi_ue_subband_t),
                ("subband_ue_diff", srsran_cqi_ue_diff_subband_t), ("subband_hl", srsran_cqi_hl_subband_t)]


class srsran_cqi_value_t(ctypes.Structure):
    _anonymous_ = ("u",)
    _fields_ = [("u", _cqi_value_u), ("data_crc", ctypes.c_bool)]


class srsran_uci_value_ack_t(ctypes.Structure):
    _fields_ = [("ack_value", u8 * 10), ("valid", ctypes.c_bool)]


class srsran_uci_value_t(ctypes.Structure):
    _fields_ = [("scheduling_request", ctypes.c_bool), ("cqi", srsran_cqi_value_t), ("ack", srsran_uci_value_ack_t),
                ("ri", u8)]


class srsran_dlsch_gpu_enc_t(ctypes.Structure):
    _fields_ = [("tbs", u32), ("Qm", u32), ("rv", u32), ("nof_e_bits", u32), ("d_data", ctypes.c_void_p),
                ("d_e_bits", ctypes.c_void_p)]


class srsran_ulsch_gpu_tb_t(ctypes.Structure):
    _fields_ = [("tbs", u32), ("Qm", u32), ("rv", u32), ("nof_e_bits", u32), ("nof_symb", u32),
                ("d_q_bits", ctypes.c_void_p), ("d_g_bits", ctypes.c_void_p), ("d_data", ctypes.c_void_p),
                ("softbuffer", ctypes.POINTER(srsran_softbuffer_rx_t)), ("new_data", u32)]


_i16p = ctypes.POINTER(ctypes.c_int16)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_bound = False


def lib():
    global _bound
    L = load_library()
    if _bound:
        return L
    SB = ctypes.POINTER(srsran_softbuffer_rx_t)
    SCH = ctypes.POINTER(srsran_sch_t)
    CFG = ctypes.POINTER(srsran_pdsch_cfg_t)
    CRC = ctypes.POINTER(srsran_crc_t)
    sig = {
        "srsran_cbsegm": ([ctypes.POINTER(srsran_cbsegm_t), u32], ctypes.c_int),
        "srsran_cbsegm_cbsize": ([u32], ctypes.c_int),
        "srsran_cbsegm_cbindex": ([u32], ctypes.c_int),
        "srsran_cbsegm_cbsize_isvalid": ([u32], ctypes.c_bool),
        "srsran_crc_init": ([CRC, u32, ctypes.c_int], ctypes.c_int),
        "srsran_crc_set_init": ([CRC, ctypes.c_uint64], ctypes.c_int),
        "srsran_crc_checksum_byte": ([CRC, _u8p, ctypes.c_int], u32),
        "srsran_crc_match_byte": ([CRC, _u8p, ctypes.c_int], ctypes.c_bool),
        "srsran_crc_attach_byte": ([CRC, _u8p, ctypes.c_int], u32),
        "srsran_mod_bits_x_symbol": ([ctypes.c_int], u32),
        "srsran_rm_turbo_gentables": ([], None),
        "srsran_rm_turbo_free_tables": ([], None),
        "srsran_tcod_init": ([ctypes.POINTER(srsran_tcod_t), u32], ctypes.c_int),
        "srsran_tcod_free": ([ctypes.POINTER(srsran_tcod_t)], None),
        "srsran_tcod_encode": ([ctypes.POINTER(srsran_tcod_t), _u8p, _u8p, u32], ctypes.c_int),
        "srsran_rm_turbo_tx_lut": ([_u8p, _u8p, _u8p, _u8p, u32, u32, u32, u32], ctypes.c_int),
        "srsran_rm_turbo_rx_lut": ([_i16p, _i16p, u32, u32, u32], ctypes.c_int),
        "srsran_rm_turbo_rx_lut_": ([_i16p, _i16p, u32, u32, u32, ctypes.c_bool], ctypes.c_int),
        "srsran_rm_turbo_rx_lut_8bit": ([ctypes.POINTER(ctypes.c_int8), ctypes.POINTER(ctypes.c_int8), u32, u32, u32],
                                        ctypes.c_int),
        "srsran_softbuffer_rx_init": ([SB, u32], ctypes.c_int),
        "srsran_softbuffer_rx_init_guru": ([SB, u32, u32], ctypes.c_int),
        "srsran_softbuffer_rx_reset": ([SB], None),
        "srsran_softbuffer_rx_reset_tbs": ([SB, u32], None),
        "srsran_softbuffer_rx_reset_cb": ([SB, u32], None),
        "srsran_softbuffer_rx_reset_cb_crc": ([SB, u32], None),
        "srsran_softbuffer_rx_free": ([SB], None),
        "srsran_softbuffer_rx_sync": ([SB], ctypes.c_int),
        "srsran_softbuffer_rx_gpu_arena": ([ctypes.c_int, ctypes.c_size_t], ctypes.c_int),
        "srsran_softbuffer_rx_gpu_ptr": ([SB], ctypes.c_void_p),
        "srsran_sch_init": ([SCH], ctypes.c_int),
        "srsran_sch_free": ([SCH], None),
        "srsran_sch_set_max_noi": ([SCH, u32], None),
        "srsran_sch_last_noi": ([SCH], ctypes.c_float),
        "srsran_dlsch_decode": ([SCH, CFG, _i16p, _u8p], ctypes.c_int),
        "srsran_dlsch_decode2": ([SCH, CFG, _i16p, _u8p, ctypes.c_int, u32], ctypes.c_int),
        "srsran_dlsch_gpu_decode_batch": ([SCH, u32, ctypes.POINTER(srsran_dlsch_gpu_tb_t), ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
        "srsran_ulsch_decode": ([SCH, ctypes.POINTER(srsran_pusch_cfg_t), _i16p, _i16p, _u8p, _u8p,
                                 ctypes.POINTER(srsran_uci_value_t)], ctypes.c_int),
        "srsran_sch_beta_cqi": ([u32], ctypes.c_float),
        "srsran_sch_beta_ack": ([u32], ctypes.c_float),
        "srsran_sch_find_Ioffset_ack": ([ctypes.c_float], u32),
        "srsran_sch_find_Ioffset_cqi": ([ctypes.c_float], u32),
        "srsran_sch_find_Ioffset_ri": ([ctypes.c_float], u32),
        "srsran_qprime_cqi_ext": ([u32, u32, u32, ctypes.c_float], u32),
        "srsran_qprime_ack_ext": ([u32, u32, u32, u32, ctypes.c_float], u32),
        "srsran_dlsch_encode2": ([SCH, CFG, _u8p, _u8p, ctypes.c_int, u32], ctypes.c_int),
        "srsran_dlsch_gpu_encode_batch": ([SCH, u32, ctypes.POINTER(srsran_dlsch_gpu_enc_t), ctypes.c_void_p],
                                          ctypes.c_int),
        "srsran_uci_cfg_total_ack": ([ctypes.POINTER(srsran_uci_cfg_t)], u32),
        "srsran_cqi_size": ([ctypes.POINTER(srsran_cqi_cfg_t)], ctypes.c_int),
        "srsran_cqi_value_pack": ([ctypes.POINTER(srsran_cqi_cfg_t), ctypes.POINTER(srsran_cqi_value_t), _u8p],
                                  ctypes.c_int),
        "srsran_cqi_value_unpack": ([ctypes.POINTER(srsran_cqi_cfg_t), _u8p, ctypes.POINTER(srsran_cqi_value_t)],
                                    ctypes.c_int),
        "srsran_ulsch_gpu_decode_batch": ([SCH, u32, ctypes.POINTER(srsran_ulsch_gpu_tb_t), ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _bound = True
    return L


def cbsegm(tbs):
    s = srsran_cbsegm_t()
    ret = lib().srsran_cbsegm(ctypes.byref(s), tbs)
    return ret, s


def crc_checksum_byte(poly, data, nbits):
    c = srsran_crc_t()
    lib().srsran_crc_init(ctypes.byref(c), poly, 24)
    d = np.ascontiguousarray(data, dtype=np.uint8)
    return lib().srsran_crc_checksum_byte(ctypes.byref(c), d.ctypes.data_as(_u8p), nbits)


def rm_turbo_rx_lut(e, softbuf, cb_idx, rv, enable_input_tdec=True):
    """In place on a copy of softbuf; returns (ret, new softbuf)."""
    e = np.ascontiguousarray(e, dtype=np.int16)
    out = np.array(softbuf, dtype=np.int16, copy=True)
    ret = lib().srsran_rm_turbo_rx_lut_(e.ctypes.data_as(_i16p), out.ctypes.data_as(_i16p), len(e), cb_idx, rv,
                                        enable_input_tdec)
    return ret, out


def softbuffer_arena(enable, nbytes=0):
    """srsran_softbuffer_rx_gpu_arena: arena on / off for soft buffers initialised from now on"""
    return lib().srsran_softbuffer_rx_gpu_arena(1 if enable else 0, nbytes)


class SoftbufferRx:
    """srsran_softbuffer_rx_t owner (device arena)."""

    def __init__(self, nof_prb=None, max_cb=None, max_cb_size=SOFTBUFFER_SIZE):
        self.s = srsran_softbuffer_rx_t()
        if nof_prb is not None:
            ret = lib().srsran_softbuffer_rx_init(ctypes.byref(self.s), nof_prb)
        else:
            ret = lib().srsran_softbuffer_rx_init_guru(ctypes.byref(self.s), max_cb, max_cb_size)
        if ret != 0:
            raise RuntimeError(f"srsran_softbuffer_rx_init failed ({ret})")

    @property
    def max_cb(self):
        return self.s.max_cb

    @property
    def device_ptr(self):
        """device address of the first code block's soft buffer (srsran_softbuffer_rx_gpu_ptr)"""
        return lib().srsran_softbuffer_rx_gpu_ptr(ctypes.byref(self.s)) or 0

    def cb_crc(self, n=None):
        n = self.s.max_cb if n is None else n
        return [bool(self.s.cb_crc[i]) for i in range(n)]

    def set_cb_crc(self, i, v):
        self.s.cb_crc[i] = bool(v)

    @property
    def tb_crc(self):
        return bool(self.s.tb_crc)

    def reset(self):
        lib().srsran_softbuffer_rx_reset(ctypes.byref(self.s))

    def reset_tbs(self, tbs):
        lib().srsran_softbuffer_rx_reset_tbs(ctypes.byref(self.s), tbs)

    def reset_cb_crc(self, n):
        lib().srsran_softbuffer_rx_reset_cb_crc(ctypes.byref(self.s), n)

    def sync(self):
        return lib().srsran_softbuffer_rx_sync(ctypes.byref(self.s))

    def read_cb(self, i, n):
        """Copy n int16 of code block i's device soft buffer to the host (test helper)."""
        import torch  # device copies go through torch's HIP runtime
        out = torch.empty(n, dtype=torch.int16)
        _memcpy_d2h(out, self.s.buffer_f[i], n * 2)
        return out.numpy()

    def read_data(self, i, n):
        import torch
        out = torch.empty(n, dtype=torch.uint8)
        _memcpy_d2h(out, self.s.data[i], n)
        return out.numpy()

    def free(self):
        if self.s.gpu:
            lib().srsran_softbuffer_rx_free(ctypes.byref(self.s))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


_hip = None


def _memcpy_d2h(host_tensor, dptr, nbytes):
    """hipMemcpy device -> host through the HIP runtime already loaded by torch."""
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so.7")
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipMemcpy.restype = ctypes.c_int
    r = _hip.hipMemcpy(ctypes.c_void_p(host_tensor.data_ptr()), ctypes.c_void_p(dptr), nbytes, 2)
    if r != 0:
        raise RuntimeError(f"hipMemcpy failed ({r})")


class Sch:
    """srsran_sch_t owner with the reference's DL-SCH decode entry points."""

    def __init__(self):
        self.q = srsran_sch_t()
        if lib().srsran_sch_init(ctypes.byref(self.q)) != 0:
            raise RuntimeError("srsran_sch_init failed (no HIP device?)")

    def set_llr8(self, on=True):
        """srsran_sch_t.llr_is_8bit: int8 e bits and the 8-bit decoders (sch.c:409-428)"""
        self.q.llr_is_8bit = bool(on)

    def set_max_noi(self, n):
        lib().srsran_sch_set_max_noi(ctypes.byref(self.q), n)

    @property
    def max_iterations(self):
        return self.q.max_iterations

    def last_noi(self):
        return lib().srsran_sch_last_noi(ctypes.byref(self.q))

    def decode(self, softbuffer, tbs, Qm, rv, e_bits, nof_layers=1, nof_tb=1, tb_idx=0):
        """srsran_dlsch_decode2 -> (ret, data bytes, avg_iterations)."""
        cfg = srsran_pdsch_cfg_t()
        cfg.grant.nof_tb = nof_tb
        tb = cfg.grant.tb[tb_idx]
        tb.mod = MOD_FROM_QM[Qm]
        tb.tbs = tbs
        tb.rv = rv
        tb.nof_bits = len(e_bits)
        tb.enabled = True
        cfg.softbuffers.rx[tb_idx] = ctypes.pointer(softbuffer.s)
        e = np.ascontiguousarray(e_bits, dtype=np.int8 if self.q.llr_is_8bit else np.int16)  # sch.c:380-381
        data = np.zeros(tbs // 8 + 64, np.uint8)
        ret = lib().srsran_dlsch_decode2(ctypes.byref(self.q), ctypes.byref(cfg), ctypes.cast(e.ctypes.data, _i16p),
                                         data.ctypes.data_as(_u8p), tb_idx, nof_layers)
        return ret, data, self.last_noi()

    def encode(self, tbs, Qm, rv, nof_bits, data, nof_layers=1, nof_tb=1, tb_idx=0):
        """srsran_dlsch_encode2 -> (ret, packed e bits)"""
        cfg = srsran_pdsch_cfg_t()
        cfg.grant.nof_tb = nof_tb
        tb = cfg.grant.tb[tb_idx]
        tb.mod, tb.tbs, tb.rv, tb.nof_bits, tb.enabled = MOD_FROM_QM[Qm], tbs, rv, nof_bits, True
        d = np.ascontiguousarray(data, dtype=np.uint8)
        e = np.zeros((nof_bits + 7) // 8, np.uint8)
        ret = lib().srsran_dlsch_encode2(ctypes.byref(self.q), ctypes.byref(cfg), d.ctypes.data_as(_u8p),
                                         e.ctypes.data_as(_u8p), tb_idx, nof_layers)
        return ret, e

    def encode_batch(self, entries, stream=None):
        """srsran_dlsch_gpu_encode_batch; entries: (tbs, Qm x layers, rv, nof_e_bits, d_data, d_e_bits)"""
        arr = (srsran_dlsch_gpu_enc_t * len(entries))()
        for i, (tbs, Qm, rv, nb, dd, de) in enumerate(entries):
            arr[i].tbs, arr[i].Qm, arr[i].rv, arr[i].nof_e_bits, arr[i].d_data, arr[i].d_e_bits = tbs, Qm, rv, nb, dd, de
        return lib().srsran_dlsch_gpu_encode_batch(ctypes.byref(self.q), len(entries), arr, stream)

    def decode_batch(self, entries, d_result, d_avg, stream=None):
        """srsran_dlsch_gpu_decode_batch over device buffers.

        entries: list of (tbs, Qm, rv, nof_e_bits, d_e_bits ptr, d_data ptr, SoftbufferRx[, new_data])."""
        arr = (srsran_dlsch_gpu_tb_t * len(entries))()
        for i, ent in enumerate(entries):
            tbs, Qm, rv, nbits, de, dd, sb = ent[:7]
            arr[i].new_data = int(ent[7]) if len(ent) > 7 else 0
            arr[i].tbs, arr[i].Qm, arr[i].rv, arr[i].nof_e_bits = tbs, Qm, rv, nbits
            arr[i].d_e_bits, arr[i].d_data = de, dd
            arr[i].softbuffer = ctypes.pointer(sb.s)
        return lib().srsran_dlsch_gpu_decode_batch(ctypes.byref(self.q), len(entries), arr, d_result, d_avg, stream)

    def ulsch_decode(self, softbuffer, tbs, Qm, rv, nof_symb, q_bits, uci_cfg=None):
        """srsran_ulsch_decode (no UCI) -> (ret, data bytes, g_bits, avg_iterations, K_segm)."""
        cfg = srsran_pusch_cfg_t()
        tb = cfg.grant.tb
        tb.mod = MOD_FROM_QM[Qm]
        tb.tbs = tbs
        tb.rv = rv
        tb.nof_bits = len(q_bits)
        tb.enabled = True
        cfg.grant.nof_symb = nof_symb
        cfg.grant.nof_re = len(q_bits) // Qm
        cfg.softbuffers.rx = ctypes.pointer(softbuffer.s)
        if uci_cfg is not None:
            uci_cfg(cfg.uci_cfg)
        q = np.ascontiguousarray(q_bits, dtype=np.int16)
        g = np.zeros_like(q)
        data = np.zeros(tbs // 8 + 64, np.uint8)
        ret = lib().srsran_ulsch_decode(ctypes.byref(self.q), ctypes.byref(cfg), q.ctypes.data_as(_i16p),
                                        g.ctypes.data_as(_i16p), None, data.ctypes.data_as(_u8p), None)
        return ret, data, g, self.last_noi(), cfg.K_segm

    def ulsch_decode_uci(self, cfg, q_bits, c_seq=None, g_bits=None, tbs=None):
        """srsran_ulsch_decode with a prepared srsran_pusch_cfg_t (UCI fields set by the caller).
        Returns (ret, data bytes, q_bits after the call, g_bits, srsran_uci_value_t)."""
        q = np.array(q_bits, dtype=np.int16, copy=True)
        g = np.zeros_like(q) if g_bits is None else np.array(g_bits, dtype=np.int16, copy=True)
        nbytes = (tbs if tbs is not None else cfg.grant.tb.tbs) // 8 + 64
        data = np.zeros(nbytes, np.uint8)
        uci = srsran_uci_value_t()
        c = None if c_seq is None else np.ascontiguousarray(c_seq, dtype=np.uint8)
        ret = lib().srsran_ulsch_decode(ctypes.byref(self.q), ctypes.byref(cfg), q.ctypes.data_as(_i16p),
                                        g.ctypes.data_as(_i16p), None if c is None else c.ctypes.data_as(_u8p),
                                        data.ctypes.data_as(_u8p), ctypes.byref(uci))
        return ret, data, q, g, uci

    def ulsch_decode_batch(self, entries, d_result, d_avg, stream=None):
        """srsran_ulsch_gpu_decode_batch. entries: (tbs, Qm, rv, nof_e_bits, nof_symb, d_q, d_g, d_data,
        SoftbufferRx[, new_data])."""
        arr = (srsran_ulsch_gpu_tb_t * max(len(entries), 1))()
        for i, ent in enumerate(entries):
            (arr[i].tbs, arr[i].Qm, arr[i].rv, arr[i].nof_e_bits, arr[i].nof_symb, arr[i].d_q_bits, arr[i].d_g_bits,
             arr[i].d_data) = ent[:8]
            arr[i].softbuffer = ctypes.pointer(ent[8].s)
            arr[i].new_data = int(ent[9]) if len(ent) > 9 else 0
        return lib().srsran_ulsch_gpu_decode_batch(ctypes.byref(self.q), len(entries), arr, d_result, d_avg, stream)

    def free(self):
        if self.q.gpu:
            lib().srsran_sch_free(ctypes.byref(self.q))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
