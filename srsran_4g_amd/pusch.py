"""Python mirror of the PUSCH receive C API (include/srsran_pusch.h): PUSCH DMRS, the UL channel
estimator (chest_ul.c) and srsran_pusch_decode (pusch.c:358-471), driven the way the reference's
pusch_test.c / enb_ul.c call them.  No CPU fallback: estimation and decoding run the HIP kernels."""
import ctypes

import numpy as np

from .sch import srsran_pusch_cfg_t, srsran_sch_t, srsran_uci_value_t
from .tdec import load_library
from .ue_dl import srsran_cell_t, srsran_tdd_config_t

u32 = ctypes.c_uint32
_f = ctypes.c_float
_cfp = ctypes.c_void_p  # cf_t*


class srsran_ul_sf_cfg_t(ctypes.Structure):
    _fields_ = [("tdd_config", srsran_tdd_config_t), ("tti", u32), ("shortened", ctypes.c_bool)]


class srsran_refsignal_dmrs_pusch_cfg_t(ctypes.Structure):
    _fields_ = [("cyclic_shift", u32), ("delta_ss", u32), ("group_hopping_en", ctypes.c_bool),
                ("sequence_hopping_en", ctypes.c_bool)]


class srsran_chest_ul_res_t(ctypes.Structure):
    _fields_ = [("ce", ctypes.POINTER(ctypes.c_float)), ("nof_re", u32), ("noise_estimate", _f),
                ("noise_estimate_dbFs", _f), ("rsrp", _f), ("rsrp_dBfs", _f), ("epre", _f), ("epre_dBfs", _f),
                ("snr", _f), ("snr_db", _f), ("cfo_hz", _f), ("ta_us", _f), ("gpu", ctypes.c_void_p)]


class srsran_chest_ul_t(ctypes.Structure):
    _fields_ = [("cell", srsran_cell_t), ("dmrs_cfg", srsran_refsignal_dmrs_pusch_cfg_t),
                ("dmrs_signal_configured", ctypes.c_bool), ("smooth_filter_len", u32), ("smooth_filter", _f * 64),
                ("gpu", ctypes.c_void_p)]


class srsran_pusch_res_t(ctypes.Structure):
    _fields_ = [("data", ctypes.POINTER(ctypes.c_uint8)), ("uci", srsran_uci_value_t), ("crc", ctypes.c_bool),
                ("avg_iterations_block", _f), ("evm", _f), ("epre_dbfs", _f)]


class srsran_pusch_t(ctypes.Structure):
    _fields_ = [("cell", srsran_cell_t), ("is_ue", ctypes.c_bool), ("ue_rnti", ctypes.c_uint16), ("max_re", u32),
                ("llr_is_8bit", ctypes.c_bool), ("ul_sch", srsran_sch_t), ("gpu", ctypes.c_void_p)]


class srsran_pusch_gpu_ue_t(ctypes.Structure):
    _fields_ = [("chest", ctypes.POINTER(srsran_chest_ul_t)), ("sf", ctypes.POINTER(srsran_ul_sf_cfg_t)),
                ("cfg", ctypes.POINTER(srsran_pusch_cfg_t)), ("d_sf_symbols", ctypes.c_void_p), ("new_data", u32)]


_bound = False


def lib():
    global _bound
    L = load_library()
    if not _bound:
        CH = ctypes.POINTER(srsran_chest_ul_t)
        RES = ctypes.POINTER(srsran_chest_ul_res_t)
        PU = ctypes.POINTER(srsran_pusch_t)
        SF = ctypes.POINTER(srsran_ul_sf_cfg_t)
        CFG = ctypes.POINTER(srsran_pusch_cfg_t)
        DM = ctypes.POINTER(srsran_refsignal_dmrs_pusch_cfg_t)
        sig = {
            "srsran_dft_precoding_valid_prb": ([u32], ctypes.c_bool),
            "srsran_dft_precoding_get_valid_prb": ([u32], u32),
            "srsran_dft_precoding_gpu": ([_cfp, _cfp, u32, u32, ctypes.c_void_p], ctypes.c_int),
            "srsran_refsignal_dmrs_pusch_gen_cell": ([ctypes.POINTER(srsran_cell_t), DM, u32, u32, u32, _cfp],
                                                     ctypes.c_int),
            "srsran_chest_ul_init": ([CH, u32], ctypes.c_int),
            "srsran_chest_ul_free": ([CH], None),
            "srsran_chest_ul_res_init": ([RES, u32], ctypes.c_int),
            "srsran_chest_ul_res_set_identity": ([RES], None),
            "srsran_chest_ul_res_free": ([RES], None),
            "srsran_chest_ul_set_cell": ([CH, srsran_cell_t], ctypes.c_int),
            "srsran_chest_ul_pregen": ([CH, DM, ctypes.c_void_p], None),
            "srsran_chest_ul_estimate_pusch": ([CH, SF, CFG, _cfp, RES], ctypes.c_int),
            "srsran_pusch_init_enb": ([PU, u32], ctypes.c_int),
            "srsran_pusch_free": ([PU], None),
            "srsran_pusch_set_cell": ([PU, srsran_cell_t], ctypes.c_int),
            "srsran_pusch_assert_grant": ([ctypes.c_void_p], ctypes.c_int),
            "srsran_pusch_decode": ([PU, SF, CFG, RES, _cfp, ctypes.POINTER(srsran_pusch_res_t)], ctypes.c_int),
            "srsran_pusch_gpu_decode_batch": ([PU, u32, ctypes.POINTER(srsran_pusch_gpu_ue_t), RES,
                                               ctypes.POINTER(srsran_pusch_res_t)], ctypes.c_int),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _bound = True
    return L


def nsymb_slot(cp):
    return 7 if cp == 0 else 6


def dmrs(cell, cfg, nof_prb, sf_idx, n_dmrs):
    r = np.zeros(2 * 12 * nof_prb, np.complex64)
    ret = lib().srsran_refsignal_dmrs_pusch_gen_cell(ctypes.byref(cell), ctypes.byref(cfg), nof_prb, sf_idx, n_dmrs,
                                                     r.ctypes.data)
    return ret, r


class ChestUl:
    """srsran_chest_ul_t + one srsran_chest_ul_res_t"""

    def __init__(self, cell, dmrs_cfg, max_prb=100):
        self.cell = cell
        self.q = srsran_chest_ul_t()
        self.res = srsran_chest_ul_res_t()
        L = lib()
        assert L.srsran_chest_ul_init(ctypes.byref(self.q), max_prb) == 0
        assert L.srsran_chest_ul_res_init(ctypes.byref(self.res), max_prb) == 0
        assert L.srsran_chest_ul_set_cell(ctypes.byref(self.q), cell) == 0
        L.srsran_chest_ul_pregen(ctypes.byref(self.q), ctypes.byref(dmrs_cfg), None)
        assert self.q.dmrs_signal_configured

    def estimate(self, sf, cfg, grid):
        g = np.ascontiguousarray(grid, dtype=np.complex64)
        ret = lib().srsran_chest_ul_estimate_pusch(ctypes.byref(self.q), ctypes.byref(sf), ctypes.byref(cfg),
                                                   g.ctypes.data, ctypes.byref(self.res))
        return ret

    def ce(self, n):
        return np.ctypeslib.as_array(self.res.ce, shape=(2 * n,)).view(np.complex64).copy()

    def free(self):
        if self.q.gpu:
            lib().srsran_chest_ul_res_free(ctypes.byref(self.res))
            lib().srsran_chest_ul_free(ctypes.byref(self.q))


class Pusch:
    def __init__(self, cell, max_prb=100):
        self.q = srsran_pusch_t()
        L = lib()
        assert L.srsran_pusch_init_enb(ctypes.byref(self.q), max_prb) == 0
        assert L.srsran_pusch_set_cell(ctypes.byref(self.q), cell) == 0

    def decode(self, sf, cfg, chest_res, grid, tbs_bytes):
        g = np.ascontiguousarray(grid, dtype=np.complex64)
        data = np.zeros(tbs_bytes + 64, np.uint8)
        out = srsran_pusch_res_t()
        out.data = data.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        ret = lib().srsran_pusch_decode(ctypes.byref(self.q), ctypes.byref(sf), ctypes.byref(cfg),
                                        ctypes.byref(chest_res), g.ctypes.data, ctypes.byref(out))
        return ret, out, data

    def free(self):
        if self.q.gpu:
            lib().srsran_pusch_free(ctypes.byref(self.q))
