"""Python mirror of the control-channel C API (include/srsran_pdcch.h): REG tables, PCFICH, PDCCH
blind decoding, DCI sizes / unpacking and the DL grant.  No CPU fallback: the decode entry points
need the HIP device."""
import ctypes

import numpy as np

from .sch import srsran_pdsch_grant_t
from .tdec import load_library
from .ue_dl import (srsran_cell_t, srsran_chest_dl_res_t, srsran_dci_cfg_t, srsran_dl_sf_cfg_t, srsran_ue_dl_cfg_t,
                    srsran_ue_dl_t)

u32 = ctypes.c_uint32
MAX_BITS = 128
FORMAT0, FORMAT1, FORMAT1A, FORMAT1B, FORMAT1C, FORMAT1D, FORMAT2, FORMAT2A, FORMAT2B = range(9)


class srsran_regs_t(ctypes.Structure):
    _fields_ = [("cell", srsran_cell_t), ("max_ctrl_symbols", u32), ("ngroups_phich", u32), ("ngroups_phich_m1", u32),
                ("phich_res", ctypes.c_int), ("phich_len", ctypes.c_int), ("phich_mi", u32),
                ("pdcch_nregs", u32 * 3), ("pcfich_re", u32 * 16), ("pdcch_re", ctypes.POINTER(u32) * 3)]


class srsran_pcfich_t(ctypes.Structure):
    _fields_ = [("cell", srsran_cell_t), ("nof_rx_antennas", u32), ("nof_symbols", u32),
                ("regs", ctypes.POINTER(srsran_regs_t)), ("data_f", ctypes.c_float * 32), ("gpu", ctypes.c_void_p)]


class srsran_pdcch_t(ctypes.Structure):
    _fields_ = [("cell", srsran_cell_t), ("nof_regs", u32 * 3), ("nof_cce", u32 * 3), ("max_bits", u32),
                ("nof_rx_antennas", u32), ("is_ue", ctypes.c_bool), ("regs", ctypes.POINTER(srsran_regs_t)),
                ("llr_cfi", u32), ("gpu", ctypes.c_void_p)]


class srsran_dci_location_t(ctypes.Structure):
    _fields_ = [("L", u32), ("ncce", u32)]


class srsran_dci_msg_t(ctypes.Structure):
    _fields_ = [("payload", ctypes.c_uint8 * MAX_BITS), ("nof_bits", u32), ("location", srsran_dci_location_t),
                ("format", ctypes.c_int), ("rnti", ctypes.c_uint16)]


class srsran_dci_tb_t(ctypes.Structure):
    _fields_ = [("mcs_idx", u32), ("rv", ctypes.c_int), ("ndi", ctypes.c_bool), ("cw_idx", u32)]


class _alloc(ctypes.Union):
    _fields_ = [("type0_rbg_bitmask", u32), ("raw", u32 * 4)]


class srsran_dci_dl_t(ctypes.Structure):
    _anonymous_ = ("alloc",)
    _fields_ = [("rnti", ctypes.c_uint16), ("format", ctypes.c_int), ("location", srsran_dci_location_t),
                ("ue_cc_idx", u32), ("alloc_type", ctypes.c_int), ("alloc", _alloc), ("tb", srsran_dci_tb_t * 2),
                ("tb_cw_swap", ctypes.c_bool), ("pinfo", u32), ("pconf", ctypes.c_bool), ("power_offset", ctypes.c_bool),
                ("tpc_pucch", ctypes.c_uint8), ("is_pdcch_order", ctypes.c_bool), ("preamble_idx", u32),
                ("prach_mask_idx", u32), ("cif", u32), ("cif_present", ctypes.c_bool), ("srs_request", ctypes.c_bool),
                ("srs_request_present", ctypes.c_bool), ("pid", u32), ("dai", u32), ("is_tdd", ctypes.c_bool),
                ("is_dwpts", ctypes.c_bool), ("sram_id", ctypes.c_bool)]


class srsran_ra_type2_t(ctypes.Structure):
    _fields_ = [("riv", u32), ("n_prb1a", ctypes.c_int), ("n_gap", ctypes.c_int), ("mode", ctypes.c_int)]


class srsran_dci_ul_t(ctypes.Structure):
    """dci.h:130-178 (format 0)"""
    _fields_ = [("rnti", ctypes.c_uint16), ("format", ctypes.c_int), ("location", srsran_dci_location_t),
                ("ue_cc_idx", u32), ("type2_alloc", srsran_ra_type2_t), ("freq_hop_fl", ctypes.c_int),
                ("tb", srsran_dci_tb_t), ("n_dmrs", u32), ("cqi_request", ctypes.c_bool), ("dai", u32),
                ("ul_idx", u32), ("is_tdd", ctypes.c_bool), ("tpc_pusch", ctypes.c_uint8), ("cif", u32),
                ("cif_present", ctypes.c_bool), ("multiple_csi_request", ctypes.c_uint8),
                ("multiple_csi_request_present", ctypes.c_bool), ("srs_request", ctypes.c_bool),
                ("srs_request_present", ctypes.c_bool), ("ra_type", ctypes.c_int), ("ra_type_present", ctypes.c_bool)]


_bound = False


def lib():
    global _bound
    L = load_library()
    if not _bound:
        R = ctypes.POINTER(srsran_regs_t)
        PC = ctypes.POINTER(srsran_pcfich_t)
        PD = ctypes.POINTER(srsran_pdcch_t)
        SF = ctypes.POINTER(srsran_dl_sf_cfg_t)
        DC = ctypes.POINTER(srsran_dci_cfg_t)
        M = ctypes.POINTER(srsran_dci_msg_t)
        CH = ctypes.POINTER(srsran_chest_dl_res_t)
        P = ctypes.c_void_p
        sig = {
            "srsran_regs_init": ([R, srsran_cell_t], ctypes.c_int),
            "srsran_regs_init_opts": ([R, srsran_cell_t, u32, ctypes.c_bool], ctypes.c_int),
            "srsran_regs_free": ([R], None),
            "srsran_regs_pdcch_ncce": ([R, u32], ctypes.c_int),
            "srsran_pcfich_init": ([PC, u32], ctypes.c_int),
            "srsran_pcfich_free": ([PC], None),
            "srsran_pcfich_set_cell": ([PC, R, srsran_cell_t], ctypes.c_int),
            "srsran_pcfich_decode": ([PC, SF, CH, P, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
            "srsran_pdcch_init_ue": ([PD, u32, u32], ctypes.c_int),
            "srsran_pdcch_free": ([PD], None),
            "srsran_pdcch_set_cell": ([PD, R, srsran_cell_t], ctypes.c_int),
            "srsran_pdcch_extract_llr": ([PD, SF, CH, P], ctypes.c_int),
            "srsran_pdcch_get_llr": ([PD, P, u32], ctypes.c_int),
            "srsran_pdcch_set_llr": ([PD, u32, P, u32], ctypes.c_int),
            "srsran_pdcch_decode_msg": ([PD, SF, DC, M], ctypes.c_int),
            "srsran_pdcch_gpu_decode_msgs": ([PD, SF, DC, M, u32, P], ctypes.c_int),
            "srsran_pdcch_ue_locations_ncce": ([u32, ctypes.POINTER(srsran_dci_location_t), u32, u32, ctypes.c_uint16],
                                               u32),
            "srsran_pdcch_common_locations_ncce": ([u32, ctypes.POINTER(srsran_dci_location_t), u32], u32),
            "srsran_dci_format_sizeof": ([ctypes.POINTER(srsran_cell_t), SF, DC, ctypes.c_int], u32),
            "srsran_dci_msg_unpack_pdsch": ([ctypes.POINTER(srsran_cell_t), SF, DC, M, ctypes.POINTER(srsran_dci_dl_t)],
                                            ctypes.c_int),
            "srsran_ra_dl_dci_to_grant": ([ctypes.POINTER(srsran_cell_t), SF, ctypes.c_int, ctypes.c_bool,
                                           ctypes.POINTER(srsran_dci_dl_t), ctypes.POINTER(srsran_pdsch_grant_t)],
                                          ctypes.c_int),
            "srsran_ra_tbs_from_idx": ([u32, u32], ctypes.c_int),
            "srsran_ue_dl_find_dl_dci": ([ctypes.POINTER(srsran_ue_dl_t), SF, ctypes.POINTER(srsran_ue_dl_cfg_t),
                                          ctypes.c_uint16, ctypes.POINTER(srsran_dci_dl_t)], ctypes.c_int),
            "srsran_ue_dl_dci_to_pdsch_grant": ([ctypes.POINTER(srsran_ue_dl_t), SF, ctypes.POINTER(srsran_ue_dl_cfg_t),
                                                 ctypes.POINTER(srsran_dci_dl_t), ctypes.POINTER(srsran_pdsch_grant_t)],
                                                ctypes.c_int),
            "srsran_ue_dl_find_ul_dci": ([ctypes.POINTER(srsran_ue_dl_t), SF, ctypes.POINTER(srsran_ue_dl_cfg_t),
                                          ctypes.c_uint16, ctypes.POINTER(srsran_dci_ul_t)], ctypes.c_int),
            "srsran_dci_msg_unpack_pusch": ([ctypes.POINTER(srsran_cell_t), SF, DC, M, ctypes.POINTER(srsran_dci_ul_t)],
                                            ctypes.c_int),
            "srsran_dci_msg_pack_pdsch": ([ctypes.POINTER(srsran_cell_t), SF, DC, ctypes.POINTER(srsran_dci_dl_t), M],
                                          ctypes.c_int),
            "srsran_dci_msg_pack_pusch": ([ctypes.POINTER(srsran_cell_t), SF, DC, ctypes.POINTER(srsran_dci_ul_t), M],
                                          ctypes.c_int),
            "srsran_ue_dl_set_mi_auto": ([ctypes.POINTER(srsran_ue_dl_t)], None),
            "srsran_ue_dl_set_mi_manual": ([ctypes.POINTER(srsran_ue_dl_t), u32], None),
            "srsran_ue_dl_set_mbsfn_area_id": ([ctypes.POINTER(srsran_ue_dl_t), ctypes.c_uint16], ctypes.c_int),
            "srsran_ue_dl_set_non_mbsfn_region": ([ctypes.POINTER(srsran_ue_dl_t), ctypes.c_uint8], None),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _bound = True
    return L


def cell(nof_prb, nof_ports, cell_id, phich_len=0, phich_res=2, cp=0):
    c = srsran_cell_t()
    c.nof_prb, c.nof_ports, c.id, c.cp = nof_prb, nof_ports, cell_id, cp
    c.phich_length, c.phich_resources = phich_len, phich_res
    return c


def unpack_pusch(c, msg, cfg=None):
    """srsran_dci_msg_unpack_pusch -> (ret, srsran_dci_ul_t)"""
    d = srsran_dci_ul_t()
    r = lib().srsran_dci_msg_unpack_pusch(ctypes.byref(c), None, ctypes.byref(cfg) if cfg is not None else None,
                                          ctypes.byref(msg), ctypes.byref(d))
    return r, d


def pack_pdsch(c, dci, cfg=None):
    """srsran_dci_msg_pack_pdsch -> (ret, srsran_dci_msg_t)"""
    m = srsran_dci_msg_t()
    r = lib().srsran_dci_msg_pack_pdsch(ctypes.byref(c), None, ctypes.byref(cfg) if cfg is not None else None,
                                        ctypes.byref(dci), ctypes.byref(m))
    return r, m


def pack_pusch(c, dci, cfg=None):
    """srsran_dci_msg_pack_pusch -> (ret, srsran_dci_msg_t)"""
    m = srsran_dci_msg_t()
    r = lib().srsran_dci_msg_pack_pusch(ctypes.byref(c), None, ctypes.byref(cfg) if cfg is not None else None,
                                        ctypes.byref(dci), ctypes.byref(m))
    return r, m


class Regs:
    def __init__(self, c, phich_mi=None, sf1_6=False):
        self.q = srsran_regs_t()
        if phich_mi is None and not sf1_6:
            ret = lib().srsran_regs_init(ctypes.byref(self.q), c)
        else:
            ret = lib().srsran_regs_init_opts(ctypes.byref(self.q), c, 1 if phich_mi is None else phich_mi, bool(sf1_6))
        if ret != 0:
            raise RuntimeError("srsran_regs_init failed")

    def pcfich_re(self):
        return np.array(self.q.pcfich_re[:], np.uint32)

    def pdcch_re(self, cfi):
        n = 4 * self.q.pdcch_nregs[cfi - 1]
        return np.ctypeslib.as_array(self.q.pdcch_re[cfi - 1], (n,)).copy()

    def free(self):
        lib().srsran_regs_free(ctypes.byref(self.q))


def dci_size(c, fmt, dci_cfg=None):
    return lib().srsran_dci_format_sizeof(ctypes.byref(c), None, ctypes.byref(dci_cfg) if dci_cfg else None, fmt)


def unpack_pdsch(c, bits, fmt, rnti, L=0, ncce=0):
    m = srsran_dci_msg_t()
    m.payload[:len(bits)] = [int(b) for b in bits]
    m.nof_bits, m.format, m.rnti = len(bits), fmt, rnti
    m.location.L, m.location.ncce = L, ncce
    d = srsran_dci_dl_t()
    r = lib().srsran_dci_msg_unpack_pdsch(ctypes.byref(c), None, None, ctypes.byref(m), ctypes.byref(d))
    return r, d


def dci_to_grant(c, dci, tti, cfi, tm):
    sf = srsran_dl_sf_cfg_t()
    sf.tti, sf.cfi = tti, cfi
    g = srsran_pdsch_grant_t()
    r = lib().srsran_ra_dl_dci_to_grant(ctypes.byref(c), ctypes.byref(sf), tm, False, ctypes.byref(dci),
                                         ctypes.byref(g))
    return r, g


def _ch(grids, ce, noise, nports):
    """host grids (nrx, 14, 12N) / full estimates (ports, nrx, 14, 12N) -> (pointer array, res, keepalive)"""
    g = [np.ascontiguousarray(x, np.complex64) for x in grids]
    e = [[np.ascontiguousarray(ce[p][r], np.complex64) for r in range(len(g))] for p in range(nports)]
    res = srsran_chest_dl_res_t()
    for p in range(nports):
        for r in range(len(g)):
            res.ce[p][r] = e[p][r].ctypes.data
    res.noise_estimate = noise
    ptrs = (ctypes.c_void_p * 4)(*([x.ctypes.data for x in g] + [None] * (4 - len(g))))
    return ptrs, res, (g, e)


class Control:
    """srsran_regs_t + srsran_pcfich_t + srsran_pdcch_t of one cell (the reference's UE objects)."""

    def __init__(self, c, nrx):
        self.c = c
        self.regs = Regs(c)
        self.pc = srsran_pcfich_t()
        self.pd = srsran_pdcch_t()
        L = lib()
        if L.srsran_pcfich_init(ctypes.byref(self.pc), nrx) or L.srsran_pdcch_init_ue(ctypes.byref(self.pd), c.nof_prb,
                                                                                       nrx):
            raise RuntimeError("control channel init failed")
        if L.srsran_pcfich_set_cell(ctypes.byref(self.pc), ctypes.byref(self.regs.q), c) or \
                L.srsran_pdcch_set_cell(ctypes.byref(self.pd), ctypes.byref(self.regs.q), c):
            raise RuntimeError("control channel set_cell failed")

    def pcfich(self, grids, ce, noise, tti):
        ptrs, res, keep = _ch(grids, ce, noise, self.c.nof_ports)
        sf = srsran_dl_sf_cfg_t()
        sf.tti = tti
        corr = ctypes.c_float()
        r = lib().srsran_pcfich_decode(ctypes.byref(self.pc), ctypes.byref(sf), ctypes.byref(res), ptrs,
                                       ctypes.byref(corr))
        if r < 0:
            raise RuntimeError("srsran_pcfich_decode failed")
        return sf.cfi, corr.value, np.array(self.pc.data_f[:], np.float32)

    def pdcch_llr(self, grids, ce, noise, tti, cfi):
        ptrs, res, keep = _ch(grids, ce, noise, self.c.nof_ports)
        sf = srsran_dl_sf_cfg_t()
        sf.tti, sf.cfi = tti, cfi
        if lib().srsran_pdcch_extract_llr(ctypes.byref(self.pd), ctypes.byref(sf), ctypes.byref(res), ptrs):
            raise RuntimeError("srsran_pdcch_extract_llr failed")
        out = np.zeros(72 * self.pd.nof_cce[cfi - 1], np.float32)
        n = lib().srsran_pdcch_get_llr(ctypes.byref(self.pd), out.ctypes.data, out.size)
        return out[:n]

    def set_llr(self, cfi, llr):
        llr = np.ascontiguousarray(llr, np.float32)
        if lib().srsran_pdcch_set_llr(ctypes.byref(self.pd), cfi, llr.ctypes.data, llr.size):
            raise RuntimeError("srsran_pdcch_set_llr failed")

    def decode(self, tti, cfi, cands, dci_cfg=None):
        """cands: [(L, ncce, format)] -> [(nof_bits, payload bits, crc_rem, corr)] (one launch)"""
        n = len(cands)
        msgs = (srsran_dci_msg_t * n)()
        for m, (L, ncce, fmt) in zip(msgs, cands):
            m.location.L, m.location.ncce, m.format = L, ncce, fmt
        corr = np.zeros(n, np.float32)
        sf = srsran_dl_sf_cfg_t()
        sf.tti, sf.cfi = tti, cfi
        r = lib().srsran_pdcch_gpu_decode_msgs(ctypes.byref(self.pd), ctypes.byref(sf),
                                                ctypes.byref(dci_cfg) if dci_cfg else None, msgs, n, corr.ctypes.data)
        if r:
            raise RuntimeError("srsran_pdcch_gpu_decode_msgs failed")
        return [(m.nof_bits, np.array(m.payload[:m.nof_bits], np.uint8), m.rnti, float(corr[i]))
                for i, m in enumerate(msgs)]

    def ncce(self, cfi):
        return self.pd.nof_cce[cfi - 1]

    def free(self):
        lib().srsran_pdcch_free(ctypes.byref(self.pd))
        lib().srsran_pcfich_free(ctypes.byref(self.pc))
        self.regs.free()


def ue_locations(ncce, sf_idx, rnti):
    locs = (srsran_dci_location_t * 16)()
    n = lib().srsran_pdcch_ue_locations_ncce(ncce, locs, 16, sf_idx, rnti)
    return [(locs[i].L, locs[i].ncce) for i in range(n)]


def common_locations(ncce):
    locs = (srsran_dci_location_t * 6)()
    n = lib().srsran_pdcch_common_locations_ncce(ncce, locs, 6)
    return [(locs[i].L, locs[i].ncce) for i in range(n)]
