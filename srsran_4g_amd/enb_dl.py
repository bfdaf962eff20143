"""Python mirror of include/srsran_enb_dl.h: downlink subframes transmitted on the GPU (DL-SCH encode,
CRS, scrambling / modulation / precoding / RE mapping, PSS / SSS / PBCH / PCFICH / PDCCH, OFDM
modulator).  No CPU fallback."""
import ctypes

from .pdcch import srsran_dci_msg_t
from .sch import srsran_pdsch_cfg_t
from .tdec import load_library
from .ue_dl import srsran_cell_t

u32 = ctypes.c_uint32


class srsran_enb_dl_gpu_t(ctypes.Structure):
    _fields_ = [("cell", srsran_cell_t), ("gpu", ctypes.c_void_p)]


class srsran_enb_dl_gpu_ctrl_t(ctypes.Structure):
    _fields_ = [("put_base", u32), ("nof_dci", u32), ("dci", ctypes.POINTER(srsran_dci_msg_t))]


class srsran_enb_dl_gpu_sf_t(ctypes.Structure):
    _fields_ = [("tti", u32), ("cfi", u32), ("cfg", ctypes.POINTER(srsran_pdsch_cfg_t)),
                ("d_data", ctypes.c_void_p * 2), ("ctrl", ctypes.POINTER(srsran_enb_dl_gpu_ctrl_t))]


_bound = False


def lib():
    global _bound
    L = load_library()
    if not _bound:
        Q = ctypes.POINTER(srsran_enb_dl_gpu_t)
        for name, args, res in (
                ("srsran_enb_dl_gpu_init", [Q, srsran_cell_t], ctypes.c_int),
                ("srsran_enb_dl_gpu_free", [Q], None),
                ("srsran_enb_dl_gpu_tx_batch", [Q, u32, ctypes.POINTER(srsran_enb_dl_gpu_sf_t), ctypes.c_void_p,
                                                ctypes.c_float, ctypes.c_void_p], ctypes.c_int),
                ("srsran_enb_dl_gpu_sf_symbols", [Q], ctypes.c_void_p),
                ("srsran_pbch_mib_pack", [ctypes.POINTER(srsran_cell_t), u32, ctypes.POINTER(ctypes.c_uint8)], None)):
            f = getattr(L, name)
            f.argtypes, f.restype = args, res
        _bound = True
    return L


class EnbDl:
    def __init__(self, cell):
        self.q = srsran_enb_dl_gpu_t()
        assert lib().srsran_enb_dl_gpu_init(ctypes.byref(self.q), cell) == 0
        self._keep = []

    def tx_batch(self, sfs, d_samples, scale=0.0, stream=None):
        """sfs: list of (tti, cfi, srsran_pdsch_cfg_t or None, [device payload pointers][, ctrl]) with ctrl =
        (put_base, [srsran_dci_msg_t, ...]) or None"""
        arr = (srsran_enb_dl_gpu_sf_t * len(sfs))()
        self._keep = []
        for i, sf in enumerate(sfs):
            tti, cfi, cfg, ptrs = sf[:4]
            ctrl = sf[4] if len(sf) > 4 else None
            arr[i].tti, arr[i].cfi = tti, cfi
            if cfg is not None:
                arr[i].cfg = ctypes.pointer(cfg)
                self._keep.append(cfg)
            for j, p in enumerate(ptrs):
                arr[i].d_data[j] = p
            if ctrl is not None:
                put_base, msgs = ctrl
                c = srsran_enb_dl_gpu_ctrl_t()
                c.put_base = 1 if put_base else 0
                m = (srsran_dci_msg_t * max(1, len(msgs)))(*msgs)
                c.nof_dci, c.dci = len(msgs), ctypes.cast(m, ctypes.POINTER(srsran_dci_msg_t))
                arr[i].ctrl = ctypes.pointer(c)
                self._keep += [c, m]
        return lib().srsran_enb_dl_gpu_tx_batch(ctypes.byref(self.q), len(sfs), arr, d_samples, scale, stream)

    def sf_symbols(self):
        """device pointer of the last batch's grids (srsran_enb_dl_gpu_sf_symbols)"""
        return lib().srsran_enb_dl_gpu_sf_symbols(ctypes.byref(self.q))

    def free(self):  # noqa: E301
        if self.q.gpu:
            lib().srsran_enb_dl_gpu_free(ctypes.byref(self.q))


def mib_pack(cell, sfn):
    """srsran_pbch_mib_pack -> 24 MIB bits (uint8)"""
    import numpy as np
    out = np.zeros(24, np.uint8)
    lib().srsran_pbch_mib_pack(ctypes.byref(cell), sfn, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return out
