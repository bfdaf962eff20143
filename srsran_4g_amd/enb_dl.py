"""Python mirror of include/srsran_enb_dl.h: PDSCH subframes transmitted on the GPU (DL-SCH encode,
CRS, scrambling / modulation / precoding / RE mapping, OFDM modulator).  No CPU fallback."""
import ctypes

from .sch import srsran_pdsch_cfg_t
from .tdec import load_library
from .ue_dl import srsran_cell_t

u32 = ctypes.c_uint32


class srsran_enb_dl_gpu_t(ctypes.Structure):
    _fields_ = [("cell", srsran_cell_t), ("gpu", ctypes.c_void_p)]


class srsran_enb_dl_gpu_sf_t(ctypes.Structure):
    _fields_ = [("tti", u32), ("cfi", u32), ("cfg", ctypes.POINTER(srsran_pdsch_cfg_t)),
                ("d_data", ctypes.c_void_p * 2)]


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
                                                ctypes.c_float, ctypes.c_void_p], ctypes.c_int)):
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
        """sfs: list of (tti, cfi, srsran_pdsch_cfg_t, [device payload pointers])"""
        arr = (srsran_enb_dl_gpu_sf_t * len(sfs))()
        self._keep = [c for (_, _, c, _) in sfs]
        for i, (tti, cfi, cfg, ptrs) in enumerate(sfs):
            arr[i].tti, arr[i].cfi, arr[i].cfg = tti, cfi, ctypes.pointer(cfg)
            for j, p in enumerate(ptrs):
                arr[i].d_data[j] = p
        return lib().srsran_enb_dl_gpu_tx_batch(ctypes.byref(self.q), len(sfs), arr, d_samples, scale, stream)

    def free(self):
        if self.q.gpu:
            lib().srsran_enb_dl_gpu_free(ctypes.byref(self.q))
