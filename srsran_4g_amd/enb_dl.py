"""Python mirror of include/srsran_enb_dl.h: downlink subframes transmitted on the GPU (DL-SCH encode,
CRS, scrambling / modulation / precoding / RE mapping, PSS / SSS / PBCH / PCFICH / PDCCH, OFDM
modulator).  No CPU fallback."""
import ctypes

from .pdcch import srsran_dci_dl_t, srsran_dci_location_t, srsran_dci_msg_t, srsran_pdcch_t, srsran_regs_t
from .sch import srsran_pdsch_cfg_t
from .tdec import load_library
from .ue_dl import srsran_cell_t, srsran_dci_cfg_t, srsran_dl_sf_cfg_t

u32 = ctypes.c_uint32


class srsran_enb_dl_gpu_t(ctypes.Structure):
    _fields_ = [("cell", srsran_cell_t), ("gpu", ctypes.c_void_p)]


class srsran_enb_dl_gpu_ctrl_t(ctypes.Structure):
    _fields_ = [("put_base", u32), ("nof_dci", u32), ("dci", ctypes.POINTER(srsran_dci_msg_t))]


class srsran_enb_dl_gpu_sf_t(ctypes.Structure):
    _fields_ = [("tti", u32), ("cfi", u32), ("cfg", ctypes.POINTER(srsran_pdsch_cfg_t)),
                ("d_data", ctypes.c_void_p * 2), ("ctrl", ctypes.POINTER(srsran_enb_dl_gpu_ctrl_t)),
                ("pdsch_scaling", ctypes.c_float)]


class srsran_enb_dl_t(ctypes.Structure):  # enb_dl.h's reference-named object (include/srsran_enb_dl.h)
    _fields_ = [("cell", srsran_cell_t), ("dl_sf", srsran_dl_sf_cfg_t), ("sf_symbols", ctypes.c_void_p * 4),
                ("out_buffer", ctypes.c_void_p * 4), ("regs", srsran_regs_t), ("pdcch", srsran_pdcch_t),
                ("nof_common_locations", u32 * 3), ("common_locations", (srsran_dci_location_t * 6) * 3),
                ("gpu", ctypes.c_void_p)]


_bound = False


def lib():
    global _bound
    L = load_library()
    if not _bound:
        Q = ctypes.POINTER(srsran_enb_dl_gpu_t)
        R = ctypes.POINTER(srsran_enb_dl_t)
        for name, args, res in (
                ("srsran_enb_dl_gpu_init", [Q, srsran_cell_t], ctypes.c_int),
                ("srsran_enb_dl_gpu_free", [Q], None),
                ("srsran_enb_dl_gpu_tx_batch", [Q, u32, ctypes.POINTER(srsran_enb_dl_gpu_sf_t), ctypes.c_void_p,
                                                ctypes.c_float, ctypes.c_void_p], ctypes.c_int),
                ("srsran_enb_dl_gpu_sf_symbols", [Q], ctypes.c_void_p),
                ("srsran_pbch_mib_pack", [ctypes.POINTER(srsran_cell_t), u32, ctypes.POINTER(ctypes.c_uint8)], None),
                ("srsran_enb_dl_init", [R, ctypes.c_void_p * 4, u32], ctypes.c_int),
                ("srsran_enb_dl_free", [R], None),
                ("srsran_enb_dl_set_cell", [R, srsran_cell_t], ctypes.c_int),
                ("srsran_enb_dl_location_is_common_ncce", [R, ctypes.POINTER(srsran_dci_location_t)], ctypes.c_bool),
                ("srsran_enb_dl_put_base", [R, ctypes.POINTER(srsran_dl_sf_cfg_t)], None),
                ("srsran_enb_dl_put_pdcch_dl", [R, ctypes.POINTER(srsran_dci_cfg_t), ctypes.POINTER(srsran_dci_dl_t)],
                 ctypes.c_int),
                ("srsran_enb_dl_put_pdsch", [R, ctypes.POINTER(srsran_pdsch_cfg_t), ctypes.c_void_p * 2], ctypes.c_int),
                ("srsran_enb_dl_gen_signal", [R], None),
                ("srsran_enb_dl_get_maximum_signal_power_dBfs", [u32], ctypes.c_float)):
            f = getattr(L, name)
            f.argtypes, f.restype = args, res
        _bound = True
    return L


class EnbDl:
    def __init__(self, cell):
        self.q = srsran_enb_dl_gpu_t()
        assert lib().srsran_enb_dl_gpu_init(ctypes.byref(self.q), cell) == 0
        self._keep = []

    def tx_batch(self, sfs, d_samples, scale=0.0, stream=None, pdsch_scaling=0.0):
        """sfs: list of (tti, cfi, srsran_pdsch_cfg_t or None, [device payload pointers][, ctrl]) with ctrl =
        (put_base, [srsran_dci_msg_t, ...]) or None; pdsch_scaling: every subframe's precoder scaling (<= 0: 1)"""
        arr = (srsran_enb_dl_gpu_sf_t * len(sfs))()
        self._keep = []
        for i, sf in enumerate(sfs):
            tti, cfi, cfg, ptrs = sf[:4]
            ctrl = sf[4] if len(sf) > 4 else None
            arr[i].tti, arr[i].cfi = tti, cfi
            arr[i].pdsch_scaling = pdsch_scaling
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


class EnbDlRef:
    """The reference-named per-subframe object (srsran_enb_dl_init / set_cell / put_base / put_pdcch_dl /
    put_pdsch / gen_signal): out_buffer = nof_ports host arrays of SRSRAN_SF_LEN samples (complex64)."""

    def __init__(self, cell, out_buffers, max_prb=None):
        import numpy as np
        self.q = srsran_enb_dl_t()
        self.out = out_buffers
        ptrs = (ctypes.c_void_p * 4)(*([b.ctypes.data for b in out_buffers] + [None] * (4 - len(out_buffers))))
        assert lib().srsran_enb_dl_init(ctypes.byref(self.q), ptrs, max_prb or cell.nof_prb) == 0
        assert lib().srsran_enb_dl_set_cell(ctypes.byref(self.q), cell) == 0
        self.np = np

    def put_base(self, sf):
        lib().srsran_enb_dl_put_base(ctypes.byref(self.q), ctypes.byref(sf))

    def put_pdcch_dl(self, dci_cfg, dci):
        return lib().srsran_enb_dl_put_pdcch_dl(ctypes.byref(self.q), ctypes.byref(dci_cfg), ctypes.byref(dci))

    def put_pdsch(self, cfg, payloads):
        self._pl = [self.np.ascontiguousarray(p) for p in payloads]
        ptrs = (ctypes.c_void_p * 2)(*([p.ctypes.data for p in self._pl] + [None] * (2 - len(self._pl))))
        return lib().srsran_enb_dl_put_pdsch(ctypes.byref(self.q), ctypes.byref(cfg), ptrs)

    def gen_signal(self):
        lib().srsran_enb_dl_gen_signal(ctypes.byref(self.q))

    def sf_symbols(self, port, nre):
        return self.np.ctypeslib.as_array(ctypes.cast(self.q.sf_symbols[port], ctypes.POINTER(ctypes.c_float)),
                                          (2 * nre,)).view(self.np.complex64).copy()

    def is_common(self, L, ncce):
        loc = srsran_dci_location_t()
        loc.L, loc.ncce = L, ncce
        return bool(lib().srsran_enb_dl_location_is_common_ncce(ctypes.byref(self.q), ctypes.byref(loc)))

    def free(self):
        if self.q.gpu:
            lib().srsran_enb_dl_free(ctypes.byref(self.q))
