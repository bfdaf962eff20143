"""Python mirror of the DL receive C API (include/srsran_ue_dl.h): cell / subframe types, CRS
channel estimation, OFDM, PDSCH and UE DL (host-synchronous and batched).  No CPU fallback."""
import ctypes

import numpy as np

from .sch import srsran_pdsch_cfg_t, srsran_sch_t, srsran_softbuffer_rx_t
from .tdec import load_library

u32 = ctypes.c_uint32
MAX_PORTS = 4


class srsran_cell_t(ctypes.Structure):
    _fields_ = [("nof_prb", u32), ("nof_ports", u32), ("id", u32), ("cp", ctypes.c_int), ("phich_length", ctypes.c_int),
                ("phich_resources", ctypes.c_int), ("frame_type", ctypes.c_int)]


class srsran_tdd_config_t(ctypes.Structure):
    _fields_ = [("sf_config", u32), ("ss_config", u32), ("configured", ctypes.c_bool)]


class srsran_dl_sf_cfg_t(ctypes.Structure):
    _fields_ = [("tdd_config", srsran_tdd_config_t), ("tti", u32), ("cfi", u32), ("sf_type", ctypes.c_int),
                ("non_mbsfn_region", u32)]


class srsran_chest_dl_cfg_t(ctypes.Structure):
    _fields_ = [("estimator_alg", ctypes.c_int), ("noise_alg", ctypes.c_int), ("filter_type", ctypes.c_int),
                ("filter_coef", ctypes.c_float * 2), ("mbsfn_area_id", ctypes.c_uint16), ("rsrp_neighbour", ctypes.c_bool),
                ("cfo_estimate_enable", ctypes.c_bool), ("cfo_estimate_sf_mask", u32), ("sync_error_enable", ctypes.c_bool)]


F44 = (ctypes.c_float * MAX_PORTS) * MAX_PORTS


class srsran_chest_dl_res_t(ctypes.Structure):
    _fields_ = [("ce", (ctypes.c_void_p * MAX_PORTS) * MAX_PORTS), ("nof_re", u32), ("noise_estimate", ctypes.c_float),
                ("noise_estimate_dbm", ctypes.c_float), ("snr_db", ctypes.c_float), ("snr_ant_port_db", F44),
                ("rsrp", ctypes.c_float), ("rsrp_dbm", ctypes.c_float), ("rsrp_neigh", ctypes.c_float),
                ("rsrp_port_dbm", ctypes.c_float * MAX_PORTS), ("rsrp_ant_port_dbm", F44), ("rsrq", ctypes.c_float),
                ("rsrq_db", ctypes.c_float), ("rsrq_ant_port_db", F44), ("rssi_dbm", ctypes.c_float),
                ("cfo", ctypes.c_float), ("sync_error", ctypes.c_float)]


class srsran_chest_dl_t(ctypes.Structure):
    _fields_ = [("cell", srsran_cell_t), ("nof_rx_antennas", u32), ("rssi", F44), ("rsrp", F44),
                ("noise_estimate", F44), ("cfo", ctypes.c_float), ("gpu", ctypes.c_void_p)]


class srsran_ofdm_cfg_t(ctypes.Structure):
    _fields_ = [("nof_prb", u32), ("in_buffer", ctypes.c_void_p), ("out_buffer", ctypes.c_void_p), ("cp", ctypes.c_int),
                ("sf_type", ctypes.c_int), ("normalize", ctypes.c_bool), ("freq_shift_f", ctypes.c_float),
                ("rx_window_offset", ctypes.c_float), ("symbol_sz", u32), ("keep_dc", ctypes.c_bool),
                ("phase_compensation_hz", ctypes.c_double)]


class srsran_ofdm_t(ctypes.Structure):
    _fields_ = [("cfg", srsran_ofdm_cfg_t), ("max_prb", u32), ("nof_symbols", u32), ("nof_re", u32), ("slot_sz", u32),
                ("sf_sz", u32), ("gpu", ctypes.c_void_p)]


class srsran_cfo_t(ctypes.Structure):
    _fields_ = [("last_freq", ctypes.c_float), ("tol", ctypes.c_float), ("nsamples", u32), ("max_samples", u32),
                ("gpu", ctypes.c_void_p)]


class srsran_pdsch_t(ctypes.Structure):
    _fields_ = [("cell", srsran_cell_t), ("nof_rx_antennas", u32), ("max_re", u32), ("is_ue", ctypes.c_bool),
                ("llr_is_8bit", ctypes.c_bool), ("avg_evm", ctypes.c_float), ("dl_sch", srsran_sch_t),
                ("coworker_ptr", ctypes.c_void_p), ("gpu", ctypes.c_void_p)]


class srsran_pdsch_res_t(ctypes.Structure):
    _fields_ = [("payload", ctypes.c_void_p), ("crc", ctypes.c_bool), ("avg_iterations_block", ctypes.c_float),
                ("evm", ctypes.c_float)]


class srsran_pdsch_gpu_sf_t(ctypes.Structure):
    _fields_ = [("cfg", ctypes.POINTER(srsran_pdsch_cfg_t)), ("tti", u32), ("cfi", u32), ("d_grid", ctypes.c_void_p),
                ("d_ce", ctypes.c_void_p), ("ce_full", u32), ("d_noise", ctypes.c_void_p), ("noise", ctypes.c_float),
                ("d_payload", ctypes.c_void_p * 2), ("new_data", u32 * 2)]


class srsran_dci_cfg_t(ctypes.Structure):
    _fields_ = [("multiple_csi_request_enabled", ctypes.c_bool), ("cif_enabled", ctypes.c_bool),
                ("cif_present", ctypes.c_bool), ("srs_request_enabled", ctypes.c_bool),
                ("ra_format_enabled", ctypes.c_bool), ("is_not_ue_ss", ctypes.c_bool)]


class srsran_dl_cfg_t(ctypes.Structure):
    _fields_ = [("pdsch", srsran_pdsch_cfg_t), ("dci", srsran_dci_cfg_t), ("tm", ctypes.c_int),
                ("dci_common_ss", ctypes.c_bool)]


class srsran_ue_dl_cfg_t(ctypes.Structure):
    _fields_ = [("cfg", srsran_dl_cfg_t), ("chest_cfg", srsran_chest_dl_cfg_t), ("last_ri", u32),
                ("snr_to_cqi_offset", ctypes.c_float)]


class srsran_ue_dl_t(ctypes.Structure):
    _fields_ = [("cell", srsran_cell_t), ("nof_rx_antennas", u32), ("current_mbsfn_area_id", ctypes.c_uint16),
                ("pdsch", srsran_pdsch_t), ("chest", srsran_chest_dl_t), ("chest_res", srsran_chest_dl_res_t),
                ("fft", srsran_ofdm_t * MAX_PORTS), ("fft_mbsfn", srsran_ofdm_t), ("sf_symbols", ctypes.c_void_p * MAX_PORTS),
                ("gpu", ctypes.c_void_p)]


class srsran_ue_dl_gpu_sf_t(ctypes.Structure):
    _fields_ = [("tti", u32), ("cfi", u32), ("pdsch_cfg", ctypes.POINTER(srsran_pdsch_cfg_t)),
                ("d_payload", ctypes.c_void_p * 2), ("new_data", u32 * 2), ("tdd_config", srsran_tdd_config_t)]


_bound = False


class WorkerStream:
    """srsran_gpu_worker_stream_create: a PHY worker's stream on a hardware queue of its own, as a torch stream
    (`.stream`, an ExternalStream over it); free() releases it"""

    def __init__(self, device):
        import torch
        p = ctypes.c_void_p()
        if lib().srsran_gpu_worker_stream_create(ctypes.byref(p)) != 0 or not p.value:
            raise RuntimeError("srsran_gpu_worker_stream_create failed")
        self.ptr = p.value
        self.stream = torch.cuda.ExternalStream(self.ptr, device=device)

    @property
    def cuda_stream(self):
        return self.ptr

    def free(self):
        if self.ptr:
            lib().srsran_gpu_worker_stream_free(self.ptr)
            self.ptr = None


def lib():
    global _bound
    L = load_library()
    if not _bound:
        CH = ctypes.POINTER(srsran_chest_dl_t)
        RES = ctypes.POINTER(srsran_chest_dl_res_t)
        P = ctypes.c_void_p
        PD = ctypes.POINTER(srsran_pdsch_t)
        UE = ctypes.POINTER(srsran_ue_dl_t)
        sig = {
            "srsran_symbol_sz": ([u32], ctypes.c_int),
            "srsran_symbol_sz_power2": ([u32], ctypes.c_int),
            "srsran_use_standard_symbol_size": ([ctypes.c_bool], None),
            "srsran_symbol_size_is_standard": ([], ctypes.c_bool),
            "srsran_sampling_freq_hz": ([u32], ctypes.c_int),
            "srsran_nof_prb": ([u32], ctypes.c_int),
            "srsran_symbol_sz_isvalid": ([u32], ctypes.c_bool),
            "srsran_chest_dl_init": ([CH, u32, u32], ctypes.c_int),
            "srsran_chest_dl_free": ([CH], None),
            "srsran_chest_dl_set_cell": ([CH, srsran_cell_t], ctypes.c_int),
            "srsran_chest_dl_res_init": ([RES, u32], ctypes.c_int),
            "srsran_chest_dl_res_free": ([RES], None),
            "srsran_chest_dl_estimate": ([CH, ctypes.POINTER(srsran_dl_sf_cfg_t), P, RES], ctypes.c_int),
            "srsran_chest_dl_estimate_cfg": ([CH, ctypes.POINTER(srsran_dl_sf_cfg_t),
                                              ctypes.POINTER(srsran_chest_dl_cfg_t), P, RES], ctypes.c_int),
            "srsran_chest_dl_gpu_estimate": ([CH, u32, P, P, ctypes.c_int, P, P], ctypes.c_int),
            "srsran_ofdm_rx_init_cfg": ([ctypes.POINTER(srsran_ofdm_t), ctypes.POINTER(srsran_ofdm_cfg_t)], ctypes.c_int),
            "srsran_ofdm_rx_set_prb": ([ctypes.POINTER(srsran_ofdm_t), ctypes.c_int, u32], ctypes.c_int),
            "srsran_ofdm_rx_free": ([ctypes.POINTER(srsran_ofdm_t)], None),
            "srsran_ofdm_rx_sf": ([ctypes.POINTER(srsran_ofdm_t)], None),
            "srsran_ofdm_rx_sf_ng": ([ctypes.POINTER(srsran_ofdm_t), P, P], None),
            "srsran_ofdm_set_normalize": ([ctypes.POINTER(srsran_ofdm_t), ctypes.c_bool], None),
            "srsran_ofdm_rx_init_mbsfn": ([ctypes.POINTER(srsran_ofdm_t), ctypes.c_int, P, P, u32], ctypes.c_int),
            "srsran_ofdm_set_non_mbsfn_region": ([ctypes.POINTER(srsran_ofdm_t), ctypes.c_uint8], None),
            "srsran_chest_dl_set_mbsfn_area_id": ([CH, ctypes.c_uint16], ctypes.c_int),
            "srsran_ue_dl_set_non_mbsfn_region": ([UE, ctypes.c_uint8], None),
            "srsran_ofdm_rx_gpu": ([ctypes.POINTER(srsran_ofdm_t), P, P, u32, u32, ctypes.c_float, P], ctypes.c_int),
            "srsran_ofdm_rx_gpu_sc16": ([ctypes.POINTER(srsran_ofdm_t), P, ctypes.c_float, P, u32, u32, ctypes.c_float,
                                         P], ctypes.c_int),
            "srsran_ue_dl_gpu_decode_batch_sc16": ([UE, ctypes.POINTER(srsran_ue_dl_cfg_t), u32,
                                                    ctypes.POINTER(srsran_ue_dl_gpu_sf_t), P, ctypes.c_float,
                                                    ctypes.c_float, P, P, P], ctypes.c_int),
            "srsran_gpu_worker_stream_create": ([ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
            "srsran_gpu_worker_stream_free": ([P], None),
            "srsran_ofdm_tx_init_cfg": ([ctypes.POINTER(srsran_ofdm_t), ctypes.POINTER(srsran_ofdm_cfg_t)], ctypes.c_int),
            "srsran_ofdm_tx_sf": ([ctypes.POINTER(srsran_ofdm_t)], None),
            "srsran_ofdm_set_freq_shift": ([ctypes.POINTER(srsran_ofdm_t), ctypes.c_float], ctypes.c_int),
            "srsran_ofdm_set_phase_compensation": ([ctypes.POINTER(srsran_ofdm_t), ctypes.c_double], ctypes.c_int),
            "srsran_cfo_init": ([ctypes.POINTER(srsran_cfo_t), u32], ctypes.c_int),
            "srsran_cfo_free": ([ctypes.POINTER(srsran_cfo_t)], None),
            "srsran_cfo_correct": ([ctypes.POINTER(srsran_cfo_t), P, P, ctypes.c_float], None),
            "srsran_chest_dl_gpu_estimate_batch": ([CH, P, u32, P, ctypes.c_size_t, P, ctypes.c_size_t, P, P],
                                                   ctypes.c_int),
            "srsran_pdsch_init_ue": ([PD, u32, u32], ctypes.c_int),
            "srsran_pdsch_init_enb": ([PD, u32], ctypes.c_int),
            "srsran_pdsch_encode": ([PD, ctypes.POINTER(srsran_dl_sf_cfg_t), ctypes.POINTER(srsran_pdsch_cfg_t),
                                     ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
            "srsran_pdsch_free": ([PD], None),
            "srsran_pdsch_set_cell": ([PD, srsran_cell_t], ctypes.c_int),
            "srsran_pdsch_enable_coworker": ([PD], ctypes.c_int),
            "srsran_pdsch_decode": ([PD, ctypes.POINTER(srsran_dl_sf_cfg_t), ctypes.POINTER(srsran_pdsch_cfg_t), RES,
                                     P, ctypes.POINTER(srsran_pdsch_res_t)], ctypes.c_int),
            "srsran_pdsch_gpu_decode_batch": ([PD, u32, ctypes.POINTER(srsran_pdsch_gpu_sf_t), P, P, P], ctypes.c_int),
            "srsran_pdsch_gpu_last_llr": ([PD, u32, u32, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(u32)],
                                          ctypes.c_int),
            "srsran_pdsch_gpu_last_evm": ([PD, u32, u32, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
            "srsran_ue_dl_init": ([UE, P, u32, u32], ctypes.c_int),
            "srsran_ue_dl_free": ([UE], None),
            "srsran_ue_dl_set_cell": ([UE, srsran_cell_t], ctypes.c_int),
            "srsran_ue_dl_decode_fft_estimate": ([UE, ctypes.POINTER(srsran_dl_sf_cfg_t),
                                                  ctypes.POINTER(srsran_ue_dl_cfg_t)], ctypes.c_int),
            "srsran_ue_dl_decode_fft_estimate_noguru": ([UE, ctypes.POINTER(srsran_dl_sf_cfg_t),
                                                         ctypes.POINTER(srsran_ue_dl_cfg_t), P], ctypes.c_int),
            "srsran_ue_dl_decode_pdsch": ([UE, ctypes.POINTER(srsran_dl_sf_cfg_t), ctypes.POINTER(srsran_pdsch_cfg_t),
                                           ctypes.POINTER(srsran_pdsch_res_t)], ctypes.c_int),
            "srsran_ue_dl_gpu_decode_batch": ([UE, ctypes.POINTER(srsran_ue_dl_cfg_t), u32,
                                               ctypes.POINTER(srsran_ue_dl_gpu_sf_t), P, ctypes.c_float, P, P, P],
                                              ctypes.c_int),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _bound = True
    return L


def use_standard_symbol_size(enabled):
    """srsran_use_standard_symbol_size: the library defaults to the reference's non-standard rates
    (100 PRB -> N = 1536); srsUE and the C3 workload (N = 2048) switch standard rates on."""
    lib().srsran_use_standard_symbol_size(bool(enabled))


def symbol_size_is_standard():
    return bool(lib().srsran_symbol_size_is_standard())


def cell(nof_prb=100, nof_ports=2, cell_id=1, phich_res=2, cp=0, tdd=False, phich_len=0):
    """FDD (tdd=True: TDD), normal CP (cp=1: extended), normal PHICH duration (phich_len=1: extended), Ng = 1
    (phich_res 2) as the reference's test cells"""
    c = srsran_cell_t()
    c.nof_prb, c.nof_ports, c.id, c.cp = nof_prb, nof_ports, cell_id, cp
    c.phich_resources = phich_res
    c.phich_length = phich_len
    c.frame_type = 1 if tdd else 0
    return c


def sf_cfg(tti, cfi=0, tdd=None, mbsfn=False):
    """srsran_dl_sf_cfg_t; tdd = (uplink-downlink configuration, special-subframe configuration) or None; mbsfn:
    sf_type = SRSRAN_SF_MBSFN"""
    sf = srsran_dl_sf_cfg_t()
    sf.tti, sf.cfi = tti, cfi
    sf.sf_type = 1 if mbsfn else 0
    if tdd is not None:
        sf.tdd_config.sf_config, sf.tdd_config.ss_config, sf.tdd_config.configured = tdd[0], tdd[1], True
    return sf


def srsue_chest_cfg():
    """srsUE defaults (srsue/src/phy/phy_common.cc:83-107 + main.cc option defaults)."""
    c = srsran_chest_dl_cfg_t()
    c.estimator_alg = 0  # AVERAGE
    c.noise_alg = 0      # REFS
    c.filter_type = 0    # GAUSS
    c.filter_coef[0], c.filter_coef[1] = 4, 1.0
    c.cfo_estimate_enable = True
    c.cfo_estimate_sf_mask = 1023
    return c


def chest_cfg(estimator=0, noise_alg=0, filter_order=4, filter_std=1.0, sync_error=False, filter_type=0,
              mbsfn_area_id=0):
    """srsran_chest_dl_cfg_t with srsUE's ue.conf knobs (phy_common.cc:83-108): interpolate_subframe_enabled
    (estimator 1 INTERPOLATE), snr_estim_alg (noise_alg 0 refs / 1 pss / 2 empty), estimator_fil_order /
    _stddev (order 0 = estimator_fil_auto), correct_sync_error; filter_type 0 GAUSS / 1 TRIANGLE (w = filter_order)
    / 2 NONE"""
    c = srsue_chest_cfg()
    c.estimator_alg, c.noise_alg = estimator, noise_alg
    c.filter_type = filter_type
    c.filter_coef[0], c.filter_coef[1] = filter_order, filter_std
    c.sync_error_enable = bool(sync_error)
    c.mbsfn_area_id = mbsfn_area_id
    return c


def mbsfn_chest_cfg(area=1):
    """srsUE's estimator configuration for MBSFN subframes (cc_worker.cc:96-100, 336-338): TRIANGLE 0.1,
    INTERPOLATE, PSS noise"""
    return chest_cfg(estimator=1, noise_alg=1, filter_order=0.1, filter_std=0.0, filter_type=1, mbsfn_area_id=area)


class OfdmRx:
    """srsran_ofdm_t receiver (srsran_ue_dl configuration).  mbsfn: an MBSFN object (srsran_ofdm_rx_init_mbsfn,
    extended CP) with its own in / out buffers, which it transforms whatever srsran_ofdm_rx_sf_ng is given
    (ofdm.c:576-578); non_mbsfn_region: srsran_ofdm_set_non_mbsfn_region."""

    def __init__(self, nof_prb, normalize=False, cp=0, mbsfn=False, non_mbsfn_region=2, keep_dc=False,
                 freq_shift_f=0.0, rx_window_offset=0.0, phase_compensation_hz=0.0, tx=False):
        self.q = srsran_ofdm_t()
        self.mbsfn = mbsfn
        if mbsfn:
            n = symbol_sz_for(nof_prb)
            self.inb = np.zeros(15 * n, np.complex64)
            self.outb = np.zeros(12 * 12 * nof_prb, np.complex64)
            if lib().srsran_ofdm_rx_init_mbsfn(ctypes.byref(self.q), 1, self.inb.ctypes.data, self.outb.ctypes.data,
                                               nof_prb):
                raise RuntimeError("srsran_ofdm_rx_init_mbsfn failed")
            lib().srsran_ofdm_set_non_mbsfn_region(ctypes.byref(self.q), non_mbsfn_region)
            return
        self.cfg = srsran_ofdm_cfg_t()
        self.cfg.nof_prb = nof_prb
        self.cfg.normalize = normalize
        self.cfg.cp = cp
        self.cfg.keep_dc = keep_dc
        self.cfg.freq_shift_f = freq_shift_f
        self.cfg.rx_window_offset = rx_window_offset
        self.cfg.phase_compensation_hz = phase_compensation_hz
        init = lib().srsran_ofdm_tx_init_cfg if tx else lib().srsran_ofdm_rx_init_cfg
        self.ret = init(ctypes.byref(self.q), ctypes.byref(self.cfg))
        if self.ret:
            raise RuntimeError("srsran_ofdm_%s_init_cfg failed" % ("tx" if tx else "rx"))

    def tx(self, grid):
        """srsran_ofdm_tx_sf through the configured buffers (an object made with tx=True)"""
        g = np.ascontiguousarray(grid, np.complex64)
        assert g.size == 2 * self.q.nof_symbols * self.q.nof_re
        out = np.zeros(self.q.sf_sz, np.complex64)
        self.q.cfg.in_buffer, self.q.cfg.out_buffer = g.ctypes.data, out.ctypes.data
        lib().srsran_ofdm_tx_sf(ctypes.byref(self.q))
        self.q.cfg.in_buffer = self.q.cfg.out_buffer = None
        return out

    def rx_inplace(self, x):
        """srsran_ofdm_rx_sf_ng on the caller's array (the frequency shift multiplies it in place, ofdm.c:569-571)"""
        assert x.dtype == np.complex64 and x.flags.c_contiguous and x.size == self.q.sf_sz
        out = np.zeros(2 * self.q.nof_symbols * self.q.nof_re, np.complex64)
        lib().srsran_ofdm_rx_sf_ng(ctypes.byref(self.q), x.ctypes.data, out.ctypes.data)
        return out

    @property
    def symbol_sz(self):
        return self.q.cfg.symbol_sz

    def rx(self, samples):
        x = np.ascontiguousarray(samples, np.complex64)
        assert x.size == self.q.sf_sz
        out = np.zeros(2 * self.q.nof_symbols * self.q.nof_re, np.complex64)
        if self.mbsfn:  # the configured buffers (the _ng arguments are ignored for MBSFN objects)
            self.inb[:] = x
            lib().srsran_ofdm_rx_sf_ng(ctypes.byref(self.q), out.ctypes.data, out.ctypes.data)
            return self.outb.copy()
        lib().srsran_ofdm_rx_sf_ng(ctypes.byref(self.q), x.ctypes.data, out.ctypes.data)
        return out

    def free(self):
        if self.q.gpu:
            lib().srsran_ofdm_rx_free(ctypes.byref(self.q))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def symbol_sz_for(nof_prb):
    return lib().srsran_symbol_sz(nof_prb)


def cfo_correct(x, freq):
    h = srsran_cfo_t()
    x = np.ascontiguousarray(x, np.complex64)
    if lib().srsran_cfo_init(ctypes.byref(h), x.size):
        raise RuntimeError("srsran_cfo_init failed")
    out = np.zeros_like(x)
    lib().srsran_cfo_correct(ctypes.byref(h), x.ctypes.data, out.ctypes.data, freq)
    lib().srsran_cfo_free(ctypes.byref(h))
    return out


class ChestDl:
    def __init__(self, cell_, nof_rx):
        self.q = srsran_chest_dl_t()
        if lib().srsran_chest_dl_init(ctypes.byref(self.q), cell_.nof_prb, nof_rx):
            raise RuntimeError("srsran_chest_dl_init failed (no HIP device?)")
        if lib().srsran_chest_dl_set_cell(ctypes.byref(self.q), cell_):
            raise RuntimeError("srsran_chest_dl_set_cell failed")
        self.res = srsran_chest_dl_res_t()
        lib().srsran_chest_dl_res_init(ctypes.byref(self.res), cell_.nof_prb)
        self.cell = cell_
        self.nrx = nof_rx

    def set_mbsfn_area_id(self, area):
        return lib().srsran_chest_dl_set_mbsfn_area_id(ctypes.byref(self.q), area)

    def estimate(self, grids, tti, cfg=None, tdd=None, mbsfn=False):
        """grids: (nrx, 14*12*nof_prb) complex64 -> (ce[port][rx] arrays, res); tdd = (sf_config, ss_config);
        mbsfn: an MBSFN subframe (rows 12 / 13 of the returned estimate are those of the previous call)"""
        grids = [np.ascontiguousarray(g, np.complex64) for g in grids]
        ptrs = (ctypes.c_void_p * MAX_PORTS)(*[g.ctypes.data for g in grids] + [None] * (MAX_PORTS - len(grids)))
        sf = sf_cfg(tti, 0, tdd, mbsfn)
        if cfg is None:
            rc = lib().srsran_chest_dl_estimate(ctypes.byref(self.q), ctypes.byref(sf), ctypes.addressof(ptrs),
                                                ctypes.byref(self.res))
        else:
            rc = lib().srsran_chest_dl_estimate_cfg(ctypes.byref(self.q), ctypes.byref(sf), ctypes.byref(cfg),
                                                    ctypes.addressof(ptrs), ctypes.byref(self.res))
        if rc:
            raise RuntimeError(f"srsran_chest_dl_estimate failed ({rc})")
        n = (12 if self.cell.cp else 14) * 12 * self.cell.nof_prb
        ce = np.zeros((self.cell.nof_ports, self.nrx, n), np.complex64)
        for p in range(self.cell.nof_ports):
            for r in range(self.nrx):
                ctypes.memmove(ce[p, r].ctypes.data, self.res.ce[p][r], n * 8)
        return ce, self.res

    def free(self):
        if self.q.gpu:
            lib().srsran_chest_dl_res_free(ctypes.byref(self.res))
            lib().srsran_chest_dl_free(ctypes.byref(self.q))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# ---------------- PDSCH / UE DL ----------------
SCHEME = {"port0": 0, "diversity": 1, "sm": 2, "cdd": 3}
MOD_FROM_QM = {1: 0, 2: 1, 4: 2, 6: 3, 8: 4}


def pdsch_cfg(nof_prb, nof_re, tbs, Qm, rv=(0, 0), scheme="cdd", pmi=0, rnti=0x1234, max_iterations=8,
              csi_enable=True, power_scale=False, p_a=0.0, p_b=0, softbuffers=(), zf=False, cp=0, nof_ports=2,
              meas_evm=False, nsl=None):
    """srsran_pdsch_cfg_t for a full-bandwidth grant of len(tbs) codewords on as many layers
    (srsUE defaults: csi_enable, 8 half-iterations, MMSE, no power scaling); cp=1: extended CP;
    transmit diversity runs on nof_ports layers (2 or 4); nsl: the grant's symbols per slot (a TDD special
    subframe's DwPTS, srsran_ra_dl_compute_nof_re)."""
    c = srsran_pdsch_cfg_t()
    g = c.grant
    g.tx_scheme = SCHEME[scheme]
    g.pmi = pmi
    for s in range(2):
        for n in range(nof_prb):
            g.prb_idx[s][n] = True
    g.nof_prb = nof_prb
    g.nof_re = nof_re
    g.nof_symb_slot[0] = g.nof_symb_slot[1] = 6 if cp else 7
    if nsl is not None:
        g.nof_symb_slot[0], g.nof_symb_slot[1] = nsl
    g.nof_tb = len(tbs)
    g.nof_layers = nof_ports if scheme == "diversity" else len(tbs)
    for i, t in enumerate(tbs):
        tb = g.tb[i]
        tb.mod = MOD_FROM_QM[Qm[i]]
        tb.tbs = t
        tb.rv = rv[i]
        tb.nof_bits = nof_re * Qm[i]
        tb.cw_idx = i
        tb.enabled = True
    c.rnti = rnti
    c.max_nof_iterations = max_iterations
    c.decoder_type = 0 if zf else 1
    c.p_a, c.p_b = p_a, p_b
    c.power_scale, c.csi_enable = power_scale, csi_enable
    c.meas_evm_en = bool(meas_evm)
    for i, sb in enumerate(softbuffers):
        c.softbuffers.rx[i] = ctypes.pointer(sb.s)
    return c


class Pdsch:
    """srsran_pdsch_t (UE side)."""

    def __init__(self, cell_, nof_rx, enb=False):
        self.q = srsran_pdsch_t()
        if enb:
            if lib().srsran_pdsch_init_enb(ctypes.byref(self.q), cell_.nof_prb):
                raise RuntimeError("srsran_pdsch_init_enb failed (no HIP device?)")
        elif lib().srsran_pdsch_init_ue(ctypes.byref(self.q), cell_.nof_prb, nof_rx):
            raise RuntimeError("srsran_pdsch_init_ue failed (no HIP device?)")
        if lib().srsran_pdsch_set_cell(ctypes.byref(self.q), cell_):
            raise RuntimeError("srsran_pdsch_set_cell failed")
        self.cell = cell_
        self.nrx = nof_rx

    def set_llr8(self, on=True):
        """the 8-bit LLR chain: pdsch.llr_is_8bit and pdsch.dl_sch.llr_is_8bit, as srsUE's pdsch_8bit_decoder sets
        them (cc_worker.cc:108-110)"""
        self.q.llr_is_8bit = bool(on)
        self.q.dl_sch.llr_is_8bit = bool(on)

    def encode(self, cfg, tti, cfi, payloads, grids):
        """srsran_pdsch_encode into (a copy of) the ports' host grids -> (ret, grids)"""
        g = [np.array(x, np.complex64, copy=True) for x in grids]
        gp = (ctypes.c_void_p * MAX_PORTS)(*[x.ctypes.data for x in g] + [None] * (MAX_PORTS - len(g)))
        pl = [np.ascontiguousarray(p, np.uint8) for p in payloads]
        dp = (ctypes.c_void_p * 2)(*[p.ctypes.data for p in pl] + [None] * (2 - len(pl)))
        sf = srsran_dl_sf_cfg_t()
        sf.tti, sf.cfi = tti, cfi
        ret = lib().srsran_pdsch_encode(ctypes.byref(self.q), ctypes.byref(sf), ctypes.byref(cfg), ctypes.addressof(dp),
                                        ctypes.addressof(gp))
        return ret, g

    def decode(self, cfg, tti, cfi, grids, ce, noise, acked=(False, False)):
        """srsran_pdsch_decode on host grids (nrx, n) and full estimates (nports, nrx, n).
        Returns (ret, [(crc, payload bytes, avg_iterations_block)])."""
        grids = [np.ascontiguousarray(g, np.complex64) for g in grids]
        ce = np.ascontiguousarray(ce, np.complex64)
        sf = srsran_dl_sf_cfg_t()
        sf.tti, sf.cfi = tti, cfi
        res = srsran_chest_dl_res_t()
        for p in range(ce.shape[0]):
            for r in range(ce.shape[1]):
                res.ce[p][r] = ce[p, r].ctypes.data
        res.noise_estimate = noise
        ptrs = (ctypes.c_void_p * MAX_PORTS)(*[g.ctypes.data for g in grids] + [None] * (MAX_PORTS - len(grids)))
        ntb = cfg.grant.nof_tb
        pls = [np.zeros(cfg.grant.tb[i].tbs // 8 + 64, np.uint8) for i in range(ntb)]
        data = (srsran_pdsch_res_t * 2)()
        for i in range(ntb):
            data[i].payload = pls[i].ctypes.data
            data[i].crc = bool(acked[i])
        ret = lib().srsran_pdsch_decode(ctypes.byref(self.q), ctypes.byref(sf), ctypes.byref(cfg), ctypes.byref(res),
                                        ctypes.addressof(ptrs), data)
        self.last_evm = [float(data[i].evm) for i in range(ntb)]  # NAN unless cfg.meas_evm_en
        return ret, [(data[i].crc, pls[i], data[i].avg_iterations_block) for i in range(ntb)]

    def free(self):
        if self.q.gpu:
            lib().srsran_pdsch_free(ctypes.byref(self.q))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class UeDl:
    """srsran_ue_dl_t: host-synchronous decode_fft_estimate / decode_pdsch and the device batch."""

    def __init__(self, cell_, nof_rx, tdd=None, inputs=False):
        """tdd = (sf_config, ss_config): the TDD configuration every call's srsran_dl_sf_cfg_t carries; inputs: give
        srsran_ue_dl_init input buffers (the guru path, fft_estimate_guru; MBSFN subframes need them)"""
        self.tdd = tdd
        self.q = srsran_ue_dl_t()
        self.inb = None
        ptrs = None
        if inputs:
            self.inb = [np.zeros(15 * symbol_sz_for(cell_.nof_prb), np.complex64) for _ in range(nof_rx)]
            ptrs = (ctypes.c_void_p * MAX_PORTS)(*[b.ctypes.data for b in self.inb] + [None] * (MAX_PORTS - nof_rx))
        if lib().srsran_ue_dl_init(ctypes.byref(self.q), ptrs, cell_.nof_prb, nof_rx):
            raise RuntimeError("srsran_ue_dl_init failed (no HIP device?)")
        if lib().srsran_ue_dl_set_cell(ctypes.byref(self.q), cell_):
            raise RuntimeError("srsran_ue_dl_set_cell failed")
        self.cell = cell_
        self.nrx = nof_rx
        self.cfg = srsran_ue_dl_cfg_t()
        self.cfg.chest_cfg = srsue_chest_cfg()

    def set_llr8(self, on=True):
        """srsUE's pdsch_8bit_decoder (cc_worker.cc:108-110): ue_dl.pdsch.llr_is_8bit and its dl_sch's"""
        self.q.pdsch.llr_is_8bit = bool(on)
        self.q.pdsch.dl_sch.llr_is_8bit = bool(on)

    def fft_estimate(self, samples, tti, cfi):
        x = [np.ascontiguousarray(v, np.complex64) for v in samples]
        ptrs = (ctypes.c_void_p * MAX_PORTS)(*[v.ctypes.data for v in x] + [None] * (MAX_PORTS - len(x)))
        sf = sf_cfg(tti, cfi, self.tdd)
        ret = lib().srsran_ue_dl_decode_fft_estimate_noguru(ctypes.byref(self.q), ctypes.byref(sf),
                                                            ctypes.byref(self.cfg), ctypes.addressof(ptrs))
        self.last_cfi = sf.cfi  # decoded from the PCFICH (1/2-port cells), else the caller's
        return ret

    def fft_estimate_guru(self, samples, tti, cfi, mbsfn=False):
        """srsran_ue_dl_decode_fft_estimate on the buffers given to srsran_ue_dl_init (inputs=True): samples copied
        into them first; mbsfn: an MBSFN subframe (self.cfg.chest_cfg should then be mbsfn_chest_cfg)"""
        for b, v in zip(self.inb, samples):
            b[:] = np.asarray(v, np.complex64)
        sf = sf_cfg(tti, cfi, self.tdd, mbsfn)
        ret = lib().srsran_ue_dl_decode_fft_estimate(ctypes.byref(self.q), ctypes.byref(sf), ctypes.byref(self.cfg))
        self.last_cfi = sf.cfi
        return ret

    def set_non_mbsfn_region(self, n):
        lib().srsran_ue_dl_set_non_mbsfn_region(ctypes.byref(self.q), n)

    def chest_res_ce(self):
        """the last estimate (chest_res.ce) as (nports, nrx, 14 * 12 * nof_prb)"""
        n = (12 if self.cell.cp else 14) * 12 * self.cell.nof_prb
        ce = np.zeros((self.cell.nof_ports, self.nrx, n), np.complex64)
        for p in range(self.cell.nof_ports):
            for r in range(self.nrx):
                ctypes.memmove(ce[p, r].ctypes.data, self.q.chest_res.ce[p][r], n * 8)
        return ce

    def find_dl_dci(self, tti, cfi, rnti, tm=2, common_ss=True, mbsfn=False):
        """srsran_ue_dl_find_dl_dci (after fft_estimate) -> list of srsran_dci_dl_t"""
        from . import pdcch as PD
        PD.lib()
        sf = sf_cfg(tti, cfi, self.tdd, mbsfn)
        self.cfg.cfg.tm = tm
        self.cfg.cfg.dci_common_ss = common_ss
        out = (PD.srsran_dci_dl_t * 5)()
        n = lib().srsran_ue_dl_find_dl_dci(ctypes.byref(self.q), ctypes.byref(sf), ctypes.byref(self.cfg), rnti, out)
        if n < 0:
            raise RuntimeError("srsran_ue_dl_find_dl_dci failed")
        return [out[i] for i in range(n)]

    def find_ul_dci(self, tti, cfi, rnti):
        """srsran_ue_dl_find_ul_dci (the format 0 DCIs the last find_dl_dci found) -> [srsran_dci_ul_t]"""
        from . import pdcch as PD
        PD.lib()
        sf = sf_cfg(tti, cfi, self.tdd)
        out = (PD.srsran_dci_ul_t * 5)()
        n = lib().srsran_ue_dl_find_ul_dci(ctypes.byref(self.q), ctypes.byref(sf), ctypes.byref(self.cfg), rnti, out)
        if n < 0:
            raise RuntimeError("srsran_ue_dl_find_ul_dci failed")
        return [out[i] for i in range(n)]

    def set_mi(self, mi_idx=None):
        """srsran_ue_dl_set_mi_auto (None) / srsran_ue_dl_set_mi_manual(mi_idx)"""
        if mi_idx is None:
            lib().srsran_ue_dl_set_mi_auto(ctypes.byref(self.q))
        else:
            lib().srsran_ue_dl_set_mi_manual(ctypes.byref(self.q), mi_idx)

    def set_mbsfn_area_id(self, area):
        return lib().srsran_ue_dl_set_mbsfn_area_id(ctypes.byref(self.q), area)

    def dci_to_grant(self, dci, tti, cfi, tm=2):
        from . import pdcch as PD
        PD.lib()
        sf = sf_cfg(tti, cfi, self.tdd)
        self.cfg.cfg.tm = tm
        g = PD.srsran_pdsch_grant_t()
        r = lib().srsran_ue_dl_dci_to_pdsch_grant(ctypes.byref(self.q), ctypes.byref(sf), ctypes.byref(self.cfg),
                                                   ctypes.byref(dci), ctypes.byref(g))
        return r, g

    def grids(self):
        n = (12 if self.cell.cp else 14) * 12 * self.cell.nof_prb
        out = np.zeros((self.nrx, n), np.complex64)
        for r in range(self.nrx):
            ctypes.memmove(out[r].ctypes.data, self.q.sf_symbols[r], n * 8)
        return out

    def decode_pdsch(self, cfg, tti, cfi):
        sf = sf_cfg(tti, cfi, self.tdd)
        ntb = cfg.grant.nof_tb
        pls = [np.zeros(cfg.grant.tb[i].tbs // 8 + 64, np.uint8) for i in range(ntb)]
        data = (srsran_pdsch_res_t * 2)()
        for i in range(ntb):
            data[i].payload = pls[i].ctypes.data
        ret = lib().srsran_ue_dl_decode_pdsch(ctypes.byref(self.q), ctypes.byref(sf), ctypes.byref(cfg), data)
        return ret, [(data[i].crc, pls[i], data[i].avg_iterations_block) for i in range(ntb)]

    @staticmethod
    def batch_entries(sfs, tdd=None):
        """sfs: list of (tti, cfi, srsran_pdsch_cfg_t, [d_payload ptrs], [new_data]) -> ctypes array
        (keep the cfg objects alive while the array is used); tdd = (sf_config, ss_config) of a TDD cell."""
        arr = (srsran_ue_dl_gpu_sf_t * len(sfs))()
        for i, (tti, cfi, cfg, pls, nd) in enumerate(sfs):
            arr[i].tti, arr[i].cfi = tti, cfi
            if tdd is not None:
                t = arr[i].tdd_config
                t.sf_config, t.ss_config, t.configured = tdd[0], tdd[1], True
            arr[i].pdsch_cfg = ctypes.pointer(cfg)
            for t, p in enumerate(pls):
                arr[i].d_payload[t] = p
                arr[i].new_data[t] = nd[t]
        return arr

    def gpu_decode_batch(self, sfs, d_samples, d_result, d_avg, cfo=0.0, stream=None):
        """srsran_ue_dl_gpu_decode_batch; sfs: entry list (see batch_entries) or a prebuilt array."""
        arr = sfs if isinstance(sfs, ctypes.Array) else self.batch_entries(sfs, self.tdd)
        return lib().srsran_ue_dl_gpu_decode_batch(ctypes.byref(self.q), ctypes.byref(self.cfg), len(arr), arr,
                                                   d_samples, cfo, d_result, d_avg, stream)

    def gpu_decode_batch_sc16(self, sfs, d_samples, scale, d_result, d_avg, cfo=0.0, stream=None):
        """srsran_ue_dl_gpu_decode_batch_sc16: d_samples int16 I/Q, converted x scale in the OFDM load"""
        arr = sfs if isinstance(sfs, ctypes.Array) else self.batch_entries(sfs, self.tdd)
        return lib().srsran_ue_dl_gpu_decode_batch_sc16(ctypes.byref(self.q), ctypes.byref(self.cfg), len(arr), arr,
                                                        d_samples, scale, cfo, d_result, d_avg, stream)

    def last_llr(self, sf, tb):
        """srsran_pdsch_gpu_last_llr of the UE's PDSCH object after a batch: (device pointer, count)"""
        d, n = ctypes.c_void_p(), u32()
        if lib().srsran_pdsch_gpu_last_llr(ctypes.byref(self.q.pdsch), sf, tb, ctypes.byref(d), ctypes.byref(n)):
            raise RuntimeError(f"no LLRs for subframe {sf} TB {tb} in the last batch")
        return d.value, n.value

    def last_evm(self, sf, tb):
        """srsran_pdsch_gpu_last_evm of the UE's PDSCH object after a batch: device pointer of one float"""
        d = ctypes.c_void_p()
        if lib().srsran_pdsch_gpu_last_evm(ctypes.byref(self.q.pdsch), sf, tb, ctypes.byref(d)):
            raise RuntimeError(f"no EVM for subframe {sf} TB {tb} in the last batch")
        return d.value

    def free(self):
        if self.q.gpu:
            lib().srsran_ue_dl_free(ctypes.byref(self.q))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
