"""Python mirror of the PDSCH LLR-stage C API (include/srsran_phch.h).

Binds the HIP demapper / descrambler of the in-tree library; no CPU fallback."""
import ctypes

import numpy as np

from .tdec import load_library

_i16p = ctypes.POINTER(ctypes.c_int16)
_bound = False


def lib():
    global _bound
    L = load_library()
    if not _bound:
        L.srsran_demod_soft_demodulate_s.argtypes = [ctypes.c_int, ctypes.c_void_p, _i16p, ctypes.c_int]
        L.srsran_demod_soft_demodulate_s.restype = ctypes.c_int
        L.srsran_sequence_apply_s.argtypes = [_i16p, _i16p, ctypes.c_uint32, ctypes.c_uint32]
        L.srsran_sequence_apply_s.restype = None
        L.srsran_sequence_pdsch_apply_s.argtypes = [_i16p, _i16p, ctypes.c_uint16, ctypes.c_int, ctypes.c_uint32,
                                                    ctypes.c_uint32, ctypes.c_uint32]
        L.srsran_sequence_pdsch_apply_s.restype = None
        L.srsran_pdsch_gpu_llr.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p]
        L.srsran_pdsch_gpu_llr.restype = ctypes.c_int
        P = ctypes.c_void_p
        L.srsran_predecoding_type.argtypes = [P, P, P, P] + [ctypes.c_int] * 6 + [ctypes.c_float, ctypes.c_float]
        L.srsran_predecoding_type.restype = ctypes.c_int
        L.srsran_predecoding_gpu.argtypes = [P, P, P, P, P] + [ctypes.c_int] * 6 + [ctypes.c_float, ctypes.c_float, P]
        L.srsran_predecoding_gpu.restype = ctypes.c_int
        _bound = True
    return L


QM = (1, 2, 4, 6, 8)


def demod_s(mod, sym):
    sym = np.ascontiguousarray(sym, dtype=np.complex64)
    out = np.zeros(sym.size * QM[mod], np.int16)
    rc = lib().srsran_demod_soft_demodulate_s(mod, sym.ctypes.data, out.ctypes.data_as(_i16p), sym.size)
    if rc:
        raise RuntimeError(f"srsran_demod_soft_demodulate_s failed ({rc})")
    return out


def sequence_apply_s(llr, seed):
    x = np.ascontiguousarray(llr, dtype=np.int16)
    out = np.zeros_like(x)
    lib().srsran_sequence_apply_s(x.ctypes.data_as(_i16p), out.ctypes.data_as(_i16p), x.size, seed)
    return out


def sequence_pdsch_apply_s(llr, rnti, q, nslot, cell_id):
    x = np.ascontiguousarray(llr, dtype=np.int16)
    out = np.zeros_like(x)
    lib().srsran_sequence_pdsch_apply_s(x.ctypes.data_as(_i16p), out.ctypes.data_as(_i16p), rnti, q, nslot,
                                        cell_id, x.size)
    return out


def gpu_llr(mod, d_sym, nsym, scramble, seed, d_llr, stream=None, d_csi=None, d_csi_max=None):
    return lib().srsran_pdsch_gpu_llr(mod, d_sym, nsym, int(scramble), seed, d_csi, d_csi_max, d_llr, stream)


def _ptrs(arrs, n=4):
    return (ctypes.c_void_p * n)(*[a.ctypes.data if a is not None else None for a in arrs] + [None] * (n - len(arrs)))


def predecode(scheme, y, h, nlayers, codebook, scaling, noise):
    """srsran_predecoding_type (host-synchronous GPU). y: (nrx, n), h: (nports, nrx, n) complex64."""
    y = np.ascontiguousarray(y, np.complex64)
    h = np.ascontiguousarray(h, np.complex64)
    nrx, n = y.shape
    nports = h.shape[0]
    x = np.zeros((max(nlayers, 1), n), np.complex64)
    csi = np.zeros((2, n), np.float32)
    ys = _ptrs([y[r] for r in range(nrx)])
    hs = ((ctypes.c_void_p * 4) * 4)()
    for p in range(nports):
        for r in range(nrx):
            hs[p][r] = h[p, r].ctypes.data
    xs = _ptrs([x[l] for l in range(nlayers)])
    cs = _ptrs([csi[0], csi[1]], 2)
    rc = lib().srsran_predecoding_type(ctypes.addressof(ys), ctypes.addressof(hs), ctypes.addressof(xs),
                                       ctypes.addressof(cs), nrx, nports, nlayers, codebook, n, scheme, scaling, noise)
    if rc < 0:
        raise RuntimeError(f"srsran_predecoding_type failed ({rc})")
    if scheme == 1:  # transmit diversity: n/2 (4 ports: m_ap) symbols per layer, one CSI row
        return x[:nlayers, : (n // 2 if nlayers == 2 else rc)], csi[:1]
    return x[:nlayers], csi[:nlayers]


def predecode_gpu(scheme, d_y, d_h, d_x, d_csi, d_csi_max, nrx, nports, nlayers, codebook, n, scaling, noise,
                  stream=None):
    """srsran_predecoding_gpu: device pointer lists d_y[rx], d_h[port][rx], d_x[layer], d_csi[2]."""
    P = ctypes.c_void_p
    ys = (P * 4)(*(list(d_y) + [None] * (4 - len(d_y))))
    hs = ((P * 4) * 4)()
    for p in range(nports):
        for r in range(nrx):
            hs[p][r] = d_h[p][r]
    xs = (P * 4)(*(list(d_x) + [None] * (4 - len(d_x))))
    cs = (P * 2)(*d_csi)
    return lib().srsran_predecoding_gpu(ctypes.addressof(ys), ctypes.addressof(hs), ctypes.addressof(xs),
                                        ctypes.addressof(cs), d_csi_max, nrx, nports, nlayers, codebook, n, scheme,
                                        scaling, noise, stream)
