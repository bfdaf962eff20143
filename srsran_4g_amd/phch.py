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
                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        L.srsran_pdsch_gpu_llr.restype = ctypes.c_int
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


def gpu_llr(mod, d_sym, nsym, scramble, seed, d_llr, stream=None):
    return lib().srsran_pdsch_gpu_llr(mod, d_sym, nsym, int(scramble), seed, d_llr, stream)
