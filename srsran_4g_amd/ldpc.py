"""Python mirror of the srsran_ldpc_decoder_* C API (include/srsran_ldpc.h).

Binds the C-ABI library with ctypes so tests and bench.py drive the GPU NR LDPC decoder the way
the reference's own tests drive lib/src/phy/fec/ldpc/ldpc_decoder.c (ldpc_dec_avx2_test.c,
ldpc_rm_chain_test.c).  There is no Python or CPU fallback: without the library or a HIP device
the calls raise.
"""
import ctypes

import numpy as np

from . import tdec
from .sch import srsran_crc_t

# ldpc_decoder.h:38-50
DEC_F, DEC_S, DEC_C, DEC_C_FLOOD, DEC_C_AVX2, DEC_C_AVX2_FLOOD, DEC_C_AVX512, DEC_C_AVX512_FLOOD = range(8)
BG1, BG2 = 0, 1
BG_SHAPE = {BG1: (46, 68, 22), BG2: (42, 52, 10)}  # (M, Nfull, K)
MAX_CNCT = 20


class srsran_ldpc_decoder_args_t(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("bg", ctypes.c_int), ("ls", ctypes.c_uint16),
                ("scaling_fctr", ctypes.c_float), ("max_nof_iter", ctypes.c_uint32)]


class srsran_ldpc_decoder_t(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("bg", ctypes.c_int), ("ls", ctypes.c_uint16),
                ("max_nof_iter", ctypes.c_uint32), ("bgN", ctypes.c_uint8), ("liftN", ctypes.c_uint16),
                ("bgM", ctypes.c_uint8), ("liftM", ctypes.c_uint16), ("bgK", ctypes.c_uint8),
                ("liftK", ctypes.c_uint16), ("pcm", ctypes.POINTER(ctypes.c_uint16)),
                ("var_indices", ctypes.c_void_p), ("scaling_fctr", ctypes.c_float), ("free", ctypes.c_void_p),
                ("decode_f", ctypes.c_void_p), ("decode_s", ctypes.c_void_p), ("decode_c", ctypes.c_void_p)]


_sig = False


def _lib():
    global _sig
    L = tdec.load_library()
    if not _sig:
        P = ctypes.c_void_p
        L.srsran_ldpc_decoder_init.argtypes = [ctypes.POINTER(srsran_ldpc_decoder_t),
                                               ctypes.POINTER(srsran_ldpc_decoder_args_t)]
        L.srsran_ldpc_decoder_free.argtypes = [ctypes.POINTER(srsran_ldpc_decoder_t)]
        L.srsran_ldpc_decoder_free.restype = None
        for n in ("decode_c", "decode_s", "decode_f"):
            getattr(L, "srsran_ldpc_decoder_" + n).argtypes = [ctypes.POINTER(srsran_ldpc_decoder_t), P, P,
                                                               ctypes.c_uint32]
        L.srsran_ldpc_decoder_decode_crc_c.argtypes = [ctypes.POINTER(srsran_ldpc_decoder_t), P, P, ctypes.c_uint32,
                                                       ctypes.POINTER(srsran_crc_t)]
        L.srsran_ldpc_decoder_gpu_decode_batch.argtypes = [ctypes.POINTER(srsran_ldpc_decoder_t), P, ctypes.c_uint32,
                                                           ctypes.c_uint32, ctypes.c_uint32,
                                                           ctypes.POINTER(srsran_crc_t), P, ctypes.c_uint32,
                                                           ctypes.c_int, P, P]
        L.srsran_ldpc_decoder_gpu_decode_batch_s.argtypes = L.srsran_ldpc_decoder_gpu_decode_batch.argtypes
        L.create_compact_pcm.argtypes = [P, P, ctypes.c_int, ctypes.c_uint16]
        L.srsran_crc_init.argtypes = [ctypes.POINTER(srsran_crc_t), ctypes.c_uint32, ctypes.c_int]
        _sig = True
    return L


def compact_pcm(bg, ls):
    M, N, _ = BG_SHAPE[bg]
    pcm = np.zeros(M * N, np.uint16)
    pos = np.zeros((M, MAX_CNCT), np.int8)
    r = _lib().create_compact_pcm(pcm.ctypes.data, pos.ctypes.data, bg, ls)
    if r != 0:
        raise ValueError(f"invalid lifting size {ls}")
    return pcm.reshape(M, N), pos


def make_crc(poly, order):
    c = srsran_crc_t()
    if _lib().srsran_crc_init(ctypes.byref(c), poly, order) != 0:
        raise ValueError("crc init")
    return c


class LdpcDecoder:
    """srsran_ldpc_decoder_t on the GPU (one HIP stream per object)."""

    def __init__(self, bg, ls, dtype=DEC_C_AVX2, scaling=0.8, max_nof_iter=10):
        self.q = srsran_ldpc_decoder_t()
        args = srsran_ldpc_decoder_args_t(dtype, bg, ls, scaling, max_nof_iter)
        if _lib().srsran_ldpc_decoder_init(ctypes.byref(self.q), ctypes.byref(args)) != 0:
            raise RuntimeError("srsran_ldpc_decoder_init failed (no HIP device, or unsupported configuration)")
        self.bg, self.ls, self.dtype = bg, ls, dtype
        M, N, K = BG_SHAPE[bg]
        self.liftK, self.n_llr = K * ls, (N - 2) * ls

    def free(self):
        if self.q.ptr:
            _lib().srsran_ldpc_decoder_free(ctypes.byref(self.q))

    def decode_c(self, llrs, length=None, crc=None):
        """Host-synchronous decode of one codeword: (return value, message bits)."""
        llrs = np.ascontiguousarray(llrs, np.int8)
        assert llrs.size == self.n_llr
        out = np.zeros(self.liftK, np.uint8)
        L = self.n_llr if length is None else length
        if crc is None:
            r = _lib().srsran_ldpc_decoder_decode_c(ctypes.byref(self.q), llrs.ctypes.data, out.ctypes.data, L)
        else:
            c = make_crc(*crc)
            r = _lib().srsran_ldpc_decoder_decode_crc_c(ctypes.byref(self.q), llrs.ctypes.data, out.ctypes.data, L,
                                                        ctypes.byref(c))
        return r, out

    def decode_s(self, llrs, length=None):
        """Host-synchronous 16-bit decode (SRSRAN_LDPC_DECODER_S): (return value, message bits)."""
        llrs = np.ascontiguousarray(llrs, np.int16)
        assert llrs.size == self.n_llr
        out = np.zeros(self.liftK, np.uint8)
        r = _lib().srsran_ldpc_decoder_decode_s(ctypes.byref(self.q), llrs.ctypes.data, out.ctypes.data,
                                                self.n_llr if length is None else length)
        return r, out

    def gpu_decode_batch(self, d_llrs, llr_stride, nof_cw, d_message, message_stride, length=None, crc=None,
                         packed=False, d_ret=None, stream=None):
        """Asynchronous batch over device pointers (ints); returns the C status."""
        c = make_crc(*crc) if crc is not None else None
        self._crc_keep = c
        fn = (_lib().srsran_ldpc_decoder_gpu_decode_batch_s if self.dtype == DEC_S
              else _lib().srsran_ldpc_decoder_gpu_decode_batch)
        return fn(
            ctypes.byref(self.q), d_llrs, llr_stride, nof_cw, self.n_llr if length is None else length,
            ctypes.byref(c) if c is not None else None, d_message, message_stride, int(packed), d_ret, stream)
