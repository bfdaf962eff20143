"""ctypes bindings for the NR LDPC parity checkers (TEST INFRASTRUCTURE ONLY).

* ``OracleLdpc``  -- this repo's plain-C restatement (``ldpc_oracle.c`` in liboracle.so)
* ``RefLdpc``     -- the reference's own LDPC decoder / encoder compiled from /root/reference
  into ``_ref/libsrsref.so`` (``ref_ldpc_harness.c``)
* ``load_examples`` -- the reference's golden examples (lib/src/phy/fec/ldpc/test/examplesBG*.dat)
  as committed fixtures (tests/golden/ldpc_examples.npz)
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libsrsref.so")
EXAMPLES = os.path.join(HERE, "..", "tests", "golden", "ldpc_examples.npz")

# base graph geometry (base_graph.h:46-56): bg -> (M, Nfull, K)
BG_SHAPE = {0: (46, 68, 22), 1: (42, 52, 10)}
LIFT_SIZES = sorted({a << j for a in (2, 3, 5, 7, 9, 11, 13, 15) for j in range(8) if (a << j) <= 384})
assert len(LIFT_SIZES) == 51

# srsran_ldpc_decoder_type_t (ldpc_decoder.h:38-50)
DEC_F, DEC_S, DEC_C, DEC_C_FLOOD, DEC_C_AVX2, DEC_C_AVX2_FLOOD = 0, 1, 2, 3, 4, 5
SCALE_C, SCALE_SIMD = 0, 1

CRC24A, CRC24B, CRC16 = 0x1864CFB, 0x1800063, 0x11021  # phy_common.h:72-74


def lift(bg, ls):
    """(liftK, liftN, n_llr) for a base graph and lifting size."""
    M, N, K = BG_SHAPE[bg]
    return K * ls, N * ls, N * ls - 2 * ls


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleLdpc:
    def __init__(self):
        L = ctypes.CDLL(ORACLE_SO)
        self.L = L
        L.oracle_ldpc_ls_index.argtypes = [ctypes.c_int]
        L.oracle_ldpc_pcm.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_ldpc_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_ldpc_decode_c.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.c_void_p]
        L.oracle_ldpc_decode_s.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.c_void_p]

    def pcm(self, bg, ls):
        M, N, _ = BG_SHAPE[bg]
        pcm = np.zeros(M * N, np.uint16)
        pos = np.zeros((M, 20), np.int8)
        assert self.L.oracle_ldpc_pcm(bg, ls, _p(pcm), _p(pos)) == 0
        return pcm.reshape(M, N), pos

    def encode(self, bg, ls, msg):
        """Full lifted codeword (liftN bits, the first 2*ls included)."""
        K, N, _ = lift(bg, ls)
        msg = np.ascontiguousarray(msg, np.uint8)
        assert msg.size == K
        cw = np.zeros(N, np.uint8)
        assert self.L.oracle_ldpc_encode(bg, ls, _p(msg), _p(cw)) == 0
        return cw

    def decode_c(self, bg, ls, llrs, scaling=0.8, max_iter=10, length=None, crc=None, scale_mode=SCALE_SIMD):
        K, N, n = lift(bg, ls)
        llrs = np.ascontiguousarray(llrs, np.int8)
        assert llrs.size == n
        out = np.zeros(K, np.uint8)
        poly, order = crc if crc else (0, 0)
        r = self.L.oracle_ldpc_decode_c(bg, ls, scale_mode, scaling, max_iter, _p(llrs),
                                        n if length is None else length, poly, order, _p(out))
        return r, out

    def decode_s(self, bg, ls, llrs, scaling=0.8, max_iter=10, length=None, crc=None):
        K, N, n = lift(bg, ls)
        llrs = np.ascontiguousarray(llrs, np.int16)
        assert llrs.size == n
        out = np.zeros(K, np.uint8)
        poly, order = crc if crc else (0, 0)
        r = self.L.oracle_ldpc_decode_s(bg, ls, scaling, max_iter, _p(llrs), n if length is None else length,
                                        poly, order, _p(out))
        return r, out


def ref_available():
    return os.path.exists(REF_SO)


class RefLdpc:
    def __init__(self):
        L = ctypes.CDLL(REF_SO, mode=os.RTLD_LAZY)
        self.L = L
        L.ref_ldpc_decode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                      ctypes.c_void_p]
        L.ref_ldpc_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.ref_ldpc_decode_many.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
        L.create_compact_pcm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint16]

    def pcm(self, bg, ls):
        M, N, _ = BG_SHAPE[bg]
        pcm = np.zeros(M * N, np.uint16)
        pos = np.zeros((M, 20), np.int8)
        assert self.L.create_compact_pcm(_p(pcm), _p(pos), bg, ls) == 0
        return pcm.reshape(M, N), pos

    def encode(self, bg, ls, msg):
        """Codeword without the 2*ls punctured bits (srsran_ldpc_encoder_encode)."""
        K, N, n = lift(bg, ls)
        msg = np.ascontiguousarray(msg, np.uint8)
        cw = np.zeros(n, np.uint8)
        assert self.L.ref_ldpc_encode(bg, ls, _p(msg), _p(cw)) == 0
        return cw

    def decode(self, dtype, bg, ls, llrs, scaling=0.8, max_iter=10, length=None, crc=None):
        K, N, n = lift(bg, ls)
        bits = 16 if dtype == DEC_S else 8
        llrs = np.ascontiguousarray(llrs, np.int16 if bits == 16 else np.int8)
        assert llrs.size == n
        out = np.zeros(K, np.uint8)
        poly, order = crc if crc else (0, 0)
        r = self.L.ref_ldpc_decode(dtype, bg, ls, scaling, max_iter, _p(llrs), bits, n if length is None else length,
                                   poly, order, _p(out))
        assert r > -100, "reference decoder init failed"
        return r, out


    def decode_many(self, dtype, bg, ls, llrs2d, scaling=0.8, max_iter=10):
        """Every row through one decoder object (CPU throughput sample); returns the messages."""
        K, N, n = lift(bg, ls)
        llrs2d = np.ascontiguousarray(llrs2d, np.int8)
        out = np.zeros((llrs2d.shape[0], K), np.uint8)
        assert self.L.ref_ldpc_decode_many(dtype, bg, ls, scaling, max_iter, _p(llrs2d), llrs2d.shape[1],
                                           llrs2d.shape[0], _p(out)) == 0
        return out


def load_examples(path=EXAMPLES):
    """{(bg, ls): (msgs uint8 [n, liftK] with FILLER=254, cwds uint8 [n, liftN-2ls] with FILLER)}"""
    z = np.load(path)
    out = {}
    for key in z.files:
        if not key.endswith("_msg"):
            continue
        bg, ls = (int(v) for v in key[:-4].split("_"))
        K, N, n = lift(bg, ls)
        msg = np.unpackbits(z[key], axis=1)[:, :K]
        cw = np.unpackbits(z[f"{bg}_{ls}_cw"], axis=1)[:, :n]
        fm, fc = z[f"{bg}_{ls}_fill"]
        if fm:
            msg[:, K - fm:] = 254
        if fc:
            cfill = z[f"{bg}_{ls}_cfill"]
            cw[:, cfill] = 254
        out[(bg, ls)] = (msg, cw)
    return out


def noisy_llrs(cw_bits, rng, snr_db=2.0, amp=8.0, dtype=np.int8, clip=127):
    """BPSK (bit 1 -> negative LLR, the decoders' convention) + AWGN, quantised."""
    x = 1.0 - 2.0 * cw_bits.astype(np.float64)
    sigma = 10 ** (-snr_db / 20)
    y = x + sigma * rng.standard_normal(x.shape)
    return np.clip(np.round(amp * y), -clip, clip).astype(dtype)
