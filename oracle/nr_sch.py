"""ctypes bindings for the NR shared-channel parity checkers (TEST INFRASTRUCTURE ONLY).

* ``OracleNr`` -- this repo's plain-C restatement (``nr_sch_oracle.c`` in liboracle.so)
* ``RefNr``    -- the reference's sch_nr.c / ldpc_rm.c / cbsegm.c / softbuffer.c compiled from
  /root/reference into ``_ref/libsrsref.so`` (``ref_nr_harness.c``)
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libsrsref.so")

TB_INFO_FIELDS = ("bg", "Qm", "G", "A", "L_tb", "L_cb", "B", "Bp", "Kp", "Kr", "F", "Nref", "Z", "Nl", "C")
MAX_CB_SIZE = 384 * 66  # SRSRAN_LDPC_MAX_LEN_ENCODED_CB
MAX_NOF_CB = 41         # SRSRAN_SCH_NR_MAX_NOF_CB_LDPC
u32 = ctypes.c_uint32
P = ctypes.c_void_p


class oracle_nr_tb_info_t(ctypes.Structure):
    _fields_ = [("bg", ctypes.c_int)] + [(n, u32) for n in ("Qm", "G", "A", "L_tb", "L_cb", "B", "Bp", "Kp", "Kr",
                                                            "F", "Nref", "Z", "Nl", "C")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n in TB_INFO_FIELDS}


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def ref_available():
    return os.path.exists(REF_SO)


class OracleNr:
    def __init__(self):
        L = ctypes.CDLL(ORACLE_SO)
        self.L = L
        L.oracle_nr_cbsegm.argtypes = [ctypes.c_int, u32, ctypes.POINTER(u32 * 6)]
        L.oracle_nr_tb_info.argtypes = [u32, ctypes.c_double, u32, u32, u32, ctypes.c_int, u32, ctypes.c_int,
                                        ctypes.POINTER(oracle_nr_tb_info_t)]
        L.oracle_nr_E.argtypes = [ctypes.POINTER(oracle_nr_tb_info_t), u32]
        L.oracle_nr_E.restype = u32
        L.oracle_ldpc_rm_rx_c.argtypes = [P, P, u32, u32, ctypes.c_int, u32, u32, u32, u32]
        L.oracle_nr_sch_decode.argtypes = [ctypes.POINTER(oracle_nr_tb_info_t), u32, P, ctypes.c_float, ctypes.c_int,
                                           P, u32, P, P, u32, P, ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_float)]

    def cbsegm(self, bg, tbs):
        out = (u32 * 6)()
        assert self.L.oracle_nr_cbsegm(bg, tbs, ctypes.byref(out)) == 0
        return dict(zip(("tbs", "L_tb", "L_cb", "C", "K", "Z"), list(out)))

    def tb_info(self, tbs, R, Qm, G, Nl, lbrm=False, nof_prb=52, mcs256=False):
        t = oracle_nr_tb_info_t()
        assert self.L.oracle_nr_tb_info(tbs, R, Qm, G, Nl, int(lbrm), nof_prb, int(mcs256), ctypes.byref(t)) == 0
        return t

    def E(self, t, j):
        return int(self.L.oracle_nr_E(ctypes.byref(t), j))

    def rm_rx(self, e, out, F, bg, ls, rv, Qm, Nref):
        """In place on `out` (int8 [>= N]); returns n_llr."""
        e = np.ascontiguousarray(e, np.int8)
        return self.L.oracle_ldpc_rm_rx_c(_p(e), _p(out), e.size, F, bg, ls, rv, Qm, Nref)

    def decode(self, t, rv, e_bits, state, scaling=0.8, max_iter=10):
        """state = dict(softbuf [C, MAX_CB_SIZE] int8, cb_crc [C] u8, cb_data [C, 1056] u8), updated in place.
        Returns (tb_crc, avg_iter, payload)."""
        e_bits = np.ascontiguousarray(e_bits, np.int8)
        payload = np.zeros(t.A // 8 + 8, np.uint8)
        crc = ctypes.c_int()
        avg = ctypes.c_float()
        sb, cc, cd = state["softbuf"], state["cb_crc"], state["cb_data"]
        assert self.L.oracle_nr_sch_decode(ctypes.byref(t), rv, _p(e_bits), scaling, max_iter, _p(sb), sb.shape[1],
                                           _p(cc), _p(cd), cd.shape[1], _p(payload), ctypes.byref(crc),
                                           ctypes.byref(avg)) == 0
        return crc.value, avg.value, payload[:t.A // 8]


def new_state(C):
    return {"softbuf": np.zeros((max(C, 1), MAX_CB_SIZE), np.int8), "cb_crc": np.zeros(max(C, 1), np.uint8),
            "cb_data": np.zeros((max(C, 1), 1056), np.uint8)}


class RefNr:
    def __init__(self):
        L = ctypes.CDLL(REF_SO, mode=os.RTLD_LAZY)
        self.L = L
        L.ref_nr_softbuffer_new.argtypes = [u32, u32]
        L.ref_nr_softbuffer_new.restype = P
        L.ref_nr_softbuffer_free.argtypes = [P]
        L.ref_nr_softbuffer_reset.argtypes = [P]
        L.ref_nr_softbuffer_get.argtypes = [P, u32, P, u32, P, u32]
        L.ref_nr_decode.argtypes = [P, u32, ctypes.c_int, ctypes.c_int, u32, u32, u32, ctypes.c_double, u32, u32,
                                    ctypes.c_float, u32, P, P, ctypes.POINTER(ctypes.c_int),
                                    ctypes.POINTER(ctypes.c_float)]
        L.ref_nr_tb_info.argtypes = [u32, ctypes.c_int, ctypes.c_int, u32, u32, u32, ctypes.c_double, u32,
                                     ctypes.POINTER(u32 * 15)]
        L.ref_ldpc_rm_rx_c.argtypes = [P, P, u32, u32, ctypes.c_int, u32, u32, u32, u32]
        L.ref_cbsegm_ldpc.argtypes = [ctypes.c_int, u32, ctypes.POINTER(u32 * 6)]
        L.ref_nr_encode.argtypes = [u32, ctypes.c_int, ctypes.c_int, u32, u32, u32, ctypes.c_double, u32, u32, P, P]
        L.ref_nr_rx_new.argtypes = [u32, ctypes.c_float, u32]
        L.ref_nr_rx_new.restype = P
        L.ref_nr_rx_free.argtypes = [P]
        L.ref_nr_rx_decode.argtypes = [P, P, ctypes.c_int, ctypes.c_int, u32, u32, u32, ctypes.c_double, u32, u32, P, P,
                                       ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_float)]
        L.ref_ra_nr_tbs.argtypes = [u32, ctypes.c_double, ctypes.c_double, u32, u32]
        L.ref_ra_nr_tbs.restype = u32

    def tbs(self, N_re, R, Qm, layers, S=1.0):
        """srsran_ra_nr_tbs: a valid NR TBS for N_re resource elements."""
        return int(self.L.ref_ra_nr_tbs(N_re, S, R, Qm, layers))

    def cbsegm(self, bg, tbs):
        out = (u32 * 6)()
        assert self.L.ref_cbsegm_ldpc(bg, tbs, ctypes.byref(out)) == 0
        return dict(zip(("tbs", "L_tb", "L_cb", "C", "K", "Z"), list(out)))

    def tb_info(self, tbs, R, Qm, G, Nl, lbrm=False, nof_prb=52, mcs256=False):
        out = (u32 * 15)()
        assert self.L.ref_nr_tb_info(nof_prb, int(mcs256), int(lbrm), Qm, Nl, tbs, R, G, ctypes.byref(out)) == 0
        return dict(zip(TB_INFO_FIELDS, list(out)))

    def rm_rx(self, e, out, F, bg, ls, rv, Qm, Nref):
        e = np.ascontiguousarray(e, np.int8)
        return self.L.ref_ldpc_rm_rx_c(_p(e), _p(out), e.size, F, bg, ls, rv, Qm, Nref)

    def encode(self, tbs, R, Qm, G, Nl, rv, payload, lbrm=False, nof_prb=52, mcs256=False):
        payload = np.ascontiguousarray(payload, np.uint8)
        e = np.zeros(G, np.uint8)
        assert self.L.ref_nr_encode(nof_prb, int(mcs256), int(lbrm), Qm, Nl, tbs, R, rv, G, _p(payload), _p(e)) == 0
        return e

    class Softbuffer:
        def __init__(self, L, max_cb=MAX_NOF_CB, max_cb_size=MAX_CB_SIZE):
            self.L, self.h = L, L.ref_nr_softbuffer_new(max_cb, max_cb_size)
            assert self.h

        def reset(self):
            self.L.ref_nr_softbuffer_reset(self.h)

        def get(self, r):
            buf = np.zeros(MAX_CB_SIZE, np.int8)
            data = np.zeros(1056, np.uint8)
            ok = self.L.ref_nr_softbuffer_get(self.h, r, _p(buf), buf.size, _p(data), data.size)
            return ok, buf, data

        def free(self):
            self.L.ref_nr_softbuffer_free(self.h)

    def softbuffer(self):
        return RefNr.Softbuffer(self.L)

    def decode(self, sb, tbs, R, Qm, G, Nl, rv, e_bits, scaling=0.8, max_iter=10, lbrm=False, nof_prb=52,
               mcs256=False):
        e_bits = np.ascontiguousarray(e_bits, np.int8)
        payload = np.zeros(tbs // 8 + 8, np.uint8)
        crc = ctypes.c_int()
        avg = ctypes.c_float()
        r = self.L.ref_nr_decode(sb.h, nof_prb, int(mcs256), int(lbrm), Qm, Nl, tbs, R, rv, G, scaling, max_iter,
                                 _p(e_bits), _p(payload), ctypes.byref(crc), ctypes.byref(avg))
        assert r == 0, r
        return crc.value, avg.value, payload[:tbs // 8]


class RefNrRx:
    """A persistent reference receiver (srsran_sch_nr_init_rx once) for timing: decode() into a soft buffer."""

    def __init__(self, ref, nof_prb, scaling=0.8, max_iter=10):
        self.L = ref.L
        self.h = self.L.ref_nr_rx_new(nof_prb, scaling, max_iter)
        assert self.h

    def decode(self, sb, tbs, R, Qm, G, Nl, rv, e_bits, lbrm=False, mcs256=False):
        e_bits = np.ascontiguousarray(e_bits, np.int8)
        payload = np.zeros(tbs // 8 + 8, np.uint8)
        crc = ctypes.c_int()
        avg = ctypes.c_float()
        r = self.L.ref_nr_rx_decode(self.h, sb.h, int(mcs256), int(lbrm), Qm, Nl, tbs, R, rv, G, _p(e_bits),
                                    _p(payload), ctypes.byref(crc), ctypes.byref(avg))
        assert r == 0, r
        return crc.value, avg.value, payload[:tbs // 8]

    def free(self):
        if self.h:
            self.L.ref_nr_rx_free(self.h)
            self.h = None
