"""oracle/uci.py -- TEST INFRASTRUCTURE ONLY: ctypes view of the UCI-on-PUSCH checker.

  RefUci : the reference's uci.c / block.c compiled into oracle/_ref/libsrsref.so, driven by
           oracle/ref_uci_harness.c (which restates the unbuildable sch.c / cqi.c orchestration):
             rx(cfg, q, g, c)    srsran_ulsch_decode up to decode_tb (ACK / RI / de-interleave / CQI)
             tx(cfg, uci, e)     srsran_ulsch_encode on unpacked bits: the type of every PUSCH bit
  scramble_llrs : the PUSCH bit stream -> descrambled soft bits, as pusch.c:307-331 (scrambling,
           placeholder "x" = 1, repetition "y" = the previous scrambled bit) and pusch.c:435-441
           (descrambling by the same sequence) would leave them, through an AWGN channel.
The cfg / uci arguments are ctypes structures with the reference's layout (the library's mirrors in
srsran_4g_amd/sch.py; tests check the sizes against the harness).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SO = os.path.join(HERE, "_ref", "libsrsref.so")

TYPE_PLACEHOLDER, TYPE_REPETITION = 2, 3  # ref_ulsch_uci_tx's q_types codes


def ref_available():
    return os.path.exists(REF_SO)


class RefUci:
    def __init__(self):
        L = ctypes.CDLL(REF_SO, mode=os.RTLD_LAZY)
        for n in ("ref_ulsch_uci_rx", "ref_ulsch_uci_tx", "ref_cqi_size", "ref_cqi_pack", "ref_cqi_unpack"):
            getattr(L, n).restype = ctypes.c_int
        L.ref_sizeof_pusch_cfg.restype = ctypes.c_uint32
        L.ref_sizeof_uci_value.restype = ctypes.c_uint32
        L.srsran_qprime_cqi_ext.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float]
        L.srsran_qprime_cqi_ext.restype = ctypes.c_uint32
        L.srsran_qprime_ack_ext.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_float]
        L.srsran_qprime_ack_ext.restype = ctypes.c_uint32
        self.L = L

    def sizes(self):
        return self.L.ref_sizeof_pusch_cfg(), self.L.ref_sizeof_uci_value()

    def cqi_size(self, cqi_cfg):
        return self.L.ref_cqi_size(ctypes.byref(cqi_cfg))

    def cqi_pack(self, cqi_cfg, value):
        buf = np.zeros(64, np.uint8)
        n = self.L.ref_cqi_pack(ctypes.byref(cqi_cfg), ctypes.byref(value), buf.ctypes.data_as(ctypes.c_void_p))
        return buf[:n]

    def cqi_unpack(self, cqi_cfg, bits, value):
        buf = np.zeros(64, np.uint8)
        buf[:len(bits)] = bits
        return self.L.ref_cqi_unpack(ctypes.byref(cqi_cfg), buf.ctypes.data_as(ctypes.c_void_p), ctypes.byref(value))

    def rx(self, cfg, q_bits, c_seq, uci, g_bits=None):
        """-> (ret, q after, g, (Q'_RI, Q'_CQI, G, Q'_ACK)); cfg and uci updated in place"""
        q = np.array(q_bits, dtype=np.int16, copy=True)
        g = np.zeros_like(q) if g_bits is None else np.array(g_bits, dtype=np.int16, copy=True)
        c = np.ascontiguousarray(c_seq, dtype=np.uint8)
        out = np.zeros(4, np.uint32)
        ret = self.L.ref_ulsch_uci_rx(ctypes.byref(cfg), q.ctypes.data_as(ctypes.c_void_p),
                                      g.ctypes.data_as(ctypes.c_void_p), c.ctypes.data_as(ctypes.c_void_p),
                                      ctypes.byref(uci), out.ctypes.data_as(ctypes.c_void_p))
        return ret, q, g, tuple(int(v) for v in out)

    def tx_sizes(self, cfg, uci):
        """(Q'_RI, Q'_CQI, G) of the transmitter"""
        out = np.zeros(4, np.uint32)
        t = np.zeros(cfg.grant.tb.nof_bits, np.uint8)
        ret = self.L.ref_ulsch_uci_tx(ctypes.byref(cfg), ctypes.byref(uci), None, t.ctypes.data_as(ctypes.c_void_p),
                                      out.ctypes.data_as(ctypes.c_void_p))
        assert ret == 0
        return tuple(int(v) for v in out[:3])

    def tx(self, cfg, uci, e_bits):
        out = np.zeros(4, np.uint32)
        t = np.zeros(cfg.grant.tb.nof_bits, np.uint8)
        e = np.ascontiguousarray(e_bits, dtype=np.uint8)
        if e.size == 0:
            e = np.zeros(1, np.uint8)
        ret = self.L.ref_ulsch_uci_tx(ctypes.byref(cfg), ctypes.byref(uci), e.ctypes.data_as(ctypes.c_void_p),
                                      t.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p))
        assert ret == 0
        return t, tuple(int(v) for v in out)


def scramble_llrs(types, c_seq, rng, amp=100.0, sigma=0.0):
    """PUSCH bit types (0/1, placeholder, repetition) -> int16 descrambled LLRs (positive = 1)"""
    t = np.asarray(types)
    c = np.asarray(c_seq, dtype=np.uint8)
    s = np.where(t <= 1, t, 0).astype(np.uint8) ^ c  # x / y positions hold 0 before scrambling
    s[t == TYPE_PLACEHOLDER] = 1
    rep = np.nonzero((t == TYPE_REPETITION) & (np.arange(t.size) > 1))[0]
    s[rep] = s[rep - 1]
    x = (2.0 * (s ^ c) - 1.0) * amp
    if sigma > 0:
        x = x + rng.standard_normal(x.size) * sigma * amp
    return np.clip(np.trunc(x), -32767, 32767).astype(np.int16)
