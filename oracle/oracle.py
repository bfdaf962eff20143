"""ctypes bindings for the CPU parity checkers (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module.  It wraps two libraries built by oracle/Makefile:

* ``liboracle.so`` -- this repo's plain-C restatement (``tdec_oracle.c``)
* ``_ref/libsrsref.so`` -- the reference decoder compiled from /root/reference
  (present wherever it was built; it travels to the GPU box as a build artefact)
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libsrsref.so")

CB_SIZES = (
    [40 + 8 * i for i in range(60)]
    + [528 + 16 * i for i in range(32)]
    + [1056 + 32 * i for i in range(32)]
    + [2112 + 64 * i for i in range(64)]
)
assert len(CB_SIZES) == 188 and CB_SIZES[-1] == 6144

SEGM_FIELDS = ("F", "C", "K1", "K2", "K1_idx", "K2_idx", "C1", "C2", "tbs")
SOFTBUF_LEN = 18600  # SOFTBUFFER_SIZE, softbuffer.h:56
LTE_CRC24A = 0x1864CFB  # phy_common.h:72
LTE_CRC24B = 0x1800063  # phy_common.h:73

_i16p = ctypes.POINTER(ctypes.c_int16)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_i8p = ctypes.POINTER(ctypes.c_int8)


def _ptr(a, t):
    return a.ctypes.data_as(t)


def nof_subblocks(K):
    """AUTO 16-bit dispatch of turbodecoder.c:381-393 (AVX2 build)."""
    if K % 16 == 0 and K > 800:
        return 16
    if K % 8 == 0 and K > 400:
        return 8
    return 0


def tdec8_subblocks(K):
    """srsran_tdec_autoimp_get_subblocks_8bit (turbodecoder.c:410-424, AVX2 build)."""
    if K % 32 == 0 and K > 2048:
        return 32
    if K % 16 == 0 and K > 800:
        return 16
    return nof_subblocks(K)


def in_len(K, layout_sb):
    return 3 * (K + 32) + 12 if (layout_sb and nof_subblocks(K)) else 3 * K + 12


class _Lib:
    def __init__(self, path, prefix, lazy=False):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        mode = os.RTLD_LAZY if lazy else ctypes.DEFAULT_MODE
        self.lib = ctypes.CDLL(path, mode=mode)
        self.run = getattr(self.lib, prefix + "tdec_run")
        self.run.argtypes = [ctypes.c_uint32, _i16p, ctypes.c_int, ctypes.c_uint32, _u8p, _i16p]
        self.run.restype = ctypes.c_int

    def tdec_run(self, K, llr, layout_sb=False, nof_iterations=8, trace=False):
        llr = np.ascontiguousarray(llr, dtype=np.int16)
        assert llr.size >= in_len(K, layout_sb)
        out = np.zeros(K // 8, dtype=np.uint8)
        tr = np.zeros((nof_iterations, K), dtype=np.int16) if trace else None
        rc = self.run(K, _ptr(llr, _i16p), int(bool(layout_sb)), nof_iterations, _ptr(out, _u8p),
                      _ptr(tr, _i16p) if trace else None)
        if rc:
            raise ValueError(f"tdec_run failed K={K} rc={rc}")
        return (out, tr) if trace else out


def aligned(n, dtype, align=64):
    """Zeroed array whose data pointer is `align`-byte aligned (the reference's SSE loads need it)."""
    dt = np.dtype(dtype)
    buf = np.zeros(n * dt.itemsize + align, np.uint8)
    off = (-buf.ctypes.data) % align
    return buf[off:off + n * dt.itemsize].view(dt)


class _PhyMixin:
    """PDSCH LLR stages: soft demapping and descrambling (int16)."""

    def demod_s(self, mod, sym):
        sym = np.asarray(sym, dtype=np.complex64)
        x = aligned(sym.size, np.complex64)
        x[:] = sym
        bits = (1, 2, 4, 6, 8)[mod]
        out = aligned(sym.size * bits, np.int16)
        rc = self._demod_fn()(mod, x.ctypes.data_as(ctypes.c_void_p), _ptr(out, _i16p), sym.size)
        if rc:
            raise ValueError(rc)
        return out.copy()

    def predecode(self, scheme, y, h, nlayers, codebook, scaling, noise):
        """srsran_predecoding_type with CSI outputs. y: (nrx, n) complex64, h: (nports, nrx, n).
        Returns x (nlayers, n) complex64 and csi (nlayers, n) float32."""
        y = np.asarray(y, np.complex64)
        h = np.asarray(h, np.complex64)
        nrx, n = y.shape
        nports = h.shape[0]
        ya = aligned(y.size, np.complex64).reshape(y.shape)
        ya[:] = y
        ha = aligned(h.size, np.complex64).reshape(h.shape)
        ha[:] = h
        xa = aligned(max(nlayers, 2) * n, np.complex64).reshape(max(nlayers, 2), n)
        ca = aligned(max(nlayers, 2) * n, np.float32).reshape(max(nlayers, 2), n)
        rc = self._predecode(scheme, ya, ha, xa, ca, nrx, nports, nlayers, codebook, n, scaling, noise)
        if rc < 0:
            raise ValueError(rc)
        if scheme == 1:  # transmit diversity: n/2 (n/4, 4 ports) symbols per layer, one CSI row
            m = n // 2 if nlayers == 2 else (((n - 2) // 4 if n >= 2 else 0) if n % 4 else n // 4)
            return xa[:nlayers, :m].copy(), ca[:1].copy()
        return xa[:nlayers].copy(), ca[:nlayers].copy()

    def sequence_apply_s(self, llr, seed):
        x = aligned(len(llr), np.int16)
        x[:] = llr
        out = aligned(len(llr), np.int16)
        f = self._seq_fn()
        f(_ptr(x, _i16p), _ptr(out, _i16p), len(llr), seed)
        return out.copy()

    def demod_b(self, mod, sym):
        """int8 soft demapping (srsran_demod_soft_demodulate_b) of complex64 symbols."""
        sym = np.asarray(sym, dtype=np.complex64)
        x = aligned(sym.size, np.complex64)
        x[:] = sym
        out = aligned(sym.size * (1, 2, 4, 6, 8)[mod], np.int8)
        f = self._demod_b_fn()
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, _i8p, ctypes.c_int]
        if f(mod, x.ctypes.data_as(ctypes.c_void_p), _ptr(out, _i8p), sym.size):
            raise ValueError(mod)
        return out.copy()

    def sequence_apply_c(self, llr, seed):
        """int8 descrambling (srsran_sequence_apply_c)."""
        x = aligned(len(llr), np.int8)
        x[:] = llr
        out = aligned(len(llr), np.int8)
        f = self._seq_c_fn()
        f.argtypes = [_i8p, _i8p, ctypes.c_uint32, ctypes.c_uint32]
        f(_ptr(x, _i8p), _ptr(out, _i8p), len(llr), seed)
        return out.copy()


class Oracle(_Lib, _PhyMixin):
    """The repo's C restatement."""

    def _demod_fn(self):
        f = self.lib.oracle_demod_soft_s
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, _i16p, ctypes.c_int]
        return f

    def _seq_fn(self):
        f = self.lib.oracle_sequence_apply_s
        f.argtypes = [_i16p, _i16p, ctypes.c_uint32, ctypes.c_uint32]
        return f

    def _demod_b_fn(self):
        return self.lib.oracle_demod_soft_b

    def _seq_c_fn(self):
        return self.lib.oracle_sequence_apply_c

    def csi_correction_b(self, mod, csi, e):
        e = np.array(e, dtype=np.int8, copy=True)
        csi = np.ascontiguousarray(csi, dtype=np.float32)
        f = self.lib.oracle_csi_correction_b
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, _i8p, ctypes.c_uint32]
        f(mod, csi.ctypes.data, _ptr(e, _i8p), e.size)
        return e

    def _predecode(self, scheme, ya, ha, xa, ca, nrx, nports, nlayers, codebook, n, scaling, noise):
        f = self.lib.oracle_predecode
        f.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_float, ctypes.c_float]
        return f(scheme, nrx, nports, nlayers, codebook, ya.ctypes.data, ha.ctypes.data, xa.ctypes.data,
                 ca.ctypes.data, n, scaling, noise)

    def csi_correction(self, mod, csi, e):
        e = np.array(e, dtype=np.int16, copy=True)
        csi = np.ascontiguousarray(csi, dtype=np.float32)
        f = self.lib.oracle_csi_correction
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, _i16p, ctypes.c_uint32]
        f(mod, csi.ctypes.data, _ptr(e, _i16p), e.size)
        return e

    def crs_pilots(self, cell_id, nof_prb, pp, sf):
        out = np.zeros(4 * 2 * nof_prb, np.complex64)
        f = self.lib.oracle_crs_pilots
        f.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_void_p]
        f(cell_id, nof_prb, pp, sf, out.ctypes.data)
        return out[: (4 if pp == 0 else 2) * 2 * nof_prb]

    def gauss_filter(self, order, std):
        f = np.zeros(16, np.float32)
        g = self.lib.oracle_gauss_filter
        g.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_float]
        g.restype = ctypes.c_uint32
        n = g(f.ctypes.data, order, std)
        return f[:n]

    def chest_dl(self, grids, nof_prb, cell_id, nports, sf_idx, symbol_sz, cp=0, nsym=(4, 2)):
        """CRS channel estimate (srsUE defaults). grids: (nrx, 2*nsymb*12*nof_prb), nsymb = 7 (cp 0) or
        6 (cp 1, extended); nsym = CRS symbols of ports 0-1 / 2-3 (fewer in a TDD special subframe, crs_nsym)
        -> (ce (nports, nrx, n), stats)."""
        grids = np.ascontiguousarray(grids, np.complex64)
        nrx, n = grids.shape
        assert n == (12 if cp else 14) * 12 * nof_prb
        ce = np.zeros((nports, nrx, n), np.complex64)
        out = np.zeros(4, np.float32)
        f = self.lib.oracle_chest_dl_tdd
        f.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 9 + [ctypes.c_void_p, ctypes.c_void_p]
        f(grids.ctypes.data, nof_prb, cell_id, nports, nrx, sf_idx, symbol_sz, cp, nsym[0], nsym[1], ce.ctypes.data,
          out.ctypes.data)
        return ce, dict(noise=float(out[0]), rsrp=float(out[1]), rssi=float(out[2]), cfo=float(out[3]))

    def chest_dl_ext(self, grids, nof_prb, cell_id, nports, sf_idx, symbol_sz, cp=0, estimator=0, noise_alg=0,
                     filt_order=4, filt_std=1.0, sync=False, noise_state=None, nsym=(4, 2), filter_type=0):
        """chest_dl.c with the options beyond srsUE's defaults (oracle_chest_dl_ext_f): estimator 0 AVERAGE /
        1 INTERPOLATE, noise_alg 0 REFS / 1 PSS / 2 EMPTY, filter_type 0 GAUSS (filt_order 0 = automatic) / 1 TRIANGLE
        (w = filt_order) / 2 NONE, sync = correct_sync_error.
        -> (ce (nports, nrx, n), stats dict, corrected grids, noise_state (4, 4) after the call)"""
        grids = np.array(grids, np.complex64, copy=True)
        nrx, n = grids.shape
        ce = np.zeros((nports, nrx, n), np.complex64)
        out = np.zeros(5, np.float32)
        ns = np.zeros((4, 4), np.float32) if noise_state is None else np.array(noise_state, np.float32, copy=True)
        pss = np.zeros(62, np.complex64)
        self.lib.oracle_pss_generate.argtypes = [ctypes.c_uint32, ctypes.c_void_p]
        self.lib.oracle_pss_generate(cell_id % 3, pss.ctypes.data)
        f = self.lib.oracle_chest_dl_ext_f
        f.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 10 + [ctypes.c_float, ctypes.c_float, ctypes.c_uint32] + \
            [ctypes.c_void_p] * 2 + [ctypes.c_uint32] * 2 + [ctypes.c_void_p] * 2
        f(grids.ctypes.data, nof_prb, cell_id, nports, nrx, sf_idx, symbol_sz, cp, estimator, noise_alg, filter_type,
          float(filt_order), filt_std, 1 if sync else 0, pss.ctypes.data, ns.ctypes.data, nsym[0], nsym[1],
          ce.ctypes.data, out.ctypes.data)
        st = dict(noise=float(out[0]), rsrp=float(out[1]), rssi=float(out[2]), cfo=float(out[3]),
                  sync_error=float(out[4]))
        return ce, st, grids, ns

    def mbsfn_pilots(self, nof_prb, area, sf):
        """srsran_refsignal_mbsfn_gen_seq's pilots of subframe sf: (3, 6 N_RB) complex64"""
        out = np.zeros(18 * nof_prb, np.complex64)
        f = self.lib.oracle_mbsfn_pilots
        f.argtypes = [ctypes.c_uint32] * 3 + [ctypes.c_void_p]
        f(nof_prb, area, sf, out.ctypes.data)
        return out.reshape(3, 6 * nof_prb)

    def chest_dl_mbsfn(self, grids, nof_prb, cell_id, nports, sf_idx, area, noise_alg=1, filter_type=1, coef0=0.1,
                       coef1=0.0, noise_state=None, cp=0, ce_init=None):
        """srsran_chest_dl_estimate_cfg of an MBSFN subframe (oracle_chest_dl_mbsfn): INTERPOLATE, filter_type 0
        GAUSS (coef0 order, 0 = automatic; coef1 stddev) / 1 TRIANGLE (w = coef0; srsUE's MBSFN configuration:
        TRIANGLE 0.1, PSS noise) / 2 NONE.  ce_init: the estimate buffers before the call (rows 12 / 13 are not
        written).  -> (ce (nports, nrx, n), noise estimate, noise_state after the call)"""
        grids = np.ascontiguousarray(grids, np.complex64)
        nrx, n = grids.shape
        ce = np.zeros((nports, nrx, n), np.complex64) if ce_init is None else np.array(ce_init, np.complex64, copy=True)
        ns = np.zeros((4, 4), np.float32) if noise_state is None else np.array(noise_state, np.float32, copy=True)
        out = np.zeros(1, np.float32)
        f = self.lib.oracle_chest_dl_mbsfn
        f.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 9 + [ctypes.c_float] * 2 + [ctypes.c_void_p] * 3
        if f(grids.ctypes.data, nof_prb, cell_id, nports, nrx, sf_idx, cp, area, noise_alg, filter_type, coef0, coef1,
             ns.ctypes.data, ce.ctypes.data, out.ctypes.data):
            raise ValueError("oracle_chest_dl_mbsfn: ports 0 / 1 only")
        return ce, float(out[0]), ns

    def sequence_bits(self, seed, n):
        c = np.zeros(n, np.uint8)
        self.lib.oracle_sequence_bits.argtypes = [ctypes.c_uint32, _u8p, ctypes.c_uint32]
        self.lib.oracle_sequence_bits(seed, _ptr(c, _u8p), n)
        return c

    def pdsch_seed(self, rnti, q, nslot, cell_id):
        f = self.lib.oracle_pdsch_seed
        f.argtypes = [ctypes.c_uint16, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32]
        f.restype = ctypes.c_uint32
        return f(rnti, q, nslot, cell_id)

    def __init__(self):
        super().__init__(ORACLE_SO, "oracle_")
        L = self.lib
        L.oracle_tcod_encode.argtypes = [ctypes.c_uint32, _u8p, _u8p]
        L.oracle_natural_to_sb.argtypes = [ctypes.c_uint32, _i16p, _i16p]
        L.oracle_qpp.argtypes = [ctypes.c_uint32, _u16p, _u16p]
        L.oracle_tdec_run_batch.argtypes = [ctypes.c_uint32, _i16p, ctypes.c_uint32, ctypes.c_int,
                                            ctypes.c_uint32, _u8p, ctypes.c_uint32]

    def encode(self, K, bits):
        bits = np.ascontiguousarray(bits, dtype=np.uint8)
        out = np.zeros(3 * K + 12, dtype=np.uint8)
        if self.lib.oracle_tcod_encode(K, _ptr(bits, _u8p), _ptr(out, _u8p)):
            raise ValueError(K)
        return out

    def natural_to_sb(self, K, llr):
        llr = np.ascontiguousarray(llr, dtype=np.int16)
        out = np.zeros(in_len(K, True), dtype=np.int16)
        self.lib.oracle_natural_to_sb(K, _ptr(llr, _i16p), _ptr(out, _i16p))
        return out

    def qpp(self, K):
        f = np.zeros(K, dtype=np.uint16)
        r = np.zeros(K, dtype=np.uint16)
        self.lib.oracle_qpp(K, _ptr(f, _u16p), _ptr(r, _u16p))
        return f, r

    # ---- DL-SCH pieces (sch_oracle.c) ----
    def _sch_sigs(self):
        L = self.lib
        u32 = ctypes.c_uint32
        L.oracle_crc_checksum_byte.argtypes = [u32, ctypes.c_int, _u8p, u32]
        L.oracle_crc_checksum_byte.restype = u32
        L.oracle_crc_bits.argtypes = [u32, ctypes.c_int, _u8p, u32]
        L.oracle_crc_bits.restype = u32
        L.oracle_cbsegm.argtypes = [u32, ctypes.POINTER(u32)]
        L.oracle_rm_rx_table.argtypes = [u32, u32, ctypes.c_int, _u16p]
        L.oracle_rm_turbo_rx.argtypes = [u32, u32, ctypes.c_int, _i16p, u32, _i16p]
        L.oracle_rm_turbo_tx.argtypes = [u32, u32, _u8p, u32, _u8p]
        L.oracle_dlsch_decode_tb.argtypes = [u32, u32, u32, u32, _i16p, u32, _i16p, u32, _u8p, _u8p, u32, _u8p,
                                             ctypes.POINTER(u32), ctypes.POINTER(ctypes.c_float)]
        L.oracle_dlsch_encode_tb.argtypes = [u32, u32, u32, u32, _u8p, _u8p]
        L.oracle_dlsch_encode_tb_x.argtypes = [u32, u32, u32, u32, _u8p, _u8p, u32]

    def crc_byte(self, poly, order, data, nbits):
        self._sch_sigs()
        data = np.ascontiguousarray(data, dtype=np.uint8)
        return self.lib.oracle_crc_checksum_byte(poly, order, _ptr(data, _u8p), nbits)

    def crc_bits(self, poly, order, bits):
        self._sch_sigs()
        bits = np.ascontiguousarray(bits, dtype=np.uint8)
        return self.lib.oracle_crc_bits(poly, order, _ptr(bits, _u8p), bits.size)

    def cbsegm(self, tbs):
        self._sch_sigs()
        out = (ctypes.c_uint32 * 9)()
        rc = self.lib.oracle_cbsegm(tbs, out)
        return rc, dict(zip(SEGM_FIELDS, list(out)))

    def rm_rx_table(self, K, rv, layout_sb):
        self._sch_sigs()
        t = np.zeros(3 * K + 12, dtype=np.uint16)
        self.lib.oracle_rm_rx_table(K, rv, int(bool(layout_sb)), _ptr(t, _u16p))
        return t

    def rm_turbo_rx(self, K, rv, layout_sb, e, softbuf):
        self._sch_sigs()
        e = np.ascontiguousarray(e, dtype=np.int16)
        sb = np.ascontiguousarray(softbuf, dtype=np.int16).copy()
        self.lib.oracle_rm_turbo_rx(K, rv, int(bool(layout_sb)), _ptr(e, _i16p), e.size, _ptr(sb, _i16p))
        return sb

    def rm_turbo_tx(self, K, rv, coded, E):
        self._sch_sigs()
        coded = np.ascontiguousarray(coded, dtype=np.uint8)
        out = np.zeros(E, dtype=np.uint8)
        self.lib.oracle_rm_turbo_tx(K, rv, _ptr(coded, _u8p), E, _ptr(out, _u8p))
        return out

    def dlsch_encode(self, tbs, Qm, rv, nof_e_bits, tb_bytes, tb_crc_xor=0):
        self._sch_sigs()
        tb_bytes = np.ascontiguousarray(tb_bytes, dtype=np.uint8)
        e = np.zeros(nof_e_bits, dtype=np.uint8)
        n = self.lib.oracle_dlsch_encode_tb_x(tbs, Qm, rv, nof_e_bits, _ptr(tb_bytes, _u8p), _ptr(e, _u8p),
                                              tb_crc_xor)
        if n < 0:
            raise ValueError(f"encode failed tbs={tbs}")
        return e

    def ulsch_deinterleave(self, q_bits, Qm, nof_symb):
        """ulsch_deinterleave without RI bits (sch.c:994-1021): q (PUSCH order) -> g."""
        f = self.lib.oracle_ulsch_deinterleave
        f.argtypes = [_i16p, _i16p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        q = np.ascontiguousarray(q_bits, dtype=np.int16)
        g = np.zeros_like(q)
        f(_ptr(q, _i16p), _ptr(g, _i16p), Qm, q.size // Qm, nof_symb)
        return g

    def dlsch_decode(self, tbs, Qm, rv, e_llr, max_iterations, state=None):
        """decode_tb (sch.c:509-573). state = (softbuf[C,18600], cb_crc[C], cb_data[C,768]) for HARQ.

        Returns (ret, data, noi, avg, state); data is the whole zero-initialised payload
        buffer (tbs/8 + 8 bytes) so bytes written past tbs/8 (CRC bytes) are compared too."""
        self._sch_sigs()
        return _dlsch_decode(self.lib.oracle_dlsch_decode_tb, self.cbsegm(tbs)[1], tbs, Qm, rv, e_llr,
                             max_iterations, state)

    def dlsch_decode8(self, tbs, Qm, rv, e_llr, max_iterations, state=None):
        """decode_tb with llr_is_8bit (sch.c:409-428): int8 e bits; soft buffer rows hold int8 LLRs in the 8-bit
        decoder's layout.  Same returns as dlsch_decode."""
        self._sch_sigs()
        return _dlsch_decode(self.lib.oracle_dlsch_decode_tb8, self.cbsegm(tbs)[1], tbs, Qm, rv, e_llr,
                             max_iterations, state, llr8=True)

    def tdec8_run(self, K, llr, nof_iterations=8, trace=False):
        """C restatement of the 8-bit window decoders (nsb 16 / 32, SB layout input)."""
        f = self.lib.oracle_tdec8_run
        f.argtypes = [ctypes.c_uint32, _i8p, ctypes.c_uint32, _u8p, _i8p]
        llr = np.ascontiguousarray(llr, dtype=np.int8)
        out = np.zeros(K // 8, dtype=np.uint8)
        tr = np.zeros((nof_iterations, K), dtype=np.int8) if trace else None
        if f(K, _ptr(llr, _i8p), nof_iterations, _ptr(out, _u8p), _ptr(tr, _i8p) if trace else None):
            raise ValueError(K)
        return (out, tr) if trace else out

    def run_batch(self, K, llr2d, layout_sb, nof_iterations):
        llr2d = np.ascontiguousarray(llr2d, dtype=np.int16)
        n = llr2d.shape[0]
        out = np.zeros((n, K // 8), dtype=np.uint8)
        rc = self.lib.oracle_tdec_run_batch(K, _ptr(llr2d, _i16p), llr2d.shape[1], int(bool(layout_sb)),
                                            nof_iterations, _ptr(out, _u8p), n)
        if rc:
            raise ValueError(rc)
        return out


def _dlsch_decode(fn, segm, tbs, Qm, rv, e_llr, max_iterations, state, llr8=False):
    C = max(1, segm["C"])
    if state is None:
        state = (np.zeros((C, SOFTBUF_LEN), np.int16), np.zeros(C, np.uint8), np.zeros((C, 768), np.uint8))
    sb, crc, cbd = state
    ep = _i8p if llr8 else _i16p
    e_llr = np.ascontiguousarray(e_llr, dtype=np.int8 if llr8 else np.int16)
    data = np.zeros(tbs // 8 + 8, dtype=np.uint8)
    noi = (ctypes.c_uint32 * C)()
    avg = ctypes.c_float(0)
    u32 = ctypes.c_uint32
    fn.argtypes = [u32, u32, u32, u32, ep, u32, _i16p, u32, _u8p, _u8p, u32, _u8p, ctypes.POINTER(u32),
                   ctypes.POINTER(ctypes.c_float)]
    ret = fn(tbs, Qm, rv, e_llr.size, _ptr(e_llr, ep), max_iterations, _ptr(sb, _i16p), sb.shape[1],
             _ptr(crc, _u8p), _ptr(cbd, _u8p), cbd.shape[1], _ptr(data, _u8p), noi, ctypes.byref(avg))
    return ret, data, list(noi), avg.value, state


class Reference(_Lib, _PhyMixin):
    """The reference decoder compiled from /root/reference (oracle/_ref)."""

    def _demod_fn(self):
        f = self.lib.srsran_demod_soft_demodulate_s
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, _i16p, ctypes.c_int]
        return f

    def _seq_fn(self):
        f = self.lib.srsran_sequence_apply_s
        f.argtypes = [_i16p, _i16p, ctypes.c_uint32, ctypes.c_uint32]
        return f

    def _predecode(self, scheme, ya, ha, xa, ca, nrx, nports, nlayers, codebook, n, scaling, noise):
        # every buffer separately aligned like srsran_vec_cf_malloc (the SIMD bodies use aligned
        # loads), with slack: the CDD scalar tail writes index n when n is odd (precoding.c:1105-1118)
        P = ctypes.c_void_p
        keep = []

        def buf(src, dtype):
            b = aligned(n + 8, dtype)
            if src is not None:
                b[:n] = src
            keep.append(b)
            return b

        ys = (P * 4)(*[buf(ya[r], np.complex64).ctypes.data if r < nrx else None for r in range(4)])
        hs = ((P * 4) * 4)()
        for p in range(nports):
            for r in range(nrx):
                hs[p][r] = buf(ha[p, r], np.complex64).ctypes.data
        xb = [buf(None, np.complex64) for _ in range(xa.shape[0])]
        cb = [buf(None, np.float32) for _ in range(2)]
        xs = (P * 4)(*[xb[l].ctypes.data if l < len(xb) else None for l in range(4)])
        cs = (P * 2)(cb[0].ctypes.data, cb[1].ctypes.data)
        f = self.lib.srsran_predecoding_type
        f.argtypes = [P, P, P, P] + [ctypes.c_int] * 6 + [ctypes.c_float, ctypes.c_float]
        rc = f(ctypes.addressof(ys), ctypes.addressof(hs), ctypes.addressof(xs), ctypes.addressof(cs), nrx, nports,
               nlayers, codebook, n, scheme, scaling, noise)
        for l in range(xa.shape[0]):
            xa[l] = xb[l][:n]
        ca[0] = cb[0][:n]
        ca[1] = cb[1][:n]
        return rc

    def _demod_b_fn(self):
        return self.lib.srsran_demod_soft_demodulate_b

    def _seq_c_fn(self):
        return self.lib.srsran_sequence_apply_c

    def csi_correction(self, mod, csi, e, llr8=False):
        """csi_correction (pdsch.c:523-618) restated in ref_pdsch_tx_harness.c and built with the reference's
        flags; e int16 (int8 with llr8) LLRs of one codeword, csi nof_bits / Qm values."""
        dt = np.int8 if llr8 else np.int16
        ea = aligned(len(e) + 16, dt)
        ea[:len(e)] = e
        ca = aligned(len(csi) + 8, np.float32)
        ca[:len(csi)] = csi
        f = self.lib.ref_csi_correction
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
        f(mod, ca.ctypes.data, ea.ctypes.data, len(e), 1 if llr8 else 0)
        return ea[:len(e)].copy()

    def evm_b(self, mod, sym, llr, nof_bits, max_bits):
        """srsran_evm_run_b (evm.h) on int8 demodulated LLRs."""
        s = aligned(len(sym) + 8, np.complex64)
        s[:len(sym)] = sym
        l = aligned(len(llr) + 16, np.int8)
        l[:len(llr)] = llr
        f = self.lib.ref_evm_run_b
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        f.restype = ctypes.c_float
        return f(mod, s.ctypes.data, l.ctypes.data, nof_bits, max_bits)

    def sequence_pdsch_apply_s(self, llr, rnti, q, nslot, cell_id):
        x = aligned(len(llr), np.int16)
        x[:] = llr
        out = aligned(len(llr), np.int16)
        f = self.lib.srsran_sequence_pdsch_apply_s
        f.argtypes = [_i16p, _i16p, ctypes.c_uint16, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        f(_ptr(x, _i16p), _ptr(out, _i16p), rnti, q, nslot, cell_id, len(llr))
        return out.copy()

    def __init__(self):
        super().__init__(REF_SO, "ref_", lazy=True)
        L = self.lib
        L.ref_tcod_encode.argtypes = [ctypes.c_uint32, _u8p, _u8p]
        L.ref_rm_turbo_rx_lut.argtypes = [_i16p, _i16p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        L.ref_crc_checksum_byte.argtypes = [ctypes.c_uint32, ctypes.c_int, _u8p, ctypes.c_uint32]
        L.ref_crc_checksum_byte.restype = ctypes.c_uint32

    def encode(self, K, bits):
        bits = np.ascontiguousarray(bits, dtype=np.uint8)
        out = np.zeros(3 * K + 12, dtype=np.uint8)
        if self.lib.ref_tcod_encode(K, _ptr(bits, _u8p), _ptr(out, _u8p)):
            raise ValueError(K)
        return out

    def tdec8_run(self, K, llr, layout_sb=False, nof_iterations=8, trace=False):
        """srsran_tdec_run_all_8bit (AUTO, AVX2 build) on one int8 code block (ref_tdec8_run)."""
        f = self.lib.ref_tdec8_run
        f.argtypes = [ctypes.c_uint32, _i8p, ctypes.c_int, ctypes.c_uint32, _u8p, _i8p]
        f.restype = ctypes.c_int
        sb = layout_sb and tdec8_subblocks(K) > 0
        n = 3 * (K + 32) + 12 if sb else 3 * K + 12
        llr = np.ascontiguousarray(llr, dtype=np.int8)
        assert llr.size >= n
        out = np.zeros(K // 8, dtype=np.uint8)
        tr = np.zeros((nof_iterations, K), dtype=np.int8) if trace else None
        if f(K, _ptr(llr, _i8p), int(bool(layout_sb)), nof_iterations, _ptr(out, _u8p), _ptr(tr, _i8p) if trace else None):
            raise ValueError(f"tdec8_run failed K={K}")
        return (out, tr) if trace else out

    def interleaver(self, K, win):
        """forward / reverse tables of srsran_tc_interl_LTE_gen_interl(K, win) (tc_interl_lte.c:69-107)."""

        class Interl(ctypes.Structure):
            _fields_ = [("forward", _u16p), ("reverse", _u16p), ("max_long_cb", ctypes.c_uint32)]

        h = Interl()
        L = self.lib
        L.srsran_tc_interl_init.argtypes = [ctypes.POINTER(Interl), ctypes.c_uint32]
        L.srsran_tc_interl_LTE_gen_interl.argtypes = [ctypes.POINTER(Interl), ctypes.c_uint32, ctypes.c_uint32]
        L.srsran_tc_interl_free.argtypes = [ctypes.POINTER(Interl)]
        if L.srsran_tc_interl_init(ctypes.byref(h), K) or L.srsran_tc_interl_LTE_gen_interl(ctypes.byref(h), K, win):
            raise ValueError(K)
        fwd = np.ctypeslib.as_array(h.forward, shape=(K,)).copy()
        rev = np.ctypeslib.as_array(h.reverse, shape=(K,)).copy()
        L.srsran_tc_interl_free(ctypes.byref(h))
        return fwd, rev

    def crc_byte(self, poly, order, data, nbits):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        return self.lib.ref_crc_checksum_byte(poly, order, _ptr(data, _u8p), nbits)

    def cbsegm(self, tbs):
        f = self.lib.ref_cbsegm
        f.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
        out = (ctypes.c_uint32 * 9)()
        rc = f(tbs, out)
        return rc, dict(zip(SEGM_FIELDS, list(out)))

    def dlsch_decode(self, tbs, Qm, rv, e_llr, max_iterations, state=None):
        """decode_tb glue over the reference's rm_turbo / turbo decoder / CRC (ref_harness.c)."""
        return _dlsch_decode(self.lib.ref_dlsch_decode_tb, self.cbsegm(tbs)[1], tbs, Qm, rv, e_llr,
                             max_iterations, state)

    def dlsch_decode8(self, tbs, Qm, rv, e_llr, max_iterations, state=None):
        """decode_tb glue over the reference's 8-bit rate de-matching and decoders (ref_dlsch_decode_tb8)."""
        return _dlsch_decode(self.lib.ref_dlsch_decode_tb8, self.cbsegm(tbs)[1], tbs, Qm, rv, e_llr,
                             max_iterations, state, llr8=True)

    def rm_turbo_rx(self, cb_idx, rv, e, softbuf):
        """srsran_rm_turbo_rx_lut (SB layout for window decoders, as the reference build)."""
        e = np.ascontiguousarray(e, dtype=np.int16)
        sb = np.ascontiguousarray(softbuf, dtype=np.int16).copy()
        rc = self.lib.ref_rm_turbo_rx_lut(_ptr(e, _i16p), _ptr(sb, _i16p), e.size, cb_idx, rv)
        if rc:
            raise ValueError(rc)
        return sb

    def rm_turbo_tx(self, K, rv, coded, E):
        f = self.lib.ref_rm_turbo_tx
        f.argtypes = [_u8p, ctypes.c_uint32, _u8p, ctypes.c_uint32, ctypes.c_uint32]
        coded = np.ascontiguousarray(coded, dtype=np.uint8)
        out = np.zeros(E, dtype=np.uint8)
        if f(_ptr(coded, _u8p), K, _ptr(out, _u8p), E, rv):
            raise ValueError(K)
        return out


def crs_nsym(nof_dw, cp=0):
    """srsran_refsignal_cs_nof_symbols (refsignal_dl.c:169-226) in a TDD special subframe with nof_dw DwPTS
    symbols: (ports 0-1, ports 2-3)"""
    if nof_dw >= (10 if cp else 12):
        return (4, 2)
    if nof_dw >= (8 if cp else 9):
        return (3, 2)
    if nof_dw >= (4 if cp else 5):
        return (2, 1)
    return (1, 1)


def ref_available():
    return os.path.exists(REF_SO)


def make_llrs(K, ebno_db, rng, n=1, encoder=None):
    """Synthetic AWGN code blocks in the reference test's convention.

    turbodecoder_test.c:217-255: BPSK bit1 -> +1, bit0 -> -1, noise variance
    var = 10^(-(EbNo + 10log10(1/3))/10), LLR = (int16)(100*y) (truncation).
    Returns (bits[n,K] uint8, llr[n,3K+12] int16).
    """
    enc = encoder or Oracle()
    bits = rng.integers(0, 2, size=(n, K), dtype=np.uint8)
    esno = ebno_db + 10 * np.log10(1.0 / 3.0)
    var = 10 ** (-esno / 10)
    llr = np.zeros((n, 3 * K + 12), dtype=np.int16)
    for i in range(n):
        sym = enc.encode(K, bits[i]).astype(np.float32) * 2 - 1
        y = sym + rng.standard_normal(sym.shape).astype(np.float32) * np.float32(np.sqrt(var))
        llr[i] = np.trunc(np.float32(100) * y).astype(np.int16)
    return bits, llr
