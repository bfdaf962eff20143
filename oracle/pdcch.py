"""oracle/pdcch.py -- TEST INFRASTRUCTURE ONLY: ctypes views of the PDCCH / PCFICH checkers.

  Ref : the reference's own control-channel code compiled into oracle/_ref/libsrsref.so
        (oracle/ref_pdcch_harness.c: regs.c tables, pcfich.c / pdcch.c encode and decode,
        viterbi.c, rm_conv.c)
  Ora : oracle/pdcch_oracle.c, the plain-C restatement the GPU kernel follows
  dci_pack_* : DCI payload packing for test messages (36.212 5.3.3.1; field order of
        phch/dci.c:579-640 (format 1), :710-796 (1A), :1076-1152 (2/2A))
"""
import ctypes
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SO = os.path.join(HERE, "_ref", "libsrsref.so")
ORACLE_SO = os.path.join(HERE, "liboracle.so")

u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
u32 = ctypes.c_uint32

DCI_MAX_BITS = 128
FORMAT0, FORMAT1, FORMAT1A, FORMAT1B, FORMAT1C, FORMAT1D, FORMAT2, FORMAT2A, FORMAT2B = range(9)


def ref_available():
    return os.path.exists(REF_SO)


class Ref:
    def __init__(self):
        L = ctypes.CDLL(REF_SO, mode=os.RTLD_LAZY)
        L.ref_regs_tables.argtypes = [u32, u32, u32, ctypes.c_int, ctypes.c_int, u32p, u32p, u32, u32p]
        L.ref_regs_tables_mi.argtypes = [u32, u32, u32, ctypes.c_int, ctypes.c_int, u32, u32p, u32p, u32, u32p]
        L.ref_regs_tables_opts.argtypes = [u32, u32, u32, ctypes.c_int, ctypes.c_int, u32, ctypes.c_int, u32p, u32p,
                                           u32, u32p]
        L.ref_set_cp.argtypes = [ctypes.c_int]  # process-global in the harness (normal CP until set)
        L.ref_ctrl_tx.argtypes = [u32, u32, u32, ctypes.c_int, ctypes.c_int, u32, u32, u32, u8p, u32p, u32p, u32p,
                                  u16p, f32p]
        L.ref_ctrl_tx_opts.argtypes = [u32, u32, u32, ctypes.c_int, ctypes.c_int, u32, ctypes.c_int, u32, u32, u32, u8p,
                                       u32p, u32p, u32p, u16p, f32p]
        L.ref_ctrl_rx.argtypes = [u32, u32, u32, ctypes.c_int, ctypes.c_int, u32, u32, f32p, f32p, ctypes.c_float,
                                  ctypes.POINTER(u32), ctypes.POINTER(ctypes.c_float), f32p]
        L.ref_pdcch_decode.argtypes = [u32, u32, f32p, u32, u32, u32, ctypes.c_int, u32, u8p,
                                       ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(ctypes.c_float)]
        L.ref_enb_ctrl_tx.argtypes = [u32, u32, u32, ctypes.c_int, ctypes.c_int, ctypes.c_int, u32, u32, ctypes.c_int,
                                      u32, u8p, u32p, u32p, u32p, u16p, f32p]
        L.ref_viterbi_decode_f.argtypes = [f32p, u32, u8p]
        L.ref_rm_conv_rx.argtypes = [f32p, u32, f32p, u32]
        self.L = L

    def set_cp(self, ext):
        """cyclic prefix of the reference cells built from now on (0 normal, 1 extended)"""
        self.L.ref_set_cp(int(ext))

    def regs_tables(self, nof_prb, nof_ports, cell_id, phich_len=0, phich_res=2, phich_mi=1, sf1_6=False):
        """regs.c tables of srsran_regs_init_opts(cell, phich_mi, sf1_6) (regs.c:693-783; sf1_6 =
        mbsfn_or_sf1_6_tdd, the extended-duration PHICH limited to two symbols, regs.c:329-340)"""
        maxre = 4 * 12 * nof_prb
        pc = np.zeros(16, np.uint32)
        pd = np.zeros(3 * maxre, np.uint32)
        nre = np.zeros(3, np.uint32)
        if self.L.ref_regs_tables_opts(nof_prb, nof_ports, cell_id, phich_len, phich_res, phich_mi, int(sf1_6), pc,
                                       pd, maxre, nre) != 16:
            raise RuntimeError("ref_regs_tables failed")
        return pc, [pd[c * maxre:c * maxre + nre[c]].copy() for c in range(3)]

    def ctrl_tx(self, nof_prb, nof_ports, cell_id, tti, cfi, msgs, phich_len=0, phich_res=2, phich_mi=1, sf1_6=False):
        """msgs: list of (bits uint8[nof_bits], L, ncce, rnti).  Returns [port] grids (14, 12 nof_prb).  phich_mi /
        sf1_6: the REG tables of srsran_regs_init_opts (a TDD cell's m_i; its extended-duration subframes 1 / 6)."""
        n = len(msgs)
        pl = np.zeros((max(n, 1), DCI_MAX_BITS), np.uint8)
        nb = np.zeros(max(n, 1), np.uint32)
        Ls = np.zeros(max(n, 1), np.uint32)
        nc = np.zeros(max(n, 1), np.uint32)
        rn = np.zeros(max(n, 1), np.uint16)
        for i, (bits, L, ncce, rnti) in enumerate(msgs):
            pl[i, :len(bits)] = bits
            nb[i], Ls[i], nc[i], rn[i] = len(bits), L, ncce, rnti
        g = np.zeros((nof_ports, 14, 12 * nof_prb), np.complex64)
        gf = g.view(np.float32).reshape(-1)
        if self.L.ref_ctrl_tx_opts(nof_prb, nof_ports, cell_id, phich_len, phich_res, phich_mi, int(sf1_6), tti, cfi,
                                   n, pl.reshape(-1), nb, Ls, nc, rn, gf) != 0:
            raise RuntimeError("ref_ctrl_tx failed")
        return gf.view(np.complex64).reshape(nof_ports, 14, 12 * nof_prb)

    def enb_ctrl_tx(self, nof_prb, nof_ports, cell_id, tti, cfi, msgs, put_base=True, cp=0, phich_len=0, phich_res=2):
        """srsran_enb_dl_put_base's PSS / SSS / PBCH / PCFICH (put_base) and srsran_pdcch_encode of each of
        msgs = [(bits, L, ncce, rnti)] (ref_enb_ctrl_harness.c).  Returns [port] grids (14, 12 nof_prb)."""
        n = len(msgs)
        pl = np.zeros((max(n, 1), DCI_MAX_BITS), np.uint8)
        nb = np.zeros(max(n, 1), np.uint32)
        Ls = np.zeros(max(n, 1), np.uint32)
        nc = np.zeros(max(n, 1), np.uint32)
        rn = np.zeros(max(n, 1), np.uint16)
        for i, (bits, L, ncce, rnti) in enumerate(msgs):
            pl[i, :len(bits)] = bits
            nb[i], Ls[i], nc[i], rn[i] = len(bits), L, ncce, rnti
        g = np.zeros((nof_ports, 14, 12 * nof_prb), np.complex64)
        gf = g.view(np.float32).reshape(-1)
        if self.L.ref_enb_ctrl_tx(nof_prb, nof_ports, cell_id, cp, phich_len, phich_res, tti, cfi, int(put_base), n,
                                  pl.reshape(-1), nb, Ls, nc, rn, gf) != 0:
            raise RuntimeError("ref_enb_ctrl_tx failed")
        return gf.view(np.complex64).reshape(nof_ports, 14, 12 * nof_prb)

    def ctrl_rx(self, nof_prb, nof_ports, cell_id, tti, grids, ce, noise, phich_len=0, phich_res=2):
        """grids: (nrx, 14, 12 nof_prb) complex64; ce: (ports, nrx, 14, 12 nof_prb).  Returns (cfi, corr, llr)."""
        nrx = grids.shape[0]
        g = np.ascontiguousarray(grids, np.complex64).view(np.float32).reshape(-1)
        c = np.ascontiguousarray(ce, np.complex64).view(np.float32).reshape(-1)
        llr = np.zeros(72 * 100, np.float32)
        cfi = u32()
        corr = ctypes.c_float()
        n = self.L.ref_ctrl_rx(nof_prb, nof_ports, cell_id, phich_len, phich_res, nrx, tti, g, c, noise,
                               ctypes.byref(cfi), ctypes.byref(corr), llr)
        if n < 0:
            raise RuntimeError("ref_ctrl_rx failed")
        return cfi.value, corr.value, llr[:72 * n].copy()

    def pdcch_decode(self, tti, cfi, llr, L, ncce, fmt, cif=0):
        """After ctrl_rx: srsran_pdcch_decode_msg + msg_corr -> (nof_bits, payload, crc_rem, corr)."""
        pl = np.zeros(DCI_MAX_BITS, np.uint8)
        rem = ctypes.c_uint16()
        corr = ctypes.c_float()
        llr = np.ascontiguousarray(llr, np.float32)
        nb = self.L.ref_pdcch_decode(tti, cfi, llr, len(llr) // 72, L, ncce, fmt, cif, pl, ctypes.byref(rem),
                                     ctypes.byref(corr))
        if nb < 0:
            raise RuntimeError("ref_pdcch_decode failed")
        return nb, pl[:nb].copy(), rem.value, corr.value

    def viterbi_decode_f(self, x, frame_length):
        out = np.zeros(frame_length, np.uint8)
        self.L.ref_viterbi_decode_f(np.ascontiguousarray(x, np.float32), frame_length, out)
        return out

    def rm_conv_rx(self, x, out_len):
        out = np.zeros(out_len, np.float32)
        self.L.ref_rm_conv_rx(np.ascontiguousarray(x, np.float32), len(x), out, out_len)
        return out


class Ora:
    def __init__(self):
        L = ctypes.CDLL(ORACLE_SO)
        L.ora_viterbi_decode_f.argtypes = [f32p, u32, u8p]
        L.ora_rm_conv_rx.argtypes = [f32p, u32, f32p, u32]
        L.ora_pdcch_dci_decode.argtypes = [f32p, u32, u32, u8p]
        L.ora_pdcch_dci_decode.restype = ctypes.c_uint16
        self.L = L

    def viterbi_decode_f(self, x, frame_length):
        out = np.zeros(frame_length, np.uint8)
        self.L.ora_viterbi_decode_f(np.ascontiguousarray(x, np.float32), frame_length, out)
        return out

    def rm_conv_rx(self, x, out_len):
        out = np.zeros(out_len, np.float32)
        self.L.ora_rm_conv_rx(np.ascontiguousarray(x, np.float32), len(x), out, out_len)
        return out

    def dci_decode(self, e, nof_bits):
        data = np.zeros(nof_bits + 16, np.uint8)
        rem = self.L.ora_pdcch_dci_decode(np.ascontiguousarray(e, np.float32), len(e), nof_bits, data)
        return data[:nof_bits].copy(), rem


# ---------------- DCI packing (test messages) ----------------
def riv_nbits(nof_prb):
    return int(math.ceil(math.log2(nof_prb * (nof_prb + 1) / 2)))


def type0_P(nof_prb):
    return 1 if nof_prb <= 10 else 2 if nof_prb <= 26 else 3 if nof_prb <= 63 else 4


def _bits(v, n):
    return [(v >> (n - 1 - i)) & 1 for i in range(n)]


def riv(L_crb, start, nof_prb):
    """36.213 7.1.6.3 (ra.c:37-47)"""
    if L_crb - 1 <= nof_prb // 2:
        return nof_prb * (L_crb - 1) + start
    return nof_prb * (nof_prb - L_crb + 1) + (nof_prb - 1 - start)


def dci_pack_1a(nof_prb, size, riv_v, mcs, pid, ndi, rv, tpc=0, localized=True):
    b = [1, 0 if localized else 1] + _bits(riv_v, riv_nbits(nof_prb)) + _bits(mcs, 5) + _bits(pid, 3) + [ndi] + \
        _bits(rv, 2) + _bits(tpc, 2)
    return np.array(b + [0] * (size - len(b)), np.uint8)


def dci_pack_0(nof_prb, size, riv_v, mcs, ndi, tpc=0, n_dmrs=0, cqi=0, hop=None, cif=None, csi=None, srs=None,
               ra_type=None):
    """format 0, 36.212 5.3.3.1.1: [CIF] flag 0/1A = 0, hopping flag [+ 1 or 2 hopping bits], RIV,
    MCS, NDI, TPC, DMRS cyclic shift, CQI (or 2-bit CSI) request, [SRS request], [RA type]"""
    b = (_bits(cif, 3) if cif is not None else []) + [0]
    if hop is None:
        b += [0]
        nh = 0
    else:
        nh = 1 if nof_prb < 50 else 2
        b += [1] + _bits(hop, nh)
    b += _bits(riv_v, riv_nbits(nof_prb) - nh) + _bits(mcs, 5) + [ndi] + _bits(tpc, 2) + _bits(n_dmrs, 3)
    b += _bits(csi, 2) if csi is not None else [cqi]
    b += [srs] if srs is not None else []
    b += [ra_type] if ra_type is not None else []
    assert len(b) <= size
    return np.array(b + [0] * (size - len(b)), np.uint8)


def dci_pack_1(nof_prb, size, rbg_mask, mcs, pid, ndi, rv, tpc=0):
    n = int(math.ceil(nof_prb / type0_P(nof_prb)))
    b = ([0] if nof_prb > 10 else []) + _bits(rbg_mask, n) + _bits(mcs, 5) + _bits(pid, 3) + [ndi] + _bits(rv, 2) + \
        _bits(tpc, 2)
    return np.array(b + [0] * (size - len(b)), np.uint8)


def dci_pack_2a(nof_prb, size, rbg_mask, tbs, pid, swap=0, tpc=0, pinfo=None, pinfo_bits=0):
    """tbs: [(mcs, ndi, rv)] x 2"""
    n = int(math.ceil(nof_prb / type0_P(nof_prb)))
    b = ([0] if nof_prb > 10 else []) + _bits(rbg_mask, n) + _bits(tpc, 2) + _bits(pid, 3) + [swap]
    for mcs, ndi, rv in tbs:
        b += _bits(mcs, 5) + [ndi] + _bits(rv, 2)
    if pinfo_bits:
        b += _bits(pinfo or 0, pinfo_bits)
    return np.array(b + [0] * (size - len(b)), np.uint8)


# ---- DL resource allocation type 2 (TEST INFRASTRUCTURE): ra_dl.c:225-316 and ra.c:81-124 restated ----
def type2_ngap(nof_prb, ngap1):
    """36.211 Table 6.2.3.2-1 (ra.c:81-103)"""
    if nof_prb <= 10:
        return nof_prb // 2
    if nof_prb == 11:
        return 4
    for lim, g in ((19, 8), (26, 12), (44, 18), (49, 27)):
        if nof_prb <= lim:
            return g
    if nof_prb <= 63:
        return 27 if ngap1 else 9
    if nof_prb <= 79:
        return 32 if ngap1 else 16
    return 48 if ngap1 else 16


def type2_n_vrb_dl(nof_prb, ngap1):
    """N_VRB^DL (36.211 6.2.3.2; ra.c:115-124)"""
    g = type2_ngap(nof_prb, ngap1)
    return 2 * min(g, nof_prb - g) if ngap1 else (nof_prb // g) * 2 * g


def riv_decode(riv_v, nof_prb, nof_vrb):
    """srsran_ra_type2_from_riv (ra.c:49-57): (L_crb, RB_start).  Its test L > nof_vrb - RB_start is unsigned: with
    RB_start > nof_vrb (distributed allocations, N_VRB < N_PRB) it wraps and the RIV is not flipped."""
    L, start = riv_v // nof_prb + 1, riv_v % nof_prb
    if L > (nof_vrb - start) % (1 << 32):
        L, start = nof_prb - riv_v // nof_prb + 1, nof_prb - riv_v % nof_prb - 1
    return L, start


def type2_prbs(nof_prb, riv_v, distributed, ngap1=True, fmt1c=False):
    """PRBs of a type 2 allocation per slot: ([slot 0 PRBs], [slot 1 PRBs]) or None where the reference refuses.
    Distributed VRBs by 36.211 6.2.3.2's interleaver, with the reference's N~_VRB for N_gap,2: it takes
    2 x N_VRB(N_gap,1) (ra_dl.c:257-260) where 36.211 has 2 N_gap."""
    P = type0_P(nof_prb)
    nof_vrb = type2_n_vrb_dl(nof_prb, ngap1) if distributed else nof_prb
    nof_prb_t2, step = nof_prb, 1
    if fmt1c:
        step = 2 if nof_prb < 50 else 4
        nof_vrb //= step
        nof_prb_t2 = nof_vrb
    L, start = riv_decode(riv_v, nof_prb_t2, nof_vrb)
    L, start = L * step, start * step
    if not distributed:
        prbs = list(range(start, start + L))
        return prbs, prbs
    nt = type2_n_vrb_dl(nof_prb, True) * (1 if ngap1 else 2)
    gap = type2_ngap(nof_prb, ngap1)
    n_row = -(-nt // (4 * P)) * P
    n_null = 4 * n_row - nt
    s0, s1 = [], []
    for n_vrb in range(start, start + L):
        v, blk = n_vrb % nt, nt * (n_vrb // nt)
        p1 = 2 * n_row * (v % 2) + v // 2 + blk
        p2 = n_row * (v % 4) + v // 4 + blk
        if n_null and v >= nt - n_null:
            ev = p1 - n_row if v % 2 == 1 else p1 - n_row + n_null // 2
        elif n_null and v % 4 >= 2:
            ev = p2 - n_null // 2
        else:
            ev = p2
        od = (ev + nt // 2) % nt + blk
        for n_t, out in ((ev, s0), (od, s1)):
            prb = n_t if n_t < nt // 2 else n_t + gap - nt // 2
            if not 0 <= prb < nof_prb:
                return None
            out.append(prb)
    return s0, s1


TBS_FORMAT1C = (40, 56, 72, 120, 136, 144, 176, 208, 224, 256, 280, 296, 328, 336, 392, 488, 552, 600, 632, 696, 776,
                840, 904, 1000, 1064, 1128, 1224, 1288, 1384, 1480, 1608, 1736)  # 36.213 Table 7.1.7.2.3-1
