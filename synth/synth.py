"""Synthetic eNB-side transmitter: code blocks, DL-SCH transport blocks and complete PDSCH
subframes in the time domain (tests and bench inputs; neither product nor oracle).

Written from 3GPP TS 36.211 / 36.212 (libsynth.so: synth/tx.c) plus numpy for modulation,
precoding, resource mapping and the OFDM transmitter.  The conventions are the ones srsRAN's
receiver assumes (receive side: SURVEY.md 8a):
  - turbo/LLR convention of turbodecoder_test.c:217-255 (bit 1 -> +1, LLR = trunc(100 y))
  - modulation 36.211 7.1 (bit 0 -> positive amplitude), unit average power
  - CDD for 2 ports: y0 = (x0 + x1)/2, y1 = (-1)^i (x0 - x1)/2 (36.211 6.3.4.3, srsRAN scaling)
  - spatial multiplexing rank 2: 36.211 Table 6.3.4.2.3-1 (codebook 0..2)
  - CRS 36.211 6.10.1 (c_init = 2^10 (7 (ns+1) + l + 1)(2 N_ID + 1) + 2 N_ID + 1, m' = m + 110 - N_RB)
  - PDSCH REs in (symbol, subcarrier) order skipping control symbols, CRS of every port and,
    in subframes 0 / 5, PBCH / PSS / SSS in the centre 6 PRBs (even N_RB)
  - OFDM: IFFT / N, symbol l of slot s starts after CP ceil(160N/2048) (l = 0) or ceil(144N/2048)
"""
import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None

QM = {"bpsk": 1, "qpsk": 2, "16qam": 4, "64qam": 6, "256qam": 8}


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "libsynth.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        u32 = ctypes.c_uint32
        L.synth_turbo_encode_natural.argtypes = [u32, P, P]
        L.synth_turbo_encode.argtypes = [u32, P, P, P, P]
        L.synth_dlsch_encode.argtypes = [u32, u32, u32, u32, u32, P, u32, P]
        L.synth_gold.argtypes = [u32, u32, P]
        L.synth_gold.restype = None
        L.synth_crc.argtypes = [u32, P, u32]
        L.synth_crc.restype = u32
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ---------------- channel coding ----------------
def turbo_encode(K, bits):
    """natural srsRAN decoder-input order [d0_i d1_i d2_i], 3K + 12 bits"""
    bits = np.ascontiguousarray(bits, np.uint8)
    out = np.zeros(3 * K + 12, np.uint8)
    if lib().synth_turbo_encode_natural(K, _p(bits), _p(out)):
        raise ValueError(f"K={K} is not an LTE code block size")
    return out


def make_llrs(K, ebno_db, rng, n=1):
    """AWGN code blocks in turbodecoder_test.c's convention (217-255): BPSK bit 1 -> +1,
    var = 10^(-(EbNo + 10 log10(1/3))/10), LLR = (int16)(100 y).  -> (bits[n,K], llr[n,3K+12])"""
    bits = rng.integers(0, 2, size=(n, K), dtype=np.uint8)
    var = 10 ** (-(ebno_db + 10 * np.log10(1.0 / 3.0)) / 10)
    llr = np.zeros((n, 3 * K + 12), dtype=np.int16)
    for i in range(n):
        sym = turbo_encode(K, bits[i]).astype(np.float32) * 2 - 1
        y = sym + rng.standard_normal(sym.shape).astype(np.float32) * np.float32(np.sqrt(var))
        llr[i] = np.trunc(np.float32(100) * y).astype(np.int16)
    return bits, llr


def nof_subblocks(K):
    """sub-blocks of srsRAN's AVX2 window decoder for K (turbodecoder.c:381-393)"""
    if K % 16 == 0 and K > 800:
        return 16
    if K % 8 == 0 and K > 400:
        return 8
    return 0


def natural_to_sb(K, llr):
    """natural 3K+12 decoder input -> the sub-block layout 3(K+32)+12 that srsran_rm_turbo_rx_lut
    writes for window decoders (rm_turbo.c:249-273): d^(j)_n goes to j(K+32) + (n % L) nsb + n / L,
    L = K / nsb; the 12 tail values follow at 3(K+32)."""
    llr = np.asarray(llr)
    nsb = nof_subblocks(K)
    if nsb == 0:
        return llr.copy()
    L = K // nsb
    n = np.arange(K)
    pos = (n % L) * nsb + n // L
    out = np.zeros(llr.shape[:-1] + (3 * (K + 32) + 12,), llr.dtype)
    for j in range(3):
        out[..., j * (K + 32) + pos] = llr[..., j: 3 * K: 3]
    out[..., 3 * (K + 32):] = llr[..., 3 * K:]
    return out


def dlsch_encode(tbs, Qm, rv, G, tb_bytes, Nl=1, tb_crc_xor=0):
    """36.212 5.3.2 for one TB -> G coded bits (uint8)"""
    tb = np.ascontiguousarray(tb_bytes, np.uint8)
    assert tb.size >= tbs // 8
    e = np.zeros(G, np.uint8)
    n = lib().synth_dlsch_encode(tbs, Qm, Nl, rv, G, _p(tb), tb_crc_xor, _p(e))
    if n != G:
        raise ValueError(f"dlsch_encode(tbs={tbs}, G={G}) failed ({n})")
    return e


def gold(c_init, n):
    c = np.zeros(n, np.uint8)
    lib().synth_gold(c_init, n, _p(c))
    return c


def crc24a(bits):
    b = np.ascontiguousarray(bits, np.uint8)
    return lib().synth_crc(0x1864CFB, _p(b), b.size)


# ---------------- modulation / precoding ----------------
def modulate(bits, Qm):
    """36.211 7.1: bits -> unit-power symbols (complex64)"""
    b = 1.0 - 2.0 * np.asarray(bits, np.float64).reshape(-1, Qm)
    if Qm == 1:
        s = (b[:, 0] + 1j * b[:, 0]) / math.sqrt(2)
    elif Qm == 2:
        s = (b[:, 0] + 1j * b[:, 1]) / math.sqrt(2)
    elif Qm == 4:
        s = (b[:, 0] * (2 - b[:, 2]) + 1j * b[:, 1] * (2 - b[:, 3])) / math.sqrt(10)
    elif Qm == 6:
        s = (b[:, 0] * (4 - b[:, 2] * (2 - b[:, 4])) + 1j * b[:, 1] * (4 - b[:, 3] * (2 - b[:, 5]))) / math.sqrt(42)
    elif Qm == 8:
        s = (b[:, 0] * (8 - b[:, 2] * (4 - b[:, 4] * (2 - b[:, 6])))
             + 1j * b[:, 1] * (8 - b[:, 3] * (4 - b[:, 5] * (2 - b[:, 7])))) / math.sqrt(170)
    else:
        raise ValueError(Qm)
    return s.astype(np.complex64)


def precode(x, scheme, codebook=0):
    """layers x[L][n] -> ports y[P][n]"""
    x = [np.asarray(v, np.complex128) for v in x]
    if scheme == "port0":
        return [x[0]]
    n = x[0].size
    if scheme == "cdd":
        sgn = np.where(np.arange(n) % 2 == 0, 1.0, -1.0)
        return [(x[0] + x[1]) / 2, sgn * (x[0] - x[1]) / 2]
    if scheme == "diversity":  # 36.211 6.3.3.3 layer mapping + 6.3.4.3 SFBC, 2 ports (x = one codeword)
        d = x[0]
        x0, x1 = d[0::2], d[1::2]
        y0 = np.empty(d.size, np.complex128)
        y1 = np.empty(d.size, np.complex128)
        y0[0::2], y0[1::2] = x0 / math.sqrt(2), x1 / math.sqrt(2)
        y1[0::2], y1[1::2] = -np.conj(x1) / math.sqrt(2), np.conj(x0) / math.sqrt(2)
        return [y0, y1]
    if scheme == "diversity4":  # 36.211 6.3.3.3 (4 layers) + 6.3.4.3 SFBC + FSTD, 4 ports
        d = x[0]
        m = d.size // 4
        xl = [d[j:4 * m:4] for j in range(4)]
        y = [np.zeros(4 * m, np.complex128) for _ in range(4)]
        a = 1 / math.sqrt(2)
        y[0][0::4], y[2][0::4] = xl[0] * a, -np.conj(xl[1]) * a
        y[0][1::4], y[2][1::4] = xl[1] * a, np.conj(xl[0]) * a
        y[1][2::4], y[3][2::4] = xl[2] * a, -np.conj(xl[3]) * a
        y[1][3::4], y[3][3::4] = xl[3] * a, np.conj(xl[2]) * a
        return y
    if scheme == "sm":
        W = {0: np.array([[1, 0], [0, 1]]) / math.sqrt(2), 1: np.array([[1, 1], [1, -1]]) / 2,
             2: np.array([[1, 1], [1j, -1j]]) / 2}[codebook]
        return [W[0, 0] * x[0] + W[0, 1] * x[1], W[1, 0] * x[0] + W[1, 1] * x[1]]
    raise ValueError(scheme)


# ---------------- resource grid ----------------
def crs_shift(port, l, ns=0):
    """v of 36.211 6.10.1.2 for symbol l (0..6) of slot ns"""
    if port == 0:
        return 0 if l == 0 else 3
    if port == 1:
        return 3 if l == 0 else 0
    if port == 2:
        return 3 * (ns % 2)
    if port == 3:
        return 3 + 3 * (ns % 2)
    raise ValueError(port)


def crs_symbols(nports, nsymb=7):
    return [0, nsymb - 3] if nports <= 2 else [0, 1, nsymb - 3]


def crs_values(cell_id, nof_prb, ns, l, cp=0):
    # 36.211 6.10.1.1: N_CP = 1 normal, 0 extended cyclic prefix
    c = gold((1 << 10) * (7 * (ns + 1) + l + 1) * (2 * cell_id + 1) + 2 * cell_id + (0 if cp else 1), 4 * 110)
    m = np.arange(2 * nof_prb) + 110 - nof_prb
    return ((1 - 2.0 * c[2 * m]) + 1j * (1 - 2.0 * c[2 * m + 1])) / math.sqrt(2)


def crs_grid(cell_id, nof_prb, nports, port, sf_idx, cp=0, nsymb_tx=None):
    """port's CRS in a (2 nsymb, 12 N_RB) grid (nsymb 7, or 6 with cp=1 extended); ports 2 / 3 in l = 1;
    nsymb_tx: only the first nsymb_tx symbols are transmitted (a TDD special subframe's DwPTS)"""
    ns = 6 if cp else 7
    g = np.zeros((2 * ns, 12 * nof_prb), np.complex128)
    for s in range(2):
        for l in ([0, ns - 3] if port < 2 else [1]):
            if nsymb_tx is not None and ns * s + l >= nsymb_tx:
                continue
            k = 6 * np.arange(2 * nof_prb) + (crs_shift(port, 0 if l == 0 else 4, s) + cell_id % 6) % 6
            g[ns * s + l, k] = crs_values(cell_id, nof_prb, 2 * sf_idx + s, l, cp)
    return g


# ---------------- TDD frame structure (36.211 4.2) ----------------
TDD_PATTERN = ("DSUUUDSUUU", "DSUUDDSUUD", "DSUDDDSUDD", "DSUUUDDDDD", "DSUUDDDDDD", "DSUDDDDDDD", "DSUUUDSUUD")
TDD_DWPTS = (3, 9, 10, 11, 12, 3, 9, 10, 11, 6)  # Table 4.2-1, normal CP (srsRAN uses these for both CPs)


def dwpts(tdd, sf_idx):
    """OFDM symbols a TDD subframe transmits on the downlink: all of a D subframe, the DwPTS of an S one, none of a
    U one (tdd = (uplink-downlink configuration, special-subframe configuration))"""
    t = TDD_PATTERN[tdd[0]][sf_idx]
    return 14 if t == "D" else TDD_DWPTS[tdd[1]] if t == "S" else 0


def pdsch_mask(nof_prb, nports, cell_id, cfi, sf_idx, prb=None, cp=0, tdd=None):
    """(2 nsymb, 12 N_RB) bool: REs that carry PDSCH.  tdd = (sf_config, ss_config): a TDD cell, whose SSS is the
    last symbol of subframes 0 / 5 and PSS the third symbol of subframes 1 / 6, and whose special subframes carry
    the PDSCH in their DwPTS symbols only."""
    assert nof_prb % 2 == 0 or sf_idx not in ((0, 5) if tdd is None else (0, 1, 5, 6)), \
        "odd N_RB centre PRBs not generated"
    ns = 6 if cp else 7
    nre = 12 * nof_prb
    m = np.zeros((2 * ns, nre), bool)
    prb = np.ones(nof_prb, bool) if prb is None else np.asarray(prb, bool)
    m[:, np.repeat(prb, 12)] = True
    m[: cfi + (1 if nof_prb < 10 else 0)] = False
    k = np.arange(nre)
    for s in range(2):
        for l in crs_symbols(nports, ns):
            if nports == 1:
                m[ns * s + l, (k % 6) == (crs_shift(0, 0 if l == 0 else 4) + cell_id % 6) % 6] = False
            else:
                m[ns * s + l, (k % 3) == cell_id % 3] = False
    lo, hi = 12 * (nof_prb // 2 - 3), 12 * (nof_prb // 2 + 3)
    if tdd is None:
        if sf_idx in (0, 5):
            m[ns - 2:ns, lo:hi] = False  # SSS, PSS
    else:
        if sf_idx in (0, 5):
            m[2 * ns - 1, lo:hi] = False  # SSS
        if sf_idx in (1, 6):
            m[2, lo:hi] = False  # PSS
        m[dwpts(tdd, sf_idx):] = False  # GP / UpPTS of a special subframe
    if sf_idx == 0:
        m[ns:ns + 4, lo:hi] = False  # PBCH
    return m


def pss_sequence(n_id_2):
    """36.211 6.11.1.1: the length-62 Zadoff-Chu sequence d_u(n) of root u = 25 / 29 / 34"""
    u = (25, 29, 34)[n_id_2]
    n = np.arange(62)
    e = np.where(n < 31, n * (n + 1), (n + 1) * (n + 2))
    return np.exp(-1j * np.pi * u * e / 63)


def sss_sequence(cell_id, sf_idx):
    """36.211 6.11.2.1: d(0..61) of subframe 0 or 5 (m-sequences s, c, z from x^5 + x^2 + 1, x^5 + x^3 + 1,
    x^5 + x^4 + x^2 + x + 1)"""
    n1, n2 = cell_id // 3, cell_id % 3

    def mseq(taps):
        x = [0, 0, 0, 0, 1]
        for i in range(26):
            x.append(sum(x[i + t] for t in taps) % 2)
        return 1 - 2 * np.array(x)

    s_t, c_t, z_t = mseq((2, 0)), mseq((3, 0)), mseq((4, 2, 1, 0))
    qp = n1 // 30
    q = (n1 + qp * (qp + 1) // 2) // 30
    mp = n1 + q * (q + 1) // 2
    m0 = mp % 31
    m1 = (m0 + mp // 31 + 1) % 31
    n = np.arange(31)
    s0, s1 = s_t[(n + m0) % 31], s_t[(n + m1) % 31]
    c0, c1 = c_t[(n + n2) % 31], c_t[(n + n2 + 3) % 31]
    z1m0, z1m1 = z_t[(n + m0 % 8) % 31], z_t[(n + m1 % 8) % 31]
    d = np.zeros(62)
    if sf_idx == 0:
        d[0::2], d[1::2] = s0 * c0, s1 * c1 * z1m0
    else:
        d[0::2], d[1::2] = s1 * c0, s0 * c1 * z1m1
    return d


def sync_grid(nof_prb, cell_id, sf_idx, cp=0, tdd=None):
    """(2 nsymb, 12 N_RB) grid with the PSS / SSS of the subframe (every port transmits them, enb_dl.c:333-343):
    FDD -- SSS, PSS in the last two symbols of slot 0 of subframes 0 / 5; TDD -- SSS in the last symbol of
    subframes 0 / 5, PSS in the third symbol of subframes 1 / 6.  The 5 subcarriers either side stay empty."""
    ns = 6 if cp else 7
    g = np.zeros((2 * ns, 12 * nof_prb), np.complex128)
    k = 6 * nof_prb - 31 + np.arange(62)
    if tdd is None:
        if sf_idx in (0, 5):
            g[ns - 2, k] = sss_sequence(cell_id, sf_idx)
            g[ns - 1, k] = pss_sequence(cell_id % 3)
    else:
        if sf_idx in (0, 5):
            g[2 * ns - 1, k] = sss_sequence(cell_id, sf_idx)
        if sf_idx in (1, 6):
            g[2, k] = pss_sequence(cell_id % 3)
    return g


def ofdm_tx(grid, N, cp=0):
    ns = 6 if cp else 7
    grid = np.asarray(grid).reshape(2 * ns, -1)
    nre = grid.shape[1]
    if cp:
        cp0 = cpl = math.ceil(512 * N / 2048)
    else:
        cp0, cpl = math.ceil(160 * N / 2048), math.ceil(144 * N / 2048)
    out = []
    for l in range(2 * ns):
        X = np.zeros(N, np.complex128)
        X[N - nre // 2:] = grid[l, : nre // 2]
        X[1: nre // 2 + 1] = grid[l, nre // 2:]
        t = np.fft.ifft(X)
        c = cp0 if l % ns == 0 else cpl
        out += [t[N - c:], t]
    return np.concatenate(out)


# ---------------- MBSFN subframes (36.211 6.10.2 as srsRAN's eNB places them) ----------------
def mbsfn_rs(area, nof_prb, sf_idx):
    """the MBSFN reference signal of subframe sf_idx, area N_MBSFN: (3, 6 N_RB) for the grid symbols 2 / 6 / 10 of
    the extended-CP layout -- c_init = 2^9 (7 (ns + 1) + l + 1)(2 N_MBSFN + 1) + N_MBSFN with l = symbol mod 6 of slot
    ns, r(m) = (1 - 2c(2m') + j (1 - 2c(2m' + 1))) / sqrt 2, m' = m + 3 (N_RB^max - N_RB)"""
    out = np.zeros((3, 6 * nof_prb), np.complex128)
    for i, sym in enumerate((2, 6, 10)):
        ns = 2 * sf_idx + (0 if sym < 6 else 1)
        c = gold((1 << 9) * (7 * (ns + 1) + sym % 6 + 1) * (2 * area + 1) + area, 20 * 110)
        m = np.arange(6 * nof_prb) + 3 * (110 - nof_prb)
        out[i] = ((1 - 2.0 * c[2 * m]) + 1j * (1 - 2.0 * c[2 * m + 1])) / math.sqrt(2)
    return out


def mbsfn_grid(nof_prb, cell_id, sf_idx, area, non_mbsfn_region, rng=None):
    """port 0's (12, 12 N_RB) grid of an MBSFN subframe as srsRAN's eNB fills it (enb_dl.c:345-356,
    srsran_refsignal_mbsfn_put_sf refsignal_dl.c:316-348): the CRS of symbol 0, the MBSFN reference signals at
    subcarriers 2i, 2i + 1, 2i of symbols 2 / 6 / 10, and (rng given) QPSK PMCH symbols on the other REs of the
    MBSFN region (symbols >= non_mbsfn_region).  The control region's PCFICH / PDCCH are the caller's."""
    nre = 12 * nof_prb
    g = np.zeros((12, nre), np.complex128)
    if rng is not None:
        b = rng.integers(0, 2, (12 - non_mbsfn_region, 2 * nre))
        g[non_mbsfn_region:] = ((1 - 2.0 * b[:, 0::2]) + 1j * (1 - 2.0 * b[:, 1::2])) / math.sqrt(2)
    rs = mbsfn_rs(area, nof_prb, sf_idx)
    for i, sym in enumerate((2, 6, 10)):
        g[sym] = 0 if rng is None else g[sym]
        g[sym, (1 if sym == 6 else 0) + 2 * np.arange(6 * nof_prb)] = rs[i]
    k = 6 * np.arange(2 * nof_prb) + (crs_shift(0, 0) + cell_id % 6) % 6
    g[0, k] = crs_values(cell_id, nof_prb, 2 * sf_idx, 0)
    return g


def ofdm_tx_mbsfn(grid, N, non_mbsfn_region):
    """srsRAN's MBSFN modulator (ofdm_tx_slot_mbsfn, ofdm.c:652-674, then slot 1 with extended CP): slot 0's first
    non_mbsfn_region symbols with normal cyclic prefixes, zero guard samples, extended-CP symbols after"""
    grid = np.asarray(grid).reshape(12, -1)
    nre = grid.shape[1]
    cpn0, cpn, cpe = math.ceil(160 * N / 2048), math.ceil(144 * N / 2048), math.ceil(512 * N / 2048)
    nr = non_mbsfn_region
    out = []
    for l in range(12):
        X = np.zeros(N, np.complex128)
        X[N - nre // 2:] = grid[l, : nre // 2]
        X[1: nre // 2 + 1] = grid[l, nre // 2:]
        t = np.fft.ifft(X)
        if l < 6 and l == nr:
            out.append(np.zeros(cpe - cpn0 if nr == 1 else 2 * cpe - cpn0 - cpn))
        c = cpe if (l >= 6 or l >= nr) else (cpn0 if l == 0 else cpn)
        out += [t[N - c:], t]
    return np.concatenate(out)


def symbol_sz(nof_prb, standard=True):
    """srsran_symbol_sz (phy_common.c:340-385): standard rates = power-of-two sizes (1536 for 15 MHz);
    otherwise the reference's default 3/4 rates (384 / 768 / 1536 for 25 / 50 / 100 PRB)."""
    sizes = (512, 1024, 1536, 2048) if standard else (384, 768, 1024, 1536)
    for p, n in zip((6, 15, 25, 52, 79, 110), (128, 256) + sizes):
        if nof_prb <= p:
            return n
    raise ValueError(nof_prb)


def pdsch_seed(rnti, q, ns, cell_id):
    return (rnti << 14) + (q << 13) + ((ns // 2) << 9) + cell_id


# ---------------- PCFICH (36.211 6.7, 36.212 5.3.4) ----------------
CFI_CODEWORDS = [[(i % 3) != 0 for i in range(32)], [(i % 3) != 1 for i in range(32)],
                 [(i % 3) != 2 for i in range(32)]]


def pcfich_res(nof_prb, cell_id):
    """Grid indices (symbol 0) of the 16 PCFICH REs in mapping order: 4 REGs of 36.211 6.7.4, each
    the 6 subcarriers at k0 minus the two reference-signal positions (v_shift mod 3, + 3)."""
    vo = cell_id % 3
    k_hat = 6 * (cell_id % (2 * nof_prb))
    out = []
    for q in range(4):
        k0 = (k_hat + (q * nof_prb // 2) * 6) % (12 * nof_prb)
        out += [k0 + i for i in range(6) if i not in (vo, vo + 3)]
    return np.array(out)


def pcfich_grids(nof_prb, cell_id, nports, sf_idx, cfi, cp=0):
    """Per-port (2 nsymb, 12 N_RB) grids carrying only the PCFICH of `cfi`."""
    bits = np.array(CFI_CODEWORDS[cfi - 1], np.uint8) ^ gold((sf_idx + 1) * (2 * cell_id + 1) * 512 + cell_id, 32)
    d = modulate(bits, 2)
    ports = precode([d], "diversity") if nports == 2 else precode([d], "diversity4") if nports == 4 else [d]
    k = pcfich_res(nof_prb, cell_id)
    grids = []
    for p in range(nports):
        g = np.zeros((12 if cp else 14, 12 * nof_prb), np.complex128)
        g[0, k] = ports[p]
        grids.append(g)
    return grids


def pdsch_subframe(nof_prb, cell_id, nports, tti, cfi, rnti, tbs, Qm, rv, payloads, scheme="cdd", codebook=1,
                   nrx=2, snr_db=None, rng=None, N=None, channel=None, cfo=0.0, pcfich=True, ctrl=None, cp=0,
                   sync=False, tdd=None, delay=0.0):
    """One PDSCH subframe through OFDM and a static MIMO channel.

    payloads: one uint8 array (tbs/8 bytes) per codeword.  channel: (nrx, nports) complex matrix
    (default: [[1, 1], [1, -1]] for 2 ports as phy_dl_test.c:568-583 uses, ones for 1 port).
    pcfich: also transmit the PCFICH of `cfi`; ctrl: optional per-port (14, 12 N_RB) grids added
    before the OFDM modulator (e.g. a PDCCH control region); cp=1: extended cyclic prefix;
    sync: also transmit the PSS / SSS (every port, as the reference eNB); tdd = (sf_config, ss_config): a TDD cell
    (TDD sync-signal positions; a special subframe transmits its DwPTS symbols only); delay: a timing error of that
    many samples (fractional), as a phase ramp over the subcarriers of every symbol.
    Returns (samples[nrx, sf_len] complex64, nof_re)."""
    N = N or symbol_sz(nof_prb)
    sf_idx = tti % 10
    nsymb_tx = None if tdd is None else dwpts(tdd, sf_idx)
    if nsymb_tx == 0:
        raise ValueError(f"subframe {sf_idx} is an uplink subframe of TDD configuration {tdd[0]}")
    mask = pdsch_mask(nof_prb, nports, cell_id, cfi, sf_idx, cp=cp, tdd=tdd)
    nof_re = int(mask.sum())
    layers = []
    for q, pl in enumerate(payloads):
        G = nof_re * Qm
        e = dlsch_encode(tbs, Qm, rv, G, pl, Nl=2 if scheme in ("diversity", "diversity4") else 1)
        c = gold(pdsch_seed(rnti, q, 2 * sf_idx, cell_id), G)
        layers.append(modulate(e ^ c, Qm))
    ports = precode(layers, scheme, codebook)
    if len(ports) != nports:
        raise ValueError("scheme / port count mismatch")
    tx = []
    pc = pcfich_grids(nof_prb, cell_id, nports, sf_idx, cfi, cp) if pcfich else None
    sg = sync_grid(nof_prb, cell_id, sf_idx, cp, tdd) if sync else None
    for p in range(nports):
        g = crs_grid(cell_id, nof_prb, nports, p, sf_idx, cp, nsymb_tx)
        g[mask] = ports[p]
        if pc is not None:
            g = g + pc[p]
        if ctrl is not None:
            g = g + ctrl[p]
        if sg is not None:
            g = g + sg
        if nsymb_tx is not None:
            g[nsymb_tx:] = 0  # GP / UpPTS
        if delay:
            half = g.shape[1] // 2
            kf = np.concatenate([np.arange(-half, 0), np.arange(1, half + 1)])  # subcarrier frequencies (no DC)
            g = g * np.exp(-2j * np.pi * kf * delay / N)[None, :]
        tx.append(ofdm_tx(g, N, cp))
    H4 = [[1, 0.5j, -0.4, 0.3], [0.3, -0.6j, 1, 0.5]]
    H = np.asarray(channel if channel is not None else
                   ([[1, 1], [1, -1]] if nports == 2 else H4 if nports == 4 else [[1]] * nrx), np.complex128)
    rx = H @ np.stack(tx)
    if snr_db is not None:
        pw = np.mean(np.abs(rx) ** 2)
        sd = math.sqrt(pw / 10 ** (snr_db / 10) / 2)
        rx = rx + sd * (rng.standard_normal(rx.shape) + 1j * rng.standard_normal(rx.shape))
    if cfo:
        rx = rx * np.exp(2j * np.pi * cfo * np.arange(rx.shape[1]))
    return rx.astype(np.complex64), nof_re
