"""numpy OFDM transmitter / receiver with srsRAN's conventions (TEST INFRASTRUCTURE ONLY).

FFTW is not available here and no reference test pins its outputs, so the OFDM
stage is checked against numpy's FFT (double precision) and by TX -> RX round trips:
  - symbol i of slot s occupies [s*slot + cp0 + i*(N + cp), +N) (ofdm.c:169-181, 36.211 6.12)
  - cp0 = ceil(160 N / 2048), cp = ceil(144 N / 2048) (phy_common.h:125-127); extended CP
    (cp=1): 6 symbols a slot, cp0 = cp = ceil(512 N / 2048) (SRSRAN_CP_LEN_EXT)
  - receiver: forward DFT, unnormalised, grid = [X[N-nre/2 ..], X[1 .. nre/2]] (ofdm.c:497-498)
  - transmitter: the inverse mapping with an IFFT scaled by 1/N, so rx(tx(grid)) == grid
  - CFO: z[n] = x[n] exp(j 2 pi f n), n from the subframe start (cfo.c:96-107); ref_apply_cfo runs the
    reference's own srsran_vec_apply_cfo (vector_simd.c:1723-1774, compiled into _ref/libsrsref.so), whose
    float phasor recurrence drifts from the exact exponential by up to ~1e-4 over a 20 MHz subframe
"""
import ctypes
import math
import os

import numpy as np


def nsymb(ext=0):
    return 6 if ext else 7


def cp_lens(N, ext=0):
    if ext:
        return math.ceil(512 * N / 2048), math.ceil(512 * N / 2048)
    return math.ceil(160 * N / 2048), math.ceil(144 * N / 2048)


def sf_len(N, ext=0):
    cp0, cp = cp_lens(N, ext)
    ns = nsymb(ext)
    return 2 * (ns * N + cp0 + (ns - 1) * cp)


def symbol_starts(N, ext=0):
    cp0, cp = cp_lens(N, ext)
    ns = nsymb(ext)
    slot = ns * N + cp0 + (ns - 1) * cp
    return [s * slot + cp0 + i * (N + cp) for s in range(2) for i in range(ns)]


def mbsfn_symbol_starts(N, nr):
    """sample offsets of the 12 symbols of an MBSFN subframe (ofdm_rx_slot_mbsfn, ofdm.c:522-535, then slot 1 of
    the extended-CP layout): slot 0's first nr symbols after normal cyclic prefixes, the guard
    SRSRAN_NON_MBSFN_REGION_GUARD_LENGTH (phy_common.h:166-169) before symbol nr, extended cyclic prefixes after"""
    cpn0, cpn = cp_lens(N, 0)
    cpe = cp_lens(N, 1)[0]
    out, pos = [], 0
    for i in range(6):
        if i == nr:
            pos += cpe - cpn0 if nr == 1 else 2 * cpe - cpn0 - cpn
        pos += cpe if i >= nr else (cpn0 if i == 0 else cpn)
        out.append(pos)
        pos += N
    return out + symbol_starts(N, 1)[6:]


def ofdm_rx_mbsfn(x, N, nre, nr):
    x = np.asarray(x, np.complex128)
    out = np.zeros((12, nre), np.complex128)
    for l, st in enumerate(mbsfn_symbol_starts(N, nr)):
        X = np.fft.fft(x[st:st + N])
        out[l, : nre // 2] = X[N - nre // 2:]
        out[l, nre // 2:] = X[1: nre // 2 + 1]
    return out.reshape(-1)


def ofdm_tx_mbsfn(grid, N, nre, nr):
    """the eNB's MBSFN modulator (ofdm_tx_slot_mbsfn, ofdm.c:652-674): the inverse of ofdm_rx_mbsfn; the guard
    samples stay zero"""
    grid = np.asarray(grid, np.complex128).reshape(12, nre)
    cpn0, cpn = cp_lens(N, 0)
    cpe = cp_lens(N, 1)[0]
    x = np.zeros(sf_len(N, 1), np.complex128)
    for l, st in enumerate(mbsfn_symbol_starts(N, nr)):
        X = np.zeros(N, np.complex128)
        X[N - nre // 2:] = grid[l, : nre // 2]
        X[1: nre // 2 + 1] = grid[l, nre // 2:]
        t = np.fft.ifft(X)
        c = cpe if (l >= nr or l >= 6) else (cpn0 if l == 0 else cpn)
        x[st - c: st] = t[N - c:]
        x[st: st + N] = t
    return x


def ofdm_rx(x, N, nre, normalize=False, ext=0):
    x = np.asarray(x, np.complex128)
    out = np.zeros((2 * nsymb(ext), nre), np.complex128)
    for l, st in enumerate(symbol_starts(N, ext)):
        X = np.fft.fft(x[st:st + N])
        out[l, : nre // 2] = X[N - nre // 2:]
        out[l, nre // 2:] = X[1: nre // 2 + 1]
    if normalize:
        out /= math.sqrt(N)
    return out.reshape(-1)


def ofdm_tx(grid, N, nre, ext=0):
    ns = nsymb(ext)
    grid = np.asarray(grid, np.complex128).reshape(2 * ns, nre)
    cp0, cp = cp_lens(N, ext)
    x = np.zeros(sf_len(N, ext), np.complex128)
    for l, st in enumerate(symbol_starts(N, ext)):
        X = np.zeros(N, np.complex128)
        X[N - nre // 2:] = grid[l, : nre // 2]
        X[1: nre // 2 + 1] = grid[l, nre // 2:]
        t = np.fft.ifft(X)
        c = cp0 if l % ns == 0 else cp
        x[st - c: st] = t[N - c:]
        x[st: st + N] = t
    return x


def cfo(x, f):
    n = np.arange(len(x))
    return np.asarray(x, np.complex128) * np.exp(2j * np.pi * f * n)


_REF = None


def ref_available():
    return os.path.exists(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref", "libsrsref.so"))


def ref_apply_cfo(x, f):
    """srsran_cfo_correct(h, x, z, f) of the reference (SRSRAN_CFO_USE_EXP_TABLE = 0, cfo.c:33, 105):
    srsran_vec_apply_cfo over the whole buffer, 32-byte aligned as srsran_vec_malloc buffers are"""
    global _REF
    if _REF is None:
        L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref", "libsrsref.so"),
                        mode=os.RTLD_LAZY)
        L.srsran_vec_apply_cfo.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_int]
        L.srsran_vec_apply_cfo.restype = None
        _REF = L

    def aligned(n):
        b = np.zeros(n + 8, np.complex64)
        o = (-(b.ctypes.data // 8)) % 4
        return b[o:o + n]

    n = len(x)
    xi, z = aligned(n), aligned(n)
    xi[:] = x
    _REF.srsran_vec_apply_cfo(xi.ctypes.data, ctypes.c_float(f), z.ctypes.data, n)
    return z.copy()


# ---------------- srsran_ofdm_cfg_t options (ofdm.c:151-157, 357-449, 474-519, 585-690) ----------------
def shift_buffer(N, f, ext=0):
    """srsran_ofdm_set_freq_shift's table (ofdm.c:432-443): per symbol, t over cyclic prefix + body,
    cexpf(I 2 M_PI (t - cplen) f / N) -- the argument in double, rounded to float, the exponential in float"""
    cp0, cp = cp_lens(N, ext)
    ns = nsymb(ext)
    out = []
    for l in range(2 * ns):
        c = cp0 if l % ns == 0 else cp
        t = np.arange(N + c, dtype=np.float64)
        y = (2.0 * np.pi * (t - c) * np.float64(np.float32(f)) / N).astype(np.float32)
        out.append(np.cos(y) + 1j * np.sin(y))
    return np.concatenate(out).astype(np.complex64)


def window_n(N, offset, ext=0):
    """window_offset_n = roundf(cp2 x offset), offset clamped to [0, 100] (ofdm.c:151-154)"""
    if offset == 0:
        return 0
    off = min(100.0, max(0.0, offset))
    return int(np.floor(np.float32(cp_lens(N, ext)[1]) * np.float32(off) + np.float32(0.5)))


def phase_table(N, f_hz, ext=0):
    """srsran_ofdm_set_phase_compensation (ofdm.c:380-406): symbol l's phasor exp(-j 2 pi f t_l), t_l the time of
    the end of its cyclic prefix at N x 15 kHz, computed in double and cast to complex float"""
    cp0, cp = cp_lens(N, ext)
    ns = nsymb(ext)
    srate = N * 15e3
    count, out = 0, []
    for l in range(2 * ns):
        count += cp0 if l % ns == 0 else cp
        ph = -2.0 * np.pi * f_hz * (count / srate)
        out.append(np.complex64(np.cos(ph) + 1j * np.sin(ph)))
        count += N
    return np.array(out, np.complex64)


def ofdm_rx_opts(x, N, nre, normalize=False, ext=0, keep_dc=False, freq_shift=0.0, window_offset=0.0,
                 phase_hz=0.0):
    """srsran_ofdm_rx_sf with the options: the input times shift_buffer (ofdm.c:553-555), each symbol's DFT window
    window_offset_n samples into its cyclic prefix and the bins times exp(j 2 pi n k / N) (ofdm.c:491-494), the DC bin
    kept with keep_dc or a shift (ofdm.c:230, 497-498), conj(phase) (x 1/sqrt(N) when normalising) per symbol
    (ofdm.c:501-514).  Returns (grid, the shifted input)."""
    x = np.asarray(x, np.complex128)
    if freq_shift:
        x = x * shift_buffer(N, freq_shift, ext)
    wn = window_n(N, window_offset, ext)
    dc = 0 if (keep_dc or freq_shift) else 1
    ph = phase_table(N, phase_hz, ext) if phase_hz else None
    k = np.arange(N)
    out = np.zeros((2 * nsymb(ext), nre), np.complex128)
    for l, st in enumerate(symbol_starts(N, ext)):
        X = np.fft.fft(x[st - wn: st - wn + N])
        if wn:  # window_offset_buffer: cexpf of the argument rounded to float, as ofdm.c:157 builds it
            y = (np.pi * 2.0 * wn * k / N).astype(np.float32).astype(np.float64)
            X = X * (np.cos(y) + 1j * np.sin(y))
        out[l, : nre // 2] = X[N - nre // 2:]
        out[l, nre // 2:] = X[dc: dc + nre // 2]
        g = 1.0 / math.sqrt(N) if normalize else 1.0
        if ph is not None:
            out[l] *= np.conj(np.complex128(ph[l])) * g
        elif normalize:
            out[l] *= g
    return out.reshape(-1), x


def ofdm_tx_opts(grid, N, nre, normalize=False, ext=0, keep_dc=False, freq_shift=0.0, phase_hz=0.0):
    """srsran_ofdm_tx_sf with the options (ofdm.c:585-690): the unnormalised backward DFT of each symbol's bins
    (DC bin used with keep_dc or a shift), times phase (x 1/sqrt(N) when normalising), the cyclic prefix copied
    after, then the subframe times shift_buffer"""
    ns = nsymb(ext)
    grid = np.asarray(grid, np.complex128).reshape(2 * ns, nre)
    cp0, cp = cp_lens(N, ext)
    dc = 0 if (keep_dc or freq_shift) else 1
    ph = phase_table(N, phase_hz, ext) if phase_hz else None
    x = np.zeros(sf_len(N, ext), np.complex128)
    for l, st in enumerate(symbol_starts(N, ext)):
        X = np.zeros(N, np.complex128)
        X[N - nre // 2:] = grid[l, : nre // 2]
        X[dc: dc + nre // 2] = grid[l, nre // 2:]
        t = np.fft.ifft(X) * N
        g = 1.0 / math.sqrt(N) if normalize else 1.0
        if ph is not None:
            t = t * np.complex128(ph[l]) * g
        elif normalize:
            t = t * g
        c = cp0 if l % ns == 0 else cp
        x[st - c: st] = t[N - c:]
        x[st: st + N] = t
    if freq_shift:
        x = x * shift_buffer(N, freq_shift, ext)
    return x
