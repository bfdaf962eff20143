"""The index algebra of the one-wave-per-symbol OFDM kernel (ofdm_kernel.hip ofdm_rx_wave_kernel), modelled in
numpy double precision (no GPU): N = 64 x M (M = 32 at N = 2048, 24 at 1536) --

  lane l holds x[l + 64 m], m < M -> M-point DFT in registers (4 x 8 / 3 x 8: dft_reg) -> twiddle W_N^(l k2)
  -> LDS tile [k2][l] -> lane L = 2 kk + p reads T[kk][2 j + p], j < 32 -> 32-point DFT -> across the lane pair
  X[kk + M k] = Y0[k] + W_64^k Y1[k],  X[kk + M (k + 32)] = Y0[k] - W_64^k Y1[k]

-- equals the DFT, and dft_reg's two-level split (with its inner twiddles taken from the N-point table at stride
N / M) equals the M-point DFT.  The GPU kernel itself is checked against numpy in tests/test_ofdm_gpu.py."""
import numpy as np
import pytest


def W(n, k):
    return np.exp(-2j * np.pi * np.asarray(k) / n)


def dft_reg(a, R, tw_stride, tw):
    """dft_reg<M = 8 R, TS>: m = 8 m1 + m2; R-point DFTs over m1, twiddles tw[TS m2 k1], 8-point DFTs over m2,
    output k = k1 + R k2"""
    M = 8 * R
    b = np.zeros(M, complex)
    for m2 in range(8):
        t = np.fft.fft([a[8 * m1 + m2] for m1 in range(R)])
        for k1 in range(R):
            b[k1 * 8 + m2] = t[k1] * tw[tw_stride * m2 * k1]
    out = np.zeros(M, complex)
    for k1 in range(R):
        u = np.fft.fft(b[k1 * 8:(k1 + 1) * 8])
        for k2 in range(8):
            out[k1 + R * k2] = u[k2]
    return out


@pytest.mark.parametrize("N", [2048, 1536])
def test_wave_fft_decomposition_is_the_dft(N):
    M = N // 64
    R = M // 8
    tw = W(N, np.arange(N))  # the kernel's table: exp(-2 pi i m / N)
    rng = np.random.default_rng(N)
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    T = np.zeros((M, 64), complex)
    for lane in range(64):
        v = dft_reg([x[lane + 64 * m] for m in range(M)], R, 64, tw)
        assert np.abs(v - np.fft.fft([x[lane + 64 * m] for m in range(M)])).max() < 1e-9
        for k2 in range(M):
            assert lane * k2 < N  # the kernel indexes tw[l k2] without a modulo
            T[k2, lane] = v[k2] * tw[lane * k2]
    Y = {}
    for L in range(64):
        kk, p = L >> 1, L & 1
        row = kk if kk < M else 0
        Y[L] = dft_reg([T[row, 2 * j + p] for j in range(32)], 4, N // 32, tw)
    X = np.full(N, np.nan + 0j)
    for L in range(64):
        kk, p = L >> 1, L & 1
        if kk >= M:
            continue  # M = 24: lanes 48..63 idle
        for k in range(32):
            t = Y[L][k] * tw[M * k] if (p and k) else Y[L][k]
            o_lane = L ^ 1
            o = Y[o_lane][k] * tw[M * k] if ((o_lane & 1) and k) else Y[o_lane][k]
            X[kk + M * (k + 32 * p)] = (o - t) if p else (t + o)
    assert not np.isnan(X).any()  # every bin written exactly by one lane
    assert np.abs(X - np.fft.fft(x)).max() < 1e-9 * np.abs(x).sum()
