"""numpy restatement of srsRAN_4G's 8-bit window turbo decoders (TEST INFRASTRUCTURE ONLY).

turbodecoder_win.h with WINIMP_IS_SSE8 (16 sub-blocks) / WINIMP_IS_AVX8 (32 sub-blocks), lines 154-300 and
480-832, driven by turbodecoder_iter.h:72-144 (LLR_IS_8BIT) and tdec_iteration_8 (turbodecoder.c:455-483).
Vectorised over the sub-blocks the way the SIMD code is; the schedule is the one
srsran_4g_amd/csrc/tdec8bit_kernel.hip runs per lane.  Pinned to the reference's own decoders compiled into
oracle/_ref (ref_tdec8_run, tests/test_tdec8bit.py).  Only tests/ import it.
"""
import numpy as np

OVL = 40  # win_overlap_len


def _sat(v):
    return np.clip(v, -128, 127)


def _tadd(a, b):  # beta_trellis sadd: upper clamp, int8 wrap below
    z = int(a) + int(b)
    return 127 if z > 127 else ((z + 128) % 256) - 128


def _norm(k, o):
    if k != 0:
        m = o.max(axis=0)
        o[:] = _sat(o - m)


def _beta_step(o, x, y):
    xy = _sat(x + y)
    n = np.empty_like(o)
    n[0] = np.maximum(_sat(o[4] + xy), o[0])
    n[1] = np.maximum(o[4], _sat(o[0] + xy))
    n[2] = np.maximum(_sat(o[5] + y), _sat(o[1] + x))
    n[3] = np.maximum(_sat(o[5] + x), _sat(o[1] + y))
    n[4] = np.maximum(_sat(o[6] + x), _sat(o[2] + y))
    n[5] = np.maximum(_sat(o[6] + y), _sat(o[2] + x))
    n[6] = np.maximum(o[7], _sat(o[3] + xy))
    n[7] = np.maximum(_sat(o[7] + xy), o[3])
    o[:] = n


def _alpha_cand(o, x, y):
    xy = _sat(x + y)
    mb = np.stack([o[0], _sat(o[3] + y), _sat(o[4] + y), o[7], o[1], _sat(o[2] + y), _sat(o[5] + y), o[6]])
    nw = np.stack([_sat(o[1] + xy), _sat(o[2] + x), _sat(o[5] + x), _sat(o[6] + xy),
                   _sat(o[0] + xy), _sat(o[3] + x), _sat(o[4] + x), _sat(o[7] + xy)])
    return mb, nw


def _trellis(X, P, K):
    t = [0] * 8
    for k in range(K + 2, K - 1, -1):
        x, y = int(X[k]), int(P[k])
        xy = _tadd(x, y)
        mb = [_tadd(t[4], xy), t[4], _tadd(t[5], y), _tadd(t[5], x), _tadd(t[6], x), _tadd(t[6], y), t[7],
              _tadd(t[7], xy)]
        nw = [t[0], _tadd(t[0], xy), _tadd(t[1], x), _tadd(t[1], y), _tadd(t[2], y), _tadd(t[2], x),
              _tadd(t[3], xy), t[3]]
        t = [max(a, b) for a, b in zip(mb, nw)]
    return np.array(t, dtype=np.int32)


def map_pass(X, A, P, K, nsb):
    """One MAP decoder pass: SB-ordered int arrays (length >= K + 3); returns the extrinsic output (K)."""
    Ls = K // nsb
    Xr = X[:K].reshape(Ls, nsb).astype(np.int32)
    Pr = P[:K].reshape(Ls, nsb).astype(np.int32)
    if A is not None:
        Xr = _sat(A[:K].reshape(Ls, nsb).astype(np.int32) + Xr)
    beta = np.zeros((Ls + 1, 8, nsb), np.int32)
    o = np.zeros((8, nsb), np.int32)
    for k in range(OVL - 1, -1, -1):
        _beta_step(o, Xr[k], Pr[k])
        _norm(k, o)
    e = np.empty_like(o)
    e[:, :-1] = o[:, 1:]
    e[:, -1] = _trellis(X, P, K)
    o = e
    beta[Ls] = o
    for k in range(Ls - 1, -1, -1):
        _beta_step(o, Xr[k], Pr[k])
        beta[k] = o
        _norm(k, o)
    o = np.zeros((8, nsb), np.int32)
    for k in range(OVL):
        mb, nw = _alpha_cand(o, Xr[Ls - OVL + k], Pr[Ls - OVL + k])
        o = np.maximum(mb, nw)
        _norm(k, o)
    e = np.zeros_like(o)
    e[:, 1:] = o[:, :-1]
    o = e
    out = np.empty((Ls, nsb), np.int32)
    for k in range(Ls):
        mb, nw = _alpha_cand(o, Xr[k], Pr[k])
        b = beta[k + 1]
        m0 = _sat(b + mb).max(axis=0)
        m1 = _sat(b + nw).max(axis=0)
        out[k] = _sat(m1 - m0) >> 1
        o = np.maximum(mb, nw)
        _norm(k, o)
    return out.reshape(K)


def qpp_sb(K, nsb, f1, f2):
    """forward table of tc_interl_lte.c:88-106 for interl_win = nsb (SB slot order)."""
    Ls = K // nsb
    q = np.arange(K, dtype=np.int64)
    n = (q % nsb) * Ls + q // nsb
    fn = (f1 * n + f2 * n * n) % K
    return (fn % Ls) * nsb + fn // Ls


def run_all(K, llr, nof_iterations, nsb, fwd, layout_sb=True):
    """srsran_tdec_run_all_8bit for an 8-bit decoder class (nsb 16 or 32); fwd = the forward interleaver
    table of the SB layout (ref_interleaver); returns decision bytes."""
    llr = np.asarray(llr, np.int32)
    Ls = K // nsb
    tail0 = 3 * (K + 32) if layout_sb else 3 * K
    if layout_sb:
        SY, P0, P1 = llr[:K], llr[K + 32:2 * K + 32], llr[2 * (K + 32):2 * (K + 32) + K]
    else:
        i, d = np.meshgrid(np.arange(Ls), np.arange(nsb), indexing="ij")
        nat = (i + d * Ls).reshape(K)
        SY, P0, P1 = llr[3 * nat], llr[3 * nat + 1], llr[3 * nat + 2]
    tail = llr[tail0:tail0 + 12]
    SY = np.concatenate([SY, tail[0:6:2]])
    P0 = np.concatenate([P0, tail[1:6:2]])
    A2 = np.concatenate([np.zeros(K, np.int32), tail[6:12:2]])
    P1 = np.concatenate([P1, tail[7:12:2]])
    A1 = np.zeros(K, np.int32)
    E1 = np.zeros(K, np.int32)
    fwd = np.asarray(fwd, np.int64)
    for n in range(max(1, nof_iterations)):
        if n % 2 == 0:
            if n:
                A1 = _sat(A1 - E1)
            E1 = map_pass(SY, A1 if n else None, P0, K, nsb)
        else:
            if n > 1:
                E1 = _sat(E1 - A1)
            A2[:K] = E1[fwd]
            E2 = map_pass(A2, None, P1, K, nsb)
            A1 = np.empty(K, np.int32)
            A1[fwd] = E2
    src = E1 if max(1, nof_iterations) % 2 else A1
    nn = np.arange(K)
    bits = (src[(nn % Ls) * nsb + nn // Ls] > 0).astype(np.uint8)
    return np.packbits(bits)
