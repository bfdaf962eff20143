"""The reference's single-code-block transmit entry points on the GPU against the reference itself (oracle/_ref, the
reference's turbocoder.c / rm_turbo.c / bit.c compiled from /root/reference):

* srsran_tcod_encode (turbocoder.c:77-185): 3 K + 12 unpacked bits equal ref_tcod_encode's, filler bits
  (SRSRAN_TX_NULL) included, for code block sizes across the 188;
* srsran_rm_turbo_tx_lut (rm_turbo.c:345-388) on the packed streams of the reference's srsran_tcod_encode_lut:
  the circular buffer w_buff (rv 0) and every byte of the packed output -- the bits around the written range
  included (srsran_bit_copy's byte-aligned path clears the rest of its last byte, bit.c:688-694) -- equal the
  reference's, for every rv (rv > 0 reading the w_buff an rv 0 call left), out_len below and above 3 K + 12 and
  odd bit offsets."""
import ctypes
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

u8p = ctypes.POINTER(ctypes.c_uint8)


def P(a):
    return a.ctypes.data_as(u8p)


@pytest.fixture(scope="module")
def env():
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.fail("no HIP device on a GPU test run")
    import oracle as O
    if not O.ref_available():
        pytest.fail("oracle/_ref/libsrsref.so missing: the reference checker of this module was not built")
    R = ctypes.CDLL(O.REF_SO, mode=os.RTLD_LAZY)
    R.ref_tcod_encode.argtypes = [ctypes.c_uint32, u8p, u8p]
    R.ref_tcod_rm_tx_lut.argtypes = [ctypes.c_uint32, u8p, u8p, u8p, u8p, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_int]
    return S, R, tdec


@pytest.mark.parametrize("cb_idx", [0, 1, 23, 59, 60, 91, 92, 123, 124, 150, 187])
def test_tcod_encode_matches_reference(env, cb_idx):
    S, R, tdec = env
    K = tdec.CB_SIZES[cb_idx]
    rng = np.random.default_rng(cb_idx)
    h = S.srsran_tcod_t()
    assert S.lib().srsran_tcod_init(ctypes.byref(h), 6144) == 0
    try:
        for nfill in (0, 8, 24):  # filler bits lead the first code block (sch.c:265-276)
            x = rng.integers(0, 2, K).astype(np.uint8)
            x[:nfill] = 100
            want = np.zeros(3 * K + 12, np.uint8)
            assert R.ref_tcod_encode(K, P(x), P(want)) == 0
            got = np.zeros(3 * K + 12, np.uint8)
            assert S.lib().srsran_tcod_encode(ctypes.byref(h), P(x), P(got), K) == 0
            assert np.array_equal(got, want), (K, nfill, np.flatnonzero(got != want)[:8])
        assert S.lib().srsran_tcod_encode(ctypes.byref(h), P(x), P(got), 6145) != 0
    finally:
        S.lib().srsran_tcod_free(ctypes.byref(h))


def test_rm_turbo_tx_lut_matches_reference(env):
    S, R, tdec = env
    rng = np.random.default_rng(11)
    cases = [(c, rv) for c in (0, 5, 40, 59, 60, 100, 124, 150, 187) for rv in range(4)]
    cases += [(int(rng.integers(0, 188)), int(rng.integers(0, 4))) for _ in range(40)]
    for cb, rv in cases:
        K = tdec.CB_SIZES[cb]
        in_len = 3 * K + 12
        sysb = np.zeros(K // 8 + 1, np.uint8)
        sysb[:K // 8] = rng.integers(0, 256, K // 8)
        par = np.zeros((2 * K + 8) // 8 + 32, np.uint8)
        w_ref = np.zeros(in_len // 8 + 16, np.uint8)
        E = int(rng.choice([int(rng.integers(1, in_len)), in_len, int(rng.integers(in_len, 3 * in_len))]))
        woff = int(rng.integers(0, 24))
        out0 = rng.integers(0, 256, (woff + E) // 8 + 8).astype(np.uint8)
        out_ref = out0.copy()
        # the reference: encode_lut (sys gets its tail nibble, parity filled), rv 0, then rv if any
        assert R.ref_tcod_rm_tx_lut(cb, P(sysb), P(par), P(w_ref), P(out_ref), E if rv == 0 else 0, woff, 0, 1) == 0
        if rv:
            assert R.ref_tcod_rm_tx_lut(cb, P(sysb), P(par), P(w_ref), P(out_ref), E, woff, rv, 0) == 0
        w = np.zeros_like(w_ref)
        out = out0.copy()
        assert S.lib().srsran_rm_turbo_tx_lut(P(w), P(sysb), P(par), P(out), cb, E if rv == 0 else 0, woff, 0) == 0
        if rv:
            assert S.lib().srsran_rm_turbo_tx_lut(P(w), None, None, P(out), cb, E, woff, rv) == 0
        assert np.array_equal(np.unpackbits(w)[:in_len], np.unpackbits(w_ref)[:in_len]), (cb, rv)
        assert np.array_equal(out, out_ref), (cb, rv, E, woff, np.flatnonzero(out != out_ref)[:8])
    assert S.lib().srsran_rm_turbo_tx_lut(P(w), P(sysb), P(par), P(out), 188, 10, 0, 0) != 0
    assert S.lib().srsran_rm_turbo_tx_lut(P(w), P(sysb), P(par), P(out), 0, 10, 0, 4) != 0
