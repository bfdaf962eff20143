"""CPU tests of the DL-SCH oracle pieces (oracle/sch_oracle.c).

Pinned against (a) the reference's own CRC known-answer words
(lib/src/phy/fec/test/crc_test.h:35-44: 5001 bits from srand(1)/rand()%2) and
(b) the reference compiled from /root/reference (oracle/_ref): byte-wise CRC,
code-block segmentation, rate de-matching RX (all 188 K x 4 rv, with and without
circular-buffer wrap) and rate matching TX.  The decode_tb loop (sch.c) cannot be
compiled here; it is tested through noise-free and AWGN round trips built from the
pinned pieces.
"""
import ctypes

import numpy as np
import pytest

from oracle import (CB_SIZES, LTE_CRC24A, LTE_CRC24B, SOFTBUF_LEN, Oracle, Reference, make_llrs,  # noqa: F401
                    ref_available)

needs_ref = pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built")


@pytest.fixture(scope="module")
def ora():
    return Oracle()


def test_crc_reference_kat(ora):
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(1)
    bits = np.array([libc.rand() % 2 for _ in range(5001)], np.uint8)
    assert ora.crc_bits(LTE_CRC24A, 24, bits) == 0x1C5C97
    assert ora.crc_bits(LTE_CRC24B, 24, bits) == 0x36D1F0


def test_crc_byte_equals_bitwise(ora):
    rng = np.random.default_rng(1)
    for n in (8, 64, 6144, 75400):
        d = rng.integers(0, 256, n // 8, dtype=np.uint8)
        for p in (LTE_CRC24A, LTE_CRC24B):
            assert ora.crc_byte(p, 24, d, n) == ora.crc_bits(p, 24, np.unpackbits(d))


def test_rm_table_is_permutation(ora):
    for K in CB_SIZES[::9] + [6144]:
        for rv in range(4):
            t = ora.rm_rx_table(K, rv, False)
            assert np.array_equal(np.sort(t), np.arange(3 * K + 12))


def test_dlsch_roundtrip_noise_free(ora):
    rng = np.random.default_rng(2)
    for tbs, Qm, G in ((75376, 6, 86400), (1544, 2, 3600), (40, 2, 300), (19080, 4, 28800)):
        tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        e = ora.dlsch_encode(tbs, Qm, 0, G, tb)
        llr = np.where(e > 0, 100, -100).astype(np.int16)
        ret, data, noi, avg, _ = ora.dlsch_decode(tbs, Qm, 0, llr, 8)
        assert ret == 0 and np.array_equal(data[: tbs // 8], tb), tbs
        assert all(n == 2 for n in noi) and avg == 2.0


def test_dlsch_harq_combining(ora):
    """rv0 at low SNR fails, rv2 combined into the same softbuffer succeeds (sch.c:390-419)."""
    rng = np.random.default_rng(3)
    tbs, Qm, G = 6200, 2, 7200
    tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    outs = []
    state = None
    for rv in (0, 2):
        e = ora.dlsch_encode(tbs, Qm, rv, G, tb).astype(np.float32) * 2 - 1
        y = e + rng.standard_normal(e.shape).astype(np.float32) * 0.6
        llr = np.trunc(100 * y).astype(np.int16)
        ret, data, noi, avg, state = ora.dlsch_decode(tbs, Qm, rv, llr, 8, state)
        outs.append((ret, np.array_equal(data[: tbs // 8], tb)))
    assert outs == [(-1, False), (0, True)]


@needs_ref
def test_crc_matches_reference(ora):
    ref = Reference()
    rng = np.random.default_rng(4)
    for n in (8, 800, 6144, 75400):
        d = rng.integers(0, 256, n // 8, dtype=np.uint8)
        for p in (LTE_CRC24A, LTE_CRC24B):
            assert ora.crc_byte(p, 24, d, n) == ref.crc_byte(p, 24, d, n)


@needs_ref
def test_cbsegm_matches_reference(ora):
    ref = Reference()
    for tbs in list(range(16, 200000, 8))[::41] + [75376, 97896, 6120, 6200, 40, 0]:
        a = ora.cbsegm(tbs)
        b = ref.cbsegm(tbs)
        assert a[0] == b[0] and (a[0] != 0 or a[1] == b[1]), tbs


@needs_ref
def test_rm_rx_matches_reference_all_sizes(ora):
    ref = Reference()
    rng = np.random.default_rng(5)
    bad = []
    for idx, K in enumerate(CB_SIZES):
        out_len = 3 * K + 12
        for rv in range(4):
            for E in (out_len // 3, out_len, 2 * out_len + 37):
                e = rng.integers(-30000, 30000, E, dtype=np.int16)
                sb0 = rng.integers(-30000, 30000, SOFTBUF_LEN, dtype=np.int16)
                if not np.array_equal(ora.rm_turbo_rx(K, rv, True, e, sb0), ref.rm_turbo_rx(idx, rv, e, sb0)):
                    bad.append((K, rv, E))
    assert not bad


@needs_ref
def test_rm_tx_matches_reference(ora):
    ref = Reference()
    rng = np.random.default_rng(6)
    for K in CB_SIZES[::11] + [6144]:
        coded = rng.integers(0, 2, 3 * K + 12, dtype=np.uint8)
        for rv in range(4):
            for E in (300, 3 * K + 12, 3 * K + 500):
                assert np.array_equal(ora.rm_turbo_tx(K, rv, coded, E), ref.rm_turbo_tx(K, rv, coded, E))


@needs_ref
def test_dlsch_decode_matches_reference_pieces(ora):
    """Oracle decode_tb vs the same loop over the reference's rm_turbo / turbo / CRC code:
    noise-free, early-stop, partial failure and HARQ chains (decode outputs and CB flags)."""
    ref = Reference()
    rng = np.random.default_rng(12)
    for tbs, Qm, G, sigmas in ((75376, 6, 86400, (0.0, 0.45, 0.48)), (19080, 4, 28800, (0.45,)),
                               (680, 4, 2400, (0.0, 0.6)), (16, 2, 240, (0.3,))):
        for sigma in sigmas:
            tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
            so = sr = None
            for rv in (0, 2, 3):
                e = ora.dlsch_encode(tbs, Qm, rv, G, tb).astype(np.float32) * 2 - 1
                e = np.trunc(100 * (e + rng.standard_normal(e.shape).astype(np.float32) * sigma)).astype(np.int16)
                a = ora.dlsch_decode(tbs, Qm, rv, e, 8, so)
                b = ref.dlsch_decode(tbs, Qm, rv, e, 8, sr)
                so, sr = a[4], b[4]
                assert a[0] == b[0] and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3], (tbs, sigma, rv)
                assert np.array_equal(so[1], sr[1]) and np.array_equal(so[2], sr[2]), (tbs, sigma, rv)
                if a[0] == 0:
                    break


def llr8_of(e_bits, rng, sigma, scale=20.0):
    """int8 LLRs of coded bits (+-1 plus AWGN, scaled, truncated, saturated) -- the range demod_soft_demodulate_b emits."""
    y = e_bits.astype(np.float32) * 2 - 1 + rng.standard_normal(e_bits.shape).astype(np.float32) * sigma
    return np.clip(np.trunc(np.float32(scale) * y), -128, 127).astype(np.int8)


@needs_ref
def test_dlsch_decode8_matches_reference_pieces(ora):
    """decode_tb with llr_is_8bit (sch.c:409-428): the oracle (C restatement of the 8-bit window decoders and int8 rate
    de-matching) against the same loop over the reference's srsran_rm_turbo_rx_lut_8bit / 8-bit decoders / CRC, on
    every decoder class: 32 sub-blocks (K > 2048), 16 (800 < K <= 2048), the 16-bit decoders on the widened input for
    K <= 800 (8 sub-blocks and natural); noise-free, early-stop, failure and HARQ chains."""
    ref = Reference()
    rng = np.random.default_rng(13)
    for tbs, Qm, G, sigmas in ((75376, 6, 86400, (0.0, 0.5)), (1544, 2, 3600, (0.75, 0.85)), (19080, 4, 28800, (0.6,)),
                               (680, 4, 2400, (0.0, 0.9)), (16, 2, 240, (0.3,))):
        for sigma in sigmas:
            tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
            so = sr = None
            for rv in (0, 2, 3):
                e = llr8_of(ora.dlsch_encode(tbs, Qm, rv, G, tb), rng, sigma)
                a = ora.dlsch_decode8(tbs, Qm, rv, e, 8, so)
                b = ref.dlsch_decode8(tbs, Qm, rv, e, 8, sr)
                so, sr = a[4], b[4]
                assert a[0] == b[0] and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3], (tbs, sigma, rv)
                assert np.array_equal(so[1], sr[1]) and np.array_equal(so[2], sr[2]), (tbs, sigma, rv)
                if a[0] == 0:
                    break
            if sigma == 0.0:
                assert a[0] == 0 and np.array_equal(a[1][: tbs // 8], tb), tbs
