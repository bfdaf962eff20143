"""NR LDPC oracle pinned against the reference (CPU).

* base-graph tables (srsran_4g_amd/csrc/ldpc_bg_tables.inc) == the reference's create_compact_pcm
  (base_graph.c:4467) for every lifting size of both base graphs;
* the oracle encoder reproduces the reference's golden codewords (examplesBG{1,2}.dat, committed
  as tests/golden/ldpc_examples.npz) and the oracle decoder recovers their messages the way
  ldpc_dec_test.c does (symbols +-2, filler bits +2, scaling 1);
* the oracle decoder equals the reference decoder (8-bit C, 8-bit AVX2 incl. the "long" variant for
  Z > 32, 16-bit) on noisy codewords, rate-matched lengths and CRC early stop.
"""
import numpy as np
import pytest

from ldpc import (CRC16, CRC24A, CRC24B, DEC_C, DEC_C_AVX2, DEC_S, LIFT_SIZES, SCALE_C, SCALE_SIMD, OracleLdpc,
                  RefLdpc, lift, load_examples, noisy_llrs, ref_available)
from oracle import Oracle

needs_ref = pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built")


@pytest.fixture(scope="module")
def ora():
    return OracleLdpc()


@pytest.fixture(scope="module")
def examples():
    return load_examples()


def with_crc(rng, K, poly, order):
    m = rng.integers(0, 2, K).astype(np.uint8)
    c = Oracle().crc_bits(poly, order, m[:K - order])
    m[K - order:] = [(c >> (order - 1 - i)) & 1 for i in range(order)]
    return m


@needs_ref
@pytest.mark.parametrize("bg", [0, 1])
def test_tables_match_reference(ora, bg):
    ref = RefLdpc()
    for ls in LIFT_SIZES:
        p0, q0 = ref.pcm(bg, ls)
        p1, q1 = ora.pcm(bg, ls)
        assert np.array_equal(p0, p1), ls
        for r0, r1 in zip(q0, q1):
            k = list(r0).index(-1) if -1 in r0 else 20
            assert list(r0[:k]) == list(r1[:k]) and r1[k] == -1 if k < 20 else True


def test_examples_cover_all_lifting_sizes(examples):
    assert sorted(examples) == sorted((bg, ls) for bg in (0, 1) for ls in LIFT_SIZES)


def test_encoder_matches_golden(ora, examples):
    for (bg, ls), (msg, cw) in examples.items():
        for m, c in zip(msg, cw):
            mm = np.where(m == 254, 0, m).astype(np.uint8)
            got = ora.encode(bg, ls, mm)[2 * ls:]
            want = np.where(c == 254, 0, c)
            assert np.array_equal(got, want), (bg, ls)


@pytest.mark.parametrize("mode", [SCALE_C, SCALE_SIMD])
def test_decoder_recovers_golden(ora, examples, mode):
    for (bg, ls), (msg, cw) in examples.items():
        sym = np.where(cw[0] == 1, -2, 2).astype(np.int8)  # ldpc_dec_test.c: symbols = cw==1 ? -2 : 2
        r, out = ora.decode_c(bg, ls, sym, scaling=1.0, scale_mode=mode)
        m = msg[0]
        assert r == 10 and np.all((m == 254) | (out == m)), (bg, ls)


@needs_ref
@pytest.mark.parametrize("bg", [0, 1])
def test_decoder_matches_reference(ora, bg):
    ref = RefLdpc()
    rng = np.random.default_rng(11 + bg)
    for ls in LIFT_SIZES[::2] + [384]:
        K, N, n = lift(bg, ls)
        full = ora.encode(bg, ls, rng.integers(0, 2, K).astype(np.uint8))[2 * ls:]
        for snr in (0.5, 2.5):
            llr = noisy_llrs(full, rng, snr_db=snr, amp=6)
            L = n if snr > 1 else int(rng.integers((K // ls + 2) * ls - ls // 2, n + 1))
            for typ, mode in ((DEC_C, SCALE_C), (DEC_C_AVX2, SCALE_SIMD)):
                rr, ro = ref.decode(typ, bg, ls, llr, scaling=0.8, max_iter=5, length=L)
                orr, oo = ora.decode_c(bg, ls, llr, scaling=0.8, max_iter=5, length=L, scale_mode=mode)
                assert rr == orr and np.array_equal(ro, oo), (ls, snr, typ)
            l16 = llr.astype(np.int16) * 150
            rr, ro = ref.decode(DEC_S, bg, ls, l16, scaling=0.75, max_iter=4, length=L)
            orr, oo = ora.decode_s(bg, ls, l16, scaling=0.75, max_iter=4, length=L)
            assert rr == orr and np.array_equal(ro, oo), (ls, snr, "s")


@needs_ref
def test_decoder_saturation_matches_reference(ora):
    """Full-range int8 inputs (-128 included) exercise the infinity rules of both arithmetics."""
    ref = RefLdpc()
    rng = np.random.default_rng(5)
    for bg, ls in ((0, 384), (0, 20), (1, 52), (1, 3)):
        K, N, n = lift(bg, ls)
        llr = rng.integers(-128, 128, n).astype(np.int8)
        for typ, mode in ((DEC_C, SCALE_C), (DEC_C_AVX2, SCALE_SIMD)):
            for s in (0.8, 1.0, 0.55):
                rr, ro = ref.decode(typ, bg, ls, llr, scaling=s, max_iter=3)
                orr, oo = ora.decode_c(bg, ls, llr, scaling=s, max_iter=3, scale_mode=mode)
                assert rr == orr and np.array_equal(ro, oo), (bg, ls, typ, s)


@needs_ref
def test_crc_early_stop_matches_reference(ora):
    ref = RefLdpc()
    rng = np.random.default_rng(3)
    for bg, ls in ((0, 384), (0, 36), (1, 208), (1, 15)):
        K, N, n = lift(bg, ls)
        for poly, order in ((CRC24B, 24), (CRC24A, 24), (CRC16, 16)):
            m = with_crc(rng, K, poly, order)
            full = ora.encode(bg, ls, m)[2 * ls:]
            for snr in (0.0, 1.5, 4.0):
                llr = noisy_llrs(full, rng, snr_db=snr, amp=5)
                rr, ro = ref.decode(DEC_C_AVX2, bg, ls, llr, max_iter=8, crc=(poly, order))
                orr, oo = ora.decode_c(bg, ls, llr, max_iter=8, crc=(poly, order))
                assert rr == orr and np.array_equal(ro, oo), (bg, ls, poly, snr)
