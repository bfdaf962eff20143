"""CPU tests of the parity oracle (oracle/tdec_oracle.c).

1. Against the committed golden vectors (tests/golden/tdec_golden.npz, produced by
   the reference decoder compiled from /root/reference, see make_golden.py).
2. Against the reference decoder itself (oracle/_ref/libsrsref.so) on fresh random
   inputs for all 188 code-block sizes, both input layouts, every half-iteration
   (skipped where oracle/_ref has not been built).
"""
import os
import zlib

import numpy as np
import pytest

from oracle import CB_SIZES, Oracle, Reference, make_llrs, ref_available

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tdec_golden.npz")


@pytest.fixture(scope="module")
def ora():
    return Oracle()


def golden_cases():
    z = np.load(GOLDEN)
    for i in range(int(z["ncases"][0])):
        p = f"c{i:03d}_"
        yield {k[len(p):]: z[k] for k in z.files if k.startswith(p)}


def test_golden_vectors(ora):
    n = 0
    for c in golden_cases():
        K = int(c["K"][0])
        llr = c["llr"]
        sb = ora.natural_to_sb(K, llr)
        for nit in (8, 16):
            assert np.array_equal(ora.tdec_run(K, llr, False, nit), c[f"out_nat_{nit}"]), (K, nit)
            assert np.array_equal(ora.tdec_run(K, sb, True, nit), c[f"out_sb_{nit}"]), (K, nit)
        _, tr = ora.tdec_run(K, llr, False, 16, trace=True)
        crc = np.array([zlib.crc32(row.tobytes()) for row in tr], dtype=np.uint32)
        assert np.array_equal(crc, c["trace_crc"]), K
        n += 1
    assert n == 34


def test_qpp_tables_are_permutations(ora):
    for K in CB_SIZES:
        f, r = ora.qpp(K)
        assert np.array_equal(np.sort(f), np.arange(K))
        assert np.array_equal(r[f], np.arange(K))


def test_awgn_decodes(ora):
    """Sanity: at Eb/No label 5 dB (true Eb/N0 ~2 dB) a 6144-bit block decodes error-free in 8 half-iterations."""
    rng = np.random.default_rng(3)
    bits, llr = make_llrs(6144, 5.0, rng, 4, ora)
    for b, x in zip(bits, llr):
        assert np.array_equal(np.unpackbits(ora.tdec_run(6144, x, False, 8)), b)


needs_ref = pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built")


@needs_ref
def test_encoder_matches_reference(ora):
    ref = Reference()
    rng = np.random.default_rng(11)
    for K in CB_SIZES[::7] + [6144]:
        b = rng.integers(0, 2, K, dtype=np.uint8)
        assert np.array_equal(ora.encode(K, b), ref.encode(K, b)), K


@needs_ref
@pytest.mark.parametrize("layout_sb", [False, True])
def test_oracle_matches_reference_all_sizes(ora, layout_sb):
    ref = Reference()
    rng = np.random.default_rng(77 + layout_sb)
    bad = []
    for K in CB_SIZES:
        if K % 2:
            llr = rng.integers(-32768, 32768, 3 * K + 12, dtype=np.int16)
        else:
            llr = make_llrs(K, 0.5, rng, 1, ora)[1][0]
        if layout_sb:
            llr = ora.natural_to_sb(K, llr)
        a, ta = ora.tdec_run(K, llr, layout_sb, 7, trace=True)
        b, tb = ref.tdec_run(K, llr, layout_sb, 7, trace=True)
        if not (np.array_equal(a, b) and np.array_equal(ta, tb)):
            bad.append(K)
    assert not bad
