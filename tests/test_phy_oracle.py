"""CPU tests of the PDSCH LLR-stage oracle (oracle/phy_oracle.c) against the reference's
demod_soft.c / sequence.c / sequences.c compiled into oracle/_ref (AVX2 release flags).

Inputs cover the int16 rounding/saturation/wrap corners: exact .5 ties of the SSE
round-half-even blocks, truncating scalar tails (n % 4 symbols, QPSK len % 16),
saturating and wrapping magnitudes."""
import numpy as np
import pytest

from oracle import Oracle, Reference, ref_available

needs_ref = pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built")


def tie_values(scale, count, rng):
    """floats x with float32(x * scale) exactly k + 0.5."""
    out = []
    for k in rng.integers(-3000, 3000, count * 4):
        x0 = np.float32((k + 0.5) / scale)
        for cand in (x0, np.nextafter(x0, np.float32(1)), np.nextafter(x0, np.float32(-1))):
            if np.float32(cand * np.float32(scale)) == np.float32(k + 0.5):
                out.append(cand)
                break
        if len(out) >= count:
            break
    return np.array(out, np.float32)


def symbols(rng, n, scale):
    re = rng.uniform(-1.6, 1.6, n).astype(np.float32)
    im = rng.uniform(-1.6, 1.6, n).astype(np.float32)
    t = tie_values(scale, n // 4, rng)
    re[: t.size] = t
    im[n // 8: n // 8 + t.size // 2] = -t[: t.size // 2]
    nb = n // 16
    if nb:
        im[-nb:] = rng.uniform(-100, 100, nb).astype(np.float32)  # saturation / wrap
    p = rng.permutation(n)
    return (re[p] + 1j * im[p]).astype(np.complex64)


@needs_ref
@pytest.mark.parametrize("mod,scale", [(0, 100.0), (1, 141.42136), (2, 400.0), (3, 700.0), (4, 1000.0)])
def test_demod_matches_reference(mod, scale):
    ora, ref = Oracle(), Reference()
    rng = np.random.default_rng(mod)
    for n in (1, 2, 3, 4, 5, 7, 8, 13, 16, 17, 1200, 14400, 14401, 14403):
        sym = symbols(rng, n, scale)
        a = ora.demod_s(mod, sym)
        b = ref.demod_s(mod, sym)
        assert np.array_equal(a, b), (mod, n, np.flatnonzero(a != b)[:8])


@needs_ref
def test_sequence_matches_reference():
    ora, ref = Oracle(), Reference()
    rng = np.random.default_rng(7)
    for n in (0, 1, 23, 24, 25, 47, 86400, 90000):
        llr = rng.integers(-32768, 32768, n, dtype=np.int16)
        llr[: min(n, 5)] = -32768
        for seed in (0, 1, 0x1234 << 14 | 1, 0x7FFFFFFF, int(rng.integers(0, 2**31))):
            assert np.array_equal(ora.sequence_apply_s(llr, seed), ref.sequence_apply_s(llr, seed)), (n, seed)


@needs_ref
def test_pdsch_seed_matches_reference():
    ora, ref = Oracle(), Reference()
    rng = np.random.default_rng(8)
    llr = rng.integers(-1000, 1000, 3000, dtype=np.int16)
    for rnti, q, ns, cell in ((0x1234, 0, 2, 1), (0xFFFF, 1, 19, 503), (1, 0, 0, 0)):
        seed = ora.pdsch_seed(rnti, q, ns, cell)
        assert np.array_equal(ora.sequence_apply_s(llr, seed), ref.sequence_pdsch_apply_s(llr, rnti, q, ns, cell))


def test_sequence_known_properties():
    """c(n) for seed 0 is x1 alone (x2 == 0); Gold sequence is balanced."""
    ora = Oracle()
    c = ora.sequence_bits(0x1234, 100000)
    assert abs(int(c.sum()) - 50000) < 1000
    llr = np.arange(1, 101, dtype=np.int16)
    out = ora.sequence_apply_s(llr, 0x1234)
    assert np.array_equal(np.abs(out), llr) and np.array_equal(out < 0, c[:100] == 1)


def channel(rng, nports, nrx, n):
    h = (rng.standard_normal((nports, nrx, n)) + 1j * rng.standard_normal((nports, nrx, n))) * 0.7
    y = (rng.standard_normal((nrx, n)) + 1j * rng.standard_normal((nrx, n)))
    return y.astype(np.complex64), h.astype(np.complex64)


PRE_CASES = [(0, 1, 1, 1, 0), (0, 2, 1, 1, 0), (3, 2, 2, 2, 0), (2, 2, 2, 2, 0), (2, 2, 2, 2, 1), (2, 2, 2, 2, 2)]


@needs_ref
@pytest.mark.parametrize("scheme,nrx,nports,nlayers,cb", PRE_CASES)
def test_predecode_matches_reference(scheme, nrx, nports, nlayers, cb):
    """Oracle (exact IEEE float, scalar formulas) vs the reference SIMD build, whose
    rcp_ps / rcp14 approximations limit agreement to ~1e-3 relative."""
    ora, ref = Oracle(), Reference()
    rng = np.random.default_rng(scheme * 10 + nrx + cb)
    for n in (14400, 1202, 40):  # odd n: the reference CDD tail overruns (precoding.c:1105-1118)
        y, h = channel(rng, nports, nrx, n)
        for scaling, noise in ((1.0, 0.01), (0.7, 0.3)):
            xo, co = ora.predecode(scheme, y, h, nlayers, cb, scaling, noise)
            xr, cr = ref.predecode(scheme, y, h, nlayers, cb, scaling, noise)
            assert np.all(np.isfinite(xo))
            err = np.abs(xo - xr) / (np.abs(xo) + 1e-3)
            assert np.percentile(err, 99.9) < 2e-3 and err.max() < 2e-2, (n, err.max())
            cerr = np.abs(co - cr) / np.abs(co)
            assert cerr.max() < 2e-3, (n, cerr.max())
