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


@needs_ref
@pytest.mark.parametrize("mod,scale", [(0, 20.0), (1, 28.284271), (2, 30.0), (3, 40.0), (4, 50.0)])
def test_demod_b_matches_reference(mod, scale):
    """int8 demapping (srsran_demod_soft_demodulate_b, llr_is_8bit): the SSE blocks of 8 symbols (16 values for
    QPSK) round half-even and saturate, their abs/offset steps wrap (|-128| = -128); the tails truncate."""
    ora, ref = Oracle(), Reference()
    rng = np.random.default_rng(40 + mod)
    for n in (1, 2, 3, 7, 8, 9, 15, 16, 17, 23, 1200, 14400, 14401, 14407):
        sym = symbols(rng, n, scale)
        a = ora.demod_b(mod, sym)
        b = ref.demod_b(mod, sym)
        assert np.array_equal(a, b), (mod, n, np.flatnonzero(a != b)[:8])


@needs_ref
def test_sequence_c_matches_reference():
    """int8 descrambling (srsran_sequence_apply_c): -(-128) stays -128."""
    ora, ref = Oracle(), Reference()
    rng = np.random.default_rng(9)
    for n in (0, 1, 15, 16, 17, 31, 32, 33, 86400, 90001):
        llr = rng.integers(-128, 128, n, dtype=np.int8)
        llr[: min(n, 5)] = -128
        for seed in (0, 1, 0x1234 << 14 | 1, 0x7FFFFFFF, int(rng.integers(0, 2**31))):
            assert np.array_equal(ora.sequence_apply_c(llr, seed), ref.sequence_apply_c(llr, seed)), (n, seed)


@needs_ref
@pytest.mark.parametrize("llr8", [False, True])
def test_csi_correction_matches_reference_build(llr8):
    """csi_correction (pdsch.c:523-618) restated in ref_pdsch_tx_harness.c over the reference's srsran_vec_max_fi and
    built with the reference's -Ofast flags: the oracle (and the GPU) follow the build, whose scalar loops multiply by a
    hoisted 1 / csi_max instead of dividing (-freciprocal-math); int16 SSE blocks + tail, and the int8 branch."""
    ora, ref = Oracle(), Reference()
    rng = np.random.default_rng(11 + llr8)
    for mod in (1, 2, 3, 4):
        qm = (1, 2, 4, 6, 8)[mod]
        for ns in (1, 2, 3, 5, 17, 601, 1201, 7200):
            csi = (rng.random(ns) * rng.choice([0.013, 1.0, 7.3])).astype(np.float32)
            e = rng.integers(-128, 128, ns * qm) if llr8 else rng.integers(-32768, 32768, ns * qm)
            a = (ora.csi_correction_b if llr8 else ora.csi_correction)(mod, csi, e)
            b = ref.csi_correction(mod, csi, e, llr8)
            assert np.array_equal(a, b), (mod, ns, np.flatnonzero(a != b)[:8])


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


PRE_CASES = [(0, 1, 1, 1, 0), (0, 2, 1, 1, 0), (3, 2, 2, 2, 0), (2, 2, 2, 2, 0), (2, 2, 2, 2, 1), (2, 2, 2, 2, 2),
             (1, 1, 2, 2, 0), (1, 2, 2, 2, 0), (1, 4, 2, 2, 0), (1, 1, 4, 4, 0), (1, 2, 4, 4, 0), (1, 4, 4, 4, 0)]


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
            if scheme == 1:  # diversity_csi is scalar C in the reference too: bit-exact
                m = xo.shape[1]  # 4 ports: only the m_ap whole groups are decoded (precoding.c:715)
                assert np.array_equal(xo, xr[:, :m]), n
                assert np.array_equal(co[:, :nlayers * m], cr[:, :nlayers * m]), n
                continue
            err = np.abs(xo - xr) / (np.abs(xo) + 1e-3)
            assert np.percentile(err, 99.9) < 2e-3 and err.max() < 2e-2, (n, err.max())
            cerr = np.abs(co - cr) / np.abs(co)
            assert cerr.max() < 2e-3, (n, cerr.max())


def crs_positions(nof_prb, cell_id, port):
    """(symbol, subcarrier) of the CRS of `port` (36.211 6.10.1.2)."""
    pos = []
    nsym = 4 if port < 2 else 2
    for l in range(nsym):
        sym = ((l // 2 + 1) * 7 - 3 if l % 2 else (l // 2) * 7) if port < 2 else 1 + l * 7
        v = [[0, 3], [3, 0], [0, 3], [3, 0]][port][l % 2] if port < 2 else (0 if (l == 0) == (port == 2) else 3)
        f0 = (v + cell_id % 6) % 6
        pos.append([(sym, f0 + 6 * i) for i in range(2 * nof_prb)])
    return pos


def make_subframe(ora, rng, nof_prb=100, cell_id=1, nports=2, nrx=2, sf_idx=1, snr_db=30.0, flat=False):
    """Received grids of one subframe: CRS of every port + random QPSK data through a smooth channel."""
    nre = 12 * nof_prb
    X = (rng.choice([-1, 1], (nports, 14, nre)) + 1j * rng.choice([-1, 1], (nports, 14, nre))) / np.sqrt(2)
    for p in range(nports):  # CRS REs of any port are empty on the other ports
        for q in range(nports):
            for row in crs_positions(nof_prb, cell_id, q):
                for s, k in row:
                    X[p, s, k] = 0
    for p in range(nports):
        pil = ora.crs_pilots(cell_id, nof_prb, p // 2, sf_idx).reshape(-1, 2 * nof_prb)
        for l, row in enumerate(crs_positions(nof_prb, cell_id, p)):
            for i, (s, k) in enumerate(row):
                X[p, s, k] = pil[l, i]
    k = np.arange(nre)
    H = np.zeros((nports, nrx, nre), np.complex64)
    for p in range(nports):
        for r in range(nrx):
            if flat:
                H[p, r] = rng.standard_normal() + 1j * rng.standard_normal()
            else:
                a = rng.standard_normal(3) + 1j * rng.standard_normal(3)
                H[p, r] = a[0] + a[1] * np.exp(2j * np.pi * k * 0.8 / nre) + 0.3 * a[2] * np.exp(-2j * np.pi * k * 2.3 / nre)
    Y = np.einsum("prk,psk->rsk", H, X)
    sig = 10 ** (-snr_db / 20)
    Y = Y + sig * (rng.standard_normal(Y.shape) + 1j * rng.standard_normal(Y.shape)) / np.sqrt(2)
    return Y.reshape(nrx, 14 * nre).astype(np.complex64), H, X


def test_crs_pilots_are_qpsk_gold():
    ora = Oracle()
    p = ora.crs_pilots(1, 100, 0, 1)
    assert p.size == 800 and np.allclose(np.abs(p), 1.0, atol=1e-6)
    c = ora.sequence_bits(1024 * (7 * 3 + 0 + 1) * 3 + 2 + 1, 440)  # slot 2, symbol 0, cell 1
    mp = np.arange(200) + 10
    exp = ((1 - 2 * c[2 * mp].astype(np.float32)) + 1j * (1 - 2 * c[2 * mp + 1].astype(np.float32))) / np.sqrt(2)
    assert np.allclose(p[:200], exp, atol=1e-6)


def test_chest_flat_noise_free():
    """A flat channel is recovered exactly on every RE; the REFS noise estimate is ~0."""
    ora = Oracle()
    rng = np.random.default_rng(2)
    Y, H, _ = make_subframe(ora, rng, flat=True, snr_db=200)
    ce, st = ora.chest_dl(Y, 100, 1, 2, 1, 2048)
    for p in range(2):
        for r in range(2):
            assert np.allclose(ce[p, r], H[p, r][0], rtol=1e-5, atol=1e-5)
    assert st["noise"] < 1e-10


def test_chest_noise_tracks_snr():
    ora = Oracle()
    rng = np.random.default_rng(3)
    for snr in (10.0, 20.0):
        Y, H, _ = make_subframe(ora, rng, snr_db=snr)
        ce, st = ora.chest_dl(Y, 100, 1, 2, 1, 2048)
        assert 0.5 < st["noise"] / 10 ** (-snr / 10) < 2.0, (snr, st)
        err = np.abs(ce[:, :, :1200] - H) ** 2
        assert err.mean() < 10 ** (-snr / 10)


@needs_ref
def test_gauss_filter_and_conv_same_match_reference():
    import ctypes
    ora, ref = Oracle(), Reference()
    g = ref.lib.srsran_chest_set_smooth_filter_gauss
    g.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_float]
    g.restype = ctypes.c_uint32
    for order, std in ((4, 1.0), (4, 0.37), (6, 2.0), (2, 1.0)):
        fr = np.zeros(64, np.float32)
        n = g(fr.ctypes.data, order, std)
        fo = ora.gauss_filter(order, std)
        assert n == fo.size and np.allclose(fr[:n], fo, rtol=1e-6), (order, std)
    c = ref.lib.srsran_conv_same_cf
    c.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    rng = np.random.default_rng(9)
    for N in (400, 200, 24):
        x = (rng.standard_normal(N) + 1j * rng.standard_normal(N)).astype(np.complex64)
        f = ora.gauss_filter(4, 1.0)
        yr = np.zeros(N, np.complex64)
        c(x.ctypes.data, f.ctypes.data, yr.ctypes.data, N, f.size)
        yo = np.zeros(N, np.complex64)
        fo = ora.lib.oracle_conv_same
        fo.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32] * 2
        fo(x.ctypes.data, f.ctypes.data, yo.ctypes.data, N, f.size)
        assert np.allclose(yo, yr, rtol=1e-5, atol=1e-6), N  # SIMD dot products sum in a different order


def test_sync_error_pieces_vs_reference():
    """the pieces of correct_sync_error (chest_dl.c:750-804) in the oracle against the reference compiled into
    _ref: srsran_vec_apply_cfo bit for bit (its phasor recurrence and FMA roundings) and
    srsran_vec_estimate_frequency within float summation order"""
    import ctypes
    import os
    from oracle import ref_available
    if not ref_available():
        pytest.skip("oracle/_ref not built")
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    R = ctypes.CDLL(os.path.join(here, "_ref", "libsrsref.so"), mode=os.RTLD_LAZY)
    L = ctypes.CDLL(os.path.join(here, "liboracle.so"))
    R.srsran_vec_apply_cfo.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_int]
    R.srsran_vec_estimate_frequency.argtypes = [ctypes.c_void_p, ctypes.c_int]
    R.srsran_vec_estimate_frequency.restype = ctypes.c_float
    L.oracle_apply_cfo.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_uint32]
    L.oracle_estimate_frequency.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    L.oracle_estimate_frequency.restype = ctypes.c_float
    rng = np.random.default_rng(12)

    def aligned(n):
        b = np.zeros(n + 8, np.complex64)
        o = (-(b.ctypes.data // 8)) % 4
        return b[o:o + n]
    for n in (1200, 600, 300, 72, 13):
        for f in (1e-3, -2.5e-4, 0.01, 2e-4 / 6):
            x = aligned(n)
            x[:] = rng.standard_normal(n) + 1j * rng.standard_normal(n)
            z1, z2 = aligned(n), aligned(n)
            L.oracle_apply_cfo(x.ctypes.data, f, z1.ctypes.data, n)
            R.srsran_vec_apply_cfo(x.ctypes.data, f, z2.ctypes.data, n)
            assert np.array_equal(z1.view(np.uint32), z2.view(np.uint32)), (n, f)
        y = aligned(n)
        y[:] = np.exp(2j * np.pi * 0.013 * np.arange(n)) * (1 + 0.1 * rng.standard_normal(n))
        a, b = L.oracle_estimate_frequency(y.ctypes.data, n), R.srsran_vec_estimate_frequency(y.ctypes.data, n)
        assert a == pytest.approx(b, rel=1e-5, abs=1e-7), n
