"""GPU OFDM receiver and CFO correction.  The FFT stage has no pinned reference output (FFTW
is absent and no reference test holds its results): it is checked against numpy's
double-precision FFT with srsRAN's symbol timing / subcarrier mapping (oracle/ofdm_np.py) and
by TX -> RX round trips, at float32 tolerance."""
import json
import os

import numpy as np
import pytest
import torch

import ofdm_np

pytestmark = pytest.mark.gpu

# north_star: soft values within 1e-4.  The FFT has no pinned reference output, so its error is taken against
# numpy's double-precision transform, relative to the largest bin; the measured figures are written to
# $SRSRAN_AMD_FFT_STATS.
FFT_TOL = 1e-6  # measured <= 3.3e-7 (profiles/r05a_fft_stats.json); north_star asks 1e-4
FFT_STATS = {}


def _fft_check(key, got, exp):
    err = float(np.abs(got - exp).max() / np.abs(exp).max())
    FFT_STATS[key] = err
    out = os.environ.get("SRSRAN_AMD_FFT_STATS")
    if out:
        with open(out, "w") as f:
            json.dump(FFT_STATS, f, indent=1)
    assert err <= FFT_TOL, (key, err)


@pytest.fixture(scope="module")
def U():
    from srsran_4g_amd import ue_dl
    return ue_dl


@pytest.fixture(scope="module", autouse=True)
def standard_rates(U):
    """these cases run at standard rates (N = 2048 at 100 PRB, as srsUE / C3); the reference
    default (3/4 rates) is restored afterwards and tested on its own"""
    U.use_standard_symbol_size(True)
    yield
    U.use_standard_symbol_size(False)


@pytest.mark.parametrize("nof_prb", [6, 15, 25, 50, 75, 100])
def test_ofdm_rx_matches_numpy(U, nof_prb):
    rng = np.random.default_rng(nof_prb)
    rx = U.OfdmRx(nof_prb)
    N, nre = rx.symbol_sz, 12 * nof_prb
    assert N == U.lib().srsran_symbol_sz(nof_prb)
    x = (rng.standard_normal(ofdm_np.sf_len(N)) + 1j * rng.standard_normal(ofdm_np.sf_len(N))).astype(np.complex64)
    got = rx.rx(x)
    exp = ofdm_np.ofdm_rx(x, N, nre)
    _fft_check(f"N{N}", got, exp)
    # round trip of a QAM grid
    g = (rng.choice([-3, -1, 1, 3], 14 * nre) + 1j * rng.choice([-3, -1, 1, 3], 14 * nre)).astype(np.complex64)
    back = rx.rx(ofdm_np.ofdm_tx(g, N, nre).astype(np.complex64))
    assert np.abs(back - g).max() < 1e-4 * 3
    rx.free()


def test_ofdm_normalize(U):
    rng = np.random.default_rng(1)
    rx = U.OfdmRx(100, normalize=True)
    x = (rng.standard_normal(30720) + 1j * rng.standard_normal(30720)).astype(np.complex64)
    exp = ofdm_np.ofdm_rx(x, 2048, 1200, normalize=True)
    _fft_check("N2048_normalize", rx.rx(x), exp)
    rx.free()


@pytest.fixture(scope="module")
def ref_cfo():
    if not ofdm_np.ref_available():  # on a HIP box the parity checker must be there: fail, never skip
        pytest.fail("oracle/_ref/libsrsref.so missing: srsran_vec_apply_cfo (the CFO checker) was not built")
    return ofdm_np.ref_apply_cfo


@pytest.mark.parametrize("n", [30720, 23040, 15360, 1001, 8, 5])
def test_cfo_correct_bitexact_vs_reference(U, ref_cfo, n):
    """srsran_cfo_correct equals the reference's srsran_vec_apply_cfo (cfo.c:105, vector_simd.c:1723-1774,
    compiled into _ref) bit for bit: the same phasor recurrence, FMA roundings and scalar tail, at the subframe
    lengths of 20 / 15 / 10 MHz (N = 2048 / 1536 / 1024) and at lengths with a tail"""
    rng = np.random.default_rng(2 + n)
    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    for f in (1.6e-5, -3.3e-4, 1e-4, -3.3e-3, 0.01, 0.37, 0.0):
        got = U.cfo_correct(x, f)
        want = ref_cfo(x, f)
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32), err_msg=f"f={f} n={n}")
        # the reference's phasor recurrence drifts from the exact rotation (|w^8| != 1 and arg(w^8) != 8 arg(w)
        # after rounding, compounded over n/8 blocks): up to ~2e-3 of |x| over a 20 MHz subframe at f = 1e-4 --
        # which is why parity is bit-exact against srsran_vec_apply_cfo, not a tolerance against exp()
        if abs(f) <= 5e-4:
            exact = ofdm_np.cfo(x, float(np.float32(f)))
            assert np.abs(got - exact).max() <= 1e-2 * np.abs(x).max()


@pytest.mark.parametrize("f", [2.5e-4, -1.6e-5, 1.3e-3])
def test_ofdm_gpu_batch_with_cfo(U, ref_cfo, f):
    """Device batch: 3 subframes x 2 antennas, CFO folded into the sample load: equal (FFT tolerance) to the
    reference's srsran_cfo_correct on each subframe buffer followed by the numpy FFT, and the transmitted
    grids come back.  A second call with another frequency rebuilds the cached phasor table."""
    import ctypes
    rng = np.random.default_rng(3)
    rx = U.OfdmRx(100)
    nsf, nrx, L, nre = 3, 2, 30720, 1200
    grids = (rng.choice([-1, 1], (nsf, nrx, 14 * nre)) + 1j * rng.choice([-1, 1], (nsf, nrx, 14 * nre)))
    x = np.stack([np.stack([ofdm_np.cfo(ofdm_np.ofdm_tx(grids[s, r], 2048, nre), -f) for r in range(nrx)])
                  for s in range(nsf)]).astype(np.complex64)
    d_in = torch.from_numpy(x.view(np.float32).reshape(-1)).cuda()
    d_out = torch.zeros(nsf * nrx * 14 * nre * 2, dtype=torch.float32, device="cuda")
    for ff in (f / 3, f):
        assert U.lib().srsran_ofdm_rx_gpu(ctypes.byref(rx.q), d_in.data_ptr(), d_out.data_ptr(), nrx, nsf,
                                          ctypes.c_float(ff), None) == 0
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.complex64).reshape(nsf, nrx, 14 * nre)
    assert np.abs(got - grids).max() < 2e-3  # the reference's phasor drift, up to ~1e-3 by the end of a subframe
    want = np.stack([np.stack([ofdm_np.ofdm_rx(ref_cfo(x[s, r], f), 2048, nre) for r in range(nrx)])
                     for s in range(nsf)])
    _fft_check(f"N2048_batch_cfo{f:g}", got, want)
    rx.free()


def test_ofdm_gpu_cfo_table_two_streams(U, ref_cfo):
    """The cached CFO phasor table of one OFDM object used from two streams (advisor round 4): the table for
    f2 is rebuilt on stream A behind a long-running kernel; a call on stream B with the same f2 finds it in the
    cache and must wait for that rebuild instead of reading f1's table."""
    import ctypes
    rng = np.random.default_rng(4)
    rx = U.OfdmRx(100)
    nsf, nrx, nre = 2, 2, 1200
    x = (rng.standard_normal((nsf, nrx, 30720)) + 1j * rng.standard_normal((nsf, nrx, 30720))).astype(np.complex64)
    d_in = torch.from_numpy(x.view(np.float32).reshape(-1)).cuda()
    outs = [torch.zeros(nsf * nrx * 14 * nre * 2, dtype=torch.float32, device="cuda") for _ in range(2)]
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    f1, f2 = 1.1e-4, -2.7e-4
    busy = torch.randn(4096, 4096, device="cuda")
    for rep in range(3):
        lib = U.lib()
        assert lib.srsran_ofdm_rx_gpu(ctypes.byref(rx.q), d_in.data_ptr(), outs[0].data_ptr(), nrx, nsf,
                                      ctypes.c_float(f1), ctypes.c_void_p(sa.cuda_stream)) == 0
        torch.cuda.synchronize()
        with torch.cuda.stream(sa):
            for _ in range(8):
                busy = busy @ busy
                busy = busy / busy.abs().max()
        assert lib.srsran_ofdm_rx_gpu(ctypes.byref(rx.q), d_in.data_ptr(), outs[0].data_ptr(), nrx, nsf,
                                      ctypes.c_float(f2), ctypes.c_void_p(sa.cuda_stream)) == 0
        assert lib.srsran_ofdm_rx_gpu(ctypes.byref(rx.q), d_in.data_ptr(), outs[1].data_ptr(), nrx, nsf,
                                      ctypes.c_float(f2), ctypes.c_void_p(sb.cuda_stream)) == 0
        torch.cuda.synchronize()
        a = outs[0].cpu().numpy().view(np.complex64)
        b = outs[1].cpu().numpy().view(np.complex64)
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32), err_msg=f"rep {rep}")
    want = np.stack([np.stack([ofdm_np.ofdm_rx(ref_cfo(x[s, r], f2), 2048, nre) for r in range(nrx)])
                     for s in range(nsf)]).reshape(-1)
    _fft_check("N2048_two_streams", b, want)
    rx.free()


@pytest.mark.parametrize("nof_prb,N", [(25, 384), (50, 768), (75, 1024), (100, 1536)])
def test_ofdm_rx_reference_default_rates(U, nof_prb, N):
    """the reference's default 3/4 sampling rates (phy_common.c:31-35, 361-385): non-power-of-two
    FFT sizes (radix-3 stage) at 25 / 50 / 100 PRB"""
    U.use_standard_symbol_size(False)
    try:
        assert U.lib().srsran_symbol_sz(nof_prb) == N and not U.symbol_size_is_standard()
        assert U.lib().srsran_nof_prb(N) == nof_prb and U.lib().srsran_sampling_freq_hz(nof_prb) == 15000 * N
        rng = np.random.default_rng(N)
        rx = U.OfdmRx(nof_prb)
        nre = 12 * nof_prb
        assert rx.symbol_sz == N
        x = (rng.standard_normal(ofdm_np.sf_len(N)) + 1j * rng.standard_normal(ofdm_np.sf_len(N))).astype(np.complex64)
        exp = ofdm_np.ofdm_rx(x, N, nre)
        _fft_check(f"N{N}_default_rates", rx.rx(x), exp)
        rx.free()
    finally:
        U.use_standard_symbol_size(True)
