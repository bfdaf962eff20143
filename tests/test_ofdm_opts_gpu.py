"""srsran_ofdm_cfg_t options of the GPU OFDM receiver and modulator (ofdm.c:151-157, 228-233, 357-449, 474-519,
585-690) against oracle/ofdm_np.py's restatement (numpy double-precision FFT -- FFTW is absent and no reference test
pins the transform): keep_dc, freq_shift_f (the receiver's input multiplied in place, the modulator's
output), rx_window_offset (clamped and written back; window_offset_n samples into the cyclic prefix and its phase
ramp removed), phase_compensation_hz (per-symbol phasors; srsran_ofdm_rx_set_prb turns it off), and their
combinations, on the one-wave kernels (N = 2048, 1536) and the Stockham one (other N).  Tolerance: the FFT's
1e-6 of the largest bin (test_ofdm_gpu.py) widened to 2e-6 for the products by the option tables."""
import ctypes

import numpy as np
import pytest

import ofdm_np

pytestmark = pytest.mark.gpu
TOL = 2e-6


@pytest.fixture(scope="module")
def U():
    from srsran_4g_amd import tdec, ue_dl
    if not tdec.gpu_available():
        pytest.fail("no HIP device on a GPU test run")
    ue_dl.use_standard_symbol_size(True)
    yield ue_dl
    ue_dl.use_standard_symbol_size(False)


def _err(got, exp):
    return float(np.abs(got - exp).max() / np.abs(exp).max())


def _samples(rng, n):
    return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)


CASES = [  # (nof_prb, cp, keep_dc, freq_shift, window_offset, phase_hz, normalize)
    (100, 0, True, 0.0, 0.0, 0.0, False),
    (100, 0, False, 0.5, 0.0, 0.0, False),
    (100, 0, False, 0.0, 0.5, 0.0, False),
    (100, 0, False, 0.0, 0.0, 2.6e9, False),
    (100, 0, False, 0.0, 0.0, 2.6e9, True),
    (75, 0, True, 0.0, 0.3, 1.8e9, True),
    (25, 0, False, -0.5, 0.25, 3.5e9, False),
    (50, 1, True, 0.0, 1.0, 7.5e8, False),
    (6, 0, False, 0.5, 0.7, 2.1e9, True),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}prb_cp{c[1]}_dc{int(c[2])}_fs{c[3]}_w{c[4]}_ph{c[5]:g}_n{int(c[6])}"
                                             for c in CASES])
def test_rx_options_match_oracle(U, case):
    nprb, cp, keep_dc, fs, wo, ph, norm = case
    rng = np.random.default_rng(nprb * 7 + cp)
    rx = U.OfdmRx(nprb, normalize=norm, cp=cp, keep_dc=keep_dc, freq_shift_f=fs, rx_window_offset=wo,
                  phase_compensation_hz=ph)
    try:
        N, nre = rx.symbol_sz, 12 * nprb
        assert rx.cfg.rx_window_offset == pytest.approx(wo)  # in [0, 100]: unchanged by the clamp
        x = _samples(rng, ofdm_np.sf_len(N, cp))
        x0 = x.copy()
        got = rx.rx_inplace(x)
        exp, shifted = ofdm_np.ofdm_rx_opts(x0, N, nre, normalize=norm, ext=cp, keep_dc=keep_dc, freq_shift=fs,
                                            window_offset=wo, phase_hz=ph)
        assert _err(got, exp) <= TOL, _err(got, exp)
        if fs:  # the input buffer itself carries the shift afterwards (ofdm.c:569-571)
            assert _err(x, shifted) <= 1e-6
        else:
            assert np.array_equal(x, x0)
    finally:
        rx.free()


def test_window_offset_clamp_and_limit(U):
    # a negative offset is clamped to 0 and written back to the caller's configuration (ofdm.c:152)
    rx = U.OfdmRx(25, rx_window_offset=-0.5)
    try:
        assert rx.cfg.rx_window_offset == 0.0
        x = _samples(np.random.default_rng(3), rx.q.sf_sz)
        assert _err(rx.rx(x), ofdm_np.ofdm_rx(x, rx.symbol_sz, 300)) <= 1e-6
    finally:
        rx.free()
    # above 1 the window leaves the cyclic prefix (the reference reads before its buffer): refused
    with pytest.raises(RuntimeError):
        U.OfdmRx(25, rx_window_offset=1.5)


def test_setters_and_set_prb(U):
    rng = np.random.default_rng(5)
    rx = U.OfdmRx(100)
    L = U.lib()
    try:
        N = rx.symbol_sz
        x = _samples(rng, rx.q.sf_sz)
        assert L.srsran_ofdm_set_phase_compensation(ctypes.byref(rx.q), 2.4e9) == 0
        exp, _ = ofdm_np.ofdm_rx_opts(x, N, 1200, phase_hz=2.4e9)
        assert _err(rx.rx(x), exp) <= TOL
        assert L.srsran_ofdm_set_freq_shift(ctypes.byref(rx.q), 0.5) == 0
        exp, _ = ofdm_np.ofdm_rx_opts(x, N, 1200, phase_hz=2.4e9, freq_shift=0.5)
        assert _err(rx.rx(x), exp) <= TOL
        assert L.srsran_ofdm_set_freq_shift(ctypes.byref(rx.q), 0.0) == 0  # DC removed again (ofdm.c:426-428)
        exp, _ = ofdm_np.ofdm_rx_opts(x, N, 1200, phase_hz=2.4e9)
        assert _err(rx.rx(x), exp) <= TOL
        # set_prb: phase compensation back to 0 Hz (ofdm_init_mbsfn_ with a cp / nof_prb configuration)
        assert L.srsran_ofdm_rx_set_prb(ctypes.byref(rx.q), 0, 50) == 0
        assert rx.q.cfg.phase_compensation_hz == 0.0
        x = _samples(rng, rx.q.sf_sz)
        assert _err(rx.rx(x), ofdm_np.ofdm_rx(x, rx.symbol_sz, 600)) <= 1e-6
    finally:
        rx.free()


def test_rx_gpu_shift_and_cfo(U):
    """srsran_ofdm_rx_gpu on device buffers: the CFO correction, then the frequency shift, in the transform"""
    import torch
    rng = np.random.default_rng(9)
    rx = U.OfdmRx(100, freq_shift_f=0.5, keep_dc=False)
    try:
        N, n = rx.symbol_sz, rx.q.sf_sz
        x = _samples(rng, 2 * n).reshape(2, n)
        d_in = torch.from_numpy(x.view(np.float32)).cuda()
        d_out = torch.zeros((2, 14 * 1200 * 2), dtype=torch.float32, device="cuda")
        f = 1e-4
        assert U.lib().srsran_ofdm_rx_gpu(ctypes.byref(rx.q), d_in.data_ptr(), d_out.data_ptr(), 2, 1, f, None) == 0
        torch.cuda.synchronize()
        got = d_out.cpu().numpy().view(np.complex64)
        for r in range(2):
            exp, _ = ofdm_np.ofdm_rx_opts(ofdm_np.ref_apply_cfo(x[r], f), N, 1200, freq_shift=0.5)
            assert _err(got[r], exp) <= TOL
    finally:
        rx.free()


TX_CASES = [  # (nof_prb, cp, keep_dc, freq_shift, phase_hz, normalize)
    (100, 0, False, 0.0, 0.0, False),
    (100, 0, True, 0.0, 2.6e9, False),
    (75, 0, False, 0.5, 0.0, True),
    (25, 1, True, -0.5, 1.9e9, True),
    (15, 0, False, 0.5, 3.1e9, False),
]


@pytest.mark.parametrize("case", TX_CASES, ids=[f"{c[0]}prb_cp{c[1]}_dc{int(c[2])}_fs{c[3]}_ph{c[4]:g}_n{int(c[5])}"
                                                for c in TX_CASES])
def test_tx_options_match_oracle_and_round_trip(U, case):
    nprb, cp, keep_dc, fs, ph, norm = case
    rng = np.random.default_rng(nprb + 100 * cp)
    tx = U.OfdmRx(nprb, normalize=norm, cp=cp, keep_dc=keep_dc, freq_shift_f=fs, phase_compensation_hz=ph, tx=True)
    try:
        N, nre, ns = tx.symbol_sz, 12 * nprb, 2 * tx.q.nof_symbols
        g = (rng.choice([-1, 1], ns * nre) + 1j * rng.choice([-1, 1], ns * nre)).astype(np.complex64)
        got = tx.tx(g)
        exp = ofdm_np.ofdm_tx_opts(g, N, nre, normalize=norm, ext=cp, keep_dc=keep_dc, freq_shift=fs, phase_hz=ph)
        assert _err(got, exp) <= TOL, _err(got, exp)
    finally:
        tx.free()
    # the receiver with the same options undoes it (the shift's conjugate at the receiver, as eNB UL does for UE UL)
    rx = U.OfdmRx(nprb, normalize=norm, cp=cp, keep_dc=keep_dc, freq_shift_f=-fs, phase_compensation_hz=ph)
    try:
        back = rx.rx(got)
        scale = 1.0 if norm else float(N)
        assert np.abs(back / scale - g).max() < 1e-4
    finally:
        rx.free()


@pytest.mark.parametrize("nprb,cp,fs,cfo", [(100, 0, 0.0, 0.0), (75, 0, 0.0, 2e-5), (25, 1, 0.5, 0.0), (6, 0, 0.0, 0.0)])
def test_rx_gpu_sc16_equals_float(U, nprb, cp, fs, cfo):
    """srsran_ofdm_rx_gpu_sc16 on int16 I/Q == srsran_ofdm_rx_gpu on the host conversion (float)x * scale, bit for
    bit, on the one-wave kernels (N = 2048, 1536) and the Stockham one, with a CFO or a frequency shift"""
    import torch
    rng = np.random.default_rng(nprb + cp)
    rx = U.OfdmRx(nprb, cp=cp, freq_shift_f=fs)
    try:
        n = rx.q.sf_sz
        q = rng.integers(-20000, 20000, (2, 2, n, 2), dtype=np.int16)  # [sf][rx][sample][I/Q]
        scale = float(np.float32(1.0 / 32767.0))
        xf = (q[..., 0].astype(np.float32) * np.float32(scale) + 1j * (q[..., 1].astype(np.float32) * np.float32(scale)))
        d_f = torch.from_numpy(xf.astype(np.complex64).view(np.float32)).cuda()
        d_q = torch.from_numpy(q).cuda()
        nout = 2 * 2 * 2 * rx.q.nof_symbols * rx.q.nof_re
        o_f = torch.zeros(2 * nout, dtype=torch.float32, device="cuda")
        o_q = torch.zeros(2 * nout, dtype=torch.float32, device="cuda")
        L = U.lib()
        assert L.srsran_ofdm_rx_gpu(ctypes.byref(rx.q), d_f.data_ptr(), o_f.data_ptr(), 2, 2, cfo, None) == 0
        assert L.srsran_ofdm_rx_gpu_sc16(ctypes.byref(rx.q), d_q.data_ptr(), scale, o_q.data_ptr(), 2, 2, cfo,
                                         None) == 0
        torch.cuda.synchronize()
        assert torch.equal(o_f, o_q)
        assert o_f.abs().max() > 0
    finally:
        rx.free()
