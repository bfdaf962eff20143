"""MBSFN subframes, host side (no GPU): the test infrastructure the GPU tests of tests/test_mbsfn_gpu.py rely on.

* the MBSFN reference signals of the oracle (oracle_mbsfn_pilots, a restatement of refsignal_dl.c:382-422) equal
  synth/'s independent transmitter-side restatement, and the Gold generator under both is the reference's
  (pinned in tests/test_phy_oracle.py); refsignal_dl.c itself is unbuildable here (srsran/srsran.h), so the
  c_init / index expressions are parity-unpinned restatements;
* the MBSFN OFDM layout (ofdm.c:522-535 / 652-674): sample offsets, the guard, and synth's modulator inverted by
  the oracle's numpy demodulator;
* the oracle MBSFN estimator recovers a flat channel exactly from a noiseless subframe (every filter), and a
  frequency-selective one to within its interpolation error."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ofdm_np  # noqa: E402
from oracle import Oracle  # noqa: E402
from synth import synth as S  # noqa: E402


@pytest.fixture(scope="module")
def ora():
    return Oracle()


@pytest.mark.parametrize("nprb,area", [(6, 0), (25, 1), (50, 7), (100, 255)])
def test_mbsfn_pilots_match_synth(ora, nprb, area):
    for sf in (1, 3, 8):
        got = ora.mbsfn_pilots(nprb, area, sf)
        want = S.mbsfn_rs(area, nprb, sf)
        assert np.abs(got - want).max() < 1e-6
    # the sequences differ between areas and subframes
    assert np.abs(ora.mbsfn_pilots(nprb, area, 1) - ora.mbsfn_pilots(nprb, area, 2)).max() > 0.5
    assert np.abs(ora.mbsfn_pilots(nprb, area, 1) - ora.mbsfn_pilots(nprb, (area + 1) % 256, 1)).max() > 0.5


@pytest.mark.parametrize("N", [128, 512, 1536, 2048])
@pytest.mark.parametrize("nr", [1, 2])
def test_mbsfn_ofdm_layout(N, nr):
    st = ofdm_np.mbsfn_symbol_starts(N, nr)
    ext = ofdm_np.symbol_starts(N, 1)
    assert st[nr:] == ext[nr:]  # the guard realigns the MBSFN region with the extended-CP layout
    cpn0, cpn = ofdm_np.cp_lens(N, 0)
    assert st[0] == cpn0 and (nr == 1 or st[1] == cpn0 + N + cpn)
    nre = 12 * {128: 6, 512: 25, 1536: 75, 2048: 100}[N]
    rng = np.random.default_rng(N + nr)
    grid = (rng.standard_normal((12, nre)) + 1j * rng.standard_normal((12, nre))) / np.sqrt(2)
    x = S.ofdm_tx_mbsfn(grid, N, nr)
    assert x.size == ofdm_np.sf_len(N, 1) == 15 * N
    back = ofdm_np.ofdm_rx_mbsfn(x, N, nre, nr).reshape(12, nre)  # ifft (1/N) then the unnormalised FFT
    assert np.abs(back - grid).max() < 1e-9


@pytest.mark.parametrize("ftype,coef", [(1, 0.1), (2, 0.0), (0, 4.0)])
@pytest.mark.parametrize("nports", [1, 2])
def test_oracle_mbsfn_estimator_flat_channel(ora, ftype, coef, nports):
    nprb, cell_id, sf, area = 25, 11, 3, 1
    nre = 12 * nprb
    g = S.mbsfn_grid(nprb, cell_id, sf, area, 2)
    h = 0.8 - 0.3j
    grid = np.zeros((1, 14 * nre), np.complex64)
    grid[0, :12 * nre] = (h * g).reshape(-1)
    # (port 1, if configured, sends nothing in srsRAN's MBSFN subframes, enb_dl.c:348-351: only port 0 is checked)
    ce, noise, _ = ora.chest_dl_mbsfn(grid, nprb, cell_id, nports, sf, area, noise_alg=1, filter_type=ftype,
                                      coef0=coef, coef1=1.0)
    est = ce[0, 0, :12 * nre]
    assert np.abs(est - h).max() < 1e-5, np.abs(est - h).max()
    assert noise == 0.0  # PSS noise: the kept state (subframes 0 / 5 are never MBSFN)
    assert np.all(ce[0, 0, 12 * nre:] == 0)  # rows 12 / 13 are not written
    # REFS noise in an MBSFN subframe: estimate_noise_pilots cuts the 20 N_RB estimates into 3 rows of floor(20 N_RB / 3)
    # that straddle the CRS and the MBSFN pilots (chest_dl.c:331-342; the reference warns it is not supported): on a
    # flat channel every estimate is h and the residuals vanish all the same
    _, noise_refs, _ = ora.chest_dl_mbsfn(grid, nprb, cell_id, nports, sf, area, noise_alg=0, filter_type=ftype,
                                          coef0=coef, coef1=1.0)
    assert nports == 2 or noise_refs < 1e-10  # (port 1 sees no CRS of its own: its residual is not zero)


def test_oracle_mbsfn_estimator_selective_channel(ora):
    """a two-tap channel: the interpolated estimate within 2 % of the true response on every RE (TRIANGLE 0.1, srsUE's
    MBSFN configuration)"""
    nprb, cell_id, sf, area, N = 50, 77, 6, 3, 1024
    nre = 12 * nprb
    g = S.mbsfn_grid(nprb, cell_id, sf, area, 2)
    k = np.concatenate([np.arange(N - nre // 2, N), np.arange(1, nre // 2 + 1)])
    H = 1.0 + 0.3 * np.exp(-2j * np.pi * k * 3 / N)
    grid = np.zeros((1, 14 * nre), np.complex64)
    grid[0, :12 * nre] = (g * H[None, :]).reshape(-1)
    ce, _, _ = ora.chest_dl_mbsfn(grid, nprb, cell_id, 1, sf, area, noise_alg=1, filter_type=1, coef0=0.1)
    est = ce[0, 0, :12 * nre].reshape(12, nre)
    assert np.abs(est - H[None, :]).max() < 0.02 * np.abs(H).max()
