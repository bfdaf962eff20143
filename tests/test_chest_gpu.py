"""GPU parity of the DL CRS channel estimator (srsUE default configuration) against the oracle
(oracle/phy_oracle.c, a restatement of chest_dl.c / refsignal_dl.c whose buildable pieces --
Gauss filter, conv_same, Gold sequence -- are pinned to the reference in test_phy_oracle.py).
Estimates are compared at float tolerance (the reductions sum in a different order)."""
import numpy as np
import pytest
import torch

from oracle import Oracle

from test_phy_oracle import make_subframe

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ora():
    return Oracle()


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


@pytest.mark.parametrize("nof_prb,cell_id,nports,nrx,sf", [(100, 1, 2, 2, 1), (100, 5, 2, 2, 0), (50, 7, 1, 1, 6),
                                                            (25, 301, 2, 1, 9), (6, 2, 4, 2, 3), (100, 0, 1, 2, 5)])
def test_chest_matches_oracle(U, ora, nof_prb, cell_id, nports, nrx, sf):
    rng = np.random.default_rng(nof_prb + cell_id)
    Y, H, _ = make_subframe(ora, rng, nof_prb=nof_prb, cell_id=cell_id, nports=nports, nrx=nrx, sf_idx=sf, snr_db=25)
    ch = U.ChestDl(U.cell(nof_prb, nports, cell_id), nrx)
    ce, res = ch.estimate(Y, sf, U.srsue_chest_cfg())
    ceo, st = ora.chest_dl(Y, nof_prb, cell_id, nports, sf, U.lib().srsran_symbol_sz(nof_prb))
    scale = np.abs(ceo).max()
    assert np.abs(ce - ceo).max() < 2e-5 * scale
    assert res.noise_estimate == pytest.approx(st["noise"], rel=1e-4)
    assert res.rsrp == pytest.approx(st["rsrp"], rel=1e-4)
    assert res.cfo == pytest.approx(st["cfo"], rel=1e-3, abs=1e-6)
    ch.free()


def test_chest_device_rows(U, ora):
    rng = np.random.default_rng(1)
    Y, H, _ = make_subframe(ora, rng, snr_db=25)
    ch = U.ChestDl(U.cell(100, 2, 1), 2)
    d_grid = torch.from_numpy(Y.view(np.float32)).cuda()
    d_ce = torch.zeros(2 * 2 * 1200 * 2, dtype=torch.float32, device="cuda")
    d_res = torch.zeros(4, dtype=torch.float32, device="cuda")
    import ctypes
    rc = U.lib().srsran_chest_dl_gpu_estimate(ctypes.byref(ch.q), 1, d_grid.data_ptr(), d_ce.data_ptr(), 0,
                                              d_res.data_ptr(), None)
    assert rc == 0
    torch.cuda.synchronize()
    ceo, st = ora.chest_dl(Y, 100, 1, 2, 1, 2048)
    rows = d_ce.cpu().numpy().view(np.complex64).reshape(2, 2, 1200)
    assert np.abs(rows - ceo[:, :, :1200]).max() < 2e-5 * np.abs(ceo).max()
    r = d_res.cpu().numpy()
    assert r[0] == pytest.approx(st["noise"], rel=1e-4) and r[1] == pytest.approx(st["rsrp"], rel=1e-4)
    ch.free()


def test_chest_zero_cfg_auto_filter(U, ora):
    """srsran_chest_dl_estimate (zeroed cfg): Gauss filter with stddev 200 * noise."""
    rng = np.random.default_rng(2)
    Y, H, _ = make_subframe(ora, rng, snr_db=20)
    ch = U.ChestDl(U.cell(100, 2, 1), 2)
    ce, res = ch.estimate(Y, 1)
    assert np.all(np.isfinite(ce)) and res.noise_estimate > 0
    err = np.abs(ce[:, :, :1200] - H) ** 2
    assert err.mean() < 0.05
    ch.free()
