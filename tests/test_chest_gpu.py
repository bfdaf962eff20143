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
    assert res.cfo == pytest.approx(st["cfo"], rel=1e-4, abs=1e-6)  # abs: the static channel's CFO is ~0
    ch.free()


@pytest.mark.parametrize("nof_prb,cell_id,nports,nrx,sf,rot", [(100, 1, 2, 2, 1, 0.013), (50, 7, 1, 1, 6, -0.021),
                                                                (25, 301, 2, 1, 9, 0.004), (6, 2, 4, 2, 3, 0.03)])
def test_chest_cfo_estimate_matches_oracle(U, ora, nof_prb, cell_id, nports, nrx, sf, rot):
    """chest_estimate_cfo (chest_dl.c:618-641) on a subframe with a real frequency offset (a phase advance of `rot`
    rad a symbol): the GPU estimate within 1e-4 (relative) of the oracle's -- north_star's soft-value tolerance"""
    rng = np.random.default_rng(nof_prb + cell_id + 7)
    Y, H, _ = make_subframe(ora, rng, nof_prb=nof_prb, cell_id=cell_id, nports=nports, nrx=nrx, sf_idx=sf, snr_db=25)
    Y = (Y.reshape(nrx, 14, -1) * np.exp(1j * rot * np.arange(14))[None, :, None]).astype(np.complex64).reshape(nrx, -1)
    ch = U.ChestDl(U.cell(nof_prb, nports, cell_id), nrx)
    _, res = ch.estimate(Y, sf, U.srsue_chest_cfg())
    _, st = ora.chest_dl(Y, nof_prb, cell_id, nports, sf, U.lib().srsran_symbol_sz(nof_prb))
    assert abs(st["cfo"]) > 1e-4
    assert res.cfo == pytest.approx(st["cfo"], rel=1e-4)
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


def _doppler_subframe(ora, rng, nof_prb, cell_id, nports, nrx, sf_idx, snr_db=25, fd=0.02, delay=0.0, N=2048):
    """make_subframe with a channel that rotates over the subframe (phase 2 pi fd per symbol, so INTERPOLATE has
    something to follow) and, with `delay`, a timing error of `delay` samples (a phase ramp over the subcarriers
    that correct_sync_error detects from the CRS)"""
    Y, H, X = make_subframe(ora, rng, nof_prb=nof_prb, cell_id=cell_id, nports=nports, nrx=nrx, sf_idx=sf_idx,
                            snr_db=snr_db)
    nre = 12 * nof_prb
    Y = Y.reshape(nrx, 14, nre) * np.exp(2j * np.pi * fd * np.arange(14))[None, :, None]
    if delay:
        Y = Y * np.exp(-2j * np.pi * delay * np.arange(nre) / N)[None, None, :]
    return Y.reshape(nrx, 14 * nre).astype(np.complex64)


OPT_CASES = [
    # (name, nof_prb, cell_id, nports, nrx, estimator, noise_alg, order, std)
    ("interp_2port", 100, 1, 2, 2, 1, 0, 4, 1.0),
    ("interp_1port_order6", 50, 7, 1, 1, 1, 0, 6, 2.0),
    ("interp_4port", 25, 301, 4, 2, 1, 0, 4, 1.0),
    ("interp_auto_filter", 100, 4, 2, 2, 1, 0, 0, 0.0),
    ("average_pss", 100, 11, 2, 2, 0, 1, 4, 1.0),
    ("interp_pss", 50, 2, 2, 1, 1, 1, 4, 1.0),
    ("average_empty", 100, 5, 2, 2, 0, 2, 4, 1.0),
    ("interp_empty_4port", 6, 3, 4, 1, 1, 2, 2, 1.0),
    ("average_pss_auto", 25, 9, 1, 2, 0, 1, 0, 0.0),
    # TRIANGLE ({w, 1 - 2w, w}, chest_common.c:62-68; `order` = w) and NONE (no average_pilots, chest_dl.c:724-725)
    ("average_triangle", 100, 1, 2, 2, 0, 0, 0.25, 0.0, 1),
    ("interp_triangle_pss", 50, 8, 1, 1, 1, 1, 0.1, 0.0, 1),
    ("average_none", 100, 3, 2, 2, 0, 0, 0, 0.0, 2),
    ("average_none_1port", 25, 10, 1, 2, 0, 0, 0, 0.0, 2),
    ("interp_none_4port", 25, 301, 4, 2, 1, 0, 0, 0.0, 2),
    ("interp_none_empty", 50, 5, 2, 1, 1, 2, 0, 0.0, 2),
]


@pytest.mark.parametrize("case", OPT_CASES, ids=[c[0] for c in OPT_CASES])
def test_chest_options_match_oracle(U, ora, case):
    """srsUE's non-default estimator knobs (ue.conf interpolate_subframe_enabled, snr_estim_alg,
    estimator_fil_order / _stddev / _auto; chest_dl.c:437-555, 402-433, 655-745) against the oracle's
    restatement (oracle_chest_dl_ext), over a sequence of subframes on one object so that PSS / EMPTY noise is
    estimated in subframes 0 / 5 and kept in the others (q->noise_estimate, also the automatic filter's input)"""
    name, nof_prb, cell_id, nports, nrx, est, noise, order, std = case[:9]
    ftype = case[9] if len(case) > 9 else 0
    rng = np.random.default_rng(len(name) + nof_prb)
    N = U.lib().srsran_symbol_sz(nof_prb)
    ch = U.ChestDl(U.cell(nof_prb, nports, cell_id), nrx)
    cfg = U.chest_cfg(est, noise, order, std, filter_type=ftype)
    state = np.zeros((4, 4), np.float32)
    for tti in (4, 5, 6, 10, 11):
        sf = tti % 10
        Y = _doppler_subframe(ora, rng, nof_prb, cell_id, nports, nrx, sf, N=N)
        ce, res = ch.estimate(Y.copy(), tti, cfg)
        ceo, st, _, state = ora.chest_dl_ext(Y, nof_prb, cell_id, nports, sf, N, 0, est, noise, order, std,
                                             noise_state=state, filter_type=ftype)
        scale = np.abs(ceo).max()  # 0 before the first kept noise estimate with an automatic filter: the
        # reference's Gauss filter of stddev 0 is not normal, conv_same runs no taps and the estimate is all zeros
        assert np.abs(ce - ceo).max() <= 2e-5 * scale, (tti, np.abs(ce - ceo).max(), scale)
        assert res.noise_estimate == pytest.approx(st["noise"], rel=1e-4), tti
        assert res.rsrp == pytest.approx(st["rsrp"], rel=1e-4), tti
        for r in range(nrx):
            for p in range(nports):
                assert ch.q.noise_estimate[r][p] == pytest.approx(state[r, p], rel=1e-4), (tti, r, p)
    ch.free()


@pytest.mark.parametrize("delay,nports", [(0.4, 2), (-0.7, 1), (0.01, 2), (1.3, 4)])
def test_chest_sync_error_correction(U, ora, delay, nports):
    """correct_sync_error (chest_dl.c:750-804): the timing error estimated from the CRS phase slope of every
    port, and where it exceeds 0.05 samples every symbol of the grid rotated by srsran_vec_apply_cfo -- in the
    caller's buffer, as the reference corrects it in place -- before the estimate; res.sync_error"""
    nof_prb, cell_id, nrx = 50, 13, 2
    rng = np.random.default_rng(int(100 * abs(delay)) + nports)
    N = U.lib().srsran_symbol_sz(nof_prb)
    ch = U.ChestDl(U.cell(nof_prb, nports, cell_id), nrx)
    cfg = U.chest_cfg(0, 0, 4, 1.0, sync_error=True)
    Y = _doppler_subframe(ora, rng, nof_prb, cell_id, nports, nrx, 2, fd=0.0, delay=delay, N=N)
    grids = [Y[r].copy() for r in range(nrx)]
    ce, res = ch.estimate(grids, 2, cfg)
    ceo, st, Yo, _ = ora.chest_dl_ext(Y, nof_prb, cell_id, nports, 2, N, 0, 0, 0, 4, 1.0, sync=True)
    assert res.sync_error == pytest.approx(st["sync_error"], rel=1e-4, abs=1e-6)
    if abs(delay) > 0.1:
        assert abs(st["sync_error"]) > 0.05
    for r in range(nrx):  # the corrected grid is written back (or left alone below the threshold)
        assert np.abs(grids[r] - Yo[r]).max() < 1e-5 * np.abs(Yo).max(), r
    assert np.abs(ce - ceo).max() < 2e-5 * np.abs(ceo).max()
    ch.free()


def _batch_vs_host(U, ora, est, noise, nports, order=4, sync=False, delay=0.0, ftype=0, expect_ok=True):
    from synth import synth as S
    from srsran_4g_amd import sch as SCH
    import ofdm_np
    TBS = 75376 if nports == 2 else 61664
    ntb = 2 if nports == 2 else 1
    scheme = "cdd" if nports == 2 else "port0"
    cell_id = 1
    ue = U.UeDl(U.cell(100, nports, cell_id), 2)
    ue.cfg.chest_cfg = U.chest_cfg(est, noise, order, 1.0, sync_error=sync, filter_type=ftype)
    ue2 = U.UeDl(U.cell(100, nports, cell_id), 2)
    ue2.cfg.chest_cfg = U.chest_cfg(est, noise, order, 1.0, sync_error=sync, filter_type=ftype)
    rng = np.random.default_rng(40 + est + 3 * noise + nports + int(7 * order) + (11 if sync else 0) + 13 * ftype)
    ttis = (4, 5, 6, 10, 11)
    first_ok = 0
    if not expect_ok:
        first_ok = len(ttis)
    elif order == 0 and noise != 0 and ftype == 0:
        # the automatic filter's width comes from the kept PSS / EMPTY estimate, 0 before the first subframe 0 / 5:
        # a Gauss filter of stddev 0 is not normal, conv_same runs no taps and the estimate is all zeros (the
        # reference's too), so the first subframes fail in both paths; from the second subframe 0 / 5 on it is a noise
        # power (the first PSS estimate is taken against that zero estimate)
        ttis, first_ok = (5, 6, 10, 11, 15, 16), 2
    samples, entries, keep, pls_all = [], [], [], []
    d_pl = torch.zeros((len(ttis), 2, TBS // 8 + 64), dtype=torch.uint8, device="cuda")
    for b, tti in enumerate(ttis):
        pls = [rng.integers(0, 256, TBS // 8, dtype=np.uint8) for _ in range(ntb)]
        x, nre = S.pdsch_subframe(100, cell_id, nports, tti, 1, 0x1234, TBS, 6, 0, pls, scheme=scheme, snr_db=30.0,
                                  rng=rng, N=2048, sync=True, delay=delay)
        sb = [SCH.SoftbufferRx(nof_prb=100) for _ in range(ntb)]
        cfg = U.pdsch_cfg(100, nre, (TBS,) * ntb, (6,) * ntb, softbuffers=sb, scheme=scheme, nof_ports=nports)
        keep += [sb, cfg]
        samples.append(x)
        pls_all.append(pls)
        entries.append((tti, 1, cfg, [d_pl[b, q].data_ptr() for q in range(ntb)], [1] * ntb))
    d_x = torch.from_numpy(np.stack(samples).view(np.float32)).cuda()
    d_res = torch.full((ntb * len(ttis),), 7, dtype=torch.int32, device="cuda")
    d_avg = torch.zeros(ntb * len(ttis), dtype=torch.float32, device="cuda")
    assert ue.gpu_decode_batch(entries, d_x.data_ptr(), d_res.data_ptr(), d_avg.data_ptr(), 0.0, None) == \
        ntb * len(ttis)
    torch.cuda.synchronize()
    res, pl = d_res.cpu().numpy(), d_pl.cpu().numpy()
    state = np.zeros((4, 4), np.float32)
    for b, tti in enumerate(ttis):
        assert ue2.fft_estimate(samples[b], tti, 1) == 0
        grids = np.stack([ofdm_np.ofdm_rx(v, 2048, 1200) for v in samples[b]]).astype(np.complex64)
        _, st, _, state = ora.chest_dl_ext(grids, 100, cell_id, nports, tti % 10, 2048, 0, est, noise, order, 1.0,
                                           sync=sync, noise_state=state, filter_type=ftype)
        assert ue2.q.chest_res.noise_estimate == pytest.approx(st["noise"], rel=1e-4), tti
        if sync:
            assert ue2.q.chest_res.sync_error == pytest.approx(st["sync_error"], rel=1e-4, abs=1e-6), tti
            assert abs(st["sync_error"]) > 0.05
        sb = [SCH.SoftbufferRx(nof_prb=100) for _ in range(ntb)]
        cfg = U.pdsch_cfg(100, entries[b][2].grant.nof_re, (TBS,) * ntb, (6,) * ntb, softbuffers=sb, scheme=scheme,
                          nof_ports=nports)
        ret, out = ue2.decode_pdsch(cfg, tti, 1)
        keep.append(sb)
        for q in range(ntb):
            assert (res[ntb * b + q] == 0) == bool(out[q][0]), (b, q)
            if b >= first_ok:
                assert res[ntb * b + q] == 0, (b, q)
            if res[ntb * b + q] == 0:
                assert np.array_equal(pl[b, q, : TBS // 8], pls_all[b][q]), (b, q)
                assert np.array_equal(pl[b, q, : TBS // 8 + 6], out[q][1][: TBS // 8 + 6]), (b, q)
    ue.free()
    ue2.free()


@pytest.mark.parametrize("est,noise,nports", [(1, 0, 2), (0, 1, 1), (1, 1, 1), (0, 2, 2), (1, 2, 2)])
def test_ue_dl_batch_estimator_options(U, ora, est, noise, nports):
    """srsran_ue_dl_gpu_decode_batch with INTERPOLATE / PSS / EMPTY in cfg->chest_cfg decodes and equals the
    host-synchronous UE DL path subframe by subframe (kept noise carried across the batch in subframe order).
    synth/ transmits the PSS / SSS (every port, as the reference eNB), so the PSS / EMPTY estimates of subframes 0 / 5
    are noise powers: every TB decodes at 30 dB, and the host-synchronous path's noise estimate of every subframe
    equals the oracle restatement (oracle_chest_dl_ext on the numpy FFT of the same samples, the kept estimate
    carried) within 1e-4.  PSS runs on 1-port cells: with more ports the reference subtracts one port's H PSS
    from the sum every port transmitted (estimate_noise_pss, chest_dl.c:402-418), which measures the ports'
    channel difference rather than noise."""
    _batch_vs_host(U, ora, est, noise, nports)


@pytest.mark.parametrize("est,noise,nports,sync", [(0, 1, 1, False), (0, 2, 2, False), (1, 1, 1, False),
                                                   (0, 0, 2, True), (0, 1, 1, True), (1, 2, 2, True)])
def test_ue_dl_batch_auto_filter_and_sync_error(U, ora, est, noise, nports, sync):
    """the two srsUE knobs the batch used to refuse (verdict round 4): estimator_fil_auto with PSS / EMPTY noise (the
    batch runs in segments that end at subframes 0 / 5, each segment filtering with the estimate kept before it,
    chest_dl.c:703-707) and correct_sync_error (per subframe and rx the CRS phase slope, then the grid rotated in
    place, chest_dl.c:750-804) on subframes sent with a 0.4-sample timing error: the batch decodes every TB, equal to
    the host-synchronous path, whose noise estimate / sync error equal the oracle's within 1e-4"""
    _batch_vs_host(U, ora, est, noise, nports, order=0, sync=sync, delay=0.4 if sync else 0.0)


@pytest.mark.parametrize("est,noise,nports,ftype,coef", [(0, 0, 2, 1, 0.1), (1, 1, 1, 1, 0.2), (1, 0, 2, 2, 0),
                                                         (0, 0, 2, 2, 0)])
def test_ue_dl_batch_filter_types(U, ora, est, noise, nports, ftype, coef):
    """TRIANGLE and NONE filters (chest_dl.c:700-729) in the batch: equal to the host-synchronous path subframe by
    subframe.  AVERAGE with NONE interpolates the raw LS estimates of the first two CRS symbols as one comb of
    spacing 3 (interp_lin_3 over pilot_estimates, chest_dl.c:476-481): not a channel estimate, so its TBs fail --
    in both paths alike, which is what is checked there"""
    _batch_vs_host(U, ora, est, noise, nports, order=coef, ftype=ftype, expect_ok=not (est == 0 and ftype == 2))


def test_ue_dl_batch_refused_config_then_good_batch(U):
    """a batch whose estimator configuration the batch cannot run (WIENER) is refused before anything is staged or
    launched; the next good batch on the same object runs without waiting on a staging fence (advisor round 4)"""
    import time
    from synth import synth as S
    from srsran_4g_amd import sch as SCH
    TBS = 75376
    ue = U.UeDl(U.cell(100, 2, 1), 2)
    rng = np.random.default_rng(3)
    pls = [rng.integers(0, 256, TBS // 8, dtype=np.uint8) for _ in range(2)]
    x, nre = S.pdsch_subframe(100, 1, 2, 3, 1, 0x1234, TBS, 6, 0, pls, snr_db=30.0, rng=rng, N=2048)
    sb = [SCH.SoftbufferRx(nof_prb=100) for _ in range(2)]
    cfg = U.pdsch_cfg(100, nre, (TBS, TBS), (6, 6), softbuffers=sb)
    d_pl = torch.zeros((2, TBS // 8 + 64), dtype=torch.uint8, device="cuda")
    d_x = torch.from_numpy(x[None].view(np.float32)).cuda()
    d_res = torch.full((2,), 7, dtype=torch.int32, device="cuda")
    d_avg = torch.zeros(2, dtype=torch.float32, device="cuda")
    entry = [(3, 1, cfg, [d_pl[0].data_ptr(), d_pl[1].data_ptr()], [1, 1])]
    ue.cfg.chest_cfg = U.chest_cfg(0, 0)
    ue.cfg.chest_cfg.estimator_alg = 2  # WIENER: not provided
    for _ in range(3):
        assert ue.gpu_decode_batch(entry, d_x.data_ptr(), d_res.data_ptr(), d_avg.data_ptr(), 0.0, None) < 0
    ue.cfg.chest_cfg = U.chest_cfg(0, 0)
    t0 = time.time()
    for _ in range(4):
        assert ue.gpu_decode_batch(entry, d_x.data_ptr(), d_res.data_ptr(), d_avg.data_ptr(), 0.0, None) == 2
        torch.cuda.synchronize()
    assert time.time() - t0 < 5.0
    assert (d_res.cpu().numpy() == 0).all()
    assert np.array_equal(d_pl[0, : TBS // 8].cpu().numpy(), pls[0])
    ue.free()
    for b in sb:
        b.free()
