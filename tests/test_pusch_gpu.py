"""PUSCH receive on the GPU against the oracle chain (oracle/pusch.py + the reference's compiled
demapper / descrambler / uci.c / decode_tb):

  srsran_dft_precoding_gpu   every valid L_prb (1..100) against numpy's inverse FFT x sqrt(M)
                             (FFTW, the reference's DFT, is absent: float tolerance 2e-6 rms)
  srsran_chest_ul_estimate_pusch  the estimate rows, noise, CFO, TA, RSRP and EPRE against the oracle
                             estimator fed the same DMRS (rtol 1e-4 on the estimate)
  srsran_pusch_decode        CRC, payload, HARQ-ACK / RI / CQI and average iterations equal to the
                             oracle chain's, over QPSK / 16QAM / 64QAM, normal / extended CP, SRS
                             shortening, UCI, HARQ retransmission, a decoding failure and the
                             64QAM limit (enable_64qam = false)
"""
import ctypes
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
sys.path.insert(0, HERE)

import pusch as OP  # noqa: E402  (oracle/pusch.py)
import pusch_tx as TX  # noqa: E402
import uci_cases as UC  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    if not OP.ref_available():  # on a HIP box the parity checker must be there: fail, never skip
        pytest.fail("oracle/_ref/libsrsref.so missing: the reference checker of this module was not built")
    return OP.PuschOracle()


def test_dft_precoding_all_sizes(env):
    import torch

    from srsran_4g_amd import pusch as P
    L = P.lib()
    rng = np.random.default_rng(5)
    for n in range(1, 101):
        if not L.srsran_dft_precoding_valid_prb(n):
            assert L.srsran_dft_precoding_gpu(None, None, n, 1, None) != 0
            continue
        M, ns = 12 * n, int(rng.integers(1, 15))
        x = (rng.standard_normal((ns, M)) + 1j * rng.standard_normal((ns, M))).astype(np.complex64)
        d_in = torch.from_numpy(x.view(np.float32)).cuda()
        d_out = torch.zeros_like(d_in)
        assert L.srsran_dft_precoding_gpu(d_in.data_ptr(), d_out.data_ptr(), n, ns, None) == 0
        torch.cuda.synchronize()
        y = d_out.cpu().numpy().view(np.complex64)
        want = np.fft.ifft(x.astype(np.complex128), axis=1) * np.sqrt(M)
        rms = np.sqrt(np.mean(np.abs(y - want) ** 2))
        assert rms < 2e-6 * np.sqrt(np.log2(M)) + 1e-6, (n, rms)


def _setup(cell_id, cprb, cp, dcfg):
    from srsran_4g_amd import pusch as P
    from srsran_4g_amd.ue_dl import cell as make_cell
    c = make_cell(nof_prb=cprb, cell_id=cell_id)
    c.cp = cp
    d = P.srsran_refsignal_dmrs_pusch_cfg_t()
    d.cyclic_shift, d.delta_ss, d.group_hopping_en, d.sequence_hopping_en = dcfg
    return c, d


CASES = [
    # (name, cell_id, cell_prb, cp, Qm, L, n_prb, tbs, nack, ri, cqi, shortened, tti, dmrs cfg, snr)
    ("qpsk_1prb", 3, 6, 0, 2, 1, 2, 104, 0, 0, None, False, 0, (0, 0, False, False), 20.0),
    ("qpsk_6prb_ack", 1, 25, 0, 2, 6, 3, 1544, 1, 0, None, False, 4, (1, 0, True, False), 20.0),
    ("16qam_25prb_uci", 77, 50, 0, 4, 25, 10, 11064, 2, 1, (UC.WB, dict(pmi_present=True)), False, 7,
     (3, 4, True, False), 30.0),
    ("64qam_50prb_srs", 501, 100, 0, 6, 50, 40, 30576, 4, 2, (UC.HL, dict(N=13, pmi_present=True)), True, 9,
     (5, 11, False, True), 35.0),
    ("64qam_100prb", 29, 100, 0, 6, 100, 0, 61664, 0, 0, None, False, 2, (7, 29, True, False), 35.0),
    ("qpsk_ext_cp_uci", 30, 25, 1, 2, 8, 5, 1736, 3, 1, (UC.WB, dict()), False, 5, (2, 5, True, True), 25.0),
    ("16qam_75prb_cqi_only", 10, 100, 0, 4, 75, 20, 0, 0, 0, (UC.HL, dict(N=12)), False, 1, (0, 3, False, False),
     30.0),
]


def _decode_case(po, case, rv=0, softbuffers=None, meas_ta=True, rng=None, grid_override=None):
    import uci as RU

    from srsran_4g_amd import pusch as P
    from srsran_4g_amd import sch as S
    name, cell_id, cprb, cp, Qm, L, n0, tbs, nack, ri, cqi, sh, tti, dcfg, snr = case
    rng = rng or np.random.default_rng(len(name) + 100 * rv)
    cell, d = _setup(cell_id, cprb, cp, dcfg)
    sf = P.srsran_ul_sf_cfg_t()
    sf.tti, sf.shortened = tti, sh
    sb_gpu, sb_state = softbuffers if softbuffers else (S.SoftbufferRx(nof_prb=100), None)
    cfg = TX.make_cfg(cprb, Qm, L, n0, tbs, nack, ri, cqi, cp=cp, shortened=sh, rv=rv, softbuffer=sb_gpu)
    cfg.meas_ta_en = meas_ta
    cfg.meas_epre_en = True
    grid, payload, u, H, s2 = TX.pusch_subframe(po, cell_id, cprb, cp, cfg, d, tti, rng, snr_db=snr, shortened=sh,
                                                payload=getattr(_decode_case, "payload", None))
    if grid_override is not None:
        grid = grid_override(grid)

    # ---- GPU: estimator + decoder through the C-ABI
    ch = P.ChestUl(cell, d)
    assert ch.estimate(sf, cfg, grid) == 0
    nsf = grid.size
    ce_gpu = ch.ce(nsf).reshape(grid.shape)
    pu = P.Pusch(cell)
    ret, out, data = pu.decode(sf, cfg, ch.res, grid, max(tbs // 8, 1))
    assert ret == 0

    # ---- oracle: the same DMRS (pinned separately in test_pusch_host.py)
    _, r = P.dmrs(cell, d, L, tti % 10, cfg.grant.n_dmrs)
    est = po.chest(grid, cprb, cp, L, cfg.grant.n_prb_tilde, cfg.grant.n_prb, r, meas_ta=meas_ta)
    M = 12 * L
    rows = slice(n0 * 12, n0 * 12 + M)
    np.testing.assert_allclose(ce_gpu[:, rows], est["ce"][:, rows], rtol=1e-4, atol=1e-5)
    assert ch.res.noise_estimate == pytest.approx(est["noise"], rel=2e-3, abs=1e-7)
    assert ch.res.epre == pytest.approx(est["epre"], rel=1e-4)
    assert ch.res.rsrp == pytest.approx(est["rsrp"], rel=1e-3, abs=1e-7)
    assert ch.res.cfo_hz == pytest.approx(est["cfo_hz"], abs=0.5)
    if meas_ta:
        assert abs(ch.res.ta_us - est["ta_us"]) <= 0.1 + 1e-6
    dsym = po.symbols(grid, est["ce"], est["noise"], cp, sh, L, cfg.grant.n_prb_tilde)
    q = po.llrs(dsym, cfg.grant.tb.mod, cfg.rnti, tti, cell_id)
    c = po.ora.sequence_bits(OP.pusch_seed(cfg.rnti, 2 * (tti % 10), cell_id), q.size)
    rcfg = TX.make_cfg(cprb, Qm, L, n0, tbs, nack, ri, cqi, cp=cp, shortened=sh, rv=rv)
    want = S.srsran_uci_value_t()
    rret, _, g, (Qri, Qcqi, G, Qack) = RU.RefUci().rx(rcfg, q, c, want)
    if tbs:
        oret, odata, _, oavg, state = po.ora.dlsch_decode(tbs, Qm, rv, g[Qcqi * Qm:(Qcqi + G) * Qm], 8, sb_state)
        assert bool(out.crc) == (oret == 0)
        assert out.avg_iterations_block == pytest.approx(oavg, abs=0)
        if oret == 0:
            assert np.array_equal(data[:tbs // 8], odata[:tbs // 8])
    else:
        state = None
        assert not out.crc or rret == 0
    if nack:
        assert list(out.uci.ack.ack_value[:nack]) == list(want.ack.ack_value[:nack])
        assert bool(out.uci.ack.valid) == bool(want.ack.valid)
    if ri:
        assert out.uci.ri == want.ri
    if cqi:
        assert bool(out.uci.cqi.data_crc) == bool(want.cqi.data_crc)
        assert UC.cqi_fields(cfg, out.uci.cqi) == UC.cqi_fields(rcfg, want.cqi)
    assert cfg.last_O_cqi == S.lib().srsran_cqi_size(ctypes.byref(cfg.uci_cfg.cqi))
    pu.free()
    ch.free()
    return out, data, payload, u, state, sb_gpu


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_pusch_decode_matches_oracle(env, case):
    out, data, payload, u, _, sb = _decode_case(env, case)
    tbs, nack = case[7], case[8]
    if tbs:  # and, at these SNRs, it is the transmitted one
        assert out.crc and np.array_equal(data[:tbs // 8], payload)
    if nack:
        assert list(out.uci.ack.ack_value[:nack]) == list(u.ack.ack_value[:nack])
    sb.free()


def test_pusch_decode_failure_and_harq(env):
    """a low-SNR first transmission fails like the oracle's; the retransmission (rv 2) combines in
    the soft buffer and both agree again"""
    from srsran_4g_amd import sch as S
    case = ("harq_16qam", 9, 25, 0, 4, 12, 6, 4584, 0, 0, None, False, 6, (0, 0, False, False), 4.0)
    sb = S.SoftbufferRx(nof_prb=100)
    rng = np.random.default_rng(42)
    _decode_case.payload = rng.integers(0, 256, 4584 // 8, dtype=np.uint8)
    try:
        out, _, _, _, state, _ = _decode_case(env, case, rv=0, softbuffers=(sb, None), rng=rng)
        assert not out.crc
        case2 = case[:-1] + (16.0,)
        out2, data2, payload, _, _, _ = _decode_case(env, case2, rv=2, softbuffers=(sb, state), rng=rng)
        assert out2.crc and np.array_equal(data2[:4584 // 8], payload)
    finally:
        _decode_case.payload = None
        sb.free()


def test_pusch_64qam_limited(env):
    """enable_64qam = false turns a 64QAM grant into 16QAM over the same REs (pusch.c:374-380)"""
    from srsran_4g_amd import pusch as P
    from srsran_4g_amd import sch as S
    cell, d = _setup(5, 25, 0, (0, 0, False, False))
    cfg = TX.make_cfg(25, 6, 10, 0, 5160, 0, 0, None)
    cfg.enable_64qam = False
    sf = P.srsran_ul_sf_cfg_t()
    ch = P.ChestUl(cell, d)
    pu = P.Pusch(cell)
    grid = np.zeros((14, 300), np.complex64)
    assert ch.estimate(sf, cfg, grid) == 0
    ret, out, _ = pu.decode(sf, cfg, ch.res, grid, 5160 // 8)
    assert ret == 0 and cfg.grant.tb.mod == S.SRSRAN_MOD_16QAM and cfg.grant.tb.nof_bits == cfg.grant.nof_re * 4
    assert not out.crc
    pu.free()
    ch.free()


def test_invalid_grants_refused(env):
    from srsran_4g_amd import pusch as P
    cell, d = _setup(5, 25, 0, (0, 0, False, False))
    sf = P.srsran_ul_sf_cfg_t()
    ch = P.ChestUl(cell, d)
    pu = P.Pusch(cell)
    grid = np.zeros((14, 300), np.complex64)
    bad = TX.make_cfg(25, 2, 7, 0, 1000, 0, 0, None)  # 7 PRB: not 2^a 3^b 5^c
    assert ch.estimate(sf, bad, grid) != 0
    assert pu.decode(sf, bad, ch.res, grid, 200)[0] != 0
    over = TX.make_cfg(25, 2, 10, 20, 1000, 0, 0, None)  # PRB 20..29 beyond a 25-PRB cell
    assert ch.estimate(sf, over, grid) != 0
    pu.free()
    ch.free()


@pytest.mark.parametrize("mixed", [False, True], ids=["same_iterations", "mixed_iterations"])
def test_pusch_batch_matches_sync(env, mixed):
    """srsran_pusch_gpu_decode_batch over UEs of two cells (device grids): every UE's CRC, payload,
    UCI, iterations and estimator outputs equal srsran_chest_ul_estimate_pusch + srsran_pusch_decode.
    mixed_iterations: each UE has its own max_nof_iterations (pusch.c:450 sets it per decode) at SNRs where
    the turbo decoder needs several iterations, so a batch-wide limit would change iterations and payloads"""
    import torch

    from srsran_4g_amd import pusch as P
    from srsran_4g_amd import sch as S
    po = env
    picks = [CASES[1], CASES[2], CASES[5], CASES[3], CASES[0], CASES[6]]
    maxits = [1, 4, 2, 8, 3, 5]
    cells, keep, ues, want = {}, [], [], []
    rng = np.random.default_rng(11)
    for k, case in enumerate(picks):
        name, cell_id, cprb, cp, Qm, L, n0, tbs, nack, ri, cqi, sh, tti, dcfg, snr = case
        if mixed:
            snr -= 12.0
        cell, d = _setup(cell_id, cprb, cp, dcfg)
        sf = P.srsran_ul_sf_cfg_t()
        sf.tti, sf.shortened = tti, sh
        def mk(sb, a=(cprb, Qm, L, n0, tbs, nack, ri, cqi, cp, sh)):
            c = TX.make_cfg(*a[:8], cp=a[8], shortened=a[9], softbuffer=sb)
            c.meas_epre_en = True
            if mixed:
                c.max_nof_iterations = maxits[k]
            return c
        sb1, sb2 = S.SoftbufferRx(nof_prb=100), S.SoftbufferRx(nof_prb=100)
        cfg_b = mk(sb2)
        grid, payload, u, H, s2 = TX.pusch_subframe(po, cell_id, cprb, cp, cfg_b, d, tti, rng, snr_db=snr, shortened=sh)
        # the reference flow, one UE at a time
        ch = P.ChestUl(cell, d)
        cfg_s = mk(sb1)
        assert ch.estimate(sf, cfg_s, grid) == 0
        pu = P.Pusch(cell)
        ret, out_s, data_s = pu.decode(sf, cfg_s, ch.res, grid, max(tbs // 8, 1))
        assert ret == 0
        want.append((out_s, data_s.copy(), ch.res.noise_estimate, ch.res.epre, ch.res.cfo_hz, tbs, nack, cfg_s))
        pu.free()
        ch_b = P.ChestUl(cell, d)
        d_grid = torch.from_numpy(grid.view(np.float32).reshape(-1).copy()).cuda()
        data_b = np.zeros(max(tbs // 8, 1) + 64, np.uint8)
        keep += [ch, ch_b, d_grid, data_b, sb1, sb2, sf, cfg_b]
        ues.append((ch_b, sf, cfg_b, d_grid, data_b))
    n = len(ues)
    arr = (P.srsran_pusch_gpu_ue_t * n)()
    res = (P.srsran_pusch_res_t * n)()
    cres = (P.srsran_chest_ul_res_t * n)()
    for i, (ch_b, sf, cfg_b, d_grid, data_b) in enumerate(ues):
        arr[i].chest = ctypes.pointer(ch_b.q)
        arr[i].sf = ctypes.pointer(sf)
        arr[i].cfg = ctypes.pointer(cfg_b)
        arr[i].d_sf_symbols = d_grid.data_ptr()
        res[i].data = data_b.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    if mixed:  # the limits matter here: some UE ran more than one iteration in the sequential flow
        assert max(w[0].avg_iterations_block for w in want if w[5]) > 1
    pu = P.Pusch(ues[0][0].cell)
    assert P.lib().srsran_pusch_gpu_decode_batch(ctypes.byref(pu.q), n, arr, cres, res) == 0
    for i, (out_s, data_s, noise, epre, cfo, tbs, nack, cfg_s) in enumerate(want):
        assert bool(res[i].crc) == bool(out_s.crc), i
        if tbs:  # (without a TB avg_iterations is the previous decode's, as in pusch.c:457)
            assert res[i].avg_iterations_block == out_s.avg_iterations_block, i
            assert np.array_equal(ues[i][4][:tbs // 8], data_s[:tbs // 8]), i
        assert bytes(res[i].uci) == bytes(out_s.uci), i
        assert cres[i].noise_estimate == pytest.approx(noise, rel=1e-5, abs=1e-9), i
        assert cres[i].epre == pytest.approx(epre, rel=1e-5), i
        assert cres[i].cfo_hz == pytest.approx(cfo, abs=1e-3), i
        assert res[i].epre_dbfs == pytest.approx(out_s.epre_dbfs, abs=1e-3), i
    pu.free()
    for k in keep:
        if hasattr(k, "free"):
            k.free()
