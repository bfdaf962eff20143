"""Extended cyclic prefix on the GPU downlink (cell.cp = SRSRAN_CP_EXT: 6 symbols a slot, cp = 512 N /
2048, CRS in l = 0 and 3 with N_cp = 0 in the CRS c_init, refsignal_dl.c:65-119, 254-266): the OFDM
demodulator against numpy, the CRS estimator against the oracle (phy_oracle.c), srsran_pdsch_decode
bit-exact against the oracle chain (oracle/pdsch_chain.py, cp=1), the UE DL batch against the
host-synchronous path, and the GPU eNB transmitter against the CPU transmitter (synth/synth.py).
Parity is anchored as for normal CP: the pieces the oracle restates are pinned in test_phy_oracle.py;
the extended-CP RE map and grant size rest on two independent restatements (test_pdsch_map.py)."""
import numpy as np
import pytest
import torch

from oracle import Oracle
import ofdm_np
import pdsch_chain as PC
from synth import synth as SY

pytestmark = pytest.mark.gpu

RNTI = 0x1234


@pytest.fixture(scope="module")
def ora():
    return Oracle()


@pytest.fixture(scope="module")
def U():
    from srsran_4g_amd import ue_dl
    return ue_dl


@pytest.fixture(scope="module")
def SCH():
    from srsran_4g_amd import sch
    return sch


@pytest.fixture(scope="module", autouse=True)
def standard_rates(U):
    U.use_standard_symbol_size(True)
    yield
    U.use_standard_symbol_size(False)


def _subframe(rng, nof_prb, cell_id, nports, tti, cfi, scheme, tbs, Qm, snr_db=30.0):
    ncw = 2 if scheme in ("cdd", "sm") else 1
    pls = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(ncw)]
    ch = [[1], [0.5 + 0.5j]] if nports == 1 else None
    x, nre = SY.pdsch_subframe(nof_prb, cell_id, nports, tti, cfi, RNTI, tbs, Qm, 0, pls, scheme=scheme, codebook=1,
                               snr_db=snr_db, rng=rng, channel=ch, cp=1)
    return pls, x, nre


@pytest.mark.parametrize("nof_prb", [100, 25, 6])
def test_ofdm_rx_extended_cp(U, nof_prb):
    rng = np.random.default_rng(nof_prb)
    N = SY.symbol_sz(nof_prb)
    x = (rng.standard_normal(ofdm_np.sf_len(N, ext=1)) + 1j * rng.standard_normal(ofdm_np.sf_len(N, ext=1)))
    o = U.OfdmRx(nof_prb, cp=1)
    assert o.q.nof_symbols == 6 and o.q.sf_sz == 2 * (6 * N + 6 * ((512 * N + 2047) // 2048))
    got = o.rx(x.astype(np.complex64))
    want = ofdm_np.ofdm_rx(x.astype(np.complex64), N, 12 * nof_prb, ext=1)
    assert got.size == 12 * 12 * nof_prb
    assert np.abs(got - want).max() < 2e-5 * np.abs(want).max() * np.sqrt(np.log2(N))
    o.free()


@pytest.mark.parametrize("nof_prb,cell_id,nports,sf", [(100, 9, 2, 1), (100, 4, 1, 0), (50, 301, 2, 5), (6, 2, 2, 3)])
def test_chest_extended_cp(U, ora, nof_prb, cell_id, nports, sf):
    rng = np.random.default_rng(nof_prb + cell_id)
    tbs, Qm = (1800, 4) if nof_prb == 6 else (4008, 4)
    scheme = "port0" if nports == 1 else "cdd"
    _, x, _ = _subframe(rng, nof_prb, cell_id, nports, sf, 2, scheme, tbs, Qm, snr_db=25.0)
    N = SY.symbol_sz(nof_prb)
    Y = np.stack([ofdm_np.ofdm_rx(v, N, 12 * nof_prb, ext=1) for v in x]).astype(np.complex64)
    ch = U.ChestDl(U.cell(nof_prb, nports, cell_id, cp=1), Y.shape[0])
    ce, res = ch.estimate(Y, sf, U.srsue_chest_cfg())
    ceo, st = ora.chest_dl(Y, nof_prb, cell_id, nports, sf, U.lib().srsran_symbol_sz(nof_prb), cp=1)
    assert ce.shape == ceo.shape == (nports, Y.shape[0], 12 * 12 * nof_prb)
    scale = np.abs(ceo).max()
    assert np.abs(ce - ceo).max() < 2e-5 * scale
    assert res.noise_estimate == pytest.approx(st["noise"], rel=1e-4)
    assert res.rsrp == pytest.approx(st["rsrp"], rel=1e-4)
    assert res.cfo == pytest.approx(st["cfo"], rel=1e-3, abs=1e-6)
    ch.free()


CASES = [  # (nof_prb, cell_id, nports, tti, cfi, scheme, tbs, Qm)
    (100, 9, 2, 1, 1, "cdd", 55056, 6),
    (100, 9, 2, 10, 2, "cdd", 46888, 6),      # subframe 0: PBCH over both CRS symbols of slot 1
    (100, 3, 2, 5, 3, "diversity", 46888, 6),  # PSS / SSS subframe
    (100, 3, 1, 2, 1, "port0", 30576, 4),
    (50, 11, 2, 4, 1, "cdd", 22152, 6),
    (6, 2, 2, 7, 2, "cdd", 1160, 4),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[5]}_{c[0]}prb_sf{c[3] % 10}_cfi{c[4]}" for c in CASES])
@pytest.mark.parametrize("csi", [True, False])
def test_pdsch_decode_extended_cp(U, SCH, ora, case, csi):
    nof_prb, cell_id, nports, tti, cfi, scheme, tbs, Qm = case
    rng = np.random.default_rng(tbs + tti)
    pls, x, nre = _subframe(rng, nof_prb, cell_id, nports, tti, cfi, scheme, tbs, Qm)
    grids, ce, st = PC.fft_estimate(ora, x, nof_prb, cell_id, nports, tti, cp=1)
    ncw = len(pls)
    ref = PC.pdsch_decode(ora, grids, ce, st["noise"], nof_prb, cell_id, nports, tti, cfi, RNTI, [tbs] * ncw,
                          [Qm] * ncw, [0] * ncw, scheme=scheme, csi_enable=csi, cp=1)
    assert ref[0]["nof_re"] == nre
    sbs = [SCH.SoftbufferRx(nof_prb=nof_prb) for _ in range(ncw)]
    cfg = U.pdsch_cfg(nof_prb, nre, [tbs] * ncw, [Qm] * ncw, scheme=scheme, softbuffers=sbs, csi_enable=csi, cp=1)
    pd = U.Pdsch(U.cell(nof_prb, nports, cell_id, cp=1), grids.shape[0])
    ret, out = pd.decode(cfg, tti, cfi, grids, ce, st["noise"])
    assert ret == 0
    for q, (crc, payload, avg) in enumerate(out):
        r = ref[q]
        assert r["ret"] == 0 and crc
        assert np.array_equal(payload[: tbs // 8 + 6], r["data"][: tbs // 8 + 6])
        assert np.array_equal(payload[: tbs // 8], pls[q])
        assert avg == pytest.approx(r["avg"], abs=1e-6)
    # the normal-CP grant size is refused on the extended-CP cell
    cfg2 = U.pdsch_cfg(nof_prb, nre + 12, [tbs] * ncw, [Qm] * ncw, scheme=scheme, softbuffers=sbs, cp=1)
    assert pd.decode(cfg2, tti, cfi, grids, ce, st["noise"])[0] != 0
    pd.free()


def test_ue_dl_batch_extended_cp(U, SCH, ora):
    """srsran_ue_dl_gpu_decode_batch from time samples (extended-CP OFDM, estimator, PDSCH) == the
    host-synchronous srsran_ue_dl path subframe by subframe, and decodes what was sent"""
    nof_prb, cell_id, tbs = 100, 9, 46888
    rng = np.random.default_rng(12)
    cell = U.cell(nof_prb, 2, cell_id, cp=1)
    ue = U.UeDl(cell, 2)
    ttis = [0, 1, 5, 6]
    samples, payloads, entries, keep = [], [], [], []
    d_pl = torch.zeros((len(ttis), 2, tbs // 8 + 64), dtype=torch.uint8, device="cuda")
    for b, tti in enumerate(ttis):
        pls, x, nre = _subframe(rng, nof_prb, cell_id, 2, tti, 1, "cdd", tbs, 6)
        sb = [SCH.SoftbufferRx(nof_prb=nof_prb) for _ in range(2)]
        cfg = U.pdsch_cfg(nof_prb, nre, (tbs, tbs), (6, 6), softbuffers=sb, cp=1)
        samples.append(x)
        payloads.append(pls)
        keep.append((sb, cfg))
        entries.append((tti, 1, cfg, [d_pl[b, 0].data_ptr(), d_pl[b, 1].data_ptr()], [1, 1]))
    d_x = torch.from_numpy(np.stack(samples).view(np.float32)).cuda()
    d_res = torch.full((2 * len(ttis),), 7, dtype=torch.int32, device="cuda")
    d_avg = torch.zeros(2 * len(ttis), dtype=torch.float32, device="cuda")
    assert ue.gpu_decode_batch(entries, d_x.data_ptr(), d_res.data_ptr(), d_avg.data_ptr(), 0.0, None) == 2 * len(ttis)
    torch.cuda.synchronize()
    res, pl = d_res.cpu().numpy(), d_pl.cpu().numpy()
    ue2 = U.UeDl(cell, 2)
    for b, tti in enumerate(ttis):
        assert ue2.fft_estimate(samples[b], tti, 1) == 0
        sb = [SCH.SoftbufferRx(nof_prb=nof_prb) for _ in range(2)]
        cfg = U.pdsch_cfg(nof_prb, keep[b][1].grant.nof_re, (tbs, tbs), (6, 6), softbuffers=sb, cp=1)
        ret, out = ue2.decode_pdsch(cfg, tti, 1)
        assert ret == 0
        for q in range(2):
            assert res[2 * b + q] == 0 and out[q][0]
            assert np.array_equal(pl[b, q, : tbs // 8], payloads[b][q])
            assert np.array_equal(out[q][1][: tbs // 8], payloads[b][q])
    ue.free()
    ue2.free()


@pytest.mark.parametrize("nports,scheme,tti,cfi", [(2, "cdd", 3, 1), (2, "cdd", 0, 2), (1, "port0", 5, 2)])
def test_enb_tx_extended_cp(U, nports, scheme, tti, cfi):
    """srsran_enb_dl_gpu_tx_batch on an extended-CP cell == the CPU transmitter sample for sample"""
    from srsran_4g_amd import enb_dl as E
    nprb, cell_id, rnti = 100, 37, 0x4601
    tbs, Qm = (46888, 6) if scheme == "cdd" else (30576, 4)
    ntb = 2 if scheme == "cdd" else 1
    N = SY.symbol_sz(nprb)
    nre = int(SY.pdsch_mask(nprb, nports, cell_id, cfi, tti % 10, cp=1).sum())
    rng = np.random.default_rng(tbs + tti)
    payloads = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(ntb)]
    want, _ = SY.pdsch_subframe(nprb, cell_id, nports, tti, cfi, rnti, tbs, Qm, 0, payloads, scheme=scheme, nrx=nports,
                                N=N, channel=np.eye(nports), pcfich=False, cp=1)
    enb = E.EnbDl(U.cell(nprb, nports, cell_id, cp=1))
    cfg = U.pdsch_cfg(nprb, nre, [tbs] * ntb, [Qm] * ntb, scheme=scheme, rnti=rnti, cp=1)
    d_pl = [torch.from_numpy(p).cuda() for p in payloads]
    d_out = torch.zeros((nports, want.shape[1], 2), dtype=torch.float32, device="cuda")
    assert enb.tx_batch([(tti, cfi, cfg, [p.data_ptr() for p in d_pl])], d_out.data_ptr(), 1.0 / N) == 0
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.complex64)[..., 0]
    scale = np.abs(want).max()
    assert np.abs(got - want).max() < 2e-5 * scale * np.sqrt(np.log2(N))
    enb.free()


# ---------------- 4 transmit ports (TM2: SFBC + FSTD, srsran_predecoding_diversity_csi 4-port branch) ----------------
def test_predecoding_type_four_ports_matches_oracle(U, ora):
    """srsran_predecoding_type, 4-port transmit diversity with CSI, == the oracle (itself bit-exact
    against the reference's precoding.c, test_phy_oracle.py), including a trailing half group"""
    from srsran_4g_amd import phch as PH
    rng = np.random.default_rng(44)
    for nrx in (1, 2, 4):
        for n in (14400, 1202, 40):
            h = ((rng.standard_normal((4, nrx, n)) + 1j * rng.standard_normal((4, nrx, n))) * 0.7).astype(np.complex64)
            y = (rng.standard_normal((nrx, n)) + 1j * rng.standard_normal((nrx, n))).astype(np.complex64)
            for scaling in (1.0, 0.7):
                xo, co = ora.predecode(1, y, h, 4, 0, scaling, 0.01)
                xg, cg = PH.predecode(1, y, h, 4, 0, scaling, 0.01)
                m = xo.shape[1]
                assert np.array_equal(xg[:, :m], xo), (nrx, n)
                assert np.array_equal(cg[0, :4 * m], co[0, :4 * m]), (nrx, n)


@pytest.mark.parametrize("tti,cfi,cp,csi", [(1, 1, 0, True), (5, 2, 0, True), (10, 1, 0, False), (3, 2, 1, True)])
def test_pdsch_decode_four_ports(U, SCH, ora, tti, cfi, cp, csi):
    """TM2 on 4 ports: CRS estimator for ports 0..3, 4-port SFBC + FSTD predecoding with the layer
    demapping fused, DL-SCH with Nl = 2 -- bit-exact against the oracle chain and CRC-clean"""
    nof_prb, cell_id, tbs = 100, 6, 36696
    rng = np.random.default_rng(tti + 60)
    pl = [rng.integers(0, 256, tbs // 8, dtype=np.uint8)]
    x, nre = SY.pdsch_subframe(nof_prb, cell_id, 4, tti, cfi, RNTI, tbs, 6, 0, pl, scheme="diversity4", snr_db=30.0,
                               rng=rng, cp=cp)
    grids, ce, st = PC.fft_estimate(ora, x, nof_prb, cell_id, 4, tti, cp=cp)
    ref = PC.pdsch_decode(ora, grids, ce, st["noise"], nof_prb, cell_id, 4, tti, cfi, RNTI, [tbs], [6], [0],
                          scheme="diversity", csi_enable=csi, cp=cp)
    sbs = [SCH.SoftbufferRx(nof_prb=nof_prb)]
    cfg = U.pdsch_cfg(nof_prb, nre, [tbs], [6], scheme="diversity", softbuffers=sbs, csi_enable=csi, cp=cp,
                      nof_ports=4)
    pd = U.Pdsch(U.cell(nof_prb, 4, cell_id, cp=cp), grids.shape[0])
    ret, out = pd.decode(cfg, tti, cfi, grids, ce, st["noise"])
    assert ret == 0
    crc, payload, avg = out[0]
    assert ref[0]["ret"] == 0 and crc
    assert np.array_equal(payload[: tbs // 8 + 6], ref[0]["data"][: tbs // 8 + 6])
    assert np.array_equal(payload[: tbs // 8], pl[0])
    assert avg == pytest.approx(ref[0]["avg"], abs=1e-6)
    pd.free()


def test_chest_four_ports_extended_cp(U, ora):
    rng = np.random.default_rng(3)
    pl = [rng.integers(0, 256, 36696 // 8, dtype=np.uint8)]
    x, _ = SY.pdsch_subframe(100, 6, 4, 2, 1, RNTI, 36696, 6, 0, pl, scheme="diversity4", snr_db=25.0, rng=rng, cp=1)
    Y = np.stack([ofdm_np.ofdm_rx(v, 2048, 1200, ext=1) for v in x]).astype(np.complex64)
    ch = U.ChestDl(U.cell(100, 4, 6, cp=1), 2)
    ce, res = ch.estimate(Y, 2, U.srsue_chest_cfg())
    ceo, st = ora.chest_dl(Y, 100, 6, 4, 2, 2048, cp=1)
    assert np.abs(ce - ceo).max() < 2e-5 * np.abs(ceo).max()
    assert res.noise_estimate == pytest.approx(st["noise"], rel=1e-4)
    ch.free()


def test_ue_dl_batch_four_ports(U, SCH, ora):
    """srsran_ue_dl_gpu_decode_batch on a 4-port cell (TM2): OFDM, 4-port estimator, SFBC + FSTD,
    DL-SCH from time samples; every TB decodes and equals the host-synchronous path"""
    nof_prb, cell_id, tbs = 100, 6, 36696
    rng = np.random.default_rng(21)
    cell = U.cell(nof_prb, 4, cell_id)
    ue = U.UeDl(cell, 2)
    ttis = [1, 2, 5]
    samples, payloads, entries, keep = [], [], [], []
    d_pl = torch.zeros((len(ttis), 2, tbs // 8 + 64), dtype=torch.uint8, device="cuda")
    for b, tti in enumerate(ttis):
        pl = [rng.integers(0, 256, tbs // 8, dtype=np.uint8)]
        x, nre = SY.pdsch_subframe(nof_prb, cell_id, 4, tti, 1, RNTI, tbs, 6, 0, pl, scheme="diversity4", snr_db=30.0,
                                   rng=rng)
        sb = [SCH.SoftbufferRx(nof_prb=nof_prb)]
        cfg = U.pdsch_cfg(nof_prb, nre, [tbs], [6], scheme="diversity", softbuffers=sb, nof_ports=4)
        samples.append(x)
        payloads.append(pl)
        keep.append((sb, cfg))
        entries.append((tti, 1, cfg, [d_pl[b, 0].data_ptr(), d_pl[b, 1].data_ptr()], [1, 1]))
    d_x = torch.from_numpy(np.stack(samples).view(np.float32)).cuda()
    d_res = torch.full((len(ttis),), 7, dtype=torch.int32, device="cuda")
    d_avg = torch.zeros(len(ttis), dtype=torch.float32, device="cuda")
    assert ue.gpu_decode_batch(entries, d_x.data_ptr(), d_res.data_ptr(), d_avg.data_ptr(), 0.0, None) == len(ttis)
    torch.cuda.synchronize()
    res, pl = d_res.cpu().numpy(), d_pl.cpu().numpy()
    ue2 = U.UeDl(cell, 2)
    for b, tti in enumerate(ttis):
        assert res[b] == 0
        assert np.array_equal(pl[b, 0, : tbs // 8], payloads[b][0])
        assert ue2.fft_estimate(samples[b], tti, 1) == 0
        sb = [SCH.SoftbufferRx(nof_prb=nof_prb)]
        cfg = U.pdsch_cfg(nof_prb, keep[b][1].grant.nof_re, [tbs], [6], scheme="diversity", softbuffers=sb, nof_ports=4)
        ret, out = ue2.decode_pdsch(cfg, tti, 1)
        assert ret == 0 and out[0][0]
        assert np.array_equal(out[0][1][: tbs // 8 + 6], pl[b, 0, : tbs // 8 + 6])
    ue.free()
    ue2.free()


@pytest.mark.parametrize("tti,cfi,cp", [(3, 1, 0), (0, 2, 0), (5, 1, 1)])
def test_enb_tx_four_ports(U, tti, cfi, cp):
    """srsran_enb_dl_gpu_tx_batch on a 4-port cell (CRS of ports 0..3, SFBC + FSTD) == the CPU
    transmitter, and the GPU UE DL chain decodes it"""
    from srsran_4g_amd import enb_dl as E
    nprb, cell_id, rnti, tbs = 100, 37, 0x4601, 36696
    N = SY.symbol_sz(nprb)
    nre = int(SY.pdsch_mask(nprb, 4, cell_id, cfi, tti % 10, cp=cp).sum())
    assert nre % 4 == 0
    rng = np.random.default_rng(tbs + tti)
    payloads = [rng.integers(0, 256, tbs // 8, dtype=np.uint8)]
    want, _ = SY.pdsch_subframe(nprb, cell_id, 4, tti, cfi, rnti, tbs, 6, 0, payloads, scheme="diversity4", nrx=4,
                                N=N, channel=np.eye(4), pcfich=False, cp=cp)
    enb = E.EnbDl(U.cell(nprb, 4, cell_id, cp=cp))
    cfg = U.pdsch_cfg(nprb, nre, [tbs], [6], scheme="diversity", rnti=rnti, cp=cp, nof_ports=4)
    d_pl = [torch.from_numpy(p).cuda() for p in payloads]
    d_out = torch.zeros((4, want.shape[1], 2), dtype=torch.float32, device="cuda")
    assert enb.tx_batch([(tti, cfi, cfg, [p.data_ptr() for p in d_pl])], d_out.data_ptr(), 1.0 / N) == 0
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.complex64)[..., 0]
    scale = np.abs(want).max()
    assert np.abs(got - want).max() < 2e-5 * scale * np.sqrt(np.log2(N))
    enb.free()
