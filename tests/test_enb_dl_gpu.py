"""eNB downlink transmit on the GPU: srsran_enb_dl_gpu_tx_batch (DL-SCH encode,
CRS, scrambling + modulation + precoding + RE mapping, OFDM modulator) against the independent
CPU transmitter synth/synth.py (36.211 / 36.212 restated; its encoder equals the oracle's) sample
for sample, for CDD 2x2 (C3), transmit diversity and one port, several subframe indices (PSS / SSS /
PBCH holes) and CFIs; then the GPU receive chain decodes what the GPU transmitted."""
import numpy as np
import pytest

from synth import synth as SY

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    import torch
    return torch


CASES = [  # (nof_prb, nports, scheme, ntb, Qm, tbs, tti, cfi)
    (100, 2, "cdd", 2, 6, 75376, 3, 1),
    (100, 2, "cdd", 2, 6, 75376, 0, 2),
    (50, 2, "diversity", 1, 4, 12216, 5, 2),
    (25, 1, "port0", 1, 2, 2216, 7, 3),
    (6, 1, "port0", 1, 4, 1160, 2, 2),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[2]}_{c[0]}prb_sf{c[6]}_cfi{c[7]}" for c in CASES])
def test_tx_matches_cpu_transmitter(gpu, case):
    torch = gpu
    from srsran_4g_amd import enb_dl as E
    from srsran_4g_amd import ue_dl as U
    nprb, P, scheme, ntb, Qm, tbs, tti, cfi = case
    cell_id, rnti = 37, 0x4601
    U.use_standard_symbol_size(True)
    N = SY.symbol_sz(nprb)
    mask = SY.pdsch_mask(nprb, P, cell_id, cfi, tti % 10)
    nre = int(mask.sum())
    rng = np.random.default_rng(tbs + tti)
    payloads = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(ntb)]
    want, _ = SY.pdsch_subframe(nprb, cell_id, P, tti, cfi, rnti, tbs, Qm, 0, payloads, scheme=scheme, nrx=P,
                                N=N, channel=np.eye(P), pcfich=False)
    cell = U.cell(nprb, P, cell_id)
    enb = E.EnbDl(cell)
    cfg = U.pdsch_cfg(nprb, nre, [tbs] * ntb, [Qm] * ntb, scheme=scheme, rnti=rnti)
    d_pl = [torch.from_numpy(p).cuda() for p in payloads]
    sf_len = want.shape[1]
    d_out = torch.zeros((P, sf_len, 2), dtype=torch.float32, device="cuda")
    assert enb.tx_batch([(tti, cfi, cfg, [p.data_ptr() for p in d_pl])], d_out.data_ptr(), 1.0 / N) == 0
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.complex64)[..., 0]
    scale = np.abs(want).max()
    assert np.abs(got - want).max() < 2e-5 * scale * np.sqrt(np.log2(N)), np.abs(got - want).max() / scale
    enb.free()


def test_gpu_tx_to_gpu_rx(gpu):
    """C3 subframes from the GPU transmitter (reference amplitude 0.05 / sqrt(N_RB)) through the
    phy_dl_test channel [[1, 1], [1, -1]] into the GPU UE DL batch chain: every TB decodes"""
    torch = gpu
    from srsran_4g_amd import enb_dl as E
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import ue_dl as U
    nprb, P, Qm, tbs, cfi, cell_id, rnti = 100, 2, 6, 75376, 1, 11, 0x1234
    U.use_standard_symbol_size(True)
    ttis = [1, 2, 3, 4]
    rng = np.random.default_rng(5)
    cell = U.cell(nprb, P, cell_id)
    enb = E.EnbDl(cell)
    N = SY.symbol_sz(nprb)
    sfs, keep, pls = [], [], []
    for tti in ttis:
        nre = int(SY.pdsch_mask(nprb, P, cell_id, cfi, tti % 10).sum())
        p2 = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(2)]
        d = [torch.from_numpy(p).cuda() for p in p2]
        cfg = U.pdsch_cfg(nprb, nre, [tbs] * 2, [Qm] * 2, scheme="cdd", rnti=rnti)
        keep += d + [cfg]
        pls.append(p2)
        sfs.append((tti, cfi, cfg, [x.data_ptr() for x in d]))
    sf_len = 2 * (7 * N + 160 * N // 2048 + 6 * (144 * N // 2048))
    d_tx = torch.zeros((len(ttis), P, sf_len, 2), dtype=torch.float32, device="cuda")
    assert enb.tx_batch(sfs, d_tx.data_ptr()) == 0
    torch.cuda.synchronize()
    tx = d_tx.cpu().numpy().view(np.complex64)[..., 0]
    H = np.array([[1, 1], [1, -1]], np.complex64)
    rx = np.einsum("rp,bps->brs", H, tx).astype(np.complex64)
    # the host-synchronous UE DL path on each subframe
    ue = U.UeDl(cell, 2)
    for b, tti in enumerate(ttis):
        nre = int(SY.pdsch_mask(nprb, P, cell_id, cfi, tti % 10).sum())
        sbs = [S.SoftbufferRx(nof_prb=100) for _ in range(2)]
        cfg = U.pdsch_cfg(nprb, nre, [tbs] * 2, [Qm] * 2, scheme="cdd", rnti=rnti, softbuffers=sbs)
        ue.fft_estimate(list(rx[b]), tti, cfi)  # (no PCFICH is transmitted: the CFI is given below)
        ret, res = ue.decode_pdsch(cfg, tti, cfi)
        for cw in range(2):
            ok, data = res[cw][0], res[cw][1]
            assert ok and np.array_equal(data[:tbs // 8], pls[b][cw]), (tti, cw)
        for sb in sbs:
            sb.free()
    ue.free()
    enb.free()


@pytest.mark.parametrize("scheme,P,ntb,Qm,tbs,tti,cfi", [("cdd", 2, 2, 6, 75376, 1, 1), ("diversity", 2, 1, 4, 12216, 5, 2),
                                                       ("port0", 1, 1, 2, 2216, 2, 3)])
def test_pdsch_encode_host_grids(gpu, scheme, P, ntb, Qm, tbs, tti, cfi):
    """srsran_pdsch_encode (eNB, host grids): the PDSCH REs equal the CPU transmitter's precoded
    symbols times the reference's rho_a, every other RE (here the CRS already put) is left as it was"""
    from srsran_4g_amd import ue_dl as U
    nprb = 100 if scheme == "cdd" else 50 if scheme == "diversity" else 25
    cell_id, rnti = 21, 0x3311
    mask = SY.pdsch_mask(nprb, P, cell_id, cfi, tti % 10)
    nre = int(mask.sum())
    rng = np.random.default_rng(tti + tbs)
    pls = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(ntb)]
    layers = []
    for q, pl in enumerate(pls):
        G = nre * Qm
        e = SY.dlsch_encode(tbs, Qm, 0, G, pl, Nl=2 if scheme == "diversity" else 1)
        layers.append(SY.modulate(e ^ SY.gold(SY.pdsch_seed(rnti, q, 2 * (tti % 10), cell_id), G), Qm))
    # srsran_pdsch_encode's rho_a with p_a = 0 dB: sqrt 2 with more than one port (pdsch.c:492, 1066-1070)
    rho_a = np.float32(np.sqrt(2.0)) if P > 1 else np.float32(1.0)
    ports = [x * rho_a for x in SY.precode(layers, scheme)]
    crs = [SY.crs_grid(cell_id, nprb, P, p, tti % 10) for p in range(P)]
    want = []
    for p in range(P):
        g = crs[p].copy()
        g[mask] = ports[p]
        want.append(g.reshape(-1))
    cell = U.cell(nprb, P, cell_id)
    pd = U.Pdsch(cell, 1, enb=True)
    cfg = U.pdsch_cfg(nprb, nre, [tbs] * ntb, [Qm] * ntb, scheme=scheme, rnti=rnti)
    ret, got = pd.encode(cfg, tti, cfi, pls, [c.reshape(-1) for c in crs])
    assert ret == 0
    for p in range(P):
        np.testing.assert_allclose(got[p], want[p], rtol=0, atol=2e-6)
    pd.free()


def test_re_table_cache_wrap_in_and_across_batches(gpu):
    """Both RE-table caches (eNB transmitter, UE receiver; 512 tables each) wrap inside one batch and
    across consecutive batches: 600 subframes a batch, every one with its own (PRB set, subframe, CFI)
    key, transmitted by srsran_enb_dl_gpu_tx_batch and decoded by srsran_ue_dl_gpu_decode_batch;
    every TB decodes to its payload (a table freed while a batch still used it would not)"""
    torch = gpu
    import itertools
    from srsran_4g_amd import enb_dl as E
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import ue_dl as U
    nprb, P, Qm, tbs, cell_id, rnti = 6, 1, 2, 40, 23, 0x2222
    U.use_standard_symbol_size(True)
    keys = [(m, sf, cfi) for cfi in (1, 2, 3) for sf in (1, 2, 3, 4, 6, 7, 8, 9) for m in range(1, 64)]
    rng = np.random.default_rng(77)
    rng.shuffle(keys)
    cell = U.cell(nprb, P, cell_id)
    enb = E.EnbDl(cell)
    ue = U.UeDl(cell, 1)
    nb = 600
    sbs = [S.SoftbufferRx(nof_prb=nprb) for _ in range(nb)]
    N = SY.symbol_sz(nprb)
    sf_len = 2 * (7 * N + 160 * N // 2048 + 6 * (144 * N // 2048))
    for batch in (keys[:nb], keys[nb:2 * nb]):
        tx_sfs, rx_sfs, keep, pls = [], [], [], []
        for i, (m, sf, cfi) in enumerate(batch):
            prb = [(m >> n) & 1 for n in range(nprb)]
            nre = int(SY.pdsch_mask(nprb, P, cell_id, cfi, sf, prb=prb).sum())
            pl = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
            cfg = U.pdsch_cfg(nprb, nre, [tbs], [Qm], scheme="port0", rnti=rnti, nof_ports=1, softbuffers=[sbs[i]])
            for s, n in itertools.product(range(2), range(nprb)):
                cfg.grant.prb_idx[s][n] = bool(prb[n])
            cfg.grant.nof_prb = sum(prb)
            d_pl = torch.from_numpy(pl).cuda()
            d_out = torch.zeros(tbs // 8 + 64, dtype=torch.uint8, device="cuda")
            keep += [cfg, d_pl, d_out]
            pls.append(pl)
            tx_sfs.append((sf, cfi, cfg, [d_pl.data_ptr()]))
            rx_sfs.append((sf, cfi, cfg, [d_out.data_ptr()], [1]))
        d_tx = torch.zeros((nb, P, sf_len, 2), dtype=torch.float32, device="cuda")
        assert enb.tx_batch(tx_sfs, d_tx.data_ptr()) == 0
        d_res = torch.full((nb,), 7, dtype=torch.int32, device="cuda")
        d_avg = torch.zeros(nb, dtype=torch.float32, device="cuda")
        n = ue.gpu_decode_batch(rx_sfs, d_tx.data_ptr(), d_res.data_ptr(), d_avg.data_ptr())
        torch.cuda.synchronize()
        assert n == nb
        res = d_res.cpu().numpy()
        bad = [i for i in range(nb) if res[i] != 0 or not np.array_equal(keep[3 * i + 2].cpu().numpy()[: tbs // 8], pls[i])]
        assert not bad, (len(bad), bad[:10])
    for sb in sbs:
        sb.free()
    ue.free()
    enb.free()
