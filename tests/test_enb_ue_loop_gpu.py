"""The GPU eNB and the GPU UE talking to each other through the control channels, as srsENB and srsUE do
(phy/test/pdsch_pdcch_file_test.c, phy_dl_test.c): per subframe the eNB packs a DCI
(srsran_dci_msg_pack_pdsch), derives the grant from it (srsran_ra_dl_dci_to_grant), and transmits
PSS / SSS / PBCH / PCFICH / PDCCH / CRS / PDSCH in one srsran_enb_dl_gpu_tx_batch; the samples go through
a fixed channel + AWGN; the UE finds the CFI on the PCFICH (srsran_ue_dl_decode_fft_estimate), the grant
on the PDCCH (srsran_ue_dl_find_dl_dci, no injected grant), and decodes the PDSCH: the payloads equal
what was sent.  1, 2 and 4 ports; TM1 / TM2 / TM3; normal and extended CP; subframes 0 and 5 (sync and
PBCH REs around the PDSCH) and others."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

F1, F1A, F2A = 1, 2, 7
TM1, TM2, TM3 = 0, 1, 2

CASES = [  # (nof_prb, ports, nrx, cp, tm, format, mcs, tti, cfi)
    (100, 2, 2, 0, TM3, F2A, 28, 3, 2),
    (50, 2, 2, 1, TM2, F1, 20, 5, 3),
    (6, 1, 1, 0, TM1, F1A, 10, 0, 2),
    (25, 4, 2, 0, TM2, F1, 16, 10, 1),
    (15, 1, 1, 1, TM1, F1, 12, 15, 2),
]


@pytest.fixture(scope="module")
def env():
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    import torch
    return torch


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}prb_{c[1]}p_{'ext' if c[3] else 'norm'}_tm{c[4] + 1}_sf{c[7] % 10}"
                                             for c in CASES])
def test_enb_to_ue_through_pdcch(env, case):
    torch = env
    from srsran_4g_amd import enb_dl as E
    from srsran_4g_amd import pdcch as PD
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import ue_dl as U
    nprb, P, nrx, cp, tm, fmt, mcs, tti, cfi = case
    cell_id, rnti = 97, 0x4A21
    rng = np.random.default_rng(nprb * 31 + tti)
    U.use_standard_symbol_size(True)
    cell = U.cell(nprb, P, cell_id, cp=cp)
    regs = PD.Regs(cell)
    nof_cce = regs.q.pdcch_nregs[cfi - 1] // 9
    regs.free()
    # the scheduler side: DCI with a full allocation, packed, and the grant it implies
    d = PD.srsran_dci_dl_t()
    d.rnti, d.format, d.pid = rnti, fmt, 3
    for i in range(2):
        d.tb[i].rv = 1
    if fmt == F1A:
        d.alloc_type = 2
        d.raw[0] = U.lib().srsran_ra_type2_to_riv(nprb, 0, nprb)
        d.raw[1] = d.raw[2] = d.raw[3] = 0
    else:
        d.alloc_type = 0
        d.raw[0] = (1 << int(np.ceil(nprb / U.lib().srsran_ra_type0_P(nprb)))) - 1
    ntb = 2 if fmt == F2A else 1
    for i in range(ntb):  # codeword i carries TB i (no swap), as the scheduler fills the DCI
        d.tb[i].mcs_idx, d.tb[i].rv, d.tb[i].ndi, d.tb[i].cw_idx = mcs, 0, True, i
    locs = [loc for loc in PD.ue_locations(nof_cce, tti % 10, rnti) if (1 << loc[0]) <= nof_cce]
    d.location.L, d.location.ncce = max(locs)  # the highest aggregation level the cell offers
    r, msg = PD.pack_pdsch(cell, d)
    assert r == 0
    r, grant = PD.dci_to_grant(cell, d, tti, cfi, tm)
    assert r == 0 and grant.nof_tb == ntb
    qm_of = {m: q for q, m in S.MOD_FROM_QM.items()}
    qm = [qm_of[grant.tb[i].mod] for i in range(ntb)]
    cfg = U.pdsch_cfg(nprb, grant.nof_re, [grant.tb[i].tbs for i in range(ntb)], qm, rnti=rnti, cp=cp)
    cfg.grant = grant
    pls = [rng.integers(0, 256, grant.tb[i].tbs // 8, dtype=np.uint8) for i in range(ntb)]
    d_pl = [torch.from_numpy(p).cuda() for p in pls]
    # the eNB: everything of the subframe in one batch entry
    enb = E.EnbDl(cell)
    N = U.lib().srsran_symbol_sz(nprb)
    d_tx = torch.zeros((1, P, 15 * N, 2), dtype=torch.float32, device="cuda")
    assert enb.tx_batch([(tti, cfi, cfg, [p.data_ptr() for p in d_pl], (True, [msg]))], d_tx.data_ptr()) == 0
    torch.cuda.synchronize()
    tx = d_tx.cpu().numpy().view(np.complex64)[0, :, :, 0]
    enb.free()
    # the channel: phy_dl_test's [[1, 1], [1, -1]] for 2 ports, two rows of +-1 for 4, identity for 1; 30 dB
    H = {1: np.ones((1, 1)), 2: np.array([[1, 1], [1, -1]]), 4: np.array([[1, 1, 1, 1], [1, -1, 1, -1]])}[P]
    rx = (H.astype(np.complex64) @ tx).astype(np.complex64)
    sigma = np.sqrt(np.mean(np.abs(rx) ** 2) / 10 ** 3.0 / 2)
    rx = (rx + sigma * (rng.standard_normal(rx.shape) + 1j * rng.standard_normal(rx.shape))).astype(np.complex64)
    # the UE: CFI from the PCFICH, grant from the PDCCH, PDSCH
    ue = U.UeDl(cell, nrx)
    try:
        assert ue.fft_estimate(list(rx), tti, 0) == 0
        assert ue.last_cfi == cfi
        dcis = ue.find_dl_dci(tti, cfi, rnti, tm=tm)
        assert len(dcis) == 1 and dcis[0].format == fmt and dcis[0].rnti == rnti and dcis[0].pid == 3
        r, g = ue.dci_to_grant(dcis[0], tti, cfi, tm=tm)
        assert r == 0 and g.nof_tb == ntb and g.nof_re == grant.nof_re
        sbs = [S.SoftbufferRx(nof_prb=nprb) for _ in range(ntb)]
        ucfg = U.pdsch_cfg(nprb, g.nof_re, [g.tb[i].tbs for i in range(ntb)], qm, rnti=rnti, cp=cp, softbuffers=sbs)
        ucfg.grant = g
        ret, res = ue.decode_pdsch(ucfg, tti, cfi)
        assert ret == 0
        for i in range(ntb):
            assert res[i][0] and np.array_equal(res[i][1][:len(pls[i])], pls[i]), (i, bool(res[i][0]))
        assert ue.find_dl_dci(tti, cfi, rnti ^ 0x0100, tm=tm) == []
        for sb in sbs:
            sb.free()
    finally:
        ue.free()
