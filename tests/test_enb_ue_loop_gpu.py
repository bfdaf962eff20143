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


@pytest.mark.parametrize("case", [(50, 2, 2, "1c_si", 5, 1), (100, 2, 2, "1a_dist_gap2", 3, 2), (25, 1, 1, "1c_si", 7, 2),
                                  (15, 1, 1, "1a_dist", 2, 3), (50, 2, 2, "1a_dist", 4, 2)],
                         ids=["50prb_1c_si_rnti", "100prb_1a_distributed_gap2", "25prb_1c_si_rnti", "15prb_1a_distributed",
                              "50prb_1a_distributed"])
def test_enb_to_ue_distributed_vrb(env, case):
    """system information and distributed-VRB grants (ra_dl.c:225-316, 383-391; dci.c:952-1023): the eNB
    sends a format 1C DCI with the SI-RNTI in the common search space (TBS of 36.213 Table 7.1.7.2.3-1, QPSK), or a
    C-RNTI format 1A with distributed VRBs (N_gap,1 / N_gap,2), whose PRBs differ between the two slots; the UE finds
    it by srsran_ue_dl_find_dl_dci from the samples, derives the same grant and decodes the PDSCH"""
    torch = env
    from srsran_4g_amd import enb_dl as E
    from srsran_4g_amd import pdcch as PD
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import ue_dl as U
    nprb, P, nrx, kind, tti, cfi = case
    si = kind.startswith("1c")
    rnti = 0xFFFF if si else 0x3B07
    fmt = 4 if si else F1A  # SRSRAN_DCI_FORMAT1C
    tm = TM1 if P == 1 else TM2
    cell_id = 41
    rng = np.random.default_rng(nprb + tti)
    U.use_standard_symbol_size(True)
    cell = U.cell(nprb, P, cell_id)
    regs = PD.Regs(cell)
    nof_cce = regs.q.pdcch_nregs[cfi - 1] // 9
    regs.free()
    d = PD.srsran_dci_dl_t()
    d.rnti, d.format, d.pid = rnti, fmt, 1
    for i in range(2):
        d.tb[i].rv = 1
    d.alloc_type = 2
    ngap1 = kind != "1a_dist_gap2"
    step = (2 if nprb < 50 else 4) if si else 1
    ngap = {6: 3, 15: 8, 25: 12, 50: 27, 100: 48}[nprb] if ngap1 else 16
    nvrb = (2 * min(ngap, nprb - ngap) if ngap1 else (nprb // ngap) * 2 * ngap) // step
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import pdcch as OP
    # the largest allocation from VRB 1 that the reference maps inside the cell (with N_gap,2 its N~_VRB is twice
    # 36.211's, ra_dl.c:257-260, so long ones fall outside and are refused)
    riv_n = nvrb if si else nprb  # 1C: the RIV counts N_RB^step units of N_VRB^DL (36.213 7.1.6.3)
    # and, for a C-RNTI 1A at N_RB >= 50, whose RIV fits the field the N_gap bit leaves (riv_nbits - 1 bits: the
    # reference packer truncates a larger one, dci.c:751-755)
    riv_max = 1 << (OP.riv_nbits(nprb) - (1 if not si and nprb >= 50 else 0))
    L = max(n for n in range(1, max(2, nvrb // 2 + 1))
            if OP.type2_prbs(nprb, U.lib().srsran_ra_type2_to_riv(n, 1, riv_n), True, ngap1, fmt1c=si)
            and (si or U.lib().srsran_ra_type2_to_riv(n, 1, riv_n) < riv_max))
    riv = U.lib().srsran_ra_type2_to_riv(L, 1, riv_n)
    d.raw[0], d.raw[1], d.raw[2], d.raw[3] = riv, 0, 0 if ngap1 else 1, 1  # distributed
    d.tb[0].mcs_idx, d.tb[0].rv, d.tb[0].ndi, d.tb[0].cw_idx = (9 if si else 7), 0, True, 0
    locs = PD.common_locations(nof_cce) if si else \
        [loc for loc in PD.ue_locations(nof_cce, tti % 10, rnti) if (1 << loc[0]) <= nof_cce]
    d.location.L, d.location.ncce = max(locs)
    r, msg = PD.pack_pdsch(cell, d)
    assert r == 0
    r, grant = PD.dci_to_grant(cell, d, tti, cfi, tm)
    want = OP.type2_prbs(nprb, riv, True, ngap1, fmt1c=si)
    assert r == 0 and grant.nof_tb == 1 and grant.nof_prb == len(want[0])
    for s in range(2):
        assert [n for n in range(nprb) if grant.prb_idx[s][n]] == sorted(want[s])
    hops = any(grant.prb_idx[0][n] != grant.prb_idx[1][n] for n in range(nprb))
    if (nprb, kind) == (50, "1c_si"):
        # 50 PRB, format 1C: allocations come in N_RB^step = 4 VRBs from multiples of 4, and with N_gap,1 = 27 the
        # interleaver (36.211 6.2.3.2, 4 columns) maps every such group to the same PRBs in both slots -- no 1C grant of
        # this cell hops: checked over every RIV (type2_prbs of ra_dl.c:234-260); the other cases hop
        assert not hops
        assert not any((lambda w: w and sorted(w[0]) != sorted(w[1]))(
            OP.type2_prbs(nprb, U.lib().srsran_ra_type2_to_riv(n, s0, riv_n), True, ngap1, fmt1c=True))
            for n in range(1, nvrb + 1) for s0 in range(nvrb))
    else:
        assert hops  # a distributed grant: slot 1's PRBs differ from slot 0's
    grant.tb[0].rv = 0  # 1C carries no RV (36.321 5.3.1: the UE derives it from the SFN)
    qm = [{1: 2, 2: 4, 3: 6}[grant.tb[0].mod]]
    cfg = U.pdsch_cfg(nprb, grant.nof_re, [grant.tb[0].tbs], qm, rnti=rnti, scheme="port0" if P == 1 else "diversity",
                      nof_ports=P)
    cfg.grant = grant
    pls = [rng.integers(0, 256, grant.tb[0].tbs // 8, dtype=np.uint8)]
    d_pl = [torch.from_numpy(p).cuda() for p in pls]
    enb = E.EnbDl(cell)
    N = U.lib().srsran_symbol_sz(nprb)
    d_tx = torch.zeros((1, P, 15 * N, 2), dtype=torch.float32, device="cuda")
    assert enb.tx_batch([(tti, cfi, cfg, [p.data_ptr() for p in d_pl], (True, [msg]))], d_tx.data_ptr()) == 0
    torch.cuda.synchronize()
    tx = d_tx.cpu().numpy().view(np.complex64)[0, :, :, 0]
    enb.free()
    H = {1: np.ones((1, 1)), 2: np.array([[1, 1], [1, -1]])}[P]
    rx = (H.astype(np.complex64) @ tx).astype(np.complex64)
    sigma = np.sqrt(np.mean(np.abs(rx) ** 2) / 10 ** 3.0 / 2)
    rx = (rx + sigma * (rng.standard_normal(rx.shape) + 1j * rng.standard_normal(rx.shape))).astype(np.complex64)
    ue = U.UeDl(cell, nrx)
    try:
        assert ue.fft_estimate(list(rx), tti, 0) == 0
        assert ue.last_cfi == cfi
        dcis = ue.find_dl_dci(tti, cfi, rnti, tm=tm, common_ss=not si)
        assert len(dcis) == 1 and dcis[0].format == fmt and dcis[0].rnti == rnti
        r, g = ue.dci_to_grant(dcis[0], tti, cfi, tm=tm)
        assert r == 0 and g.nof_re == grant.nof_re and g.tb[0].tbs == grant.tb[0].tbs
        for s in range(2):
            assert [g.prb_idx[s][n] for n in range(nprb)] == [grant.prb_idx[s][n] for n in range(nprb)]
        g.tb[0].rv = 0
        sbs = [S.SoftbufferRx(nof_prb=nprb)]
        ucfg = U.pdsch_cfg(nprb, g.nof_re, [g.tb[0].tbs], qm, rnti=rnti, softbuffers=sbs,
                           scheme="port0" if P == 1 else "diversity", nof_ports=P)
        ucfg.grant = g
        ret, res = ue.decode_pdsch(ucfg, tti, cfi)
        assert ret == 0 and res[0][0] and np.array_equal(res[0][1][:len(pls[0])], pls[0])
        for sb in sbs:
            sb.free()
    finally:
        ue.free()
