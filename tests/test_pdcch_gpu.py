"""GPU PCFICH / PDCCH parity (through the C-ABI) against the reference's own pcfich.c / pdcch.c /
viterbi.c compiled into oracle/_ref: CFI and its LLRs, the control-region LLRs, every candidate's
decoded payload / CRC remainder, the blind search (srsran_ue_dl_find_dl_dci) and a C3 subframe
decoded from time samples with its grant taken from the PDCCH."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

pytestmark = pytest.mark.gpu

import pdcch as P  # noqa: E402  (oracle/pdcch.py)


@pytest.fixture(scope="module")
def mods():
    import torch  # noqa: F401  -- one HIP runtime for torch and the library

    from srsran_4g_amd import pdcch as PD
    from srsran_4g_amd import ue_dl as U

    return PD, U


def control_subframe(nprb, nports, cid, tti, cfi, msgs, nrx, rng, snr_db=20.0):
    """reference-encoded control region through a random flat channel + AWGN: returns the rx grids
    (nrx, 14, 12N), the exact estimates (ports, nrx, 14, 12N) and the noise variance"""
    ref = P.Ref()
    tx = ref.ctrl_tx(nprb, nports, cid, tti, cfi, msgs)
    H = (rng.standard_normal((nrx, nports)) + 1j * rng.standard_normal((nrx, nports))) / np.sqrt(2)
    y = np.einsum("rp,pls->rls", H, tx)
    sd = np.sqrt(10 ** (-snr_db / 10) / 2)
    y = y + sd * (rng.standard_normal(y.shape) + 1j * rng.standard_normal(y.shape))
    ce = np.broadcast_to(H.T[:, :, None, None], (nports, nrx, 14, 12 * nprb)).astype(np.complex64)
    return y.astype(np.complex64), np.ascontiguousarray(ce), float(2 * sd * sd)


def dci_msgs(nprb, nports, cid, tti, cfi, rng, n=3, cp=0):
    """random DCIs at non-overlapping UE-search-space locations of random C-RNTIs"""
    from srsran_4g_amd import pdcch as PD

    c = PD.cell(nprb, nports, cid, cp=cp)
    regs = PD.Regs(c)
    nof_cce = regs.q.pdcch_nregs[cfi - 1] // 9
    regs.free()
    used = np.zeros(nof_cce, bool)
    msgs = []
    for _ in range(50):
        if len(msgs) == n:
            break
        rnti = int(rng.integers(11, 0xFFF3))
        fmt = int(rng.choice([P.FORMAT1A, P.FORMAT2A, P.FORMAT1]))
        size = PD.dci_size(c, fmt)
        locs = PD.ue_locations(nof_cce, tti % 10, rnti)
        if not locs:
            continue
        L, ncce = locs[int(rng.integers(len(locs)))]
        if used[ncce:ncce + (1 << L)].any():
            continue
        used[ncce:ncce + (1 << L)] = True
        msgs.append((rng.integers(0, 2, size).astype(np.uint8), L, ncce, rnti, fmt))
    return msgs, nof_cce


CASES = [(100, 2, 1, 3, 1), (100, 2, 301, 7, 3), (50, 2, 7, 0, 2), (25, 1, 12, 4, 2), (6, 1, 2, 8, 3), (6, 2, 5, 5, 1),
         (75, 1, 100, 9, 3), (100, 4, 1, 3, 1), (50, 4, 19, 6, 3), (6, 4, 2, 5, 2)]


@pytest.mark.parametrize("nprb,nports,cid,tti,cfi", CASES)
def test_pcfich_and_pdcch_llr_vs_reference(mods, nprb, nports, cid, tti, cfi):
    PD, U = mods
    rng = np.random.default_rng(nprb * 7 + cid)
    nrx = 2
    msgs, nof_cce = dci_msgs(nprb, nports, cid, tti, cfi, rng)
    y, ce, noise = control_subframe(nprb, nports, cid, tti, cfi, [m[:4] for m in msgs], nrx, rng)
    ref = P.Ref()
    rcfi, rcorr, rllr = ref.ctrl_rx(nprb, nports, cid, tti, y, ce, noise)
    ctl = PD.Control(PD.cell(nprb, nports, cid), nrx)
    try:
        gcfi, gcorr, gdata = ctl.pcfich(y, ce, noise, tti)
        assert gcfi == rcfi == cfi
        assert abs(gcorr - rcorr) <= 1e-4 * max(1.0, abs(rcorr))
        gllr = ctl.pdcch_llr(y, ce, noise, tti, gcfi)
        assert gllr.size == rllr.size == 72 * nof_cce
        if nports >= 2:  # TX diversity: the reference's SSE / generic arithmetic, bit for bit
            assert np.array_equal(gllr, rllr)
        else:  # 1 port: the reference's SIMD MMSE uses rcp approximations
            np.testing.assert_allclose(gllr, rllr, rtol=2e-3, atol=2e-3 * np.abs(rllr).max())
    finally:
        ctl.free()


@pytest.mark.parametrize("nprb,nports,cid,tti,cfi", [c for c in CASES if c[0] in (6, 50, 100)])
def test_extended_cp_control_vs_reference(mods, nprb, nports, cid, tti, cfi):
    """extended-CP cells (regs.c:587-617): CFI, PCFICH correlation, the control-region LLRs and every
    transmitted DCI decoded from them, against the reference built for the same cell"""
    PD, U = mods
    rng = np.random.default_rng(nprb * 11 + cid)
    nrx = 2
    ref = P.Ref()
    ref.set_cp(1)
    try:
        msgs, nof_cce = dci_msgs(nprb, nports, cid, tti, cfi, rng, cp=1)
        y, ce, noise = control_subframe(nprb, nports, cid, tti, cfi, [m[:4] for m in msgs], nrx, rng)
        rcfi, rcorr, rllr = ref.ctrl_rx(nprb, nports, cid, tti, y, ce, noise)
        ctl = PD.Control(PD.cell(nprb, nports, cid, cp=1), nrx)
        try:
            gcfi, gcorr, _ = ctl.pcfich(y, ce, noise, tti)
            assert gcfi == rcfi == cfi
            assert abs(gcorr - rcorr) <= 1e-4 * max(1.0, abs(rcorr))
            gllr = ctl.pdcch_llr(y, ce, noise, tti, gcfi)
            assert gllr.size == rllr.size == 72 * nof_cce
            if nports >= 2:
                assert np.array_equal(gllr, rllr)
            else:
                np.testing.assert_allclose(gllr, rllr, rtol=2e-3, atol=2e-3 * np.abs(rllr).max())
            ctl.set_llr(cfi, rllr)
            fl = [(m[1], m[2], m[4]) for m in msgs]
            got = ctl.decode(tti, cfi, fl)
            for (bits, L, n, rnti, f), (nb, pl, rem, corr) in zip(msgs, got):
                want = ref.pdcch_decode(tti, cfi, rllr, L, n, f)
                assert (nb, rem) == (want[0], want[2]) and np.array_equal(pl, want[1])
                assert nb == len(bits) and rem == rnti and np.array_equal(pl, bits)
        finally:
            ctl.free()
    finally:
        ref.set_cp(0)


@pytest.mark.parametrize("nprb,nports,cid,tti,cfi", CASES[:5] + CASES[7:8])
def test_candidates_bit_exact_vs_reference(mods, nprb, nports, cid, tti, cfi):
    """every UE / common search-space candidate of every generated RNTI, three formats, decoded on the
    GPU from the reference's own LLRs: payload bits, CRC remainder and the mean gate equal"""
    PD, U = mods
    rng = np.random.default_rng(1000 + nprb + cid)
    nrx = 2
    msgs, nof_cce = dci_msgs(nprb, nports, cid, tti, cfi, rng)
    y, ce, noise = control_subframe(nprb, nports, cid, tti, cfi, [m[:4] for m in msgs], nrx, rng, snr_db=6.0)
    ref = P.Ref()
    rcfi, _, rllr = ref.ctrl_rx(nprb, nports, cid, tti, y, ce, noise)
    assert rcfi == cfi
    cands = set(PD.common_locations(nof_cce))
    for m in msgs:
        cands |= set(PD.ue_locations(nof_cce, tti % 10, m[3]))
    cands = sorted(cands)
    fl = [(L, n, f) for (L, n) in cands for f in (P.FORMAT1A, P.FORMAT2A, P.FORMAT1)]
    ctl = PD.Control(PD.cell(nprb, nports, cid), nrx)
    try:
        ctl.set_llr(cfi, rllr)
        got = ctl.decode(tti, cfi, fl)
        found = 0
        for (L, n, f), (nb, pl, rem, corr) in zip(fl, got):
            want = ref.pdcch_decode(tti, cfi, rllr, L, n, f)
            assert nb == want[0], (L, n, f)
            if nb:
                assert np.array_equal(pl, want[1]) and rem == want[2], (L, n, f)
                assert abs(corr - want[3]) <= 1e-4, (L, n, f, corr, want[3])
            for bits, mL, mn, rnti, mf in msgs:
                if (mL, mn) == (L, n) and len(bits) == nb and rem == rnti:
                    found += np.array_equal(pl, bits)
        assert found == len(msgs)
    finally:
        ctl.free()


def test_pure_noise_candidates_bit_exact(mods):
    """LLRs of pure noise: the Viterbi metrics wrap and tie everywhere; still equal to the reference"""
    PD, U = mods
    rng = np.random.default_rng(3)
    nprb, nports, cid, tti, cfi = 50, 2, 9, 2, 3
    y, ce, noise = control_subframe(nprb, nports, cid, tti, cfi, [], 2, rng)
    ref = P.Ref()
    ref.ctrl_rx(nprb, nports, cid, tti, y, ce, noise)
    ctl = PD.Control(PD.cell(nprb, nports, cid), 2)
    try:
        nof_cce = ctl.ncce(cfi)
        llr = (rng.standard_normal(72 * nof_cce) * 2).astype(np.float32)
        ctl.set_llr(cfi, llr)
        fl = [(L, n, f) for L in range(4) for n in range(0, nof_cce - (1 << L) + 1, 1 << L)
              for f in (P.FORMAT1A, P.FORMAT2A)]
        got = ctl.decode(tti, cfi, fl)
        for (L, n, f), (nb, pl, rem, corr) in zip(fl, got):
            want = ref.pdcch_decode(tti, cfi, llr, L, n, f)
            assert nb == want[0] and np.array_equal(pl, want[1]) and rem == want[2], (L, n, f)
    finally:
        ctl.free()


def test_find_dl_dci_and_pdsch_without_injected_grant(mods):
    """C3 (100 PRB, 2x2 TM3, 64QAM, 2 TBs): time samples -> OFDM -> CRS estimate -> PCFICH (CFI from
    the air) -> PDCCH blind search (format 2A for the C-RNTI) -> grant -> PDSCH decode; payloads equal"""
    import torch  # noqa: F401

    PD, U = mods
    from srsran_4g_amd import sch
    from synth import synth as S

    cid, tti, cfi, rnti, tbs = 1, 3, 2, 0x1234, 75376
    rng = np.random.default_rng(42)
    c = PD.cell(100, 2, cid)
    bits = P.dci_pack_2a(100, PD.dci_size(c, P.FORMAT2A), (1 << 25) - 1, [(28, 1, 0), (28, 1, 0)], pid=1)
    regs = PD.Regs(c)
    nof_cce = regs.q.pdcch_nregs[cfi - 1] // 9
    regs.free()
    L, ncce = [loc for loc in PD.ue_locations(nof_cce, tti % 10, rnti) if loc[0] == 3][0]
    ctrl = P.Ref().ctrl_tx(100, 2, cid, tti, cfi, [(bits, L, ncce, rnti)])
    # the reference encoder wrote a PCFICH too: the transmitter's own is skipped (pcfich=False)
    pls = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(2)]
    x, nre = S.pdsch_subframe(100, cid, 2, tti, cfi, rnti, tbs, 6, 0, pls, snr_db=30.0, rng=rng, pcfich=False,
                              ctrl=[ctrl[0], ctrl[1]])
    U.use_standard_symbol_size(True)
    ue = U.UeDl(U.cell(100, 2, cid), 2)
    try:
        assert ue.fft_estimate(x, tti, 0) == 0
        assert ue.last_cfi == cfi
        dcis = ue.find_dl_dci(tti, cfi, rnti, tm=2)
        assert len(dcis) == 1
        d = dcis[0]
        assert d.format == P.FORMAT2A and d.rnti == rnti and d.pid == 1 and d.type0_rbg_bitmask == (1 << 25) - 1
        r, g = ue.dci_to_grant(d, tti, cfi, tm=2)
        assert r == 0 and g.nof_tb == 2 and g.tb[0].tbs == tbs and g.nof_re == nre
        sbs = [sch.SoftbufferRx(nof_prb=100) for _ in range(2)]
        cfg = U.pdsch_cfg(100, nre, (tbs, tbs), (6, 6), softbuffers=sbs)
        cfg.grant = g
        cfg.rnti = rnti
        ret, res = ue.decode_pdsch(cfg, tti, cfi)
        assert ret == 0
        for i in range(2):
            assert res[i][0] and np.array_equal(res[i][1][:tbs // 8], pls[i])
        # a different RNTI finds nothing
        assert ue.find_dl_dci(tti, cfi, 0x4321, tm=2) == []
    finally:
        ue.free()


def test_find_dl_dci_and_pdsch_four_ports(mods):
    """4-port TM2 cell: time samples -> OFDM -> 4-port CRS estimate -> PCFICH and PDCCH with 4-port SFBC +
    FSTD -> format 1 grant -> 4-port transmit-diversity PDSCH decode; payload equal"""
    PD, U = mods
    from srsran_4g_amd import sch
    from synth import synth as S

    cid, tti, cfi, rnti, mcs = 6, 3, 2, 0x2222, 20
    rng = np.random.default_rng(43)
    c = PD.cell(100, 4, cid)
    lib = U.lib()
    tbs = lib.srsran_ra_tbs_from_idx(lib.srsran_ra_tbs_idx_from_mcs(mcs, False, False), 100)
    bits = P.dci_pack_1(100, PD.dci_size(c, P.FORMAT1), (1 << 25) - 1, mcs, 2, 1, 0)
    regs = PD.Regs(c)
    nof_cce = regs.q.pdcch_nregs[cfi - 1] // 9
    regs.free()
    L, ncce = [loc for loc in PD.ue_locations(nof_cce, tti % 10, rnti) if loc[0] == 2][0]
    ctrl = P.Ref().ctrl_tx(100, 4, cid, tti, cfi, [(bits, L, ncce, rnti)])
    pl = [rng.integers(0, 256, tbs // 8, dtype=np.uint8)]
    x, nre = S.pdsch_subframe(100, cid, 4, tti, cfi, rnti, tbs, 6, 0, pl, scheme="diversity4", snr_db=30.0, rng=rng,
                              pcfich=False, ctrl=list(ctrl[:4]))
    U.use_standard_symbol_size(True)
    ue = U.UeDl(U.cell(100, 4, cid), 2)
    try:
        assert ue.fft_estimate(x, tti, 0) == 0
        assert ue.last_cfi == cfi
        dcis = ue.find_dl_dci(tti, cfi, rnti, tm=1)
        assert len(dcis) == 1 and dcis[0].format == P.FORMAT1 and dcis[0].rnti == rnti
        r, g = ue.dci_to_grant(dcis[0], tti, cfi, tm=1)
        assert r == 0 and g.nof_tb == 1 and g.tb[0].tbs == tbs and g.nof_re == nre and g.nof_layers == 4
        sbs = [sch.SoftbufferRx(nof_prb=100)]
        cfg = U.pdsch_cfg(100, nre, [tbs], [6], scheme="diversity", softbuffers=sbs, nof_ports=4)
        cfg.grant = g
        cfg.rnti = rnti
        ret, res = ue.decode_pdsch(cfg, tti, cfi)
        assert ret == 0 and res[0][0] and np.array_equal(res[0][1][:tbs // 8], pl[0])
    finally:
        ue.free()


def test_find_ul_dci_format0_and_mi(mods):
    """srsran_ue_dl_find_ul_dci (ue_dl.c:573-611): a format 0 grant and a format 2A grant for one C-RNTI in
    the UE search space, from time samples; find_dl_dci returns the 2A and sets the format 0 aside,
    find_ul_dci unpacks it (fields as packed) and empties the list.  The search on the PHICH m_i = 1 REG
    tables chosen manually (srsran_ue_dl_set_mi_manual(1)) equals the automatic FDD choice."""
    import torch  # noqa: F401

    PD, U = mods
    from synth import synth as S

    cid, tti, cfi, rnti, tbs = 1, 3, 2, 0x1234, 75376
    rng = np.random.default_rng(43)
    c = PD.cell(100, 2, cid)
    dl_bits = P.dci_pack_2a(100, PD.dci_size(c, P.FORMAT2A), (1 << 25) - 1, [(28, 1, 0), (28, 1, 0)], pid=1)
    riv = P.riv(20, 30, 100)
    ul_bits = P.dci_pack_0(100, PD.dci_size(c, P.FORMAT0), riv, 17, 1, tpc=2, n_dmrs=5, cqi=1)
    regs = PD.Regs(c)
    nof_cce = regs.q.pdcch_nregs[cfi - 1] // 9
    regs.free()
    locs = PD.ue_locations(nof_cce, tti % 10, rnti)
    L3 = [loc for loc in locs if loc[0] == 3][0]
    L1 = [loc for loc in locs if loc[0] == 1 and not (L3[1] <= loc[1] < L3[1] + 8)][0]
    ctrl = P.Ref().ctrl_tx(100, 2, cid, tti, cfi, [(dl_bits, L3[0], L3[1], rnti), (ul_bits, L1[0], L1[1], rnti)])
    pls = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(2)]
    x, nre = S.pdsch_subframe(100, cid, 2, tti, cfi, rnti, tbs, 6, 0, pls, snr_db=30.0, rng=rng, pcfich=False,
                              ctrl=[ctrl[0], ctrl[1]])
    U.use_standard_symbol_size(True)
    ue = U.UeDl(U.cell(100, 2, cid), 2)
    try:
        assert ue.set_mbsfn_area_id(1) == 0  # cc_worker.cc:151
        for mi in (None, 1):
            ue.set_mi(mi)
            assert ue.fft_estimate(x, tti, 0) == 0 and ue.last_cfi == cfi
            dcis = ue.find_dl_dci(tti, cfi, rnti, tm=2)
            assert len(dcis) == 1 and dcis[0].format == P.FORMAT2A
            ul = ue.find_ul_dci(tti, cfi, rnti)
            assert len(ul) == 1
            u = ul[0]
            assert (u.rnti, u.format, u.location.L, u.location.ncce) == (rnti, P.FORMAT0, L1[0], L1[1])
            assert u.type2_alloc.riv == riv and u.tb.mcs_idx == 17 and u.tb.ndi and u.tpc_pusch == 2
            assert u.n_dmrs == 5 and u.cqi_request and u.freq_hop_fl == -1
            assert ue.find_ul_dci(tti, cfi, rnti) == []  # consumed
        # m_i = 0 tables: a different control region layout; the search runs (finds what it finds)
        ue.set_mi(0)
        assert ue.fft_estimate(x, tti, 0) == 0
        ue.find_dl_dci(tti, cfi, rnti, tm=2)
        ue.set_mi(None)
    finally:
        ue.free()


@pytest.mark.parametrize("tti", [1, 6, 0, 5])
def test_tdd_extended_phich_control_region(mods, tti):
    """TDD cell with the extended PHICH duration: in subframes 1 / 6 srsran_ue_dl_find_dl_dci searches the REG tables
    whose PHICH keeps to two symbols (MI_IDX + 3, ue_dl.c:59-64; srsran_regs_init_opts(..., true), regs.c:329-340),
    in the others the three-symbol ones of that subframe's m_i (uplink-downlink configuration 0: m_i = 2 in
    subframes 0 / 5, 1 in 1 / 6).  The control region comes from the reference's own pcfich.c / pdcch.c on the
    reference's tables of the same options; a DCI is found from time samples.  The manual m_i choice never takes the
    two-symbol tables (ue_dl.c:308-311), so in subframes 1 / 6 it does not find the DCI."""
    import torch  # noqa: F401

    PD, U = mods
    from synth import synth as S

    tdd, cid, rnti, tbs = (0, 7), 17, 0x4321, 2216
    sf16 = tti % 10 in (1, 6)
    mi = [2, 1, 0, 0, 0, 2, 1, 0, 0, 0][tti % 10]
    cfi = 2 if sf16 else 3  # the extended duration needs the PHICH's symbols in the control region
    rng = np.random.default_rng(200 + tti)
    c = PD.cell(100, 2, cid, 1)
    c.frame_type = 1
    bits = P.dci_pack_1a(100, PD.dci_size(c, P.FORMAT1A), P.riv(10, 5, 100), 5, 1, 1, 0)  # flag 1A, localized
    regs = PD.Regs(c, phich_mi=mi, sf1_6=sf16)
    nof_cce = regs.q.pdcch_nregs[cfi - 1] // 9
    regs.free()
    L, ncce = [loc for loc in PD.ue_locations(nof_cce, tti % 10, rnti) if loc[0] == 2][0]
    ctrl = P.Ref().ctrl_tx(100, 2, cid, tti, cfi, [(bits, L, ncce, rnti)], phich_len=1, phich_mi=mi, sf1_6=sf16)
    pls = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(2)]
    x, _ = S.pdsch_subframe(100, cid, 2, tti, cfi, rnti, tbs, 2, 0, pls, snr_db=30.0, rng=rng, pcfich=False,
                            ctrl=[ctrl[0], ctrl[1]], tdd=tdd)
    U.use_standard_symbol_size(True)
    ue = U.UeDl(U.cell(100, 2, cid, tdd=True, phich_len=1), 2, tdd=tdd)
    try:
        assert ue.fft_estimate(x, tti, 0) == 0 and ue.last_cfi == cfi
        dcis = ue.find_dl_dci(tti, cfi, rnti, tm=1)
        assert len(dcis) == 1
        d = dcis[0]
        assert (d.rnti, d.format, d.location.L, d.location.ncce) == (rnti, P.FORMAT1A, L, ncce)
        if sf16:
            ue.set_mi(mi)
            assert ue.fft_estimate(x, tti, 0) == 0
            assert all(x.location.ncce != ncce or x.rnti != rnti for x in ue.find_dl_dci(tti, cfi, rnti, tm=1))
            ue.set_mi(None)
    finally:
        ue.free()
