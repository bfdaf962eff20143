"""PUSCH receive, host side and checker (no GPU): the library's DMRS generator (refsignal_ul.c:95-358
restated in csrc/pusch_api.cpp) against the oracle built on the reference's compiled
srsran_zc_sequence_generate_lte / srsran_group_hopping_f_gh; the transform-precoding PRB rule
against dft_precoding.c:88-112; and the checker chain itself: test transmitter -> oracle channel
estimator -> equaliser / inverse DFT -> reference demapper / descrambler -> reference UCI + UL-SCH
receiver returns the transmitted payload and UCI."""
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
from srsran_4g_amd import pusch as P  # noqa: E402
from srsran_4g_amd import sch as S  # noqa: E402
from srsran_4g_amd.ue_dl import cell as make_cell  # noqa: E402

needs_ref = pytest.mark.skipif(not OP.ref_available(), reason="oracle/_ref not built")


@pytest.fixture(scope="module")
def po():
    return OP.PuschOracle()


def test_valid_prb_matches_reference():
    L = P.lib()
    if OP.ref_available():
        R = ctypes.CDLL(OP.REF_SO, mode=os.RTLD_LAZY)
        R.srsran_dft_precoding_valid_prb.restype = ctypes.c_bool
        R.srsran_dft_precoding_get_valid_prb.restype = ctypes.c_uint32
        for n in range(0, 101):
            assert L.srsran_dft_precoding_valid_prb(n) == R.srsran_dft_precoding_valid_prb(n), n
            if n:
                assert L.srsran_dft_precoding_get_valid_prb(n) == R.srsran_dft_precoding_get_valid_prb(n), n
    assert [n for n in range(1, 13) if L.srsran_dft_precoding_valid_prb(n)] == [1, 2, 3, 4, 5, 6, 8, 9, 10, 12]


@needs_ref
@pytest.mark.parametrize("cell_id", [0, 1, 29, 30, 77, 503])
def test_dmrs_matches_reference(po, cell_id):
    rng = np.random.default_rng(cell_id)
    for cp in (0, 1):
        c = make_cell(nof_prb=100, cell_id=cell_id)
        c.cp = cp
        for _ in range(12):
            d = P.srsran_refsignal_dmrs_pusch_cfg_t()
            d.cyclic_shift, d.delta_ss = int(rng.integers(0, 8)), int(rng.integers(0, 30))
            d.group_hopping_en, d.sequence_hopping_en = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
            n = int(rng.choice([1, 2, 3, 4, 5, 6, 8, 12, 25, 48, 75, 100]))
            sf, cs = int(rng.integers(0, 10)), int(rng.integers(0, 8))
            ret, r = P.dmrs(c, d, n, sf, cs)
            assert ret == 0
            want = po.dmrs(cell_id, cp, d.cyclic_shift, d.delta_ss, d.group_hopping_en, d.sequence_hopping_en, n, sf, cs)
            # same float expressions, but the ZC argument -pi q m (m + 1) / N_zc (double, rounded to
            # float) reaches ~1.4e5 rad at 100 PRB, where one float ulp is 0.016 rad, and the reference
            # is built with -Ofast (reassociation): the few elements whose argument rounds to a
            # neighbouring float differ by a few such ulps; the rest agree to float precision (a wrong
            # u, v or alpha would differ by O(1) almost everywhere)
            err = np.abs(r - want)
            assert err.max() < 0.3 and np.mean(err > 1e-3) < 0.05 and np.median(err) < 1e-5
    d = P.srsran_refsignal_dmrs_pusch_cfg_t()
    d.cyclic_shift = 8
    assert P.dmrs(make_cell(nof_prb=25, cell_id=cell_id), d, 6, 0, 0)[0] != 0


CHAIN = [
    # (name, cell_prb, Qm, L, n_prb, tbs, nack, ri, cqi, cp, shortened)
    ("qpsk_6prb", 25, 2, 6, 3, 1544, 0, 0, None, 0, False),
    ("16qam_25prb_ack", 50, 4, 25, 10, 11064, 2, 0, None, 0, False),
    ("64qam_50prb_uci_srs", 100, 6, 50, 40, 30576, 1, 1, (UC.WB, dict(pmi_present=True)), 0, True),
    ("qpsk_ext_cp", 25, 2, 8, 0, 1736, 3, 1, (UC.WB, dict()), 1, False),
]


@needs_ref
@pytest.mark.parametrize("case", CHAIN, ids=[c[0] for c in CHAIN])
def test_checker_chain_round_trip(po, case):
    import uci as RU
    name, cprb, Qm, L, n0, tbs, nack, ri, cqi, cp, sh = case
    rng = np.random.default_rng(len(name))
    cell_id, tti = 57, 3
    d = P.srsran_refsignal_dmrs_pusch_cfg_t()
    d.cyclic_shift, d.delta_ss, d.group_hopping_en = 2, 5, True
    cfg = TX.make_cfg(cprb, Qm, L, n0, tbs, nack, ri, cqi, cp=cp, shortened=sh)
    grid, payload, u, H, s2 = TX.pusch_subframe(po, cell_id, cprb, cp, cfg, d, tti, rng, snr_db=35.0, shortened=sh)
    r = po.dmrs(cell_id, cp, 2, 5, True, False, L, tti % 10, 0)
    est = po.chest(grid, cprb, cp, L, cfg.grant.n_prb_tilde, cfg.grant.n_prb, r)
    M = 12 * L
    h_true = H[n0 * 12:n0 * 12 + M]
    assert np.mean(np.abs(est["ce"][0, n0 * 12:n0 * 12 + M] - h_true) ** 2) < 0.02
    dsym = po.symbols(grid, est["ce"], est["noise"], cp, sh, L, cfg.grant.n_prb_tilde)
    q = po.llrs(dsym, cfg.grant.tb.mod, cfg.rnti, tti, cell_id)
    c = po.ora.sequence_bits(OP.pusch_seed(cfg.rnti, 2 * (tti % 10), cell_id), q.size)
    rc = TX.make_cfg(cprb, Qm, L, n0, tbs, nack, ri, cqi, cp=cp, shortened=sh)
    got = S.srsran_uci_value_t()
    ret, q2, g, (Qri, Qcqi, G, Qack) = RU.RefUci().rx(rc, q, c, got)
    if nack:
        assert list(got.ack.ack_value[:nack]) == list(u.ack.ack_value[:nack])
    if ri:
        assert got.ri == u.ri
    if cqi:
        assert got.cqi.data_crc
    oret, odata, _, _, _ = po.ora.dlsch_decode(tbs, Qm, 0, g[Qcqi * Qm:(Qcqi + G) * Qm], 8, None)
    assert oret == 0 and np.array_equal(odata[:tbs // 8], payload)
