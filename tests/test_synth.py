"""The synthetic transmitter (synth/) against the oracle (pinned to the reference): turbo
encoder, DL-SCH encoder, Gold sequence, CRS values, PDSCH RE set, modulation vs demapper."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

from oracle import CB_SIZES, Oracle  # noqa: E402
import pdsch_np  # noqa: E402
from synth import synth as S  # noqa: E402


@pytest.fixture(scope="module")
def ora():
    return Oracle()


def test_turbo_encoder_all_sizes(ora):
    rng = np.random.default_rng(1)
    for K in CB_SIZES:
        b = rng.integers(0, 2, K, dtype=np.uint8)
        assert np.array_equal(S.turbo_encode(K, b), ora.encode(K, b)), K


@pytest.mark.parametrize("tbs,Qm,rv", [(75376, 6, 0), (75376, 6, 2), (1544, 2, 1), (30576, 4, 3), (6200, 6, 0),
                                       (97896, 8, 0), (40, 2, 0)])
def test_dlsch_encoder(ora, tbs, Qm, rv):
    rng = np.random.default_rng(tbs + rv)
    tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    for G in (Qm * ((3 * tbs) // (2 * Qm) + 7), 86400 - 86400 % Qm):
        assert np.array_equal(S.dlsch_encode(tbs, Qm, rv, G, tb), ora.dlsch_encode(tbs, Qm, rv, G, tb)), (tbs, G)


def test_tb_crc_corruption(ora):
    rng = np.random.default_rng(3)
    tb = rng.integers(0, 256, 75376 // 8, dtype=np.uint8)
    a = S.dlsch_encode(75376, 6, 0, 86400, tb, tb_crc_xor=0x5A)
    b = ora.dlsch_encode(75376, 6, 0, 86400, tb, tb_crc_xor=0x5A)
    assert np.array_equal(a, b)


def test_gold(ora):
    for seed in (0, 1, 0x1234 << 14, 0x7FFFFFFF):
        assert np.array_equal(S.gold(seed, 5000), ora.sequence_bits(seed, 5000))


@pytest.mark.parametrize("cell_id,nof_prb,sf", [(1, 100, 1), (0, 6, 0), (301, 50, 7), (503, 25, 9)])
def test_crs_values(ora, cell_id, nof_prb, sf):
    ref = ora.crs_pilots(cell_id, nof_prb, 0, sf).reshape(4, -1)
    for li in range(4):
        v = S.crs_values(cell_id, nof_prb, 2 * sf + li // 2, 0 if li % 2 == 0 else 4)
        np.testing.assert_allclose(v, ref[li], atol=1e-6)


@pytest.mark.parametrize("nof_prb,nports,cell_id,cfi,sf", [(100, 2, 1, 1, 1), (100, 2, 1, 1, 0), (100, 2, 7, 2, 5),
                                                           (50, 1, 2, 3, 0), (6, 2, 5, 2, 5), (100, 1, 0, 1, 3)])
def test_pdsch_re_set(nof_prb, nports, cell_id, cfi, sf):
    m = S.pdsch_mask(nof_prb, nports, cell_id, cfi, sf)
    lstart = cfi + (1 if nof_prb < 10 else 0)
    ref = pdsch_np.re_table(nof_prb, nports, cell_id, np.ones((2, nof_prb), bool), lstart, sf)
    got = np.flatnonzero(m.reshape(-1))
    assert np.array_equal(got, np.array([t[0] for t in ref], np.int64))


@pytest.mark.parametrize("Qm,mod", [(2, 1), (4, 2), (6, 3), (8, 4)])
def test_modulation_matches_demapper(ora, Qm, mod):
    """noise-free symbols demap to LLRs whose sign gives back the bits (LLR > 0 <=> bit 1)"""
    rng = np.random.default_rng(Qm)
    bits = rng.integers(0, 2, Qm * 400, dtype=np.uint8)
    sym = S.modulate(bits, Qm)
    allb = ((np.arange(2 ** Qm)[:, None] >> np.arange(Qm - 1, -1, -1)[None, :]) & 1).astype(np.uint8)
    np.testing.assert_allclose(np.mean(np.abs(S.modulate(allb.reshape(-1), Qm)) ** 2), 1.0, rtol=1e-6)
    llr = ora.demod_s(mod, sym)
    assert np.all(llr != 0)
    assert np.array_equal((llr > 0).astype(np.uint8), bits)


def test_cdd_roundtrip(ora):
    """CDD precoding then the reference-pinned MMSE predecoder with the exact channel returns x"""
    rng = np.random.default_rng(5)
    n = 256
    x = [S.modulate(rng.integers(0, 2, 6 * n, dtype=np.uint8), 6) for _ in range(2)]
    y = S.precode(x, "cdd")
    Hm = np.array([[1, 1], [1, -1]], np.complex64)
    r = [(Hm[i, 0] * y[0] + Hm[i, 1] * y[1]).astype(np.complex64) for i in range(2)]
    h = np.zeros((2, 2, n), np.complex64)
    for p in range(2):
        for i in range(2):
            h[p, i] = Hm[i, p]
    xe, _ = ora.predecode(3, np.stack(r), h, 2, 0, 1.0, 1e-6)
    np.testing.assert_allclose(xe[0], x[0], atol=1e-3)
    np.testing.assert_allclose(xe[1], x[1], atol=1e-3)


def test_natural_to_sb(ora):
    rng = np.random.default_rng(9)
    for K in (40, 408, 512, 800, 1024, 6144, 6080, 4008):
        x = rng.integers(-300, 300, 3 * K + 12).astype(np.int16)
        assert np.array_equal(S.natural_to_sb(K, x), ora.natural_to_sb(K, x)), K
    x = rng.integers(-300, 300, (3, 3 * 6144 + 12)).astype(np.int16)
    assert np.array_equal(S.natural_to_sb(6144, x)[1], ora.natural_to_sb(6144, x[1]))


def test_make_llrs_matches_oracle_generator():
    from oracle import make_llrs
    for K in (6144, 40):
        b1, l1 = S.make_llrs(K, 4.0, np.random.default_rng(K), 3)
        b2, l2 = make_llrs(K, 4.0, np.random.default_rng(K), 3)
        assert np.array_equal(b1, b2) and np.array_equal(l1, l2)


def test_ldpc_tx_matches_oracle_encoder():
    """synth/ldpc_tx.py (bench / test inputs) encodes like the oracle (pinned on the golden examples)."""
    from ldpc import LIFT_SIZES, OracleLdpc

    from synth import ldpc_tx

    ora = OracleLdpc()
    rng = np.random.default_rng(9)
    for bg in (0, 1):
        for ls in LIFT_SIZES[::3] + [384]:
            K = (22 if bg == 0 else 10) * ls
            msgs = rng.integers(0, 2, (3, K)).astype(np.uint8)
            got = ldpc_tx.encode(bg, ls, msgs)
            for m, g in zip(msgs, got):
                assert np.array_equal(g, ora.encode(bg, ls, m)), (bg, ls)


@pytest.mark.parametrize("cell_id", [0, 1, 2, 167, 301, 503])
@pytest.mark.parametrize("sf", [0, 5])
def test_sync_signals_match_reference(cell_id, sf):
    """synth's PSS / SSS (36.211 6.11, written from the standard) equal the reference eNB's put_sync
    (srsran_pss_generate / srsran_sss_generate / pss_put_slot / sss_put_slot through ref_enb_ctrl_harness.c) on the
    PSS / SSS rows of subframes 0 and 5, including the 5 empty subcarriers either side"""
    import oracle as ORA
    if not ORA.ref_available():
        pytest.skip("oracle/_ref not built")
    import pdcch as OP
    nof_prb = 25
    ref = OP.Ref().enb_ctrl_tx(nof_prb, 1, cell_id, sf, 1, [], put_base=True)[0]
    got = S.sync_grid(nof_prb, cell_id, sf)
    lo, hi = 6 * nof_prb - 36, 6 * nof_prb + 36
    np.testing.assert_array_equal(got[5, lo:hi], ref[5, lo:hi])  # SSS (normal CP): +-1
    # PSS: the reference rounds the Zadoff-Chu phase argument (up to ~6600 rad) to float before cosf / sinf
    # (pss.c:352-363), synth evaluates it in double: within 5e-4
    np.testing.assert_allclose(got[6, lo:hi], ref[6, lo:hi], atol=5e-4)


@pytest.mark.parametrize("sf_config", range(7))
@pytest.mark.parametrize("ss_config", [0, 1, 4, 5, 9])
def test_tdd_pdsch_re_set(sf_config, ss_config):
    """synth's TDD PDSCH REs (36.211 rules: DwPTS only, SSS last symbol of 0 / 5, PSS symbol 2 of 1 / 6) equal the
    oracle's rule-based RE walk with the grant's DwPTS symbols per slot, in every downlink and special subframe"""
    for sf in range(10):
        if pdsch_np.tdd_type(sf_config, sf) == "U":
            continue
        for nports, cfi, nof_prb in ((2, 1, 100), (1, 2, 50), (4, 2, 6)):
            m = S.pdsch_mask(nof_prb, nports, 7, cfi, sf, tdd=(sf_config, ss_config))
            lstart = cfi + (1 if nof_prb < 10 else 0)
            nsl = pdsch_np.tdd_nof_symb_slot(sf_config, ss_config, sf)
            ref = pdsch_np.re_table(nof_prb, nports, 7, np.ones((2, nof_prb), bool), lstart, sf, fdd=False, nsl=nsl)
            # grid rows of slot 1 start at nsl[0] in the reference's walk; in the grid they start at row 7
            got = np.flatnonzero(m.reshape(-1))
            want = np.array([t[0] for t in ref], np.int64)
            if nsl[0] == 7:
                assert np.array_equal(got, want), (sf, nports)
            else:  # DwPTS shorter than a slot: slot 1 empty, the rows coincide
                assert nsl[1] == 0 and np.array_equal(got, want), (sf, nports)
