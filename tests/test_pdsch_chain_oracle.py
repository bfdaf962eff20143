"""CPU: the oracle chain (oracle/pdsch_chain.py) decodes synthetic eNB subframes (synth/) --
the precondition for using it as the checker of the GPU chain."""
import numpy as np
import pytest

from oracle import Oracle
import pdsch_chain as PC
from synth import synth as S

TBS = 75376


@pytest.fixture(scope="module")
def ora():
    return Oracle()


@pytest.mark.parametrize("tti,cfi,snr,scheme,pmi", [(1, 1, None, "cdd", 0), (5, 2, 30.0, "cdd", 0),
                                                     (10, 1, 25.0, "cdd", 0), (3, 1, 30.0, "sm", 1)])
def test_oracle_chain_decodes_c3(ora, tti, cfi, snr, scheme, pmi):
    rng = np.random.default_rng(tti)
    pls = [rng.integers(0, 256, TBS // 8, dtype=np.uint8) for _ in range(2)]
    x, nre = S.pdsch_subframe(100, 1, 2, tti, cfi, 0x1234, TBS, 6, 0, pls, scheme=scheme, codebook=pmi + 1,
                              snr_db=snr, rng=rng)
    g, ce, st = PC.fft_estimate(ora, x, 100, 1, 2, tti)
    res = PC.pdsch_decode(ora, g, ce, st["noise"], 100, 1, 2, tti, cfi, 0x1234, [TBS, TBS], [6, 6], [0, 0],
                          scheme=scheme, pmi=pmi)
    for q in range(2):
        assert res[q]["ret"] == 0
        assert np.array_equal(res[q]["data"][: TBS // 8], pls[q])
    assert res[0]["nof_re"] == nre


def test_oracle_chain_port0_16qam(ora):
    rng = np.random.default_rng(2)
    pl = [rng.integers(0, 256, 30576 // 8, dtype=np.uint8)]
    x, nre = S.pdsch_subframe(100, 3, 1, 4, 1, 0x1234, 30576, 4, 0, pl, scheme="port0", snr_db=25.0, rng=rng,
                              channel=[[1], [0.5 + 0.5j]])
    g, ce, st = PC.fft_estimate(ora, x, 100, 3, 1, 4)
    res = PC.pdsch_decode(ora, g, ce, st["noise"], 100, 3, 1, 4, 1, 0x1234, [30576], [4], [0], scheme="port0")
    assert res[0]["ret"] == 0 and np.array_equal(res[0]["data"][: 30576 // 8], pl[0])


def test_oracle_chain_tm2_diversity(ora):
    rng = np.random.default_rng(4)
    pl = [rng.integers(0, 256, TBS // 8, dtype=np.uint8)]
    x, nre = S.pdsch_subframe(100, 4, 2, 5, 1, 0x1234, TBS, 6, 0, pl, scheme="diversity", snr_db=30.0, rng=rng)
    g, ce, st = PC.fft_estimate(ora, x, 100, 4, 2, 5)
    res = PC.pdsch_decode(ora, g, ce, st["noise"], 100, 4, 2, 5, 1, 0x1234, [TBS], [6], [0], scheme="diversity")
    assert res[0]["ret"] == 0 and np.array_equal(res[0]["data"][: TBS // 8], pl[0])


@pytest.mark.parametrize("tti,cfi,nports,scheme,tbs,Qm", [(1, 1, 2, "cdd", 55056, 6), (10, 2, 2, "cdd", 46888, 6),
                                                          (5, 3, 2, "diversity", 46888, 6), (2, 1, 1, "port0", 30576, 4)])
def test_oracle_chain_extended_cp(ora, tti, cfi, nports, scheme, tbs, Qm):
    """extended cyclic prefix (6 symbols a slot, CRS in l = 0 / 3, N_cp = 0 in the CRS c_init,
    cp = 512 N / 2048): synth -> numpy OFDM -> oracle estimator -> oracle PDSCH decode"""
    rng = np.random.default_rng(tti + 40)
    ncw = 2 if scheme == "cdd" else 1
    pls = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(ncw)]
    ch = [[1], [0.5 + 0.5j]] if nports == 1 else None
    x, nre = S.pdsch_subframe(100, 9, nports, tti, cfi, 0x1234, tbs, Qm, 0, pls, scheme=scheme, codebook=1,
                              snr_db=30.0, rng=rng, channel=ch, cp=1)
    assert x.shape[1] == 2 * (6 * 2048 + 6 * 512)
    g, ce, st = PC.fft_estimate(ora, x, 100, 9, nports, tti, cp=1)
    assert g.shape[1] == 12 * 1200
    res = PC.pdsch_decode(ora, g, ce, st["noise"], 100, 9, nports, tti, cfi, 0x1234, [tbs] * ncw, [Qm] * ncw,
                          [0] * ncw, scheme=scheme, cp=1)
    for q in range(ncw):
        assert res[q]["ret"] == 0
        assert np.array_equal(res[q]["data"][: tbs // 8], pls[q])
    assert res[0]["nof_re"] == nre


@pytest.mark.parametrize("tti,cfi,cp", [(1, 1, 0), (5, 2, 0), (10, 1, 0), (3, 2, 1)])
def test_oracle_chain_tm2_four_ports(ora, tti, cfi, cp):
    """4 tx ports (SFBC + FSTD, 36.211 6.3.4.3; CRS of ports 2 / 3 in l = 1) through a 2 x 4 channel:
    4-port estimator, srsran_predecoding_diversity_csi (4 ports, pinned in test_phy_oracle.py), 4-layer
    demap, DL-SCH with Nl = 2"""
    rng = np.random.default_rng(tti + 60)
    tbs = 36696
    pl = [rng.integers(0, 256, tbs // 8, dtype=np.uint8)]
    x, nre = S.pdsch_subframe(100, 6, 4, tti, cfi, 0x1234, tbs, 6, 0, pl, scheme="diversity4", snr_db=30.0, rng=rng,
                              cp=cp)
    assert nre % 4 == 0
    g, ce, st = PC.fft_estimate(ora, x, 100, 6, 4, tti, cp=cp)
    res = PC.pdsch_decode(ora, g, ce, st["noise"], 100, 6, 4, tti, cfi, 0x1234, [tbs], [6], [0], scheme="diversity",
                          cp=cp)
    assert res[0]["nof_re"] == nre
    assert res[0]["ret"] == 0 and np.array_equal(res[0]["data"][: tbs // 8], pl[0])
