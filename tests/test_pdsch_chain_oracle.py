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
