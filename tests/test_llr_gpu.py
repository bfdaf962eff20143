"""GPU parity of the PDSCH LLR stages (soft demapping, descrambling, fused) against the oracle,
which is pinned to the reference's demod_soft.c / sequence.c (tests/test_phy_oracle.py).
Bit-exact int16 comparison, including SSE/scalar splits, ties, saturation and wrap."""
import numpy as np
import pytest
import torch

from oracle import Oracle

from test_phy_oracle import symbols

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ora():
    return Oracle()


@pytest.fixture(scope="module")
def P():
    from srsran_4g_amd import phch
    return phch


@pytest.mark.parametrize("mod,scale", [(0, 100.0), (1, 141.42136), (2, 400.0), (3, 700.0), (4, 1000.0)])
def test_demod(P, ora, mod, scale):
    rng = np.random.default_rng(10 + mod)
    for n in (1, 2, 3, 4, 5, 7, 8, 9, 13, 15, 16, 17, 31, 1200, 14400, 14401, 14403, 30000):
        sym = symbols(rng, n, scale)
        got = P.demod_s(mod, sym)
        exp = ora.demod_s(mod, sym)
        assert np.array_equal(got, exp), (mod, n, np.flatnonzero(got != exp)[:8])


def test_sequence(P, ora):
    rng = np.random.default_rng(20)
    for n in (1, 23, 24, 63, 64, 65, 86400, 172800, 300001):
        llr = rng.integers(-32768, 32768, n, dtype=np.int16)
        llr[: min(n, 3)] = -32768
        for seed in (0, 1, (0x1234 << 14) + 1, 0x7FFFFFFF, 0xFFFFFFFF):
            assert np.array_equal(P.sequence_apply_s(llr, seed), ora.sequence_apply_s(llr, seed)), (n, seed)


def test_sequence_pdsch(P, ora):
    rng = np.random.default_rng(21)
    llr = rng.integers(-2000, 2000, 86400, dtype=np.int16)
    for rnti, q, ns, cell in ((0x1234, 0, 2, 1), (0xFFFF, 1, 19, 503)):
        seed = ora.pdsch_seed(rnti, q, ns, cell)
        assert np.array_equal(P.sequence_pdsch_apply_s(llr, rnti, q, ns, cell), ora.sequence_apply_s(llr, seed))


@pytest.mark.parametrize("mod", [1, 2, 3, 4])
def test_fused_llr_device(P, ora, mod):
    rng = np.random.default_rng(30 + mod)
    for n in (14400, 14401, 7, 100000):
        sym = symbols(rng, n, 700.0)
        seed = int(rng.integers(0, 2**31))
        d_sym = torch.from_numpy(sym.view(np.float32)).cuda()
        d_llr = torch.zeros(n * P.QM[mod], dtype=torch.int16, device="cuda")
        assert P.gpu_llr(mod, d_sym.data_ptr(), n, True, seed, d_llr.data_ptr()) == 0
        torch.cuda.synchronize()
        exp = ora.sequence_apply_s(ora.demod_s(mod, sym), seed)
        assert np.array_equal(d_llr.cpu().numpy(), exp), (mod, n)
