"""GPU parity of MIMO predecoding (MMSE with CSI) and the PDSCH CSI correction.

The GPU kernel computes the reference's scalar MMSE formulas in IEEE float without
contraction, so it must equal the oracle (oracle/phy_oracle.c) bit for bit; the oracle
itself is pinned to the reference's precoding.c within the rcp_ps tolerance
(tests/test_phy_oracle.py).  The CSI correction is compared bit-exactly with the
oracle's restatement of pdsch.c:523-618 (SSE semantics)."""
import numpy as np
import pytest
import torch

from oracle import Oracle

from test_phy_oracle import PRE_CASES, channel, symbols

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ora():
    return Oracle()


@pytest.fixture(scope="module")
def P():
    from srsran_4g_amd import phch
    return phch


@pytest.mark.parametrize("scheme,nrx,nports,nlayers,cb", PRE_CASES + [(0, 4, 1, 1, 0)])
def test_predecode_host_api(P, ora, scheme, nrx, nports, nlayers, cb):
    rng = np.random.default_rng(100 + scheme * 10 + nrx + cb)
    for n in (14400, 1201, 7, 1):
        y, h = channel(rng, nports, nrx, n)
        for scaling, noise in ((1.0, 0.01), (0.6, 0.5), (1.0, 0.0)):
            xg, cg = P.predecode(scheme, y, h, nlayers, cb, scaling, noise)
            xo, co = ora.predecode(scheme, y, h, nlayers, cb, scaling, noise)
            assert np.array_equal(xg.view(np.uint32), xo.view(np.uint32)), (n, scaling)
            assert np.array_equal(cg.view(np.uint32), co.view(np.uint32)), (n, scaling)


def test_predecode_device_csi_max(P, ora):
    rng = np.random.default_rng(5)
    n = 14400
    y, h = channel(rng, 2, 2, n)
    dy = [torch.from_numpy(y[r].view(np.float32)).cuda() for r in range(2)]
    dh = [[torch.from_numpy(h[p, r].view(np.float32)).cuda() for r in range(2)] for p in range(2)]
    dx = [torch.zeros(2 * n, dtype=torch.float32, device="cuda") for _ in range(2)]
    dc = [torch.zeros(n, dtype=torch.float32, device="cuda") for _ in range(2)]
    dm = torch.zeros(2, dtype=torch.float32, device="cuda")
    rc = P.predecode_gpu(3, [t.data_ptr() for t in dy], [[t.data_ptr() for t in row] for row in dh],
                         [t.data_ptr() for t in dx], [t.data_ptr() for t in dc], dm.data_ptr(), 2, 2, 2, 0, n, 1.0, 0.05)
    assert rc == 0
    torch.cuda.synchronize()
    xo, co = ora.predecode(3, y, h, 2, 0, 1.0, 0.05)
    for l in range(2):
        assert np.array_equal(dx[l].cpu().numpy().view(np.complex64), xo[l])
        assert np.array_equal(dc[l].cpu().numpy(), co[l])
        assert dm[l].item() == co[l].max()


@pytest.mark.parametrize("mod", [0, 1, 2, 3, 4])
def test_llr_with_csi_correction(P, ora, mod):
    """demap -> descramble -> csi_correction, fused on the GPU, vs the oracle chain."""
    rng = np.random.default_rng(40 + mod)
    for n in (14400, 14401, 14403, 9):
        sym = symbols(rng, n, 300.0)
        csi = rng.uniform(0.05, 3.0, n).astype(np.float32)
        seed = int(rng.integers(0, 2**31))
        d_sym = torch.from_numpy(sym.view(np.float32)).cuda()
        d_csi = torch.from_numpy(csi).cuda()
        d_max = torch.tensor([csi.max()], dtype=torch.float32, device="cuda")
        d_llr = torch.zeros(n * P.QM[mod], dtype=torch.int16, device="cuda")
        assert P.gpu_llr(mod, d_sym.data_ptr(), n, True, seed, d_llr.data_ptr(), None, d_csi.data_ptr(),
                         d_max.data_ptr()) == 0
        torch.cuda.synchronize()
        e = ora.sequence_apply_s(ora.demod_s(mod, sym), seed)
        exp = ora.csi_correction(mod, csi, e)
        got = d_llr.cpu().numpy()
        assert np.array_equal(got, exp), (mod, n, np.flatnonzero(got != exp)[:8])
