"""The single-lane decoder of the 8-sub-block window class (tdecs_kernel.hip built with TDECS_NSB=8: every K
from 408 to 800, the SSE 8-block window decoder of turbodecoder_win.h) forced onto every batch size
(srsran_tdec_gpu_set_single_threshold(0)) against the oracle decoder: all 32 sizes with partly empty
workgroups, several half-iteration counts, the fused multi-size launch and DL-SCH transport blocks with
CRC early stop over HARQ."""
import numpy as np
import pytest

from oracle import CB_SIZES, Oracle, make_llrs

pytestmark = pytest.mark.gpu

K8 = [k for k in CB_SIZES if 408 <= k <= 800]


@pytest.fixture(scope="module", autouse=True, params=["tdec8s_kernel"])
def kname(request):
    """the single-lane decoder on 16-step windows (the 8-step build, the class's default, is
    tests/test_tdec_w8_gpu.py; the split variant with helper waves was retired in round 4)"""
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    with tdec.single_threshold(0), tdec.w8_max_k(0):
        yield request.param


@pytest.fixture(scope="module")
def ora():
    return Oracle()


def test_all_8class_sizes_bit_exact(ora, kname):
    from srsran_4g_amd import tdec
    assert len(K8) == 32 and all(tdec.nof_subblocks(k) == 8 for k in K8)
    rng = np.random.default_rng(801)
    dec = tdec.TurboDecoder()
    bad = []
    for j, K in enumerate(K8):
        _, llr = make_llrs(K, 1.0, rng, 1 + j % 11, ora)
        sb = np.stack([ora.natural_to_sb(K, x) for x in llr])
        if not np.array_equal(dec.run_all_batch(sb, 8, K), ora.run_batch(K, sb, True, 8)):
            bad.append(K)
        assert tdec.last_kernel() == kname + "<false>"
    dec.free()
    assert not bad, bad


@pytest.mark.parametrize("nit", [1, 2, 3, 16])
def test_half_iteration_counts(ora, nit):
    from srsran_4g_amd import tdec
    rng = np.random.default_rng(810 + nit)
    dec = tdec.TurboDecoder()
    for K in (408, 512, 704, 800):
        _, llr = make_llrs(K, 0.5, rng, 9, ora)
        sb = np.stack([ora.natural_to_sb(K, x) for x in llr])
        assert np.array_equal(dec.run_all_batch(sb, nit, K), ora.run_batch(K, sb, True, nit)), (K, nit)
    dec.free()


def test_multi_size_launch(ora):
    import torch
    from srsran_4g_amd import tdec
    rng = np.random.default_rng(820)
    Ks = [408, 800, 576, 496, 752]
    ins, outs, want = [], [], []
    for i, K in enumerate(Ks):
        n = 3 * i + 1
        _, llr = make_llrs(K, 1.5, rng, n, ora)
        sb = np.stack([ora.natural_to_sb(K, x) for x in llr])
        ins.append(torch.from_numpy(sb).cuda())
        outs.append(torch.zeros((n, K // 8), dtype=torch.uint8, device="cuda"))
        want.append(ora.run_batch(K, sb, True, 8))
    tdec.gpu_run_multi(Ks, [t.data_ptr() for t in ins], [t.shape[1] for t in ins], True,
                       [t.data_ptr() for t in outs], [t.shape[0] for t in ins], 8, None)
    torch.cuda.synchronize()
    assert tdec.last_kernel() == "tdec8s_multi_kernel"
    for K, o, w in zip(Ks, outs, want):
        assert np.array_equal(o.cpu().numpy(), w), K


def test_dlsch_early_stop_harq(ora, kname):
    """single-CB TBs (CRC24A; every TB of an 8-class K is one code block), rv 0 -> 2 -> 3 at low SNR"""
    from srsran_4g_amd import sch, tdec
    rng = np.random.default_rng(830)
    q = sch.Sch()
    for tbs, Qm, G in ((600, 2, 1440), (392, 2, 960), (760, 4, 2000)):
        rc, s = sch.cbsegm(tbs)
        assert all(408 <= k <= 800 for k in (s.K1, s.K2) if k), (tbs, s.K1, s.K2)
        tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        sb = sch.SoftbufferRx(nof_prb=100)
        state = None
        for rv, sigma in ((0, 0.9), (2, 0.9), (3, 0.5)):
            e = ora.dlsch_encode(tbs, Qm, rv, G, tb, 0).astype(np.float32) * 2 - 1
            llr = np.trunc(100 * (e + rng.standard_normal(e.shape).astype(np.float32) * sigma)).astype(np.int16)
            q.set_max_noi(8)
            ret, data, avg = q.decode(sb, tbs, Qm, rv, llr)
            assert tdec.last_kernel() == kname + "<true>"
            oret, odata, _, oavg, state = ora.dlsch_decode(tbs, Qm, rv, llr, 8, state)
            assert ret == oret, (tbs, rv)
            assert np.array_equal(data[: len(odata)], odata), (tbs, rv)
            assert avg == pytest.approx(oavg, abs=0), (tbs, rv)
            assert sb.cb_crc(s.C) == [bool(x) for x in state[1][: s.C]], (tbs, rv)
        sb.free()
    q.free()
