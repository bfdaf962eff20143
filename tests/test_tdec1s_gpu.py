"""The single-lane decoder of the generic class (tdec1s_kernel.hip: the 46 sizes K = 40 .. 400, the decoder of
turbodecoder_gen.c with wrap-around arithmetic on the natural input layout) forced onto every batch size
(srsran_tdec_gpu_set_generic_single_threshold(0); by default the quad decoder keeps this class) against the oracle decoder: all 46 sizes with batches that fill
a 64-block workgroup partly, exactly and over several workgroups, several half-iteration counts, extreme
inputs (the int16 wrap matters), the fused multi-size launch and DL-SCH transport blocks (one code block,
CRC24A) with CRC early stop over HARQ."""
import numpy as np
import pytest

from oracle import CB_SIZES, Oracle, make_llrs

pytestmark = pytest.mark.gpu

K1 = [k for k in CB_SIZES if k <= 400]


@pytest.fixture(scope="module", autouse=True)
def single():
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    with tdec.generic_single_threshold(0):
        yield


@pytest.fixture(scope="module")
def ora():
    return Oracle()


def test_all_generic_sizes_bit_exact(ora):
    from srsran_4g_amd import tdec
    assert len(K1) == 46 and all(tdec.nof_subblocks(k) in (0, 1) for k in K1)
    rng = np.random.default_rng(101)
    dec = tdec.TurboDecoder()
    bad = []
    for j, K in enumerate(K1):
        n = (1, 7, 63, 64, 65, 130)[j % 6]
        _, llr = make_llrs(K, 0.8, rng, n, ora)
        if not np.array_equal(dec.run_all_batch(llr, 8, K), ora.run_batch(K, llr, False, 8)):
            bad.append(K)
        assert tdec.last_kernel() == "tdec1s_kernel<false>"
    dec.free()
    assert not bad, bad


@pytest.mark.parametrize("nit", [1, 2, 3, 5, 16])
def test_half_iteration_counts(ora, nit):
    from srsran_4g_amd import tdec
    rng = np.random.default_rng(110 + nit)
    dec = tdec.TurboDecoder()
    for K in (40, 48, 104, 256, 400):
        _, llr = make_llrs(K, 0.3, rng, 33, ora)
        assert np.array_equal(dec.run_all_batch(llr, nit, K), ora.run_batch(K, llr, False, nit)), (K, nit)
    dec.free()


@pytest.mark.parametrize("K", [40, 208, 400])
def test_extreme_inputs(ora, K):
    """saturated, alternating and all-zero LLRs: the generic decoder's int16 wrap-around on every path"""
    from srsran_4g_amd import tdec
    rng = np.random.default_rng(K)
    n = 3 * K + 12
    llr = np.stack([np.full(n, 32767, np.int16), np.full(n, -32768, np.int16), np.zeros(n, np.int16),
                    np.where(np.arange(n) % 2, 32767, -32768).astype(np.int16),
                    rng.integers(-32768, 32767, n).astype(np.int16)])
    dec = tdec.TurboDecoder()
    assert np.array_equal(dec.run_all_batch(llr, 8, K), ora.run_batch(K, llr, False, 8))
    dec.free()


def test_multi_size_launch(ora):
    import torch
    from srsran_4g_amd import tdec
    rng = np.random.default_rng(120)
    Ks = [40, 400, 96, 328, 136]
    ins, outs, want = [], [], []
    for i, K in enumerate(Ks):
        n = 31 * i + 5
        _, llr = make_llrs(K, 1.0, rng, n, ora)
        ins.append(torch.from_numpy(llr).cuda())
        outs.append(torch.zeros((n, K // 8), dtype=torch.uint8, device="cuda"))
        want.append(ora.run_batch(K, llr, False, 8))
    tdec.gpu_run_multi(Ks, [t.data_ptr() for t in ins], [t.shape[1] for t in ins], True,
                       [t.data_ptr() for t in outs], [t.shape[0] for t in ins], 8, None)
    torch.cuda.synchronize()
    assert tdec.last_kernel() == "tdec1s_multi_kernel"
    for K, o, w in zip(Ks, outs, want):
        assert np.array_equal(o.cpu().numpy(), w), K


def test_dlsch_early_stop_harq(ora):
    """single-CB TBs of generic K (CRC24A over the TB), rv 0 -> 2 -> 3 at low SNR"""
    from srsran_4g_amd import sch, tdec
    rng = np.random.default_rng(130)
    q = sch.Sch()
    for tbs, Qm, G in ((16, 2, 120), (120, 2, 360), (376, 4, 1000), (208, 6, 540)):
        rc, s = sch.cbsegm(tbs)
        assert s.C == 1 and s.K1 <= 400, (tbs, s.K1)
        tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        sb = sch.SoftbufferRx(nof_prb=100)
        state = None
        for rv, sigma in ((0, 0.9), (2, 0.9), (3, 0.4)):
            e = ora.dlsch_encode(tbs, Qm, rv, G, tb, 0).astype(np.float32) * 2 - 1
            llr = np.trunc(100 * (e + rng.standard_normal(e.shape).astype(np.float32) * sigma)).astype(np.int16)
            q.set_max_noi(8)
            ret, data, avg = q.decode(sb, tbs, Qm, rv, llr)
            assert tdec.last_kernel() == "tdec1s_kernel<true>"
            oret, odata, _, oavg, state = ora.dlsch_decode(tbs, Qm, rv, llr, 8, state)
            assert ret == oret, (tbs, rv)
            assert np.array_equal(data[: len(odata)], odata), (tbs, rv)
            assert avg == pytest.approx(oavg, abs=0), (tbs, rv)
            assert sb.cb_crc(1) == [bool(state[1][0])], (tbs, rv)
        sb.free()
    q.free()
