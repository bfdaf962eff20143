"""The two decoders of the 16-sub-block class on the SB layout, each forced onto small batches: the lane
pair (tdec16_kernel.hip; by itself from 512 blocks a launch), the single lane per sub-block
(tdecs_kernel.hip; by itself from srsran_tdec_gpu_get_single_threshold() blocks) on 16-step windows and on
8-step windows (srsran_tdec_gpu_set_w8_max_k, the build the fused all-size class runs): every K >= 816 of
the bit-exact suites again, plain batches with block counts that leave workgroups partly empty, the
multi-size fused launch, and DL-SCH transport blocks with CRC early stop over HARQ."""
import numpy as np
import pytest

from oracle import CB_SIZES, Oracle, make_llrs

pytestmark = pytest.mark.gpu


NEVER = 1 << 30
KERNELS = {"pair": ("tdec16_kernel", 0, NEVER, None), "single": ("tdec16s_kernel", 0, 0, 0),
           "single_w8": ("tdec16sw8_kernel", 0, 0, 6144)}


@pytest.fixture(scope="module", autouse=True, params=sorted(KERNELS))
def kernel(request):
    """every test three times: the lane-pair decoder (tdec16_kernel.hip), the single-lane decoder
    (tdecs_kernel.hip) on 16-step and on 8-step windows, each forced onto every batch size"""
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    name, pair_min, single_min, w8 = KERNELS[request.param]
    with tdec.pair_threshold(pair_min), tdec.single_threshold(single_min), \
            tdec.w8_max_k(w8 if w8 is not None else tdec.load_library().srsran_tdec_gpu_get_w8_max_k()), \
            tdec.w8_fused_max_k(w8 if w8 else tdec.load_library().srsran_tdec_gpu_get_w8_fused_max_k()):
        yield name


@pytest.fixture(scope="module")
def ora():
    return Oracle()


def test_all_large_sizes_bit_exact(ora, kernel):
    """every K >= 816 (all 110 sizes), 1..7 blocks (partly empty workgroups), 8 half-iterations, SB layout"""
    from srsran_4g_amd import tdec
    rng = np.random.default_rng(1601)
    dec = tdec.TurboDecoder()
    bad = []
    for j, K in enumerate([k for k in CB_SIZES if k >= 816]):
        _, llr = make_llrs(K, 1.5, rng, 1 + j % 7, ora)
        sb = np.stack([ora.natural_to_sb(K, x) for x in llr])
        if not np.array_equal(dec.run_all_batch(sb, 8, K), ora.run_batch(K, sb, True, 8)):
            bad.append(K)
        assert tdec.last_kernel() == kernel + "<false>"
    dec.free()
    assert not bad, bad


@pytest.mark.parametrize("nit", [1, 2, 3, 5, 16])
def test_half_iteration_counts(ora, nit, kernel):
    from srsran_4g_amd import tdec
    rng = np.random.default_rng(1602 + nit)
    dec = tdec.TurboDecoder()
    for K in (816, 1056, 3136, 6144):
        _, llr = make_llrs(K, 0.5, rng, 5, ora)
        sb = np.stack([ora.natural_to_sb(K, x) for x in llr])
        assert np.array_equal(dec.run_all_batch(sb, nit, K), ora.run_batch(K, sb, True, nit)), (K, nit)
    dec.free()


def test_multi_size_launch(ora, kernel):
    """srsran_tdec_gpu_run_multi: several K >= 816 fused into one lane-pair launch"""
    import torch
    from srsran_4g_amd import tdec
    rng = np.random.default_rng(1603)
    Ks = [816, 2048, 4032, 6144, 1504]
    ins, outs, want = [], [], []
    for i, K in enumerate(Ks):
        n = 2 * i + 1
        _, llr = make_llrs(K, 2.0, rng, n, ora)
        sb = np.stack([ora.natural_to_sb(K, x) for x in llr])
        ins.append(torch.from_numpy(sb).cuda())
        outs.append(torch.zeros((n, K // 8), dtype=torch.uint8, device="cuda"))
        want.append(ora.run_batch(K, sb, True, 8))
    with tdec.w8_fused_max_k(0):  # one fused launch (the cut at w8_fused_max_k: test_tdec_fullsize_gpu.py)
        tdec.gpu_run_multi(Ks, [t.data_ptr() for t in ins], [t.shape[1] for t in ins], True,
                           [t.data_ptr() for t in outs], [t.shape[0] for t in ins], 8, None)
        torch.cuda.synchronize()
    assert tdec.last_kernel() == kernel.replace("_kernel", "_multi_kernel")
    for K, o, w in zip(Ks, outs, want):
        assert np.array_equal(o.cpu().numpy(), w), K


def test_dlsch_early_stop_harq(ora, kernel):
    """DL-SCH decode_tb with the pair kernel's CRC early stop: return, payload, average iterations,
    CB flags, over rv 0 -> 2 at low SNR (some blocks pass at rv 0, the rest after combining)"""
    from srsran_4g_amd import sch, tdec
    rng = np.random.default_rng(1604)
    q = sch.Sch()
    for tbs, Qm, G in ((75376, 6, 86400), (36696, 6, 43200), (6200, 2, 14400)):
        tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        sb = sch.SoftbufferRx(nof_prb=100)
        state = None
        for rv, sigma in ((0, 0.95), (2, 0.95), (3, 0.5)):
            e = ora.dlsch_encode(tbs, Qm, rv, G, tb, 0).astype(np.float32) * 2 - 1
            llr = np.trunc(100 * (e + rng.standard_normal(e.shape).astype(np.float32) * sigma)).astype(np.int16)
            q.set_max_noi(8)
            ret, data, avg = q.decode(sb, tbs, Qm, rv, llr)
            assert tdec.last_kernel() == kernel + "<true>"
            oret, odata, _, oavg, state = ora.dlsch_decode(tbs, Qm, rv, llr, 8, state)
            assert ret == oret, (tbs, rv)
            assert np.array_equal(data[: len(odata)], odata), (tbs, rv)
            assert avg == pytest.approx(oavg, abs=0), (tbs, rv)
            rc, s = sch.cbsegm(tbs)
            assert sb.cb_crc(s.C) == [bool(x) for x in state[1][: s.C]], (tbs, rv)
        sb.free()
    q.free()
