"""The production turbo-decoder launches at BASELINE size, checked block by block against the
reference decoder compiled from /root/reference (oracle/_ref: turbodecoder.c:536-549 driving the
AVX2 16-bit window decoders of turbodecoder_win.h), and the DL-SCH path of sch.c:371-573 with soft
buffers placed far apart in device memory.

  * configs[1]: all 188 LTE code block sizes x 1024 blocks, 8 half-iterations, one
    srsran_tdec_gpu_run_multi call (the bench's timed step): the 16-sub-block class is one fused
    launch of the single-lane decoder, its sizes up to srsran_tdec_gpu_get_w8_fused_max_k on the
    8-step-window build as a second launch (checked as well uncut, and on the lane-pair decoder),
    the 8-sub-block class the single-lane
    tdec8sw8_multi_kernel (8-step windows) and the generic class the quad decoder's fused launch.  Every block equals the reference's output
    for its pool block (the batch tiles a pool of distinct AWGN blocks at several SNRs, so decoded
    words differ from the transmitted ones in some blocks and not in others).
  * configs[0]'s shape on the GPU: K = 6144 x 1024 through srsran_tdec_gpu_run_batch, on each of the
    16-sub-block decoders (the single lane by default at this size, its 8-step-window build, lane pair, quad).
  * DL-SCH transport blocks whose soft buffers lie more than 2 GB apart: the lane-pair decoder runs
    (the descriptor list is padded where a workgroup's two blocks would straddle two far buffers) and
    every TB equals the oracle's decode_tb (return, payload, average iterations, CB CRC flags).
"""
import numpy as np
import pytest

from oracle import CB_SIZES, Oracle, Reference, make_llrs, ref_available

pytestmark = pytest.mark.gpu

POOL_EBNO = (0.0, 0.4, 0.8, 1.2, 2.0, 4.0)  # dB: low ones leave residual errors after 8 half-its


@pytest.fixture(scope="module")
def env():
    import torch
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    if not ref_available():  # on a HIP box the reference checker must be there: fail, never skip
        pytest.fail("oracle/_ref/libsrsref.so missing: the reference decoder was not built")
    return torch, tdec, Reference(), Oracle()


def _pool(ora, K, rng):
    """one AWGN block per POOL_EBNO entry, SB layout"""
    blocks = []
    for eb in POOL_EBNO:
        _, llr = make_llrs(K, eb, rng, 1, ora)
        blocks.append(ora.natural_to_sb(K, llr[0]))
    return np.stack(blocks)


def test_all188_x1024_fused_launch(env):
    torch, tdec, ref, ora = env
    rng = np.random.default_rng(3001)
    batch, iters = 1024, 8
    Ks = list(CB_SIZES)
    ins, outs, want, pools = [], [], {}, {}
    for K in Ks:
        pool = _pool(ora, K, rng)
        pools[K] = pool
        want[K] = np.stack([ref.tdec_run(K, x, True, iters) for x in pool])
        host = np.ascontiguousarray(np.tile(pool, ((batch + len(pool) - 1) // len(pool), 1))[:batch])
        ins.append(torch.from_numpy(host).cuda())
        outs.append(torch.zeros((batch, K // 8), dtype=torch.uint8, device="cuda"))
    k16 = [i for i, K in enumerate(Ks) if tdec.nof_subblocks(K) == 16]
    assert len(k16) == 110

    # the 16-sub-block class alone: the single-lane decoder (the library's choice at 112,640 blocks) as the
    # library cuts it (sizes up to srsran_tdec_gpu_get_w8_fused_max_k on 8-step windows, launched last),
    # uncut (one fused launch), then the lane-pair decoder
    lib = tdec.load_library()
    cut = lib.srsran_tdec_gpu_get_w8_fused_max_k()
    for name, single, fused_cut in (("tdec16sw8_multi_kernel" if cut >= 816 else "tdec16s_multi_kernel", None, cut),
                                    ("tdec16s_multi_kernel", None, 0), ("tdec16_multi_kernel", 1 << 30, cut)):
        with tdec.single_threshold(single if single is not None else lib.srsran_tdec_gpu_get_single_threshold()), \
                tdec.w8_fused_max_k(fused_cut):
            tdec.gpu_run_multi([Ks[i] for i in k16], [ins[i].data_ptr() for i in k16], [ins[i].shape[1] for i in k16],
                               True, [outs[i].data_ptr() for i in k16], [batch] * len(k16), iters, None)
            torch.cuda.synchronize()
            assert tdec.last_kernel() == name
        for i in k16:
            K = Ks[i]
            got = outs[i].cpu().numpy()
            exp = want[K][np.arange(batch) % len(POOL_EBNO)]
            assert np.array_equal(got, exp), f"{name} K={K}: {(got != exp).any(axis=1).sum()} blocks differ"
            outs[i].zero_()

    # all 188 sizes in one call, as the bench's timed step
    tdec.gpu_run_multi(Ks, [t.data_ptr() for t in ins], [t.shape[1] for t in ins], True,
                       [t.data_ptr() for t in outs], [batch] * len(Ks), iters, None)
    torch.cuda.synchronize()
    bad = {}
    for i, K in enumerate(Ks):
        got = outs[i].cpu().numpy()
        exp = want[K][np.arange(batch) % len(POOL_EBNO)]
        n = int((got != exp).any(axis=1).sum())
        if n:
            bad[K] = n
    assert not bad, bad
    # the pool is not trivially decodable: some reference outputs are not the transmitted words,
    # so equality above is a statement about the decoder's arithmetic, not only about success
    assert len({w.tobytes() for K in (6144, 40) for w in want[K]}) == 2 * len(POOL_EBNO)


@pytest.mark.parametrize("kernel", ["tdec16sw8_kernel<false>", "tdec16s_kernel<false>", "tdec16_kernel<false>",
                                    "tdec_kernel<16>"])
def test_k6144_x1024_batch(env, kernel):
    torch, tdec, ref, ora = env
    rng = np.random.default_rng(3002)
    K, batch = 6144, 1024
    pool = _pool(ora, K, rng)
    want = np.stack([ref.tdec_run(K, x, True, 8) for x in pool])
    d_in = torch.from_numpy(np.ascontiguousarray(np.tile(pool, (batch // len(pool) + 1, 1))[:batch])).cuda()
    d_out = torch.zeros((batch, K // 8), dtype=torch.uint8, device="cuda")
    never = 1 << 30
    L = tdec.load_library()
    pair, single, w8 = {"tdec16s_kernel<false>": (None, None, 0),  # the default at this size
                        "tdec16sw8_kernel<false>": (None, None, 6144), "tdec16_kernel<false>": (None, never, 0),
                        "tdec_kernel<16>": (never, never, 0)}[kernel]
    with tdec.pair_threshold(L.srsran_tdec_gpu_get_pair_threshold() if pair is None else pair), \
            tdec.single_threshold(L.srsran_tdec_gpu_get_single_threshold() if single is None else single), \
            tdec.w8_max_k(w8):
        tdec.gpu_run_batch(K, d_in.data_ptr(), d_in.shape[1], True, d_out.data_ptr(), batch, 8, None)
        torch.cuda.synchronize()
    assert tdec.last_kernel() == kernel
    got = d_out.cpu().numpy()
    assert np.array_equal(got, want[np.arange(batch) % len(pool)])


@pytest.mark.parametrize("kernel", ["tdec16_kernel", "tdec16s_kernel", "tdec16sw8_kernel"])
def test_dlsch_far_soft_buffers(env, kernel):
    """soft buffers > 2 GB apart (arena off, 2.4 GB buffers): the lane-pair and the single-lane decoder
    still run (the descriptor list is padded per workgroup) and every TB equals the oracle's decode_tb"""
    torch, tdec, ref, ora = env
    from srsran_4g_amd import sch as S
    rng = np.random.default_rng(3003)
    tbs, Qm, G = 75376, 6, 86400  # C3: 13 code blocks of K = 5824 per TB
    ntb = 4
    q = S.Sch()
    q.set_max_noi(8)
    S.softbuffer_arena(False)
    try:
        # max_cb x (3 * 6176 + 12) int16 each: 64000 blocks = 2.37 GB, so two buffers' bases are > 2 GB apart
        sbs = [S.SoftbufferRx(max_cb=64000, max_cb_size=3 * 6176 + 12) for _ in range(ntb)]
    finally:
        S.softbuffer_arena(True)
    ptrs = sorted(sb.device_ptr for sb in sbs)
    assert min(b - a for a, b in zip(ptrs, ptrs[1:])) >= (1 << 31)
    entries, keep, exp = [], [], []
    for i in range(ntb):
        tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        sigma = (0.3, 0.45, 0.5, 0.55)[i]
        e = ora.dlsch_encode(tbs, Qm, 0, G, tb, 0).astype(np.float32) * 2 - 1
        llr = np.trunc(100 * (e + rng.standard_normal(e.shape).astype(np.float32) * sigma)).astype(np.int16)
        d_e = torch.from_numpy(llr).cuda()
        d_data = torch.zeros(tbs // 8 + 64, dtype=torch.uint8, device="cuda")
        keep += [d_e, d_data]
        entries.append((tbs, Qm, 0, G, d_e.data_ptr(), d_data.data_ptr(), sbs[i], 1))
        exp.append(ora.dlsch_decode(tbs, Qm, 0, llr, 8))
    d_res = torch.full((ntb,), 77, dtype=torch.int32, device="cuda")
    d_avg = torch.zeros(ntb, dtype=torch.float32, device="cuda")
    with tdec.pair_threshold(0), tdec.single_threshold(1 << 30 if kernel == "tdec16_kernel" else 0), \
            tdec.w8_max_k(6144 if "w8" in kernel else 0):
        assert q.decode_batch(entries, d_res.data_ptr(), d_avg.data_ptr()) == 0
        torch.cuda.synchronize()
        assert tdec.last_kernel() == kernel + "<true>"
    res, avg = d_res.cpu().numpy(), d_avg.cpu().numpy()
    C = S.cbsegm(tbs)[1].C
    for i, (oret, odata, _, oavg, st) in enumerate(exp):
        assert res[i] == oret, i
        assert np.array_equal(keep[2 * i + 1].cpu().numpy()[: len(odata)], odata), i
        assert avg[i] == oavg, i
        sbs[i].sync()
        assert sbs[i].cb_crc(C) == [bool(x) for x in st[1][:C]], i
    for sb in sbs:
        sb.free()
    q.free()
