"""8-bit LLR turbo decoder (srsran_tdec_run_all_8bit / srsran_tdec_iteration_8bit /
srsran_tdec_gpu_run_batch_8bit) against the reference's own 8-bit decoders.

The checker is oracle/_ref: turbodecoder_win.h built as WINIMP_IS_SSE8 / WINIMP_IS_AVX8 and
turbodecoder_iter.h as LLR_IS_8BIT, driven like tdec_iteration_8 (turbodecoder.c:455-483) in
oracle/ref_harness.c (ref_tdec8_run).  CPU tests pin the numpy restatement oracle/tdec8.py (the schedule
the HIP kernel runs) to it; GPU tests compare the HIP decoder with it bit for bit on every class: the AVX2
8-bit decoder (32 sub-blocks, K > 2048), the SSE 8-bit decoder (16, 800 < K <= 2048) and the 16-bit
decoders the reference falls back on for K <= 800, in both input layouts, over several half-iteration
counts, on AWGN and saturating inputs.
"""
import numpy as np
import pytest

from oracle import CB_SIZES, Oracle, make_llrs
import oracle as O
import tdec8


@pytest.fixture(scope="module")
def ref():
    if not O.ref_available():
        pytest.fail("oracle/_ref/libsrsref.so missing: the reference checker of this module was not built")
    return O.Reference()


def to_sb(K, x):
    """natural 3K+12 -> the sub-block layout of the decoder that takes K (rm_turbo_rx_lut_8bit's layout:
    syst | 32 | parity0 | 32 | parity1 | 32 | tail, slot q = position * nsb + sub-block)."""
    nsb = O.tdec8_subblocks(K)
    Ls = K // nsb
    out = np.zeros(3 * (K + 32) + 12, x.dtype)
    i, d = np.meshgrid(np.arange(Ls), np.arange(nsb), indexing="ij")
    nat = (i + d * Ls).reshape(K)
    for s in range(3):
        out[s * (K + 32):s * (K + 32) + K] = x[3 * nat + s]
    out[3 * (K + 32):] = x[3 * K:3 * K + 12]
    return out


def _llr8(K, rng, layout_sb, ora, kind):
    """int8 code block: AWGN (natural, or permuted to the SB layout) or uniform random over int8."""
    nsb = O.tdec8_subblocks(K)
    n = 3 * (K + 32) + 12 if (layout_sb and nsb) else 3 * K + 12
    if kind == "rand":
        return rng.integers(-128, 128, size=n).astype(np.int8)
    bits, llr16 = make_llrs(K, 1.5, rng, 1, ora)
    llr = np.clip(llr16[0] // 3, -127, 127).astype(np.int16)
    if layout_sb and nsb:
        llr = to_sb(K, llr)
    return llr.astype(np.int8)


def test_subblock_dispatch():
    """srsran_tdec_autoimp_get_subblocks_8bit of an AVX2 build (turbodecoder.c:410-424)."""
    got = [O.tdec8_subblocks(K) for K in CB_SIZES]
    assert (got.count(32), got.count(16), got.count(8), got.count(0)) == (64, 46, 32, 46)
    from srsran_4g_amd import tdec
    lib = tdec.load_library()
    assert [lib.srsran_tdec_autoimp_get_subblocks_8bit(K) for K in CB_SIZES] == got


@pytest.mark.parametrize("K", [832, 2112])
@pytest.mark.parametrize("layout_sb", [False, True])
def test_restatement_matches_reference(ref, K, layout_sb):
    ora = Oracle()
    rng = np.random.default_rng(K + layout_sb)
    nsb = O.tdec8_subblocks(K)
    fwd, _ = ref.interleaver(K, nsb)
    for kind in ("awgn", "rand"):
        llr = _llr8(K, rng, layout_sb, ora, kind)
        for it in (1, 2, 3):
            assert np.array_equal(tdec8.run_all(K, llr, it, nsb, fwd, layout_sb), ref.tdec8_run(K, llr, layout_sb, it))


@pytest.mark.parametrize("K", [832, 2048, 2112, 6144])
def test_c_restatement_matches_reference_trace(ref, K):
    """oracle_tdec8_run (the C form of tdec8.py the 8-bit DL-SCH oracle runs) against the reference's decoders:
    decisions and the latest output after every half-iteration, AWGN and uniformly random int8 input."""
    ora = Oracle()
    rng = np.random.default_rng(K + 3)
    for kind in ("awgn", "rand"):
        llr = _llr8(K, rng, True, ora, kind)
        out, tr = ora.tdec8_run(K, llr, 7, trace=True)
        rout, rtr = ref.tdec8_run(K, llr, True, 7, trace=True)
        assert np.array_equal(out, rout) and np.array_equal(tr, rtr), kind


def test_reference_decodes_noise_free(ref):
    """The checker itself decodes: a noise-free encoded block comes back exactly (both 8-bit classes)."""
    ora = Oracle()
    rng = np.random.default_rng(7)
    for K in (1024, 6144):
        bits = rng.integers(0, 2, K, dtype=np.uint8)
        llr = ((ora.encode(K, bits).astype(np.int16) * 2 - 1) * 20).astype(np.int8)
        assert np.array_equal(ref.tdec8_run(K, llr, False, 4), np.packbits(bits))


# ---------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def decs():
    from srsran_4g_amd import tdec
    d_sb, d_nat = tdec.TurboDecoder(), tdec.TurboDecoder()
    d_nat.force_not_sb()
    yield d_sb, d_nat
    d_sb.free()
    d_nat.free()


GPU_SIZES = [40, 400, 408, 800, 816, 1024, 2048, 2112, 3072, 4096, 6144]


@pytest.mark.gpu
@pytest.mark.parametrize("layout_sb", [False, True])
def test_run_all_8bit_matches_reference(ref, decs, layout_sb):
    ora = Oracle()
    rng = np.random.default_rng(80 + layout_sb)
    d = decs[0] if layout_sb else decs[1]
    bad = []
    for K in GPU_SIZES:
        for kind in ("awgn", "rand"):
            llr = _llr8(K, rng, layout_sb, ora, kind)
            for it in (1, 2, 5, 8):
                got = d.run_all_8bit(llr, it, K)
                want = ref.tdec8_run(K, llr, layout_sb, it)
                if not np.array_equal(got, want):
                    bad.append((K, kind, it, int(np.count_nonzero(got != want))))
    assert not bad, bad


@pytest.mark.gpu
def test_all_8bit_sizes_sb(ref, decs):
    """Every K of the two 8-bit classes once (SB layout, AWGN, 6 half-iterations)."""
    ora = Oracle()
    rng = np.random.default_rng(81)
    bad = []
    for K in CB_SIZES:
        if O.tdec8_subblocks(K) < 16:
            continue
        llr = _llr8(K, rng, True, ora, "awgn")
        if not np.array_equal(decs[0].run_all_8bit(llr, 6, K), ref.tdec8_run(K, llr, True, 6)):
            bad.append(K)
    assert not bad, bad


@pytest.mark.gpu
def test_iteration_8bit_matches_reference_trace(ref, decs):
    """srsran_tdec_iteration_8bit: the decision after every half-iteration equals the reference's."""
    ora = Oracle()
    rng = np.random.default_rng(82)
    d = decs[0]
    for K in (1056, 5120):
        llr = _llr8(K, rng, True, ora, "awgn")
        _, trace = ref.tdec8_run(K, llr, True, 6, trace=True)
        assert d.new_cb(K) == 0
        for n in range(6):
            got = d.iteration_8bit(llr)
            assert np.array_equal(got, np.packbits((trace[n] > 0).astype(np.uint8))), (K, n)
        assert d.get_nof_iterations() == 6


@pytest.mark.gpu
@pytest.mark.parametrize("K,n", [(6144, 1024), (1024, 37), (512, 9)])
def test_gpu_run_batch_8bit(ref, K, n):
    """Device-resident batch (C1 shape for K = 6144) in the SB layout, every block against the reference."""
    torch = pytest.importorskip("torch")
    from srsran_4g_amd import tdec
    ora = Oracle()
    rng = np.random.default_rng(83 + K)
    nsb = O.tdec8_subblocks(K)
    L = 3 * (K + 32) + 12 if nsb else 3 * K + 12
    stride = L + 20
    llr = np.zeros((n, stride), np.int8)
    _, llr16 = make_llrs(K, 1.0, rng, min(n, 64), ora)
    for i in range(n):
        x = np.clip(llr16[i % len(llr16)] // 3, -127, 127).astype(np.int16)
        if i % 3 == 2:
            x = rng.integers(-128, 128, 3 * K + 12).astype(np.int16)
        llr[i, :L] = (to_sb(K, x) if nsb else x).astype(np.int8)
    d_in = torch.from_numpy(llr).cuda()
    d_out = torch.zeros((n, K // 8), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    tdec.gpu_run_batch_8bit(K, d_in.data_ptr(), stride, True, d_out.data_ptr(), n, 8, stream)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    checks = range(n) if n <= 64 else list(range(0, n, 17)) + [n - 1]
    for i in checks:
        assert np.array_equal(got[i], ref.tdec8_run(K, llr[i, :L], True, 8)), i
    if nsb >= 16:
        assert tdec.last_kernel() == f"tdec8bit_kernel<{nsb}>"


@pytest.mark.gpu
def test_rm_turbo_rx_lut_8bit_matches_reference(ref):
    """srsran_rm_turbo_rx_lut_8bit (rm_turbo.c:447-483, SSE 8-bit path): accumulate with int8 wrap-around on
    the 8-bit decoder's sub-block layout (32 / 16 / 8 sub-blocks, natural below K = 408), every rv, E below
    and above 3K + 12 (wrapped reads), onto a non-zero soft buffer."""
    import ctypes
    from srsran_4g_amd import tdec
    i8p = ctypes.POINTER(ctypes.c_int8)
    mine = tdec.load_library().srsran_rm_turbo_rx_lut_8bit
    theirs = ref.lib.srsran_rm_turbo_rx_lut_8bit
    for f in (mine, theirs):
        f.argtypes = [i8p, i8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        f.restype = ctypes.c_int
    ref.lib.srsran_rm_turbo_gentables()
    rng = np.random.default_rng(84)
    bad = []
    for K in (40, 400, 512, 800, 1024, 2048, 2112, 6144):
        idx = CB_SIZES.index(K)
        nsb = O.tdec8_subblocks(K)
        n = 3 * (K + 32) + 12 if nsb else 3 * K + 12
        for rv in range(4):
            for E in (3 * K // 2 + 7, 5 * (3 * K + 12) // 2):
                e = rng.integers(-128, 128, E).astype(np.int8)
                base = rng.integers(-128, 128, n).astype(np.int8)
                a, b = base.copy(), base.copy()
                assert mine(e.ctypes.data_as(i8p), a.ctypes.data_as(i8p), E, idx, rv) == 0
                assert theirs(e.ctypes.data_as(i8p), b.ctypes.data_as(i8p), E, idx, rv) == 0
                if not np.array_equal(a, b):
                    bad.append((K, rv, E, int(np.count_nonzero(a != b))))
    assert not bad, bad
