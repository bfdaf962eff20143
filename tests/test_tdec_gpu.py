"""GPU parity tests: HIP turbo decoder (through the C-ABI) vs the CPU oracle.

Modelled on the reference's turbodecoder_test.c (AWGN code blocks, srsran_tdec_run_all)
but with an actual check: hard-decision bytes must be identical to the oracle
(pinned bit-exact to the reference decoder, see tests/test_oracle.py) for every one
of the 188 code-block sizes, both input layouts, several half-iteration counts and
saturating / degenerate inputs.  Integer work => the bar is bit-exact.
"""
import ctypes

import numpy as np
import pytest

from oracle import CB_SIZES, Oracle, make_llrs
from srsran_4g_amd import tdec

pytestmark = pytest.mark.gpu


def decisions(llr_rows):
    """Hard decisions (turbodecoder_gen.c:260-277) of trace rows -> bytes."""
    bits = (np.asarray(llr_rows) > 0).astype(np.uint8)
    return np.packbits(bits, axis=-1)


@pytest.fixture(scope="module")
def ora():
    return Oracle()


@pytest.fixture(scope="module")
def dec():
    d = tdec.TurboDecoder()
    yield d
    d.free()


@pytest.fixture(scope="module")
def dec_nat():
    d = tdec.TurboDecoder()
    d.force_not_sb()
    yield d
    d.free()


def _inputs(ora, K, rng, n, layout_sb):
    _, llr = make_llrs(K, 0.5, rng, n, ora)
    llr[n // 2:] = rng.integers(-32768, 32768, size=(n - n // 2, 3 * K + 12), dtype=np.int16)
    if layout_sb:
        llr = np.stack([ora.natural_to_sb(K, x) for x in llr])
    return llr


@pytest.mark.parametrize("layout_sb", [False, True])
def test_all_188_sizes(ora, dec, dec_nat, layout_sb):
    rng = np.random.default_rng(100 + layout_sb)
    d = dec if layout_sb else dec_nat
    bad = []
    for K in CB_SIZES:
        llr = _inputs(ora, K, rng, 4, layout_sb)
        got = d.run_all_batch(llr, 8, K)
        want = ora.run_batch(K, llr, layout_sb, 8)
        if not np.array_equal(got, want):
            bad.append(K)
    assert not bad, f"mismatching K: {bad}"


@pytest.mark.parametrize("K", [40, 400, 408, 800, 816, 1504, 6144])
@pytest.mark.parametrize("nit", [1, 2, 3, 4, 5, 16])
def test_half_iteration_counts(ora, dec, K, nit):
    rng = np.random.default_rng(K * 31 + nit)
    llr = _inputs(ora, K, rng, 6, True)
    got = dec.run_all_batch(llr, nit, K)
    want = ora.run_batch(K, llr, True, nit)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("K", [40, 256, 416, 688, 1024, 6144])
def test_iteration_api_per_half_iteration(ora, dec, K):
    """srsran_tdec_iteration: the decision after every half-iteration (sch.c:426-456 usage)."""
    rng = np.random.default_rng(K)
    llr = _inputs(ora, K, rng, 2, True)
    for x in llr:
        _, trace = ora.tdec_run(K, x, True, 10, trace=True)
        want = decisions(trace)
        assert dec.new_cb(K) == 0
        for n in range(10):
            got = dec.iteration(x)
            assert np.array_equal(got, want[n]), f"K={K} half-iteration {n}"
        assert dec.get_nof_iterations() == 10


def test_run_all_single(ora, dec_nat):
    rng = np.random.default_rng(5)
    for K in (40, 6144, 2112):
        _, llr = make_llrs(K, 1.0, rng, 1, ora)
        got = dec_nat.run_all(llr[0], 8, K)
        assert np.array_equal(got, ora.tdec_run(K, llr[0], False, 8))
        assert dec_nat.get_nof_iterations() == 8


@pytest.mark.parametrize("K", [40, 512, 6144])
def test_degenerate_inputs(ora, dec, K):
    """All-zero, all-max, all-min and alternating extremes (saturation / wrap paths)."""
    n = tdec.input_len(K, True)
    rows = [np.zeros(n, np.int16), np.full(n, 32767, np.int16), np.full(n, -32768, np.int16),
            np.where(np.arange(n) % 2 == 0, 32767, -32768).astype(np.int16)]
    llr = np.stack(rows)
    got = dec.run_all_batch(llr, 8, K)
    want = ora.run_batch(K, llr, True, 8)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("ncb", [1, 3, 17, 63])
def test_ragged_batches(ora, dec, ncb):
    """Batch sizes that leave partially filled waves (16 CBs/wave generic, 2/wave K<=800)."""
    rng = np.random.default_rng(ncb)
    for K in (40, 528, 1088):
        llr = _inputs(ora, K, rng, ncb, True) if ncb > 1 else _inputs(ora, K, rng, 2, True)[:1]
        got = dec.run_all_batch(llr, 6, K)
        assert np.array_equal(got, ora.run_batch(K, llr, True, 6))


def test_empty_batch(dec):
    llr = np.zeros((0, tdec.input_len(6144, True)), np.int16)
    assert dec.run_all_batch(llr, 8, 6144).shape == (0, 768)


def test_invalid_sizes(dec):
    assert dec.new_cb(41) != 0
    assert dec.new_cb(6145) != 0


def test_gpu_run_multi_mixed_sizes(ora):
    """srsran_tdec_gpu_run_multi: several sizes decoded concurrently, joined into one stream."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(77)
    Ks = [40, 400, 408, 800, 816, 5824, 6144, 1056]
    ncbs = [17, 5, 3, 64, 9, 13, 2, 33]
    ins, outs, want = [], [], []
    for K, n in zip(Ks, ncbs):
        llr = _inputs(ora, K, rng, n, True)
        ins.append(torch.from_numpy(llr).cuda())
        outs.append(torch.zeros((n, K // 8), dtype=torch.uint8, device="cuda"))
        want.append(ora.run_batch(K, llr, True, 8))
    stream = torch.cuda.current_stream().cuda_stream
    tdec.gpu_run_multi(Ks, [t.data_ptr() for t in ins], [t.shape[1] for t in ins], True,
                       [t.data_ptr() for t in outs], ncbs, 8, stream)
    torch.cuda.current_stream().synchronize()
    for K, o, w in zip(Ks, outs, want):
        assert np.array_equal(o.cpu().numpy(), w), K


def test_config1_full_batch(ora):
    """BASELINE config 1/2 shape: K=6144 x 1024 CBs, 8 half-iterations, AWGN, device-resident."""
    torch = pytest.importorskip("torch")
    K, n = 6144, 1024
    rng = np.random.default_rng(2024)
    _, llr = make_llrs(K, 1.0, rng, n, ora)
    sb = np.stack([ora.natural_to_sb(K, x) for x in llr])
    d_in = torch.from_numpy(sb).cuda()
    d_out = torch.zeros((n, K // 8), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    tdec.gpu_run_batch(K, d_in.data_ptr(), sb.shape[1], True, d_out.data_ptr(), n, 8, stream)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    want = ora.run_batch(K, sb, True, 8)
    assert np.array_equal(got, want)
