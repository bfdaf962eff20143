"""GPU NR LDPC decoder parity through the C-ABI (srsran_ldpc_decoder_*), against the oracle
restatement (itself pinned against the reference decoder, tests/test_ldpc_oracle.py) and the
reference's golden examples.  Bit-exact: message bits and return values (iterations / CRC)."""
import numpy as np
import pytest

from ldpc import CRC16, CRC24A, CRC24B, LIFT_SIZES, SCALE_C, SCALE_SIMD, OracleLdpc, lift, load_examples, noisy_llrs
from oracle import Oracle
from srsran_4g_amd import ldpc as G
from srsran_4g_amd import tdec

pytestmark = pytest.mark.gpu

MODES = {G.DEC_C: SCALE_C, G.DEC_C_AVX2: SCALE_SIMD, G.DEC_C_AVX512: SCALE_SIMD}


@pytest.fixture(scope="module")
def ora():
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    return OracleLdpc()


def with_crc(rng, K, poly, order):
    m = rng.integers(0, 2, K).astype(np.uint8)
    c = Oracle().crc_bits(poly, order, m[:K - order])
    m[K - order:] = [(c >> (order - 1 - i)) & 1 for i in range(order)]
    return m


@pytest.mark.parametrize("bg", [0, 1])
def test_golden_examples(ora, bg):
    """ldpc_dec_avx2_test.c: symbols +-2 (filler +2), scaling 1, message bits recovered."""
    ex = load_examples()
    for ls in LIFT_SIZES:
        msg, cw = ex[(bg, ls)]
        dec = G.LdpcDecoder(bg, ls, G.DEC_C_AVX2, scaling=1.0)
        for m, c in zip(msg, cw):
            r, out = dec.decode_c(np.where(c == 1, -2, 2).astype(np.int8))
            assert r == 10 and np.all((m == 254) | (out == m)), (bg, ls)
        dec.free()


@pytest.mark.parametrize("bg", [0, 1])
@pytest.mark.parametrize("dtype", [G.DEC_C, G.DEC_C_AVX2])
def test_all_lifting_sizes_vs_oracle(ora, bg, dtype):
    rng = np.random.default_rng(100 + bg + dtype)
    for ls in LIFT_SIZES:
        K, N, n = lift(bg, ls)
        dec = G.LdpcDecoder(bg, ls, dtype, scaling=0.8, max_nof_iter=6)
        full = ora.encode(bg, ls, rng.integers(0, 2, K).astype(np.uint8))[2 * ls:]
        for snr, L in ((0.5, int(rng.integers((K // ls + 2) * ls - ls // 2, n + 1))), (2.0, n)):
            llr = noisy_llrs(full, rng, snr_db=snr, amp=6)
            got = dec.decode_c(llr, length=L)
            want = ora.decode_c(bg, ls, llr, scaling=0.8, max_iter=6, length=L, scale_mode=MODES[dtype])
            assert got[0] == want[0] and np.array_equal(got[1], want[1]), (ls, snr, L)
        dec.free()


def test_saturating_inputs(ora):
    rng = np.random.default_rng(7)
    for bg, ls in ((0, 384), (0, 20), (1, 52), (1, 3), (0, 2)):
        K, N, n = lift(bg, ls)
        llr = rng.integers(-128, 128, n).astype(np.int8)
        for dtype in (G.DEC_C, G.DEC_C_AVX512):
            for s in (0.8, 1.0, 0.55):
                dec = G.LdpcDecoder(bg, ls, dtype, scaling=s, max_nof_iter=3)
                got = dec.decode_c(llr)
                want = ora.decode_c(bg, ls, llr, scaling=s, max_iter=3, scale_mode=MODES[dtype])
                assert got[0] == want[0] and np.array_equal(got[1], want[1]), (bg, ls, dtype, s)
                dec.free()


def test_crc_early_stop(ora):
    rng = np.random.default_rng(3)
    for bg, ls in ((0, 384), (0, 36), (1, 208), (1, 15), (0, 7)):
        K, N, n = lift(bg, ls)
        dec = G.LdpcDecoder(bg, ls, G.DEC_C_AVX2, max_nof_iter=8)
        for poly, order in ((CRC24B, 24), (CRC24A, 24), (CRC16, 16)):
            m = with_crc(rng, K, poly, order)
            full = ora.encode(bg, ls, m)[2 * ls:]
            for snr in (-0.5, 1.5, 4.0):
                llr = noisy_llrs(full, rng, snr_db=snr, amp=5)
                got = dec.decode_c(llr, crc=(poly, order))
                want = ora.decode_c(bg, ls, llr, max_iter=8, crc=(poly, order))
                assert got[0] == want[0] and np.array_equal(got[1], want[1]), (bg, ls, poly, snr)
        dec.free()


@pytest.mark.parametrize("bg,ls,ncw", [(0, 384, 40), (1, 384, 33), (0, 104, 21), (1, 15, 70), (0, 2, 300),
                                       (1, 36, 17)])
def test_batch_vs_oracle(ora, bg, ls, ncw):
    """Batch entry point: several codewords per workgroup, strides, CRC stop, packed output, d_ret."""
    import torch

    rng = np.random.default_rng(ls * 7 + bg)
    K, N, n = lift(bg, ls)
    stride = n + 5
    llrs = np.zeros((ncw, stride), np.int8)
    crc = (CRC24B, 24)
    for i in range(ncw):
        m = with_crc(rng, K, *crc)
        full = ora.encode(bg, ls, m)[2 * ls:]
        llrs[i, :n] = noisy_llrs(full, rng, snr_db=float(rng.uniform(-1.0, 3.0)), amp=5)
    dec = G.LdpcDecoder(bg, ls, G.DEC_C_AVX2, max_nof_iter=8)
    d_in = torch.from_numpy(llrs).cuda()
    for use_crc in (False, True):
        d_out = torch.zeros((ncw, K + 3), dtype=torch.uint8, device="cuda")
        d_ret = torch.full((ncw,), 255, dtype=torch.uint8, device="cuda")
        assert dec.gpu_decode_batch(d_in.data_ptr(), stride, ncw, d_out.data_ptr(), K + 3,
                                    crc=crc if use_crc else None, d_ret=d_ret.data_ptr()) == 0
        torch.cuda.synchronize()
        out, ret = d_out.cpu().numpy(), d_ret.cpu().numpy()
        for i in range(ncw):
            want = ora.decode_c(bg, ls, llrs[i, :n], max_iter=8, crc=crc if use_crc else None)
            assert ret[i] == want[0] and np.array_equal(out[i, :K], want[1]), (i, use_crc)
        if K % 8 == 0:
            d_pk = torch.zeros((ncw, K // 8), dtype=torch.uint8, device="cuda")
            assert dec.gpu_decode_batch(d_in.data_ptr(), stride, ncw, d_pk.data_ptr(), K // 8,
                                        crc=crc if use_crc else None, packed=True) == 0
            torch.cuda.synchronize()
            assert np.array_equal(np.unpackbits(d_pk.cpu().numpy(), axis=1), out[:, :K])
    dec.free()


def test_compact_pcm_matches_oracle(ora):
    for bg in (0, 1):
        for ls in LIFT_SIZES:
            p, q = G.compact_pcm(bg, ls)
            p0, q0 = ora.pcm(bg, ls)
            assert np.array_equal(p, p0) and np.array_equal(q, q0)


def test_16bit_decoder_vs_oracle(ora):
    """SRSRAN_LDPC_DECODER_S (ldpc_dec_s.c): int16 LLRs, 15-bit messages, decode_s and the batch."""
    import torch

    rng = np.random.default_rng(16)
    for bg in (0, 1):
        for ls in LIFT_SIZES[::3] + [384]:
            K, N, n = lift(bg, ls)
            dec = G.LdpcDecoder(bg, ls, G.DEC_S, scaling=0.75, max_nof_iter=5)
            full = ora.encode(bg, ls, rng.integers(0, 2, K).astype(np.uint8))[2 * ls:]
            for snr, amp in ((0.5, 900.0), (2.0, 20000.0)):  # the second saturates (INT16 infinity)
                llr = noisy_llrs(full, rng, snr_db=snr, amp=amp, dtype=np.int16, clip=32767)
                llr[rng.integers(0, n, 8)] = -32768
                L = int(rng.integers((K // ls + 2) * ls - ls // 2, n + 1)) if snr < 1 else n
                got = dec.decode_s(llr, length=L)
                want = ora.decode_s(bg, ls, llr, scaling=0.75, max_iter=5, length=L)
                assert got[0] == want[0] and np.array_equal(got[1], want[1]), (bg, ls, snr)
            assert dec.decode_c(np.zeros(n, np.int8))[0] == -1  # 8-bit call on a 16-bit decoder
            dec.free()
        # batch
        ls, ncw = 208, 9
        K, N, n = lift(bg, ls)
        dec = G.LdpcDecoder(bg, ls, G.DEC_S, scaling=0.8, max_nof_iter=6)
        llrs = np.stack([noisy_llrs(ora.encode(bg, ls, rng.integers(0, 2, K).astype(np.uint8))[2 * ls:], rng,
                                    snr_db=1.0, amp=700.0, dtype=np.int16, clip=32767) for _ in range(ncw)])
        d_in = torch.from_numpy(llrs).cuda()
        d_out = torch.zeros((ncw, K), dtype=torch.uint8, device="cuda")
        assert dec.gpu_decode_batch(d_in.data_ptr(), n, ncw, d_out.data_ptr(), K) == 0
        torch.cuda.synchronize()
        out = d_out.cpu().numpy()
        for i in range(ncw):
            assert np.array_equal(out[i], ora.decode_s(bg, ls, llrs[i], scaling=0.8, max_iter=6)[1]), i
        dec.free()
