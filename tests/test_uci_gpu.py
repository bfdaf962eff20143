"""UCI on PUSCH on the GPU: srsran_ulsch_decode with HARQ-ACK / RI / CQI multiplexed (sch.c:994-1193)
against the reference's uci.c / block.c compiled into oracle/_ref (oracle/ref_uci_harness.c).

Per case the reference transmitter (srsran_uci_encode_* + the UL-SCH multiplexing of
ref_ulsch_uci_tx) builds the PUSCH bit stream, scramble_llrs turns it into descrambled soft bits
(noise-free and noisy), and the library's srsran_ulsch_decode must return exactly what the
reference receiver returns: the HARQ-ACK bits and their `valid` flag, the RI, the CQI report and
its CRC flag, q_bits with the ACK positions zeroed, the de-interleaved g_bits (RI cells skipped),
and -- with a TB -- decode_tb's return / payload over g's UL-SCH part (the oracle's decode_tb).
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
sys.path.insert(0, HERE)

import uci as RU  # noqa: E402  (oracle/uci.py)
import uci_cases as UC  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    from oracle import Oracle
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    if not RU.ref_available():  # on a HIP box the parity checker must be there: fail, never skip
        pytest.fail("oracle/_ref/libsrsref.so missing: the reference checker of this module was not built")
    q = S.Sch()
    q.set_max_noi(8)
    yield S, q, Oracle(), RU.RefUci()
    q.free()


def _run(env, case, sigma, seed, I=(9, 6, 8), amp=100.0):
    S, q, ora, ref = env
    name, Qm, L, ns, tbs, nack, ri, cqi = case
    rng = np.random.default_rng(seed)
    cfg = UC.make_cfg(Qm, L, ns, tbs, nack, ri, cqi, I=I)
    u = UC.random_uci(cfg, rng)
    Qri, Qcqi, G = ref.tx_sizes(cfg, u)
    e = np.zeros(0, np.uint8)
    payload = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    if tbs:
        e = ora.dlsch_encode(tbs, Qm, 0, G * Qm, payload)
    types, _ = ref.tx(cfg, u, e)
    c = rng.integers(0, 2, types.size).astype(np.uint8)
    qb = RU.scramble_llrs(types, c, rng, amp=amp, sigma=sigma)

    # reference receiver
    rcfg = UC.make_cfg(Qm, L, ns, tbs, nack, ri, cqi, I=I)
    want = S.srsran_uci_value_t()
    rret, rq, rg, (rQri, rQcqi, rG, rQack) = ref.rx(rcfg, qb, c, want)

    # library, on the GPU
    sb = S.SoftbufferRx(nof_prb=100)
    gcfg = UC.make_cfg(Qm, L, ns, tbs, nack, ri, cqi, I=I, softbuffer=sb)
    gcfg.max_nof_iterations = 8
    ret, data, gq, gg, got = q.ulsch_decode_uci(gcfg, qb, c_seq=c)
    sb.free()

    assert np.array_equal(gq, rq), "q_bits after the ACK zeroing"
    assert np.array_equal(gg, rg), "de-interleaved g_bits"
    assert gcfg.K_segm == rcfg.K_segm
    if nack:
        assert list(got.ack.ack_value[:nack]) == list(want.ack.ack_value[:nack])
        assert bool(got.ack.valid) == bool(want.ack.valid)
    if ri:
        assert got.ri == want.ri
    if cqi:
        assert bool(got.cqi.data_crc) == bool(want.cqi.data_crc)
        assert UC.cqi_fields(gcfg, got.cqi) == UC.cqi_fields(rcfg, want.cqi)
        assert bool(gcfg.uci_cfg.cqi.rank_is_not_one) == bool(rcfg.uci_cfg.cqi.rank_is_not_one)
    if tbs:
        oret, odata, _, _, _ = ora.dlsch_decode(tbs, Qm, 0, rg[rQcqi * Qm:(rQcqi + rG) * Qm], 8, None)
        assert ret == oret
        if oret == 0:
            assert np.array_equal(data[:tbs // 8], odata[:tbs // 8])
    else:
        assert ret == rret
    return ret, got, u, (rQri, rQcqi, rG, rQack), want


@pytest.mark.parametrize("case", UC.CASES, ids=[c[0] for c in UC.CASES])
def test_uci_noise_free_matches_reference(env, case):
    name, Qm, L, ns, tbs, nack, ri, cqi = case
    ret, got, u, _, want = _run(env, case, 0.0, len(name))
    # and the values are the transmitted ones
    if nack:
        assert list(got.ack.ack_value[:nack]) == list(u.ack.ack_value[:nack])
    if ri:
        assert got.ri == u.ri
    if cqi:
        assert got.cqi.data_crc
    if tbs:
        assert ret == 0


@pytest.mark.parametrize("sigma", [0.5, 1.0, 2.5])
@pytest.mark.parametrize("case", UC.CASES, ids=[c[0] for c in UC.CASES])
def test_uci_noisy_matches_reference(env, case, sigma):
    """noisy soft bits: decisions, valid flags and CRC failures agree with the reference"""
    _run(env, case, sigma, 1000 + int(sigma * 10) + len(case[0]))


@pytest.mark.parametrize("I", [(2, 0, 0), (15, 12, 14), (5, 3, 10)])
def test_uci_offsets(env, I):
    """other beta offsets: Q'_ACK / Q'_RI / Q'_CQI and so every position set change"""
    for case in UC.CASES[:6]:
        _run(env, case, 0.3, 7 + sum(I), I=I)


@pytest.mark.parametrize("amp", [12.0, 3000.0, 16000.0])
def test_uci_amplitudes(env, amp):
    """small and near-saturating LLRs: the accumulator clamp (uci.c:689-690), int16 wrap of the
    2-bit sums (uci.c:532-534) and the amplitude threshold on `valid` (uci.c:695-711)"""
    for case in UC.CASES:
        _run(env, case, 0.4, 31 + int(amp), amp=amp)
