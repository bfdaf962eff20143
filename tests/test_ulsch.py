"""UL-SCH receive, data part (srsran_ulsch_decode without UCI, sch.c:994-1021 and 1122-1193): the channel
de-interleaver and decode_tb over its output.

CPU: the oracle's de-interleaver (restated from ulsch_interleave_gen + srsran_vec_lut_sis) inverts the
synthetic transmit interleaver (restated independently from ulsch_interleave_qm2/4/6).  sch.c itself is
not compiled here -- it includes srsran/srsran.h, which needs the CMake-generated srsran/version.h -- so
the de-interleaver is pinned by that round trip, and decode_tb by tests/test_sch_oracle.py.
GPU: srsran_ulsch_decode / srsran_ulsch_gpu_decode_batch against the oracle (de-interleaver + decode_tb):
g_bits, return code, payload, average iterations, soft-buffer flags, over HARQ retransmissions.
"""
import numpy as np
import pytest

from oracle import Oracle
from synth.ulsch_tx import ulsch_interleave

# (Qm, L_prb, N_symb, tbs): QPSK / 16QAM / 64QAM, normal (12) and SRS-shortened (11) subframes, C = 1 .. 9
CASES = [(2, 6, 12, 1544), (4, 25, 12, 11064), (6, 50, 11, 30576), (2, 1, 12, 56), (4, 100, 12, 51024)]


@pytest.fixture(scope="module")
def ora():
    return Oracle()


@pytest.mark.parametrize("Qm,L,nsymb,tbs", CASES)
def test_deinterleaver_inverts_transmit_interleaver(ora, Qm, L, nsymb, tbs):
    nb = L * 12 * nsymb * Qm
    g = np.random.default_rng(nb).integers(-300, 300, nb).astype(np.int16)
    q = ulsch_interleave(g, Qm, nsymb)
    assert not np.array_equal(q, g) or nb == Qm
    assert np.array_equal(ora.ulsch_deinterleave(q, Qm, nsymb), g)


def _ul_llrs(ora, tbs, Qm, rv, nb, payload, sigma, rng, nsymb):
    e = ora.dlsch_encode(tbs, Qm, rv, nb, payload).astype(np.float32) * 2 - 1
    e = e + rng.standard_normal(e.shape).astype(np.float32) * sigma
    g = np.trunc(100 * e).astype(np.int16)
    return g, ulsch_interleave(g, Qm, nsymb)


@pytest.mark.gpu
@pytest.mark.parametrize("Qm,L,nsymb,tbs", CASES)
def test_ulsch_decode_matches_oracle(ora, Qm, L, nsymb, tbs):
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    q = S.Sch()
    q.set_max_noi(8)
    nb = L * 12 * nsymb * Qm
    rng = np.random.default_rng(tbs)
    payload = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    sb = S.SoftbufferRx(nof_prb=100)
    state = None
    for rv, sigma in ((0, 0.9), (2, 0.7), (3, 0.5), (1, 0.2)):
        g_ref, qb = _ul_llrs(ora, tbs, Qm, rv, nb, payload, sigma, rng, nsymb)
        ret, data, g, avg, K_segm = q.ulsch_decode(sb, tbs, Qm, rv, nsymb, qb)
        assert np.array_equal(g, ora.ulsch_deinterleave(qb, Qm, nsymb)) and np.array_equal(g, g_ref)
        oret, odata, onoi, oavg, state = ora.dlsch_decode(tbs, Qm, rv, g, 8, state)
        assert ret == oret and avg == pytest.approx(oavg, abs=0), rv
        assert np.array_equal(data[:len(odata)], odata), rv
        rc, s = S.cbsegm(tbs)
        assert K_segm == s.C1 * s.K1 + s.C2 * s.K2
        assert sb.cb_crc(s.C) == [bool(x) for x in state[1][:s.C]], rv
        if ret == 0:
            break
    assert ret == 0 and np.array_equal(data[:tbs // 8], payload)
    sb.free()
    q.free()


@pytest.mark.gpu
def test_ulsch_batch_matches_oracle(ora):
    import torch

    from srsran_4g_amd import sch as S
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    q = S.Sch()
    q.set_max_noi(8)
    rng = np.random.default_rng(77)
    entries, keep, wants = [], [], []
    for Qm, L, nsymb, tbs in CASES:
        nb = L * 12 * nsymb * Qm
        payload = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        g, qb = _ul_llrs(ora, tbs, Qm, 0, nb, payload, 0.6, rng, nsymb)
        d_q = torch.from_numpy(qb).cuda()
        d_g = torch.zeros(nb, dtype=torch.int16, device="cuda")
        d_d = torch.zeros(tbs // 8 + 64, dtype=torch.uint8, device="cuda")
        sb = S.SoftbufferRx(nof_prb=100)
        keep += [d_q, d_g, d_d, sb]
        entries.append((tbs, Qm, 0, nb, nsymb, d_q.data_ptr(), d_g.data_ptr(), d_d.data_ptr(), sb, 1))
        wants.append((ora.dlsch_decode(tbs, Qm, 0, g, 8, None), g, d_g, d_d, tbs))
    d_res = torch.full((len(entries),), 77, dtype=torch.int32, device="cuda")
    d_avg = torch.zeros(len(entries), dtype=torch.float32, device="cuda")
    assert q.ulsch_decode_batch(entries, d_res.data_ptr(), d_avg.data_ptr()) == 0
    torch.cuda.synchronize()
    res, avg = d_res.cpu().numpy(), d_avg.cpu().numpy()
    for i, ((oret, odata, onoi, oavg, st), g, d_g, d_d, tbs) in enumerate(wants):
        assert np.array_equal(d_g.cpu().numpy(), g), i
        assert res[i] == oret and avg[i] == pytest.approx(oavg, abs=0), i
        if oret == 0:
            assert np.array_equal(d_d.cpu().numpy()[:tbs // 8], odata[:tbs // 8]), i
    for k in keep:
        if isinstance(k, S.SoftbufferRx):
            k.free()
    q.free()
