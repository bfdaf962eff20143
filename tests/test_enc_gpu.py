"""DL-SCH transmit on the GPU: srsran_dlsch_encode2 / srsran_dlsch_gpu_encode_batch
(TB CRC24A, segmentation with CRC24B, turbo encoding, rate matching: sch.c:240-359, turbocoder.c,
rm_turbo.c:345-388) against the oracle's encoder (oracle/sch_oracle.c, pinned to the reference's
compiled rm_turbo.c and turbocoder.c by tests/test_sch_oracle.py / test_oracle.py), bit for bit on
the packed e bits: every code block size as a single-block TB, multi-block TBs with K- / K+ blocks,
all four rv, two layers (Qm x 2), E not a multiple of 8; and an encode -> decode round trip."""
import numpy as np
import pytest

from oracle import Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    q = S.Sch()
    yield S, q, Oracle()
    q.free()


def _want(ora, tbs, Qm, rv, G, payload):
    return np.packbits(ora.dlsch_encode(tbs, Qm, rv, G, payload))


def _single_cb_tbs(S):
    """TBS whose segmentation is one block of each size K (tbs = K - 24), where cbsegm gives F = 0"""
    from srsran_4g_amd.tdec import CB_SIZES
    out = []
    for K in CB_SIZES:
        tbs = K - 24
        rc, s = S.cbsegm(tbs)
        if rc == 0 and s.C == 1 and s.F == 0 and tbs > 0 and tbs % 8 == 0:
            out.append(tbs)
    return out


def test_encode_every_block_size(env):
    S, q, ora = env
    rng = np.random.default_rng(1)
    sizes = _single_cb_tbs(S)
    assert len(sizes) > 150
    for tbs in sizes:
        Qm, rv = int(rng.choice([2, 4, 6])), int(rng.integers(0, 4))
        G = Qm * int(rng.integers((tbs + 24) // Qm // 2 + 1, 3 * (tbs + 24) // Qm + 10))
        payload = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        ret, e = q.encode(tbs, Qm, rv, G, payload)
        assert ret == 0
        assert np.array_equal(e, _want(ora, tbs, Qm, rv, G, payload)), (tbs, Qm, rv, G)


@pytest.mark.parametrize("tbs,Qm,G", [(75376, 6, 86400), (51024, 4, 57600), (6200, 2, 12000), (30576, 6, 39600),
                                      (7992, 4, 9000), (97896, 6, 86400 + 36)])
@pytest.mark.parametrize("rv", [0, 1, 2, 3])
def test_encode_multi_block(env, tbs, Qm, G, rv):
    S, q, ora = env
    rc, s = S.cbsegm(tbs)
    if rc or s.F:
        pytest.skip("filler bits")
    rng = np.random.default_rng(tbs + rv)
    payload = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    ret, e = q.encode(tbs, Qm, rv, G, payload)
    assert ret == 0 and np.array_equal(e, _want(ora, tbs, Qm, rv, G, payload))


def test_encode_two_layers(env):
    """one TB on two layers: encode_tb sees Qm x 2 (sch.c:633-636)"""
    S, q, ora = env
    rng = np.random.default_rng(3)
    tbs, Qm, G = 61664, 6, 2 * 6 * 6000
    payload = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    ret, e = q.encode(tbs, Qm, 0, G, payload, nof_layers=2, nof_tb=1)
    assert ret == 0 and np.array_equal(e, _want(ora, tbs, 2 * Qm, 0, G, payload))


def test_encode_batch_and_round_trip(env):
    import torch
    S, q, ora = env
    rng = np.random.default_rng(9)
    cases = [(75376, 6, 86400, 0), (1544, 2, 3456, 1), (30576, 6, 39600, 2), (11064, 4, 14400, 3), (104, 2, 288, 0)]
    ents, keep, wants = [], [], []
    for tbs, Qm, G, rv in cases:
        payload = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        d_in = torch.from_numpy(payload).cuda()
        d_out = torch.zeros((G + 7) // 8, dtype=torch.uint8, device="cuda")
        keep += [d_in, d_out]
        ents.append((tbs, Qm, rv, G, d_in.data_ptr(), d_out.data_ptr()))
        wants.append((_want(ora, tbs, Qm, rv, G, payload), d_out, payload, tbs, Qm, rv, G))
    assert q.encode_batch(ents) == 0
    torch.cuda.synchronize()
    q.set_max_noi(8)
    for want, d_out, payload, tbs, Qm, rv, G in wants:
        e = d_out.cpu().numpy()
        assert np.array_equal(e, want), tbs
        if rv == 0:  # and the receiver gets the payload back from it
            bits = np.unpackbits(e)[:G]
            sb = S.SoftbufferRx(nof_prb=100)
            ret, data, _ = q.decode(sb, tbs, Qm, 0, (bits.astype(np.int16) * 2 - 1) * 100)
            assert ret == 0 and np.array_equal(data[:tbs // 8], payload)
            sb.free()


def test_encode_refusals(env):
    S, q, ora = env
    ret, _ = q.encode(1000, 2, 0, 2000, np.zeros(125, np.uint8))  # 1000 + 24 needs filler bits
    rc, s = S.cbsegm(1000)
    assert (ret != 0) == bool(s.F)
