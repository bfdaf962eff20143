"""GPU NR SCH receive parity through the C-ABI (srsran_dlsch_nr_decode / srsran_ulsch_nr_decode /
srsran_sch_nr_gpu_decode_batch) against the oracle restatement of sch_nr.c (itself pinned against the
compiled reference, tests/test_nr_sch_oracle.py): TB CRC, average iterations, payload, and the whole
soft-buffer state (per-CB CRC flags, int8 soft bits, saved CB payloads) after every HARQ transmission.
Inputs come from synth/nr_tx.py (pinned against the reference encoder in tests/test_synth.py)."""
import numpy as np
import pytest
import torch

from nr_sch import OracleNr, new_state, oracle_nr_tb_info_t
from srsran_4g_amd import sch_nr as S
from srsran_4g_amd import tdec
from synth.nr_tx import NrCodeblocks, aligned_tbs, bpsk_llrs, rm_params

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ora():
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    return OracleNr()


@pytest.fixture(scope="module")
def q(ora):
    s = S.SchNr(nof_prb=273, max_nof_iter=6)
    yield s
    s.free()


_llrs = bpsk_llrs
_tbs = aligned_tbs


def _ot(t):
    """The product's TB info as the oracle's struct (the two are asserted equal field by field)."""
    o = oracle_nr_tb_info_t()
    for k, v in t.as_dict().items():
        setattr(o, k, v)
    return o


def _check_state(sb, st, t, tag):
    sb.sync()
    _, Ncb = rm_params(t, 0)
    for r in range(t.C):
        assert sb.s.cb_crc[r] == bool(st["cb_crc"][r]), (tag, r)
        assert np.array_equal(S.read_cb8(sb, r, Ncb), st["softbuf"][r][:Ncb]), (tag, r)
        if st["cb_crc"][r]:
            n = (t.Kp - t.L_cb + 7) // 8
            assert np.array_equal(sb.read_data(r, n), st["cb_data"][r][:n]), (tag, r)


# (N_re, R, Qm, layers, lbrm, nof_prb): BG1/BG2, C = 1 and C > 1, CRC16 / CRC24A TB CRC, LBRM
NR_CASES = [(400, 0.3, 2, 1, False, 52), (3000, 0.5, 4, 1, False, 52), (12 * 13 * 52, 0.6, 6, 2, False, 52),
            (12 * 12 * 106, 0.75, 6, 2, True, 106), (100, 0.2, 2, 1, False, 25), (12 * 12 * 100, 0.9, 8, 2, True, 273),
            (12 * 13 * 30, 0.2, 4, 1, True, 52), (12 * 13 * 273, 0.85, 8, 1, False, 273)]


@pytest.mark.parametrize("case", NR_CASES)
@pytest.mark.parametrize("uplink", [False, True])
def test_decode_harq_matches_oracle(ora, q, case, uplink):
    n_re, R, Qm, Nl, lbrm, nof_prb = case
    rng = np.random.default_rng(n_re + uplink)
    tbs = _tbs(n_re, R, Qm, Nl)
    G = n_re * Qm * Nl
    t = S.tb_info(tbs, R, Qm, G, Nl, lbrm=lbrm, nof_prb=nof_prb, mcs256=Qm == 8)
    assert t.as_dict() == ora.tb_info(tbs, R, Qm, G, Nl, lbrm=lbrm, nof_prb=nof_prb, mcs256=Qm == 8).as_dict()
    pl = rng.integers(0, 256, tbs // 8).astype(np.uint8)
    enc = NrCodeblocks(t, pl)
    q.carrier.nof_prb = nof_prb
    S.lib().srsran_sch_nr_set_carrier(S.ctypes.byref(q.q), S.ctypes.byref(q.carrier))
    sb = S.nr_softbuffer()
    st = new_state(t.C)
    base = {2: -1.0, 4: 3.0, 6: 7.0, 8: 12.0}[Qm] + 6 * (R - 0.5)
    last = None
    for rv, d in ((0, -1.5), (2, 0.0), (3, 1.0), (1, 6.0)):
        llr = _llrs(rng, enc.rate_match(rv), base + d)
        ret, crc, avg, got = q.decode(sb, tbs, R, Qm, G, Nl, rv, llr, lbrm=lbrm, mcs256=Qm == 8, uplink=uplink)
        assert ret == 0
        want = ora.decode(_ot(t), rv, llr, st, max_iter=6)
        assert crc == bool(want[0]) and avg == pytest.approx(want[1], abs=1e-6), (rv, crc, avg, want[:2])
        if all(st["cb_crc"][:t.C]):
            assert np.array_equal(got, want[2])
        _check_state(sb, st, t, rv)
        last = crc
    assert last  # the clean last retransmission decodes
    assert np.array_equal(got, pl)
    sb.free()


def test_noise_free_single_pass(ora, q):
    rng = np.random.default_rng(9)
    for n_re, R, Qm in ((12 * 13 * 273, 0.93, 8), (12 * 13 * 273, 0.5, 2), (600, 0.4, 6)):
        tbs = _tbs(n_re, R, Qm, 1)
        G = n_re * Qm
        t = S.tb_info(tbs, R, Qm, G, 1, nof_prb=273, mcs256=Qm == 8)
        pl = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        e = NrCodeblocks(t, pl).rate_match(0)
        sb = S.nr_softbuffer()
        ret, crc, avg, got = q.decode(sb, tbs, R, Qm, G, 1, 0, np.where(e == 1, -20, 20).astype(np.int8),
                                      mcs256=Qm == 8)
        want = ora.decode(_ot(t), 0, np.where(e == 1, -20, 20).astype(np.int8), new_state(t.C), max_iter=6)
        assert ret == 0 and crc and np.array_equal(got, pl), (tbs, t.C)
        assert avg == pytest.approx(want[1], abs=1e-6)
        sb.free()


def test_batch_matches_sequential_oracle(ora, q):
    """Several TBs (BG1 / BG2, different Z, C = 1 and C > 1, first and re-transmissions) in one batch."""
    rng = np.random.default_rng(21)
    q.carrier.nof_prb = 273
    S.lib().srsran_sch_nr_set_carrier(S.ctypes.byref(q.q), S.ctypes.byref(q.carrier))
    cases = [(400, 0.3, 2, 1), (12 * 13 * 52, 0.6, 6, 2), (3000, 0.5, 4, 1), (12 * 12 * 100, 0.9, 8, 2),
             (100, 0.2, 2, 1), (12 * 13 * 100, 0.45, 6, 1)]
    tbs_l, objs = [], []
    for n_re, R, Qm, Nl in cases:
        tbs = _tbs(n_re, R, Qm, Nl)
        G = n_re * Qm * Nl
        t = S.tb_info(tbs, R, Qm, G, Nl, nof_prb=273, mcs256=Qm == 8)
        pl = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        objs.append(dict(t=t, tbs=tbs, R=R, Qm=Qm, G=G, Nl=Nl, pl=pl, enc=NrCodeblocks(t, pl), sb=S.nr_softbuffer(),
                         st=new_state(t.C), base={2: -1.0, 4: 3.0, 6: 7.0, 8: 12.0}[Qm] + 6 * (R - 0.5)))
        tbs_l.append(tbs)
    for rv, d in ((0, -1.0), (2, 0.5), (1, 6.0)):
        entries, keep = [], []
        d_crc = torch.full((len(objs),), 77, dtype=torch.uint8, device="cuda")
        d_avg = torch.zeros(len(objs), dtype=torch.float32, device="cuda")
        wants = []
        for o in objs:
            llr = _llrs(rng, o["enc"].rate_match(rv), o["base"] + d)
            d_e = torch.from_numpy(llr).cuda()
            d_p = torch.zeros(o["tbs"] // 8 + 8, dtype=torch.uint8, device="cuda")
            cfg = S.make_cfg(mcs256=o["Qm"] == 8)
            tb = S.make_tb(o["tbs"], o["R"], o["Qm"], o["G"], o["Nl"], rv, o["sb"])
            keep += [d_e, d_p, cfg, tb]
            entries.append((cfg, tb, d_e.data_ptr(), d_p.data_ptr()))
            o["d_p"] = d_p
            wants.append(ora.decode(_ot(o["t"]), rv, llr, o["st"], max_iter=6))
        assert q.decode_batch(entries, d_crc.data_ptr(), d_avg.data_ptr()) == 0
        torch.cuda.synchronize()
        crc, avg = d_crc.cpu().numpy(), d_avg.cpu().numpy()
        for i, o in enumerate(objs):
            assert crc[i] == want_crc(wants[i]) and avg[i] == pytest.approx(wants[i][1], abs=1e-6), (rv, i)
            if all(o["st"]["cb_crc"][:o["t"].C]):
                assert np.array_equal(o["d_p"].cpu().numpy()[:o["tbs"] // 8], wants[i][2]), (rv, i)
            _check_state(o["sb"], o["st"], o["t"], (rv, i))
    for o in objs:
        assert np.array_equal(o["d_p"].cpu().numpy()[:o["tbs"] // 8], o["pl"])
        o["sb"].free()


def want_crc(w):
    return 1 if w[0] else 0


def test_tb_crc_mismatch_with_all_cbs_ok(ora, q):
    """Every CB passes its CRC24B but the TB CRC does not match: crc false, payload still assembled."""
    rng = np.random.default_rng(3)
    tbs = _tbs(12 * 13 * 52, 0.6, 6, 1)
    G = 12 * 13 * 52 * 6
    t = S.tb_info(tbs, 0.6, 6, G, 1)
    assert t.C > 1
    pl = rng.integers(0, 256, tbs // 8).astype(np.uint8)
    enc = NrCodeblocks(t, pl)
    # corrupt the TB CRC bits inside the last CB, then recompute that CB's own CRC so it still passes
    from synth.ldpc_tx import encode as ldpc_encode
    from synth.nr_tx import CRC24B, _unpack, crc_bits
    cb_len = t.Kp - t.L_cb
    bits = np.concatenate([np.unpackbits(pl), np.zeros(24, np.uint8)])
    seg = bits[(t.C - 1) * cb_len:t.C * cb_len].copy()
    seg[-1] ^= 1
    msg = np.zeros(t.Kr, np.uint8)
    msg[:cb_len] = seg
    msg[cb_len:t.Kp] = _unpack(crc_bits(seg, CRC24B, 24), 24)
    enc.cw[t.C - 1] = ldpc_encode(t.bg, t.Z, msg)[2 * t.Z:]
    llr = np.where(enc.rate_match(0) == 1, -20, 20).astype(np.int8)
    sb = S.nr_softbuffer()
    st = new_state(t.C)
    ret, crc, avg, got = q.decode(sb, tbs, 0.6, 6, G, 1, 0, llr)
    want = ora.decode(_ot(t), 0, llr, st, max_iter=6)
    assert ret == 0 and not crc and not want[0]
    assert np.array_equal(got, want[2])
    _check_state(sb, st, t, "tbcrc")
    sb.free()


def test_input_checks(ora, q):
    a = S.srsran_sch_nr_args_t()
    a.decoder_use_flooded = True
    x = S.srsran_sch_nr_t()
    assert S.lib().srsran_sch_nr_init_rx(S.ctypes.byref(x), S.ctypes.byref(a)) != 0
    # soft buffer with too few code blocks
    tbs = _tbs(12 * 13 * 52, 0.6, 6, 1)
    G = 12 * 13 * 52 * 6
    small = S.SoftbufferRx(max_cb=2, max_cb_size=S.MAX_CB_SIZE)
    ret, *_ = q.decode(small, tbs, 0.6, 6, G, 1, 0, np.zeros(G, np.int8))
    assert ret != 0
    small.free()
    # soft buffer blocks too short for the lifting size
    short = S.SoftbufferRx(max_cb=41, max_cb_size=6144)
    ret, *_ = q.decode(short, tbs, 0.6, 6, G, 1, 0, np.zeros(G, np.int8))
    assert ret != 0
    short.free()


def test_batch_new_data_reuses_soft_buffers(ora, q):
    """new_data = 1 on a soft buffer left by an earlier TB (flags set, soft bits accumulated) behaves as a
    freshly reset buffer: same results and state as the oracle from an empty state."""
    rng = np.random.default_rng(33)
    q.carrier.nof_prb = 273
    S.lib().srsran_sch_nr_set_carrier(S.ctypes.byref(q.q), S.ctypes.byref(q.carrier))
    n_re, R, Qm, Nl = 12 * 13 * 60, 0.7, 6, 1
    tbs = _tbs(n_re, R, Qm, Nl)
    G = n_re * Qm * Nl
    t = S.tb_info(tbs, R, Qm, G, Nl, nof_prb=273)
    sb = S.nr_softbuffer()
    for it, (rv, snr) in enumerate(((0, 20.0), (0, 6.0), (2, 5.0), (0, 4.0))):
        pl = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        llr = _llrs(rng, NrCodeblocks(t, pl).rate_match(rv), snr)
        st = new_state(t.C)
        want = ora.decode(_ot(t), rv, llr, st, max_iter=6)
        d_e = torch.from_numpy(llr).cuda()
        d_p = torch.zeros(tbs // 8 + 8, dtype=torch.uint8, device="cuda")
        d_crc = torch.full((1,), 77, dtype=torch.uint8, device="cuda")
        d_avg = torch.zeros(1, dtype=torch.float32, device="cuda")
        cfg, tb = S.make_cfg(), S.make_tb(tbs, R, Qm, G, Nl, rv, sb)
        assert q.decode_batch([(cfg, tb, d_e.data_ptr(), d_p.data_ptr(), 1)], d_crc.data_ptr(), d_avg.data_ptr()) == 0
        torch.cuda.synchronize()
        assert int(d_crc.cpu()[0]) == want_crc(want) and float(d_avg.cpu()[0]) == pytest.approx(want[1], abs=1e-6)
        _check_state(sb, st, t, it)
        if want[0]:  # rv 2 alone carries no systematic bits: both converge to the all-zero codeword,
            # whose zero-initialised CRCs pass (sch_nr.c behaves the same), hence want[2] rather than pl
            assert np.array_equal(d_p.cpu().numpy()[:tbs // 8], want[2])
            assert it == 2 or np.array_equal(want[2], pl)
    sb.free()


# (Qm, R x 1024) of 38.214 Table 5.1.3.1-1 (MCS 0, 5, 9, 10, 13, 17, 22, 28)
MCS_SUBSET = [(2, 120), (2, 379), (2, 679), (4, 340), (4, 490), (6, 438), (6, 616), (6, 948)]


@pytest.mark.parametrize("n_prb", [1, 7, 25, 52, 106, 273])
def test_prb_mcs_rv_sweep_noise_free(ora, q, n_prb):
    """sch_nr_test.c:176-235: every (PRB count, MCS, rv), LLRs +-10 of the encoded bits, a reset soft
    buffer per decode; rv 0 must decode.  Here every decode is also compared with the oracle."""
    q.carrier.nof_prb = 273
    S.lib().srsran_sch_nr_set_carrier(S.ctypes.byref(q.q), S.ctypes.byref(q.carrier))
    rng = np.random.default_rng(n_prb)
    for Qm, r1024 in MCS_SUBSET:
        R = r1024 / 1024
        n_re = 12 * 12 * n_prb
        tbs = _tbs(n_re, R, Qm, 1)
        G = n_re * Qm
        t = S.tb_info(tbs, R, Qm, G, 1, nof_prb=273)
        pl = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        enc = NrCodeblocks(t, pl)
        for rv in range(4):
            llr = np.where(enc.rate_match(rv) == 1, -10, 10).astype(np.int8)
            sb = S.nr_softbuffer(max_cb=max(t.C, 1))
            ret, crc, avg, got = q.decode(sb, tbs, R, Qm, G, 1, rv, llr)
            st = new_state(t.C)
            want = ora.decode(_ot(t), rv, llr, st, max_iter=6)
            assert ret == 0 and crc == bool(want[0]) and avg == pytest.approx(want[1], abs=1e-6), (Qm, r1024, rv)
            _check_state(sb, st, t, (Qm, r1024, rv))
            if rv == 0:
                assert crc and np.array_equal(got, pl), (n_prb, Qm, r1024, tbs)
            sb.free()
