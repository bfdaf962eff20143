"""The 8-bit LLR chain on the GPU (srsUE's pdsch_8bit_decoder: ue_dl.pdsch.llr_is_8bit and
ue_dl.pdsch.dl_sch.llr_is_8bit, srsue/src/phy/lte/cc_worker.cc:108-110) against the oracle:

  pdsch.c:691-737   demod_b, sequence_pdsch_apply_c, the 8-bit CSI correction, srsran_evm_run_b
  sch.c:409-428     srsran_rm_turbo_rx_lut_8bit + srsran_tdec_iteration_8bit with the CRC early stop

The oracle pieces (oracle/phy_oracle.c, oracle/tdec_oracle.c oracle_tdec8_run, oracle/sch_oracle.c
oracle_dlsch_decode_tb8) are pinned to the reference build in tests/test_phy_oracle.py,
tests/test_tdec8bit.py and tests/test_sch_oracle.py.  Bit-exact: decode_tb's return, every payload byte,
average iterations; int8 LLRs of the PDSCH stage fed the oracle's grids and estimates.
"""
import numpy as np
import pytest
import torch

from oracle import Oracle, Reference, ref_available
import pdsch_chain as PC
from synth import synth as S
from test_sch_oracle import llr8_of

pytestmark = pytest.mark.gpu

TBS = 75376


@pytest.fixture(scope="module")
def ora():
    return Oracle()


@pytest.fixture(scope="module")
def U():
    from srsran_4g_amd import ue_dl
    ue_dl.use_standard_symbol_size(True)
    yield ue_dl
    ue_dl.use_standard_symbol_size(False)


@pytest.fixture(scope="module")
def SCH():
    from srsran_4g_amd import sch
    return sch


# (tbs, Qm, G, sigma): every decoder class -- 32 sub-blocks (K > 2048), 16 (800 < K <= 2048), the 16-bit decoders
# on the widened row (8 sub-blocks, natural K <= 400) -- noise-free, early stops spread over half-iterations, failures
DL8_CASES = [(75376, 6, 86400, 0.0), (75376, 6, 86400, 0.5), (1544, 2, 3600, 0.8), (19080, 4, 28800, 0.6),
             (680, 4, 2400, 0.9), (16, 2, 240, 0.3), (6200, 2, 7200, 0.9)]


@pytest.mark.parametrize("case", range(len(DL8_CASES)))
def test_dlsch8_host_sync_matches_oracle(SCH, ora, case):
    """srsran_dlsch_decode2 with llr_is_8bit over a HARQ chain (rv 0, 2, 3 combined in one soft buffer) against
    oracle_dlsch_decode_tb8."""
    tbs, Qm, G, sigma = DL8_CASES[case]
    rng = np.random.default_rng(500 + case)
    sch = SCH.Sch()
    sch.set_llr8(True)
    sch.set_max_noi(8)
    sb = SCH.SoftbufferRx(nof_prb=100)
    tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    state = None
    for rv in (0, 2, 3):
        e = llr8_of(ora.dlsch_encode(tbs, Qm, rv, G, tb), rng, sigma)
        ret, data, noi = sch.decode(sb, tbs, Qm, rv, e)
        want = ora.dlsch_decode8(tbs, Qm, rv, e, 8, state)
        state = want[4]
        assert ret == want[0], (rv, ret, want[0])
        n = tbs // 8 + 6
        assert np.array_equal(data[:n], want[1][:n]), rv
        assert noi == pytest.approx(want[3], abs=1e-6), rv
        assert sb.cb_crc(len(state[1])) == [bool(v) for v in state[1]], rv
        if ret == 0:
            assert np.array_equal(data[: tbs // 8], tb)
            break


def test_dlsch8_batch_matches_oracle(SCH, ora):
    """srsran_dlsch_gpu_decode_batch with llr_is_8bit: TBs of every decoder class in one batch (one launch per K on
    the 8-bit window decoders, the widened rows of K <= 800 on the 16-bit ones), new transmissions over dirty soft
    buffers, then a retransmission round combined into the same buffers."""
    rng = np.random.default_rng(77)
    sch = SCH.Sch()
    sch.set_llr8(True)
    sch.set_max_noi(8)
    cases = DL8_CASES[1:]
    sbs = [SCH.SoftbufferRx(nof_prb=100) for _ in cases]
    tbs_data = [rng.integers(0, 256, t // 8, dtype=np.uint8) for t, _, _, _ in cases]
    states = [None] * len(cases)
    d_data = torch.zeros((len(cases), TBS // 8 + 64), dtype=torch.uint8, device="cuda")
    for rnd, rv in enumerate((0, 2)):
        es = [llr8_of(ora.dlsch_encode(t, Qm, rv, G, tbs_data[i]), rng, s) for i, (t, Qm, G, s) in enumerate(cases)]
        d_e = [torch.from_numpy(e).cuda() for e in es]
        entries = [(t, Qm, rv, G, d_e[i].data_ptr(), d_data[i].data_ptr(), sbs[i], 1 if rnd == 0 else 0)
                   for i, (t, Qm, G, _) in enumerate(cases)]
        if rnd == 0:  # dirty buffers: a new transmission must not combine with them
            for i, (t, Qm, G, _) in enumerate(cases):
                junk = rng.integers(-128, 128, G).astype(np.int8)
                sch.decode(sbs[i], t, Qm, 1, junk)
        d_data.zero_()  # bytes decode_tb does not write (skipped blocks' CRC tails) compare as the oracle's zeros
        d_res = torch.full((len(cases),), 7, dtype=torch.int32, device="cuda")
        d_avg = torch.zeros(len(cases), dtype=torch.float32, device="cuda")
        assert sch.decode_batch(entries, d_res.data_ptr(), d_avg.data_ptr()) == 0
        torch.cuda.synchronize()
        res, avg, data = d_res.cpu().numpy(), d_avg.cpu().numpy(), d_data.cpu().numpy()
        for i, (t, Qm, G, _) in enumerate(cases):
            want = ora.dlsch_decode8(t, Qm, rv, es[i], 8, states[i])
            states[i] = want[4]
            assert res[i] == want[0], (rnd, i)
            assert np.array_equal(data[i, : t // 8 + 6], want[1][: t // 8 + 6]), (rnd, i)
            assert avg[i] == pytest.approx(want[3], abs=1e-6), (rnd, i)


def _case(ora, rng, nof_prb=100, cell_id=1, nports=2, tti=1, cfi=1, tbs=(TBS, TBS), Qm=(6, 6), scheme="cdd",
          pmi=0, snr_db=30.0, **kw):
    pls = [rng.integers(0, 256, t // 8, dtype=np.uint8) for t in tbs]
    cb = pmi + 1 if len(tbs) == 2 else pmi
    x, nre = S.pdsch_subframe(nof_prb, cell_id, nports, tti, cfi, 0x1234, tbs[0], Qm[0], 0, pls, scheme=scheme,
                              codebook=cb, snr_db=snr_db, rng=rng, **kw)
    grids, ce, st = PC.fft_estimate(ora, x, nof_prb, cell_id, nports, tti)
    return pls, x, nre, grids, ce, st


PD8_CASES = [
    dict(),                                                                   # C3, 64QAM CDD
    dict(snr_db=13.0, fail=True),                                             # CB failures
    dict(nports=1, scheme="port0", tbs=(30576,), Qm=(4,), cell_id=3, channel=[[1], [0.5 + 0.5j]]),
    dict(scheme="diversity", tbs=(TBS,), Qm=(6,), tti=5, cell_id=4),
    dict(nof_prb=6, cell_id=2, tbs=(680, 680), Qm=(4, 4), cfi=2, tti=7),      # K = 704: widened rows, 8 sub-blocks
    dict(nof_prb=6, cell_id=5, tbs=(328,), Qm=(2,), nports=1, scheme="port0", tti=2),  # K = 352: widened, natural
    dict(nof_prb=25, cell_id=9, tbs=(1544, 1544), Qm=(2, 2), tti=3),         # QPSK, K = 1568: 16 sub-blocks
]


@pytest.mark.parametrize("case", range(len(PD8_CASES)))
@pytest.mark.parametrize("csi", [True, False])
def test_pdsch8_decode_bitexact(U, SCH, ora, case, csi):
    """srsran_pdsch_decode with llr_is_8bit on the oracle's grids and estimates == the oracle chain with llr8."""
    kw = dict(PD8_CASES[case])
    rng = np.random.default_rng(600 + case)
    fail = kw.pop("fail", False)
    nof_prb, cell_id, nports = kw.pop("nof_prb", 100), kw.pop("cell_id", 1), kw.pop("nports", 2)
    tti, cfi = kw.pop("tti", 1), kw.pop("cfi", 1)
    tbs, Qm = kw.pop("tbs", (TBS, TBS)), kw.pop("Qm", (6, 6))
    scheme, pmi = kw.pop("scheme", "cdd"), kw.pop("pmi", 0)
    pls, x, nre, grids, ce, st = _case(ora, rng, nof_prb, cell_id, nports, tti, cfi, tbs, Qm, scheme, pmi, **kw)
    ref = PC.pdsch_decode(ora, grids, ce, st["noise"], nof_prb, cell_id, nports, tti, cfi, 0x1234, list(tbs),
                          list(Qm), [0] * len(tbs), scheme=scheme, pmi=pmi, csi_enable=csi, llr8=True)
    sbs = [SCH.SoftbufferRx(nof_prb=nof_prb) for _ in tbs]
    cfg = U.pdsch_cfg(nof_prb, nre, tbs, Qm, scheme=scheme, pmi=pmi, softbuffers=sbs, csi_enable=csi)
    pd = U.Pdsch(U.cell(nof_prb, nports, cell_id), grids.shape[0])
    pd.set_llr8(True)
    ret, out = pd.decode(cfg, tti, cfi, grids, ce, st["noise"])
    assert ret == 0
    for q, (crc, payload, avg) in enumerate(out):
        r = ref[q]
        assert crc == (r["ret"] == 0), q
        n = tbs[q] // 8 + 6
        assert np.array_equal(payload[:n], r["data"][:n]), q
        assert avg == pytest.approx(r["avg"], abs=1e-6), q
        if not fail:
            assert crc and np.array_equal(payload[: tbs[q] // 8], pls[q])
    pd.free()


def test_pdsch8_flags_must_match(U, SCH, ora):
    """pdsch.llr_is_8bit without dl_sch.llr_is_8bit (int8 LLRs into an int16 decoder) is refused."""
    rng = np.random.default_rng(9)
    pls, x, nre, grids, ce, st = _case(ora, rng)
    sbs = [SCH.SoftbufferRx(nof_prb=100) for _ in range(2)]
    cfg = U.pdsch_cfg(100, nre, (TBS, TBS), (6, 6), softbuffers=sbs)
    pd = U.Pdsch(U.cell(100, 2, 1), 2)
    pd.q.llr_is_8bit = True
    ret, _ = pd.decode(cfg, 1, 1, grids, ce, st["noise"])
    assert ret != 0
    pd.free()


@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("case", [0, 2, 4, 6])
def test_pdsch8_evm_matches_reference(U, SCH, ora, case):
    """meas_evm_en with llr_is_8bit (pdsch.c:699-704): srsran_evm_run_b of the reference (evm.h, compiled into _ref)
    on the oracle chain's equalised symbols and int8 demodulated LLRs; rtol 5e-5 (summation order)."""
    kw = dict(PD8_CASES[case])
    rng = np.random.default_rng(700 + case)
    kw.pop("fail", False)
    nof_prb, cell_id, nports = kw.pop("nof_prb", 100), kw.pop("cell_id", 1), kw.pop("nports", 2)
    tti, cfi = kw.pop("tti", 1), kw.pop("cfi", 1)
    tbs, Qm = kw.pop("tbs", (TBS, TBS)), kw.pop("Qm", (6, 6))
    scheme, pmi = kw.pop("scheme", "cdd"), kw.pop("pmi", 0)
    pls, x, nre, grids, ce, st = _case(ora, rng, nof_prb, cell_id, nports, tti, cfi, tbs, Qm, scheme, pmi, **kw)
    ref = PC.pdsch_decode(ora, grids, ce, st["noise"], nof_prb, cell_id, nports, tti, cfi, 0x1234, list(tbs),
                          list(Qm), [0] * len(tbs), scheme=scheme, pmi=pmi, llr8=True)
    max_bits = max(U.lib().srsran_ra_tbs_from_idx(33, 6), U.lib().srsran_ra_tbs_from_idx(33, nof_prb))
    mods = {2: 1, 4: 2, 6: 3, 8: 4}
    R = Reference()
    want = [R.evm_b(mods[Qm[q]], r["sym"], r["demod"], nre * Qm[q], max_bits) for q, r in enumerate(ref)]
    sbs = [SCH.SoftbufferRx(nof_prb=nof_prb) for _ in tbs]
    cfg = U.pdsch_cfg(nof_prb, nre, tbs, Qm, scheme=scheme, pmi=pmi, softbuffers=sbs, meas_evm=True,
                      nof_ports=nports)
    pd = U.Pdsch(U.cell(nof_prb, nports, cell_id), grids.shape[0])
    pd.set_llr8(True)
    ret, _ = pd.decode(cfg, tti, cfi, grids, ce, st["noise"])
    assert ret == 0
    for q in range(len(tbs)):
        assert np.isfinite(want[q]) and pd.last_evm[q] == pytest.approx(want[q], rel=5e-5), q
    pd.free()


def test_ue_dl8_batch_decodes_and_llrs_agree(U, SCH, ora):
    """srsran_ue_dl_gpu_decode_batch with the 8-bit chain from time samples: every TB decodes, and the int8 LLRs
    (srsran_pdsch_gpu_last_llr) agree with the oracle chain's llr8 LLRs on the same samples (GPU FFT / estimator
    rounding differs, FFT parity unpinned: >= 99.9 % equal, |delta| <= 1)."""
    rng = np.random.default_rng(11)
    ue = U.UeDl(U.cell(100, 2, 1), 2)
    ue.set_llr8(True)
    ttis = (1, 5, 10)
    entries, samples, wants, keep = [], [], [], []
    d_pl = torch.zeros((len(ttis), 2, TBS // 8 + 64), dtype=torch.uint8, device="cuda")
    for b, tti in enumerate(ttis):
        pls, x, nre, grids, ce, st = _case(ora, rng, tti=tti)
        wants.append((pls, PC.pdsch_decode(ora, grids, ce, st["noise"], 100, 1, 2, tti, 1, 0x1234, [TBS, TBS], [6, 6],
                                           [0, 0], llr8=True)))
        sb = [SCH.SoftbufferRx(nof_prb=100) for _ in range(2)]
        cfg = U.pdsch_cfg(100, nre, (TBS, TBS), (6, 6), softbuffers=sb)
        keep += [sb, cfg]
        samples.append(x)
        entries.append((tti, 1, cfg, [d_pl[b, 0].data_ptr(), d_pl[b, 1].data_ptr()], [1, 1]))
    d_x = torch.from_numpy(np.stack(samples).view(np.float32)).cuda()
    d_res = torch.full((2 * len(ttis),), 7, dtype=torch.int32, device="cuda")
    d_avg = torch.zeros(2 * len(ttis), dtype=torch.float32, device="cuda")
    assert ue.gpu_decode_batch(entries, d_x.data_ptr(), d_res.data_ptr(), d_avg.data_ptr(), 0.0, None) == 2 * len(ttis)
    torch.cuda.synchronize()
    res, pl = d_res.cpu().numpy(), d_pl.cpu().numpy()
    for b in range(len(ttis)):
        pls, want = wants[b]
        for q in range(2):
            assert res[2 * b + q] == 0 and np.array_equal(pl[b, q, : TBS // 8], pls[q]), (b, q)
            d, n = ue.last_llr(b, q)
            assert n == want[q]["llr"].size
            got = torch.empty(n, dtype=torch.int8)
            SCH._memcpy_d2h(got, d, n)
            delta = np.abs(got.numpy().astype(np.int32) - want[q]["llr"].astype(np.int32))
            assert (delta == 0).mean() >= 0.999 and delta.max() <= 1, (b, q, (delta == 0).mean(), delta.max())
    ue.free()

