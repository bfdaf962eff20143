"""NR shared-channel oracle pinned against the reference (CPU): LDPC code block segmentation, TB info
(incl. limited-buffer rate matching), LDPC rate de-matching with HARQ accumulation, and the whole
srsran_dlsch_nr_decode (decoded payload, TB CRC, average iterations, per-CB soft-buffer state) over
HARQ retransmissions, against lib/src/phy/phch/sch_nr.c compiled from the reference."""
import numpy as np
import pytest

from nr_sch import MAX_CB_SIZE, OracleNr, RefNr, new_state, ref_available

needs_ref = pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built")


@pytest.fixture(scope="module")
def ora():
    return OracleNr()


@pytest.fixture(scope="module")
def ref():
    return RefNr()


@needs_ref
def test_cbsegm_matches_reference(ora, ref):
    for bg in (0, 1):
        for tbs in list(range(8, 4000, 8))[::5] + [4008, 8424, 8448, 20000, 100000, 300000, 1213032]:
            assert ora.cbsegm(bg, tbs) == ref.cbsegm(bg, tbs), (bg, tbs)


@needs_ref
@pytest.mark.parametrize("lbrm", [False, True])
def test_tb_info_matches_reference(ora, ref, lbrm):
    rng = np.random.default_rng(4)
    for _ in range(60):
        Qm = int(rng.choice([2, 4, 6, 8]))
        Nl = int(rng.integers(1, 5))
        nof_prb = int(rng.choice([25, 52, 79, 106, 133, 162, 217, 273]))
        R = float(rng.uniform(0.1, 0.93))
        n_re = int(rng.integers(100, 12 * 13 * nof_prb))
        n_re = min(n_re, int(330000 / (R * Qm * Nl)))  # the reference holds at most 41 CBs (sch_nr.h:28)
        tbs = ref.tbs(n_re, R, Qm, Nl)
        G = n_re * Qm * Nl
        a = ora.tb_info(tbs, R, Qm, G, Nl, lbrm=lbrm, nof_prb=nof_prb, mcs256=Qm == 8).as_dict()
        assert a == ref.tb_info(tbs, R, Qm, G, Nl, lbrm=lbrm, nof_prb=nof_prb, mcs256=Qm == 8)


@needs_ref
def test_rm_rx_matches_reference(ora, ref):
    rng = np.random.default_rng(5)
    for it in range(60):
        bg = int(rng.integers(0, 2))
        ls = [2, 3, 16, 36, 104, 208, 384][it % 7]
        K, N = (22 if bg == 0 else 10) * ls, (66 if bg == 0 else 50) * ls
        Qm = [1, 2, 4, 6, 8][it % 5]
        E = Qm * int(rng.integers(1, 2 * N // Qm))
        F = int(rng.integers(0, K // 3))
        rv = int(rng.integers(0, 4))
        Nref = int(rng.integers(N // 2, N + 1)) if it % 3 == 0 else MAX_CB_SIZE
        e = rng.integers(-128, 128, E).astype(np.int8)
        init = rng.integers(-63, 64, N + 8).astype(np.int8)
        x, y = init.copy(), init.copy()
        assert ora.rm_rx(e, x, F, bg, ls, rv, Qm, Nref) == ref.rm_rx(e, y, F, bg, ls, rv, Qm, Nref)
        assert np.array_equal(x, y), it


def _llrs(rng, e, snr, amp=10.0):
    x = 1.0 - 2.0 * e
    y = x + 10 ** (-snr / 20) * rng.standard_normal(x.shape)
    return np.clip(np.round(amp * y), -127, 127).astype(np.int8)


# (N_re, R, Qm, layers, lbrm, nof_prb): BG1/BG2, C = 1 and C > 1, 16/24-bit TB CRC, LBRM
NR_CASES = [(400, 0.3, 2, 1, False, 52), (3000, 0.5, 4, 1, False, 52), (12 * 13 * 52, 0.6, 6, 2, False, 52),
            (12 * 12 * 106, 0.75, 6, 2, True, 106), (100, 0.2, 2, 1, False, 25), (12 * 12 * 100, 0.9, 8, 2, True, 273),
            (12 * 13 * 30, 0.2, 4, 1, True, 52)]


@needs_ref
@pytest.mark.parametrize("case", NR_CASES)
def test_decode_matches_reference(ora, ref, case):
    n_re, R, Qm, Nl, lbrm, nof_prb = case
    rng = np.random.default_rng(n_re)
    tbs = ref.tbs(n_re, R, Qm, Nl)
    G = n_re * Qm * Nl
    t = ora.tb_info(tbs, R, Qm, G, Nl, lbrm=lbrm, nof_prb=nof_prb, mcs256=Qm == 8)
    pl = rng.integers(0, 256, tbs // 8).astype(np.uint8)
    sb = ref.softbuffer()
    st = new_state(t.C)
    base = {2: -1.0, 4: 3.0, 6: 7.0, 8: 12.0}[Qm] + 6 * (R - 0.5)
    crcs = []
    for rv, d in ((0, -1.5), (2, 0.0), (3, 1.0), (1, 6.0)):
        e = ref.encode(tbs, R, Qm, G, Nl, rv, pl, lbrm=lbrm, nof_prb=nof_prb, mcs256=Qm == 8)
        llr = _llrs(rng, e, base + d)
        a = ref.decode(sb, tbs, R, Qm, G, Nl, rv, llr, max_iter=6, lbrm=lbrm, nof_prb=nof_prb, mcs256=Qm == 8)
        b = ora.decode(t, rv, llr, st, max_iter=6)
        assert a[0] == b[0] and a[1] == pytest.approx(b[1], abs=1e-6), (rv, a[:2], b[:2])
        if a[0]:
            assert np.array_equal(a[2], b[2]) and np.array_equal(a[2], pl)
        for r in range(t.C):
            ok, buf, data = sb.get(r)
            assert ok == st["cb_crc"][r], (rv, r)
            assert np.array_equal(buf, st["softbuf"][r]), (rv, r)
            if ok:
                n = (t.Kp - t.L_cb + 7) // 8
                assert np.array_equal(data[:n], st["cb_data"][r][:n]), (rv, r)
        crcs.append(a[0])
    sb.free()
    assert crcs[-1] == 1  # the last, clean retransmission always decodes
