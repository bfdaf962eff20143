"""Fixtures generated from the reference's compiled pieces (tests/golden/make_phy_golden.py):
the oracle (CPU) and the GPU path (through the C-ABI) against them.  Integer stages: equality.
Predecoding: the reference's SIMD bodies use rcp_ps approximations, so the oracle / GPU (exact
IEEE float) agree with them to 2e-3 relative (99.9th percentile) -- except TX diversity,
whose reference body is scalar and matches exactly."""
import os

import numpy as np
import pytest

from oracle import Oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "phy_golden.npz")


@pytest.fixture(scope="module")
def G():
    return np.load(GOLD)


@pytest.fixture(scope="module")
def ora():
    return Oracle()


def _keys(G, prefix, suffix):
    return sorted(k[: -len(suffix)] for k in G.files if k.startswith(prefix) and k.endswith(suffix))


def _check_pre(x, csi, G, p, scheme):
    xr, cr = G[p + "x"], G[p + "csi"]
    if scheme == 1:
        assert np.array_equal(x, xr) and np.array_equal(csi, cr)
        return
    err = np.abs(x - xr) / (np.abs(x) + 1e-3)
    assert np.percentile(err, 99.9) < 2e-3 and err.max() < 2e-2
    assert (np.abs(csi - cr) / np.abs(csi)).max() < 2e-3


# ---------------- oracle (CPU) ----------------
def test_oracle_demod(G, ora):
    for p in _keys(G, "demod_", "_in"):
        mod = int(p.split("_")[1][1:])
        assert np.array_equal(ora.demod_s(mod, G[p + "_in"]), G[p + "_out"]), p


def test_oracle_sequences(G, ora):
    for p in _keys(G, "seq_", "_in"):
        assert np.array_equal(ora.sequence_apply_s(G[p + "_in"], int(G[p + "_seed"][0])), G[p + "_out"]), p
    for p in _keys(G, "pdsch_seq_", "_in"):
        rnti, q, ns, cell = (int(v) for v in G[p + "_args"])
        seed = ora.pdsch_seed(rnti, q, ns, cell)
        assert np.array_equal(ora.sequence_apply_s(G[p + "_in"], seed), G[p + "_out"]), p


def test_oracle_predecoding(G, ora):
    for p in _keys(G, "pre_", "args"):
        scheme, nrx, nports, nl, cb = (int(v) for v in G[p + "args"])
        x, csi = ora.predecode(scheme, G[p + "y"], G[p + "h"], nl, cb, 1.0, 0.05)
        _check_pre(x, csi, G, p, scheme)


def test_oracle_rate_dematching(G, ora):
    from oracle import CB_SIZES
    for p in _keys(G, "rm_", "_e"):
        idx, rv = int(p.split("_")[1][1:]), int(p.split("_")[2][2:])
        K = CB_SIZES[idx]
        nsb = 16 if (K % 16 == 0 and K > 800) else 8 if (K % 8 == 0 and K > 400) else 0
        out = ora.rm_turbo_rx(K, rv, bool(nsb), G[p + "_e"], G[p + "_sb0"])
        assert np.array_equal(out, G[p + "_out"]), p


def test_oracle_decode_tb(G, ora):
    for p in _keys(G, "tb_", "_llr"):
        tbs, qm, rv, iters = (int(v) for v in G[p + "_args"])
        ret, data, noi, avg, _ = ora.dlsch_decode(tbs, qm, rv, G[p + "_llr"], iters)
        assert ret == int(G[p + "_ret"][0]), p
        assert np.array_equal(data, G[p + "_data"]), p
        assert avg == pytest.approx(float(G[p + "_avg"][0]), abs=1e-6), p


# ---------------- GPU (C-ABI) ----------------
@pytest.mark.gpu
def test_gpu_demod_sequences(G):
    from srsran_4g_amd import phch
    for p in _keys(G, "demod_", "_in"):
        mod = int(p.split("_")[1][1:])
        assert np.array_equal(phch.demod_s(mod, G[p + "_in"]), G[p + "_out"]), p
    for p in _keys(G, "seq_", "_in"):
        assert np.array_equal(phch.sequence_apply_s(G[p + "_in"], int(G[p + "_seed"][0])), G[p + "_out"]), p
    for p in _keys(G, "pdsch_seq_", "_in"):
        rnti, q, ns, cell = (int(v) for v in G[p + "_args"])
        assert np.array_equal(phch.sequence_pdsch_apply_s(G[p + "_in"], rnti, q, ns, cell), G[p + "_out"]), p


@pytest.mark.gpu
def test_gpu_predecoding(G):
    from srsran_4g_amd import phch
    for p in _keys(G, "pre_", "args"):
        scheme, nrx, nports, nl, cb = (int(v) for v in G[p + "args"])
        x, csi = phch.predecode(scheme, G[p + "y"], G[p + "h"], nl, cb, 1.0, 0.05)
        _check_pre(np.asarray(x), np.asarray(csi), G, p, scheme)


@pytest.mark.gpu
def test_gpu_rate_dematching(G):
    from srsran_4g_amd import sch
    for p in _keys(G, "rm_", "_e"):
        idx, rv = int(p.split("_")[1][1:]), int(p.split("_")[2][2:])
        ret, out = sch.rm_turbo_rx_lut(G[p + "_e"], G[p + "_sb0"], idx, rv)
        assert ret == 0 and np.array_equal(out, G[p + "_out"]), p


@pytest.mark.gpu
def test_gpu_decode_tb(G):
    from srsran_4g_amd import sch
    q = sch.Sch()
    for p in _keys(G, "tb_", "_llr"):
        tbs, qm, rv, iters = (int(v) for v in G[p + "_args"])
        q.set_max_noi(iters)
        sb = sch.SoftbufferRx(nof_prb=100)
        ret, data, avg = q.decode(sb, tbs, qm, rv, G[p + "_llr"])
        assert ret == int(G[p + "_ret"][0]), p
        n = G[p + "_data"].size
        assert np.array_equal(data[:n], G[p + "_data"]), p
        assert avg == pytest.approx(float(G[p + "_avg"][0]), abs=1e-6), p
        sb.free()
    q.free()
