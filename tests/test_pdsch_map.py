"""CPU test of the PDSCH RE map (host code in srsran_4g_amd/csrc/pdsch_map.cpp, a restatement
of srsran_pdsch_cp, pdsch.c:136-220) against an independent rule-based restatement
(oracle/pdsch_np.py) and against the reference's own PRB copy routines (prb_dl.c compiled into
oracle/_ref, driven by oracle/ref_pdsch_map_harness.c): cells of 6..100 PRB (odd and even), 1/2/4
ports, normal and extended CP, all subframes, CFI 1..3, full and partial PRB allocations."""
import ctypes
import os

import numpy as np
import pytest

import oracle as ORA
import pdsch_np
from srsran_4g_amd import sch as S
from srsran_4g_amd import ue_dl as U


def product_table(nof_prb, nports, cell_id, mask, lstart, sf_idx, cp=0):
    cell = U.cell(nof_prb, nports, cell_id)
    cell.cp = cp
    g = S.srsran_pdsch_grant_t()
    g.nof_symb_slot[0] = g.nof_symb_slot[1] = 6 if cp else 7
    for s in range(2):
        for n in range(nof_prb):
            g.prb_idx[s][n] = bool(mask[s][n])
    f = S.lib().srsran_pdsch_re_table
    f.argtypes = [ctypes.POINTER(U.srsran_cell_t), ctypes.POINTER(S.srsran_pdsch_grant_t), ctypes.c_uint32,
                  ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
    f.restype = ctypes.c_int
    n = f(ctypes.byref(cell), ctypes.byref(g), lstart, sf_idx, None, 0)
    out = np.zeros(max(n, 1), np.uint32)
    f(ctypes.byref(cell), ctypes.byref(g), lstart, sf_idx, out.ctypes.data, n)
    return out[:n]


@pytest.mark.parametrize("nof_prb", [6, 15, 25, 50, 75, 100, 27])
@pytest.mark.parametrize("nports", [1, 2, 4])
def test_re_table_matches_rules(nof_prb, nports):
    rng = np.random.default_rng(nof_prb * 10 + nports)
    for sf_idx in range(10):
        for lstart in (1, 2, 3):
            full = [[1] * nof_prb, [1] * nof_prb]
            part = [list(rng.integers(0, 2, nof_prb))] * 2
            for mask in (full, part):
                cell_id = int(rng.integers(0, 504))
                got = product_table(nof_prb, nports, cell_id, mask, lstart, sf_idx)
                exp = pdsch_np.re_table(nof_prb, nports, cell_id, mask, lstart, sf_idx)
                assert len(got) == len(exp), (sf_idx, lstart)
                assert np.array_equal(got & 0x7FFFFFFF, [e[0] for e in exp])
                assert np.array_equal((got >> 31).astype(bool), [e[1] for e in exp])


def test_c3_grant_size():
    """100 PRB, 2 ports, CFI 1, subframe 1: 14400 PDSCH REs (SURVEY 8, C3 grant)."""
    got = product_table(100, 2, 1, [[1] * 100, [1] * 100], 1, 1)
    assert len(got) == 14400


@pytest.mark.parametrize("nof_prb", [6, 15, 25, 50, 100, 27])
@pytest.mark.parametrize("nports", [1, 2, 4])
def test_re_table_extended_cp(nof_prb, nports):
    """extended CP: 6 symbols a slot, CRS in l = 0 and 3 (SRSRAN_SYMBOL_HAS_REF), PSS / SSS in l = 4, 5
    of slot 0 and PBCH in l = 0..3 of slot 1 of the centre PRBs"""
    rng = np.random.default_rng(nof_prb * 10 + nports + 5)
    for sf_idx in range(10):
        for lstart in (1, 2, 3):
            full = [[1] * nof_prb, [1] * nof_prb]
            part = [list(rng.integers(0, 2, nof_prb))] * 2
            for mask in (full, part):
                cell_id = int(rng.integers(0, 504))
                got = product_table(nof_prb, nports, cell_id, mask, lstart, sf_idx, cp=1)
                exp = pdsch_np.re_table(nof_prb, nports, cell_id, mask, lstart, sf_idx, cp=1)
                assert len(got) == len(exp), (sf_idx, lstart)
                assert np.array_equal(got & 0x7FFFFFFF, [e[0] for e in exp])
                assert np.array_equal((got >> 31).astype(bool), [e[1] for e in exp])
                assert got.size == 0 or (got & 0x7FFFFFFF).max() < 12 * 12 * nof_prb


def ra_nof_re(nof_prb, nports, cell_id, mask, cfi, tti, cp):
    cell = U.cell(nof_prb, nports, cell_id)
    cell.cp = cp
    sf = U.srsran_dl_sf_cfg_t()
    sf.tti, sf.cfi = tti, cfi
    g = S.srsran_pdsch_grant_t()
    for s in range(2):
        for n in range(nof_prb):
            g.prb_idx[s][n] = bool(mask[s][n])
    f = S.lib().srsran_ra_dl_grant_nof_re
    f.argtypes = [ctypes.POINTER(U.srsran_cell_t), ctypes.POINTER(U.srsran_dl_sf_cfg_t),
                  ctypes.POINTER(S.srsran_pdsch_grant_t)]
    f.restype = ctypes.c_uint32
    return f(ctypes.byref(cell), ctypes.byref(sf), ctypes.byref(g))


@pytest.mark.parametrize("cp", [0, 1])
@pytest.mark.parametrize("nof_prb", [6, 25, 50, 100, 15, 75])
def test_ra_nof_re_matches_re_map(cp, nof_prb):
    """srsran_ra_dl_grant_nof_re (ra_dl.c:42-168 restated in dci_api.cpp) counts exactly the REs
    srsran_pdsch_cp walks (1 and 2 ports; srsran_pdsch_decode refuses a grant where they differ)"""
    rng = np.random.default_rng(nof_prb + 100 * cp)
    for nports in (1, 2):
        for tti in range(10):
            for cfi in (1, 2, 3):
                mask = [list(rng.integers(0, 2, nof_prb))] * 2 if tti % 2 else [[1] * nof_prb] * 2
                cell_id = int(rng.integers(0, 504))
                lstart = cfi + (1 if nof_prb < 10 else 0)
                if cp and lstart == 4:
                    # extended CP with 4 control symbols (6 PRB, CFI 3): both CRS symbols of slot 0 lie
                    # in the control region, yet ra_dl.c:126-131 still subtracts them (unsigned, so a
                    # PRB with no PDSCH symbol left wraps): the reference's own grant disagrees with
                    # srsran_pdsch_cp there, and srsran_pdsch_decode rejects such a grant
                    continue
                n_map = len(pdsch_np.re_table(nof_prb, nports, cell_id, mask, lstart, tti, cp=cp))
                assert ra_nof_re(nof_prb, nports, cell_id, mask, cfi, tti, cp) == n_map, (nports, tti, cfi)


def ref_table(nof_prb, nports, cell_id, mask, lstart, sf_idx, cp):
    R = ctypes.CDLL(ORA.REF_SO, mode=os.RTLD_LAZY)
    f = R.ref_pdsch_get_indices
    f.argtypes = [ctypes.c_uint32] * 6 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    f.restype = ctypes.c_int
    m = np.ascontiguousarray(np.asarray(mask, np.uint8).reshape(2, nof_prb))
    out = np.zeros(2 * 7 * 12 * nof_prb, np.uint32)
    n = f(nof_prb, nports, cell_id, cp, lstart, sf_idx, m.ctypes.data, out.ctypes.data, out.size)
    return out[:n]


@pytest.mark.skipif(not ORA.ref_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("cp", [0, 1])
@pytest.mark.parametrize("nof_prb", [6, 15, 25, 27, 50, 75, 100])
def test_re_table_matches_reference_prb_dl(cp, nof_prb):
    """pdsch_map.cpp == the reference's prb_cp_ref / prb_cp / prb_cp_half walk, index for index"""
    rng = np.random.default_rng(nof_prb + 7 * cp)
    for nports in (1, 2, 4):
        for sf_idx in range(10):
            for lstart in (1, 2, 3, 4):
                full = [[1] * nof_prb, [1] * nof_prb]
                part = [list(rng.integers(0, 2, nof_prb))] * 2
                for mask in (full, part):
                    cell_id = int(rng.integers(0, 504))
                    got = product_table(nof_prb, nports, cell_id, mask, lstart, sf_idx, cp=cp)
                    want = ref_table(nof_prb, nports, cell_id, mask, lstart, sf_idx, cp)
                    assert np.array_equal(got & 0x7FFFFFFF, want), (nports, sf_idx, lstart)
