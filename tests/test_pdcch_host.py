"""PDCCH / PCFICH host side and oracle, no GPU: the library's REG tables and search spaces against
the reference's regs.c / pdcch.c compiled into oracle/_ref, the Viterbi / rate-matching
restatement (oracle/pdcch_oracle.c) against the reference's AVX2 16-bit decoder, DCI sizes and
unpacking, and the DCI -> PDSCH grant."""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pdcch as P  # noqa: E402  (oracle/pdcch.py)
from srsran_4g_amd import pdcch as PD  # noqa: E402

needs_ref = pytest.mark.skipif(not P.ref_available(), reason="oracle/_ref not built")

CELLS = [(100, 2, 1, 2), (50, 1, 7, 0), (25, 2, 300, 1), (6, 1, 2, 3), (75, 2, 101, 2), (15, 1, 44, 1),
         (100, 1, 503, 3), (50, 2, 5, 0), (6, 2, 11, 2), (100, 2, 0, 0), (100, 4, 1, 2), (50, 4, 7, 0), (6, 4, 2, 3),
         (25, 4, 301, 1), (15, 4, 44, 3)]


@needs_ref
@pytest.mark.parametrize("nprb,nports,cid,ng", CELLS)
def test_regs_tables_match_reference(nprb, nports, cid, ng):
    ref = P.Ref()
    pc, pd = ref.regs_tables(nprb, nports, cid, 0, ng)
    r = PD.Regs(PD.cell(nprb, nports, cid, 0, ng))
    try:
        assert np.array_equal(r.pcfich_re(), pc)
        for cfi in (1, 2, 3):
            assert np.array_equal(r.pdcch_re(cfi), pd[cfi - 1]), cfi
    finally:
        r.free()


@needs_ref
@pytest.mark.parametrize("nprb,nports,cid,ng", CELLS)
def test_regs_tables_extended_cp_match_reference(nprb, nports, cid, ng):
    """extended-CP cells (regs.c:587-617: symbol 3 of the 4-symbol control region carries CRS)"""
    ref = P.Ref()
    ref.set_cp(1)
    try:
        pc, pd = ref.regs_tables(nprb, nports, cid, 0, ng)
    finally:
        ref.set_cp(0)
    r = PD.Regs(PD.cell(nprb, nports, cid, 0, ng, cp=1))
    try:
        assert np.array_equal(r.pcfich_re(), pc)
        for cfi in (1, 2, 3):
            assert np.array_equal(r.pdcch_re(cfi), pd[cfi - 1]), cfi
    finally:
        r.free()


@needs_ref
@pytest.mark.parametrize("mi", [0, 2])
@pytest.mark.parametrize("nprb,nports,cid,ng", CELLS[:8])
def test_regs_tables_phich_mi_match_reference(nprb, nports, cid, ng, mi):
    """srsran_regs_init_opts with PHICH m_i 0 / 2 (srsran_ue_dl_set_mi_manual's tables)"""
    ref = P.Ref()
    pc, pd = ref.regs_tables(nprb, nports, cid, 0, ng, phich_mi=mi)
    r = PD.Regs(PD.cell(nprb, nports, cid, 0, ng), phich_mi=mi)
    try:
        assert np.array_equal(r.pcfich_re(), pc)
        for cfi in (1, 2, 3):
            assert np.array_equal(r.pdcch_re(cfi), pd[cfi - 1]), cfi
    finally:
        r.free()


EXT_CELLS = [(100, 2, 1, 2), (50, 1, 7, 3), (25, 2, 300, 1), (6, 1, 2, 3), (75, 2, 101, 2), (15, 4, 44, 3),
             (100, 4, 503, 0), (6, 2, 11, 2)]


@needs_ref
@pytest.mark.parametrize("sf1_6", [False, True])
@pytest.mark.parametrize("mi", [0, 1, 2])
@pytest.mark.parametrize("nprb,nports,cid,ng", EXT_CELLS)
def test_regs_tables_extended_phich_match_reference(nprb, nports, cid, ng, mi, sf1_6):
    """extended PHICH duration (regs.c:249-350): the PHICH spread over symbols 0-2, or over symbols 0-1 in MBSFN /
    TDD subframe 1 and 6 tables (srsran_regs_init_opts(..., mbsfn_or_sf1_6_tdd), ue_dl.c:59-64, 198) -- the REGs left
    to the PCFICH / PDCCH equal the reference's for every CFI"""
    ref = P.Ref()
    pc, pd = ref.regs_tables(nprb, nports, cid, 1, ng, phich_mi=mi, sf1_6=sf1_6)
    c = PD.cell(nprb, nports, cid, 1, ng)
    r = PD.Regs(c, phich_mi=mi, sf1_6=sf1_6)
    try:
        assert np.array_equal(r.pcfich_re(), pc)
        for cfi in (1, 2, 3):
            assert np.array_equal(r.pdcch_re(cfi), pd[cfi - 1]), cfi
    finally:
        r.free()
    if mi and ng:  # the tables differ from the normal-duration ones: the PHICH left symbol 0 for symbols 1-2
        rn = PD.Regs(PD.cell(nprb, nports, cid, 0, ng), phich_mi=mi)
        try:
            assert not np.array_equal(rn.pdcch_re(3), pd[2])
        finally:
            rn.free()


@needs_ref
def test_viterbi_and_rm_conv_restatement_match_reference():
    ref, ora = P.Ref(), P.Ora()
    rng = np.random.default_rng(11)
    for trial in range(200):
        fl = int(rng.integers(20, 144))
        if trial % 3 == 0:  # pure noise: every tie-break and wrap of the metrics matters
            x = (rng.standard_normal(3 * fl) * 3).astype(np.float32)
        else:
            bits = rng.integers(0, 2, 3 * fl)
            x = ((2.0 * bits - 1) + rng.standard_normal(3 * fl) * (0.3 + 0.3 * (trial % 5))).astype(np.float32)
        assert np.array_equal(ref.viterbi_decode_f(x, fl), ora.viterbi_decode_f(x, fl)), trial
    for trial in range(100):
        nb = int(rng.integers(8, 112))
        E = 72 << int(rng.integers(0, 4))
        x = (rng.standard_normal(E) * 2).astype(np.float32)
        assert np.array_equal(ref.rm_conv_rx(x, 3 * (nb + 16)), ora.rm_conv_rx(x, 3 * (nb + 16))), trial


@needs_ref
def test_search_spaces_match_reference():
    """srsran_pdcch_ue_locations_ncce / common_locations_ncce vs pdcch.c compiled into _ref"""
    L = ctypes.CDLL(P.REF_SO, mode=os.RTLD_LAZY)
    LocArr = PD.srsran_dci_location_t * 22
    L.srsran_pdcch_ue_locations_ncce.argtypes = [ctypes.c_uint32, LocArr, ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_uint16]
    L.srsran_pdcch_ue_locations_ncce.restype = ctypes.c_uint32
    L.srsran_pdcch_common_locations_ncce.argtypes = [ctypes.c_uint32, LocArr, ctypes.c_uint32]
    L.srsran_pdcch_common_locations_ncce.restype = ctypes.c_uint32
    rng = np.random.default_rng(5)
    for _ in range(300):
        ncce, sf, rnti = int(rng.integers(2, 88)), int(rng.integers(0, 10)), int(rng.integers(11, 0xFFF3))
        a = LocArr()
        n = L.srsran_pdcch_ue_locations_ncce(ncce, a, 16, sf, rnti)
        assert PD.ue_locations(ncce, sf, rnti) == [(a[i].L, a[i].ncce) for i in range(n)]
        n = L.srsran_pdcch_common_locations_ncce(ncce, a, 6)
        assert PD.common_locations(ncce) == [(a[i].L, a[i].ncce) for i in range(n)]


@needs_ref
def test_dci_sizes_match_harness_restatement():
    """the library's sizes (dci_api.cpp) vs the harness's (ref_pdcch_harness.c), both from dci.c"""
    L = ctypes.CDLL(P.REF_SO, mode=os.RTLD_LAZY)
    L.srsran_dci_format_sizeof.argtypes = [ctypes.POINTER(PD.srsran_cell_t), ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int]
    L.srsran_dci_format_sizeof.restype = ctypes.c_uint32
    for nprb in (6, 15, 25, 50, 75, 100, 12, 27, 64, 81):
        for ports in (1, 2):
            c = PD.cell(nprb, ports, 1)
            for f in (P.FORMAT0, P.FORMAT1, P.FORMAT1A, P.FORMAT2, P.FORMAT2A):
                assert PD.dci_size(c, f) == L.srsran_dci_format_sizeof(ctypes.byref(c), None, None, f), (nprb, f)


def test_dci_sizes_known_values():
    """36.212 5.3.3.1 sizes for 20 MHz / 1.4 MHz FDD, 2 ports (1A padded to format 0, 1 and 2A
    off the ambiguous sizes)"""
    c = PD.cell(100, 2, 1)
    assert [PD.dci_size(c, f) for f in (P.FORMAT0, P.FORMAT1A, P.FORMAT1, P.FORMAT2, P.FORMAT2A, P.FORMAT1C)] == \
        [28, 28, 39, 51, 48, 15]
    c = PD.cell(6, 2, 1)
    assert [PD.dci_size(c, f) for f in (P.FORMAT0, P.FORMAT1A, P.FORMAT1, P.FORMAT2, P.FORMAT2A)] == [21, 21, 19, 31, 28]


def test_dci_unpack_round_trip_and_grant():
    c = PD.cell(100, 2, 1)
    n2a = PD.dci_size(c, P.FORMAT2A)
    bits = P.dci_pack_2a(100, n2a, (1 << 25) - 1, [(28, 1, 0), (28, 0, 2)], pid=5, swap=1)
    r, d = PD.unpack_pdsch(c, bits, P.FORMAT2A, 0x1234)
    assert r == 0 and d.alloc_type == 0 and d.type0_rbg_bitmask == (1 << 25) - 1 and d.pid == 5 and d.tb_cw_swap
    assert (d.tb[0].mcs_idx, d.tb[0].ndi, d.tb[0].rv, d.tb[0].cw_idx) == (28, True, 0, 1)
    assert (d.tb[1].mcs_idx, d.tb[1].ndi, d.tb[1].rv, d.tb[1].cw_idx) == (28, False, 2, 0)
    r, g = PD.dci_to_grant(c, d, 3, 1, 2)  # TM3, CFI 1, subframe 3
    assert r == 0 and g.nof_tb == 2 and g.nof_prb == 100 and g.tx_scheme == 3 and g.nof_layers == 2
    from synth import synth as S
    assert g.tb[0].tbs == 75376 and g.tb[1].tbs == 75376 and g.nof_re == int(S.pdsch_mask(100, 2, 1, 1, 3).sum())
    for sf, cfi in ((0, 2), (5, 3), (1, 3)):  # PBCH / sync subframes: ra_re_x_prb vs the RE mask
        r, g = PD.dci_to_grant(c, d, sf, cfi, 2)
        assert r == 0 and g.nof_re == int(S.pdsch_mask(100, 2, 1, cfi, sf).sum()), (sf, cfi)
    # format 1A, localized RIV, C-RNTI
    n1a = PD.dci_size(c, P.FORMAT1A)
    riv = P.riv(10, 20, 100)
    bits = P.dci_pack_1a(100, n1a, riv, 9, 2, 1, 3)
    r, d = PD.unpack_pdsch(c, bits, P.FORMAT1A, 0x4601)
    assert r == 0 and d.alloc_type == 2 and d.pid == 2 and (d.tb[0].mcs_idx, d.tb[0].ndi, d.tb[0].rv) == (9, True, 3)
    r, g = PD.dci_to_grant(c, d, 1, 2, 2)
    assert r == 0 and g.nof_prb == 10 and list(np.nonzero(np.array(g.prb_idx[0][:100]))[0]) == list(range(20, 30))
    assert g.tb[0].tbs == PD.lib().srsran_ra_tbs_from_idx(9, 10) and g.tx_scheme == 1  # TM3, 1 TB -> diversity
    # format 1 type 0, 50 PRB, every other RBG
    c50 = PD.cell(50, 1, 3)
    n1 = PD.dci_size(c50, P.FORMAT1)
    mask = int("10" * 8 + "1", 2)  # 17 RBGs of P = 3
    bits = P.dci_pack_1(50, n1, mask, 15, 1, 0, 1)
    r, d = PD.unpack_pdsch(c50, bits, P.FORMAT1, 0x100)
    assert r == 0 and d.type0_rbg_bitmask == mask and d.tb[0].mcs_idx == 15
    r, g = PD.dci_to_grant(c50, d, 2, 1, 0)
    assert r == 0 and g.nof_prb == 9 * 3 - 1  # the last RBG holds 2 PRBs


@pytest.mark.parametrize("nprb", [6, 15, 25, 50, 75, 100])
def test_dci_format0_unpack_round_trip(nprb):
    """srsran_dci_msg_unpack_pusch (dci.c:492-566, 1369-1395) on format 0 payloads packed field by field
    from 36.212 5.3.3.1.1 (oracle/pdcch.py dci_pack_0): hopping off / on (1 or 2 hopping bits by
    bandwidth), CIF, 2-bit CSI request, SRS request, RA type; a 1A flag is refused.  (dci.c includes the
    CMake-generated srsran.h and is not compiled into oracle/_ref: parity unpinned beyond this.)"""
    c = PD.cell(nprb, 2, 1)
    rng = np.random.default_rng(nprb)
    nriv = P.riv_nbits(nprb)
    for trial in range(40):
        cfg = PD.srsran_dci_cfg_t()
        kw = {}
        if trial % 4 == 1:
            cfg.cif_enabled = True
            kw["cif"] = int(rng.integers(0, 8))
        if trial % 5 == 2:
            cfg.multiple_csi_request_enabled = True
            kw["csi"] = int(rng.integers(0, 4))
        if trial % 6 == 3:
            cfg.srs_request_enabled = True
            kw["srs"] = int(rng.integers(0, 2))
        if trial % 7 == 4:
            cfg.ra_format_enabled = True
            kw["ra_type"] = int(rng.integers(0, 2))
        nh = 1 if nprb < 50 else 2
        hop = int(rng.integers(0, 1 << nh)) if trial % 2 else None
        riv = int(rng.integers(0, 1 << (nriv - (nh if hop is not None else 0))))
        mcs, ndi, tpc, dmrs, cqi = (int(rng.integers(0, 32)), int(rng.integers(0, 2)), int(rng.integers(0, 4)),
                                    int(rng.integers(0, 8)), int(rng.integers(0, 2)))
        size = PD.dci_size(c, P.FORMAT0, cfg)
        bits = P.dci_pack_0(nprb, size, riv, mcs, ndi, tpc, dmrs, cqi, hop=hop, **kw)
        m = PD.srsran_dci_msg_t()
        m.payload[:size] = [int(b) for b in bits]
        m.nof_bits, m.format, m.rnti = size, P.FORMAT0, 0x4601
        m.location.L, m.location.ncce = 2, 8
        r, d = PD.unpack_pusch(c, m, cfg)
        assert r == 0
        assert (d.rnti, d.format, d.location.L, d.location.ncce) == (0x4601, P.FORMAT0, 2, 8)
        assert d.type2_alloc.riv == riv and d.tb.mcs_idx == mcs and d.tb.ndi == bool(ndi)
        assert d.tpc_pusch == tpc and d.n_dmrs == dmrs
        assert d.freq_hop_fl == (-1 if hop is None else hop)
        assert (d.cif_present, d.cif) == ((True, kw["cif"]) if "cif" in kw else (False, 0))
        if "csi" in kw:
            assert d.multiple_csi_request_present and d.multiple_csi_request == kw["csi"] and not d.cqi_request
        else:
            assert not d.multiple_csi_request_present and d.cqi_request == bool(cqi)
        assert (d.srs_request_present, d.srs_request) == ((True, bool(kw["srs"])) if "srs" in kw else (False, False))
        assert (d.ra_type_present, d.ra_type) == ((True, kw["ra_type"]) if "ra_type" in kw else (False, 0))
    # the 0/1A flag set: format 1A, refused
    m = PD.srsran_dci_msg_t()
    m.payload[0], m.nof_bits = 1, PD.dci_size(c, P.FORMAT0)
    assert PD.unpack_pusch(c, m)[0] != 0
