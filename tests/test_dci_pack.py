"""DCI packing (the eNB side of srsran_enb_dl_put_pdcch_dl / _ul): srsran_dci_msg_pack_pdsch / _pusch
(dci.c:415-490, 579-639, 710-795, 952-988, 1076-1151, 1243-1367) against

  * the reference's own test (phch/test/dci_test.c: a format 1A PDCCH order on a 52-PRB cell packed and
    unpacked back to the same fields),
  * the field-by-field 36.212 5.3.3.1 packers of oracle/pdcch.py (formats 0, 1, 2A), bit for bit,
  * pack -> srsran_dci_msg_unpack_* round trips of every format both directions provide, over cell
    sizes 6..100 PRB, both allocation types, C-RNTI / SI-RNTI format 1A, hopping format 0,
  * srsran_pbch_mib_pack's 24 bits (pbch.c) on hand-checked MIBs.

Host code only (no GPU)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pdcch as OP  # noqa: E402  (oracle/pdcch.py)
from srsran_4g_amd import pdcch as PD  # noqa: E402

F0, F1, F1A, F1B, F1C, F1D, F2, F2A, F2B = range(9)
LOC, DIST = 0, 1
ALLOC0, ALLOC1, ALLOC2 = 0, 1, 2


def _cell(nprb, ports=1, cell_id=0):
    return PD.cell(nprb, ports, cell_id)


def _dl(rnti, fmt, **kw):
    d = PD.srsran_dci_dl_t()
    d.rnti, d.format = rnti, fmt
    for i in range(2):
        d.tb[i].rv = 1  # disabled second TB unless set
    for k, v in kw.items():
        setattr(d, k, v)
    return d


def _type2(d, riv, mode=LOC, n_gap=0, n_prb1a=0):
    d.alloc_type = ALLOC2
    d.raw[0], d.raw[1], d.raw[2], d.raw[3] = riv, n_prb1a, n_gap, mode


def _type1(d, vrb_bitmask, subset, shift):
    d.alloc_type = ALLOC1
    d.raw[0], d.raw[1], d.raw[2] = vrb_bitmask, subset, 1 if shift else 0


def test_reference_pdcch_order_round_trip():
    """dci_test.c test_pdcch_orders: format 1A PDCCH order, 52 PRB, C-RNTI 0x1234"""
    c = _cell(52)
    d = _dl(0x1234, F1A, is_pdcch_order=True, preamble_idx=0, prach_mask_idx=0)
    r, m = PD.pack_pdsch(c, d)
    assert r == 0 and m.nof_bits == PD.dci_size(c, F1A)
    r, u = PD.unpack_pdsch(c, list(m.payload[:m.nof_bits]), F1A, 0x1234)
    assert r == 0 and u.is_pdcch_order and u.preamble_idx == 0 and u.prach_mask_idx == 0
    # a non-zero preamble / mask as well
    d = _dl(0x1234, F1A, is_pdcch_order=True, preamble_idx=37, prach_mask_idx=9)
    r, m = PD.pack_pdsch(c, d)
    r, u = PD.unpack_pdsch(c, list(m.payload[:m.nof_bits]), F1A, 0x1234)
    assert r == 0 and u.is_pdcch_order and u.preamble_idx == 37 and u.prach_mask_idx == 9


@pytest.mark.parametrize("nprb", [6, 15, 25, 50, 75, 100])
def test_format0_matches_field_packer_and_round_trips(nprb):
    rng = np.random.default_rng(nprb)
    c = _cell(nprb)
    size = PD.dci_size(c, F0)
    nb = OP.riv_nbits(nprb)
    for trial in range(24):
        hop = None if trial % 3 == 0 else int(rng.integers(0, 2 if nprb < 50 else 4))
        nh = 0 if hop is None else (1 if nprb < 50 else 2)
        riv = int(rng.integers(0, 1 << (nb - nh)))
        mcs, ndi, tpc, dmrs, cqi = (int(rng.integers(0, 32)), int(rng.integers(0, 2)), int(rng.integers(0, 4)),
                                    int(rng.integers(0, 8)), int(rng.integers(0, 2)))
        d = PD.srsran_dci_ul_t()
        d.rnti, d.format = 0x4601, F0
        d.freq_hop_fl = -1 if hop is None else hop
        d.type2_alloc.riv = riv
        d.tb.mcs_idx, d.tb.ndi, d.tpc_pusch, d.n_dmrs, d.cqi_request = mcs, bool(ndi), tpc, dmrs, bool(cqi)
        r, m = PD.pack_pusch(c, d)
        assert r == 0 and m.nof_bits == size
        want = OP.dci_pack_0(nprb, size, riv, mcs, ndi, tpc, dmrs, cqi, hop=hop)
        assert np.array_equal(np.array(m.payload[:size], np.uint8), want), trial
        r, u = PD.unpack_pusch(c, m)
        assert r == 0
        assert (u.type2_alloc.riv, u.tb.mcs_idx, bool(u.tb.ndi), u.tpc_pusch, u.n_dmrs, bool(u.cqi_request)) == \
            (riv, mcs, bool(ndi), tpc, dmrs, bool(cqi))
        assert u.freq_hop_fl == (-1 if hop is None else hop)


def test_format0_srs_and_csi_fields():
    c = _cell(50)
    cfg = PD.srsran_dci_cfg_t()
    cfg.srs_request_enabled = True
    cfg.multiple_csi_request_enabled = True
    d = PD.srsran_dci_ul_t()
    d.rnti, d.format, d.freq_hop_fl = 0x50, F0, -1
    d.type2_alloc.riv, d.tb.mcs_idx, d.cqi_request = 77, 12, True
    d.srs_request, d.srs_request_present = True, True
    r, m = PD.pack_pusch(c, d, cfg)
    size = PD.dci_size(c, F0, cfg)
    assert r == 0 and m.nof_bits == size
    want = OP.dci_pack_0(50, size, 77, 12, 0, csi=2, srs=1)  # the 2-bit CSI field: request bit, then 0
    assert np.array_equal(np.array(m.payload[:size], np.uint8), want)


@pytest.mark.parametrize("nprb", [6, 15, 25, 50, 100])
def test_format1_type0_matches_field_packer(nprb):
    rng = np.random.default_rng(100 + nprb)
    c = _cell(nprb)
    size = PD.dci_size(c, F1)
    nrbg = int(np.ceil(nprb / OP.type0_P(nprb)))
    for _ in range(16):
        mask, mcs, pid, ndi, rv = (int(rng.integers(0, 1 << nrbg)), int(rng.integers(0, 32)), int(rng.integers(0, 8)),
                                   int(rng.integers(0, 2)), int(rng.integers(0, 4)))
        d = _dl(0x4601, F1, alloc_type=ALLOC0, pid=pid)
        d.raw[0] = mask
        d.tb[0].mcs_idx, d.tb[0].ndi, d.tb[0].rv = mcs, bool(ndi), rv
        r, m = PD.pack_pdsch(c, d)
        assert r == 0 and m.nof_bits == size
        want = OP.dci_pack_1(nprb, size, mask, mcs, pid, ndi, rv)
        assert np.array_equal(np.array(m.payload[:size], np.uint8), want)
        r, u = PD.unpack_pdsch(c, list(m.payload[:size]), F1, 0x4601)
        assert r == 0 and u.raw[0] == mask and u.tb[0].mcs_idx == mcs and u.pid == pid and u.tb[0].rv == rv


@pytest.mark.parametrize("nprb", [15, 50, 100])
def test_format1_type1_round_trip(nprb):
    rng = np.random.default_rng(200 + nprb)
    c = _cell(nprb)
    P = OP.type0_P(nprb)
    lp = int(np.ceil(np.log2(P)))
    nbm = int(np.ceil(nprb / P)) - lp - 1
    for _ in range(12):
        vrb, sub, sh = int(rng.integers(0, 1 << nbm)), int(rng.integers(0, P)), bool(rng.integers(0, 2))
        d = _dl(0x4601, F1, pid=3)
        _type1(d, vrb, sub, sh)
        d.tb[0].mcs_idx, d.tb[0].rv = 9, 2
        r, m = PD.pack_pdsch(c, d)
        assert r == 0
        r, u = PD.unpack_pdsch(c, list(m.payload[:m.nof_bits]), F1, 0x4601)
        assert r == 0 and u.alloc_type == ALLOC1
        assert (u.raw[0], u.raw[1], bool(u.raw[2] & 0xff)) == (vrb, sub, sh)


@pytest.mark.parametrize("nprb", [6, 25, 50, 100])
@pytest.mark.parametrize("rnti", [0x4601, 0xFFFF])
def test_format1A_round_trip(nprb, rnti):
    rng = np.random.default_rng(nprb + rnti)
    c = _cell(nprb)
    nb = OP.riv_nbits(nprb)
    for trial in range(16):
        mode = DIST if (trial % 2 and nprb >= 50) else LOC
        n_gap = int(rng.integers(0, 2)) if mode == DIST else 0
        user = rnti < 0xFFF4
        gap_bit = 1 if (user and mode == DIST and nprb >= 50) else 0
        riv = int(rng.integers(0, 1 << (nb - gap_bit)))
        d = _dl(rnti, F1A, pid=int(rng.integers(0, 8)))
        _type2(d, riv, mode, n_gap, n_prb1a=int(rng.integers(0, 2)) if not user else 0)
        d.tb[0].mcs_idx, d.tb[0].rv = int(rng.integers(0, 32)), int(rng.integers(0, 4))
        d.tb[0].ndi = bool(rng.integers(0, 2)) if user else False
        r, m = PD.pack_pdsch(c, d)
        assert r == 0 and m.nof_bits == PD.dci_size(c, F1A)
        r, u = PD.unpack_pdsch(c, list(m.payload[:m.nof_bits]), F1A, rnti)
        assert r == 0 and not u.is_pdcch_order
        assert (u.raw[0], u.raw[3], u.tb[0].mcs_idx, u.tb[0].rv, u.pid) == (riv, mode, d.tb[0].mcs_idx, d.tb[0].rv, d.pid)
        if mode == DIST and nprb >= 50:
            assert u.raw[2] == n_gap
        if user:
            assert bool(u.tb[0].ndi) == bool(d.tb[0].ndi)
        else:
            assert u.raw[1] == d.raw[1]  # N_PRB^1A


@pytest.mark.parametrize("ports", [2, 4])
@pytest.mark.parametrize("fmt", [F2, F2A])
def test_format2x_matches_field_packer_and_round_trips(ports, fmt):
    rng = np.random.default_rng(ports * 10 + fmt)
    for nprb in (25, 50, 100):
        c = _cell(nprb, ports)
        size = PD.dci_size(c, fmt)
        nrbg = int(np.ceil(nprb / OP.type0_P(nprb)))
        pbits = (3 if ports <= 2 else 6) if fmt == F2 else (0 if ports <= 2 else 2)
        for _ in range(8):
            mask, pid, swap = int(rng.integers(0, 1 << nrbg)), int(rng.integers(0, 8)), int(rng.integers(0, 2))
            tbs = [(int(rng.integers(0, 29)), int(rng.integers(0, 2)), int(rng.integers(0, 4))) for _ in range(2)]
            pinfo = int(rng.integers(0, 1 << pbits)) if pbits else 0
            d = _dl(0x4601, fmt, alloc_type=ALLOC0, pid=pid, tb_cw_swap=bool(swap), pinfo=pinfo)
            d.raw[0] = mask
            for i, (mcs, ndi, rv) in enumerate(tbs):
                d.tb[i].mcs_idx, d.tb[i].ndi, d.tb[i].rv = mcs, bool(ndi), rv
            r, m = PD.pack_pdsch(c, d)
            assert r == 0 and m.nof_bits == size
            want = OP.dci_pack_2a(nprb, size, mask, tbs, pid, swap=swap, pinfo=pinfo, pinfo_bits=pbits)
            assert np.array_equal(np.array(m.payload[:size], np.uint8), want)
            r, u = PD.unpack_pdsch(c, list(m.payload[:size]), fmt, 0x4601)
            assert r == 0 and u.raw[0] == mask and u.pid == pid and u.pinfo == pinfo
            assert [(u.tb[i].mcs_idx, bool(u.tb[i].ndi), u.tb[i].rv) for i in range(2)] == \
                [(a, bool(b), e) for a, b, e in tbs]


@pytest.mark.parametrize("nprb", [25, 100])
def test_format2B_round_trip(nprb):
    """format 2B (dci.c:1076-1151 / 1153-1245): the scrambling identity in the swap flag's place, no precoding
    field; the swap flag itself is left as the caller had it"""
    rng = np.random.default_rng(nprb + 2)
    c = _cell(nprb, 2)
    size = PD.dci_size(c, F2B)
    assert size == PD.dci_size(c, F2A)  # 2 ports: format 2A carries no precoding bits either
    nrbg = int(np.ceil(nprb / OP.type0_P(nprb)))
    for _ in range(8):
        mask, pid, sram = int(rng.integers(0, 1 << nrbg)), int(rng.integers(0, 8)), bool(rng.integers(0, 2))
        d = _dl(0x4601, F2B, alloc_type=ALLOC0, pid=pid, sram_id=sram)
        d.raw[0] = mask
        d.tb[0].mcs_idx, d.tb[0].rv, d.tb[1].mcs_idx, d.tb[1].rv = 11, 0, 20, 2
        r, m = PD.pack_pdsch(c, d)
        assert r == 0 and m.nof_bits == size
        # the same bits as a format 2A message whose swap flag carries the identity
        want = OP.dci_pack_2a(nprb, size, mask, [(11, 0, 0), (20, 0, 2)], pid, swap=int(sram), pinfo=0, pinfo_bits=0)
        assert np.array_equal(np.array(m.payload[:size], np.uint8), want)
        r, u = PD.unpack_pdsch(c, list(m.payload[:size]), F2B, 0x4601)
        assert r == 0 and u.raw[0] == mask and u.pid == pid and bool(u.sram_id) == sram and not u.tb_cw_swap
        assert (u.tb[0].mcs_idx, u.tb[1].mcs_idx, u.tb[1].rv) == (11, 20, 2)


@pytest.mark.parametrize("nprb", [6, 25, 50, 100])
def test_format1C_size(nprb):
    c = _cell(nprb)
    d = _dl(0xFFFF, F1C)
    _type2(d, 5, DIST, 0)
    d.tb[0].mcs_idx = 7
    r, m = PD.pack_pdsch(c, d)
    assert r == 0 and m.nof_bits == PD.dci_size(c, F1C)
    # type 2 localized is refused, as dci.c:968-971
    _type2(d, 5, LOC, 0)
    assert PD.pack_pdsch(c, d)[0] != 0


def test_wrong_allocation_types_refused():
    c = _cell(25)
    d = _dl(0x4601, F1A, alloc_type=ALLOC0)
    assert PD.pack_pdsch(c, d)[0] != 0
    d = _dl(0x4601, F1)
    _type2(d, 3)
    assert PD.pack_pdsch(c, d)[0] != 0


@pytest.mark.parametrize("nprb,phich_len,phich_res,sfn,want", [
    (100, 0, 2, 1023, "101" + "0" + "10" + "11111111" + "0" * 10),
    (6, 1, 0, 4, "000" + "1" + "00" + "00000001" + "0" * 10),
    (15, 0, 3, 517, "001" + "0" + "11" + "10000001" + "0" * 10),
    (50, 0, 1, 0, "011" + "0" + "01" + "00000000" + "0" * 10),
])
def test_mib_pack(nprb, phich_len, phich_res, sfn, want):
    from srsran_4g_amd import enb_dl as E
    c = PD.cell(nprb, 1, 1, phich_len=phich_len, phich_res=phich_res)
    assert "".join(str(b) for b in E.mib_pack(c, sfn)) == want


def _tdd_cell(nprb, ports=1, cell_id=0):
    c = PD.cell(nprb, ports, cell_id)
    c.frame_type = 1  # SRSRAN_TDD
    return c


def _sf(tti, sf_config=1, ss_config=7):
    from srsran_4g_amd import ue_dl as U
    return U.sf_cfg(tti, 1, (sf_config, ss_config))


@pytest.mark.parametrize("nprb", [6, 15, 25, 50, 75, 100])
def test_tdd_sizes(nprb):
    """TDD DCI sizes (dci.c:93-413): 4-bit HARQ process numbers and the 2-bit DAI / UL index -- format 0 and 1A
    grow by 2 / 3 bits before the 0 / 1A alignment, formats 1 / 2 / 2A by 3 bits before the ambiguity padding;
    at 100 PRB formats 0 / 1A are 31 bits (28 FDD)"""
    f, t = _cell(nprb), _tdd_cell(nprb)
    f0, f1a, t0, t1a = PD.dci_size(f, F0), PD.dci_size(f, F1A), PD.dci_size(t, F0), PD.dci_size(t, F1A)
    assert f0 == f1a and t0 == t1a and t1a >= f1a + 2
    if nprb == 100:
        assert (f1a, t1a) == (28, 31)
    nb = OP.riv_nbits(nprb)
    raw1a = 1 + 1 + nb + 5 + 4 + 1 + 2 + 2 + 2
    raw0 = 1 + 1 + nb + 5 + 1 + 2 + 3 + 2 + 1 + 1
    exp = max(raw1a, raw0)
    exp += 1 if exp in (12, 14, 16, 20, 24, 26, 32, 40, 44, 56) else 0
    assert t1a == exp
    for fmt in (F1, F2, F2A):
        if fmt != F1 and nprb < 50:
            continue
        n = PD.dci_size(t, fmt)
        assert n not in (12, 14, 16, 20, 24, 26, 32, 40, 44, 56) and n >= PD.dci_size(f, fmt) + 2


@pytest.mark.parametrize("nprb", [6, 25, 100])
def test_tdd_format1_1A_round_trip(nprb):
    """formats 1 and 1A on a TDD cell: 4-bit HARQ process numbers survive pack -> unpack; the reference's packers
    write no DAI (it stays in the zero padding), so the unpacked DAI is 0 and is_tdd is set"""
    rng = np.random.default_rng(7 * nprb)
    c = _tdd_cell(nprb)
    nrbg = int(np.ceil(nprb / OP.type0_P(nprb)))
    nb = OP.riv_nbits(nprb)
    for _ in range(12):
        pid = int(rng.integers(0, 16))
        d = _dl(0x4601, F1, alloc_type=ALLOC0, pid=pid)
        d.raw[0] = int(rng.integers(0, 1 << nrbg))
        d.tb[0].mcs_idx, d.tb[0].rv = int(rng.integers(0, 29)), int(rng.integers(0, 4))
        r, m = PD.pack_pdsch(c, d)
        assert r == 0 and m.nof_bits == PD.dci_size(c, F1)
        r, u = PD.unpack_pdsch(c, list(m.payload[:m.nof_bits]), F1, 0x4601)
        assert r == 0 and u.pid == pid and u.raw[0] == d.raw[0] and u.is_tdd and u.dai == 0
        d = _dl(0x4601, F1A, pid=pid)
        _type2(d, int(rng.integers(0, 1 << nb)))
        d.tb[0].mcs_idx = int(rng.integers(0, 29))
        r, m = PD.pack_pdsch(c, d)
        assert r == 0 and m.nof_bits == PD.dci_size(c, F1A)
        r, u = PD.unpack_pdsch(c, list(m.payload[:m.nof_bits]), F1A, 0x4601)
        assert r == 0 and u.pid == pid and u.raw[0] == d.raw[0] and u.is_tdd and u.dai == 0


def _bits(v, n):
    return [(v >> (n - 1 - i)) & 1 for i in range(n)]


@pytest.mark.parametrize("sf_config", [0, 1])
def test_tdd_format0_unpack_dai_ul_index(sf_config):
    """format 0 on a TDD cell (dci.c:535-548): after the DMRS cyclic shift, the 2-bit UL index (uplink-downlink
    configuration 0) or DAI (the others), then the CSI request -- from a hand-built 36.212 5.3.3.1.1 payload"""
    nprb = 50
    c = _tdd_cell(nprb)
    nb = OP.riv_nbits(nprb)
    riv, mcs, ndi, tpc, dmrs, v2, cqi = 777, 21, 1, 2, 5, 3, 1
    bits = [0, 0] + _bits(riv, nb) + _bits(mcs, 5) + [ndi] + _bits(tpc, 2) + _bits(dmrs, 3) + _bits(v2, 2) + [cqi]
    size = PD.dci_size(c, F0)
    bits += [0] * (size - len(bits))
    m = PD.srsran_dci_msg_t()
    m.payload[:size] = bits
    m.nof_bits, m.format, m.rnti = size, F0, 0x4601
    d = PD.srsran_dci_ul_t()
    import ctypes
    sf = _sf(3, sf_config)
    r = PD.lib().srsran_dci_msg_unpack_pusch(ctypes.byref(c), ctypes.byref(sf), None, ctypes.byref(m), ctypes.byref(d))
    assert r == 0 and d.is_tdd
    assert (d.type2_alloc.riv, d.tb.mcs_idx, d.tpc_pusch, d.n_dmrs, bool(d.cqi_request)) == (riv, mcs, tpc, dmrs, True)
    assert (d.ul_idx, d.dai) == ((v2, 0) if sf_config == 0 else (0, v2))


def test_tdd_format2_dai_before_pid():
    """format 2 on a TDD cell unpacks the DAI between the TPC command and the HARQ process number (dci.c:1185-1200),
    and a DwPTS subframe sets is_dwpts (dci.c:1317-1319)"""
    import ctypes
    nprb, ports = 50, 2
    c = _tdd_cell(nprb, ports)
    P = OP.type0_P(nprb)
    nrbg = int(np.ceil(nprb / P))
    size = PD.dci_size(c, F2)
    mask, tpc, dai, pid = 0x155, 1, 2, 13
    bits = [0] + _bits(mask, nrbg) + _bits(tpc, 2) + _bits(dai, 2) + _bits(pid, 4) + [0]
    bits += _bits(17, 5) + [1] + _bits(2, 2) + _bits(9, 5) + [0] + _bits(1, 2) + _bits(5, 3)
    bits += [0] * (size - len(bits))
    for tti, dwpts in ((4, False), (6, True)):  # configuration 1: subframe 6 is special
        m = PD.srsran_dci_msg_t()
        m.payload[:size] = bits
        m.nof_bits, m.format, m.rnti = size, F2, 0x4601
        d = PD.srsran_dci_dl_t()
        sf = _sf(tti, 1)
        r = PD.lib().srsran_dci_msg_unpack_pdsch(ctypes.byref(c), ctypes.byref(sf), None, ctypes.byref(m),
                                                 ctypes.byref(d))
        assert r == 0 and d.raw[0] == mask and d.tpc_pucch == tpc and d.dai == dai and d.pid == pid and d.is_tdd
        assert d.tb[0].mcs_idx == 17 and d.tb[1].mcs_idx == 9 and d.pinfo == 5
        assert bool(d.is_dwpts) == dwpts


def _grant(c, d, tti=1, cfi=1, tm=0):
    return PD.dci_to_grant(c, d, tti, cfi, tm)


@pytest.mark.parametrize("nprb", [6, 15, 25, 27, 50, 75, 100])
def test_distributed_vrb_grants(nprb):
    """type 2 distributed VRB allocations (format 1A with a C-RNTI, every RIV; N_gap,1 and, from 50 PRB, N_gap,2):
    srsran_ra_dl_dci_to_grant's per-slot PRBs equal the restatement of the reference's interleaver (ra_dl.c:225-316,
    36.211 6.2.3.2) in oracle/pdcch.py; where the reference refuses an allocation (a PRB beyond the cell) so does this"""
    c = _cell(nprb)
    for ngap1 in ((True,) if nprb < 50 else (True, False)):
        nvrb = OP.type2_n_vrb_dl(nprb, ngap1)
        for riv_v in range(0, nprb * (nprb + 1) // 2):
            L, st = OP.riv_decode(riv_v, nprb, nvrb)
            if L < 1 or st + L > nvrb:
                continue
            d = _dl(0x4601, F1A)
            _type2(d, riv_v, DIST, 0 if ngap1 else 1)
            d.tb[0].mcs_idx = 9
            r, g = _grant(c, d)
            want = OP.type2_prbs(nprb, riv_v, True, ngap1)
            if want is None:
                assert r != 0, riv_v
                continue
            assert r == 0, riv_v
            for s in range(2):
                assert [n for n in range(nprb) if g.prb_idx[s][n]] == sorted(want[s]), (riv_v, s)
            assert g.nof_prb == L


@pytest.mark.parametrize("nprb", [6, 15, 25, 50, 75, 100])
def test_format1C_si_rnti(nprb):
    """format 1C (SI / P / RA-RNTI): pack -> unpack (dci.c:952-988, 990-1023), the distributed allocation in units of
    N_RB^step (ra_dl.c:230-244), QPSK and the TBS of 36.213 Table 7.1.7.2.3-1 (ra_dl.c:383-391)"""
    c = _cell(nprb)
    step = 2 if nprb < 50 else 4
    rng = np.random.default_rng(nprb)
    # N_gap,1 only: the format's size takes the RIV width of N_gap,1 (dci.c:231-240, as 36.212 5.3.3.1.4), while the
    # reference's packer and unpacker size the RIV by the message's own gap, so an N_gap,2 1C is not of the format's
    # size (a reference quirk, restated as is)
    for ngap1 in (True,):
        nvrb = OP.type2_n_vrb_dl(nprb, ngap1) // step
        for _ in range(24):
            L = int(rng.integers(1, nvrb + 1))
            st = int(rng.integers(0, nvrb - L + 1))
            riv_v = OP.riv(L, st, nvrb)
            mcs = int(rng.integers(0, 32))
            d = _dl(0xFFFF, F1C)
            _type2(d, riv_v, DIST, 0 if ngap1 else 1)
            d.tb[0].mcs_idx = mcs
            r, m = PD.pack_pdsch(c, d)
            assert r == 0 and m.nof_bits == PD.dci_size(c, F1C)
            r, u = PD.unpack_pdsch(c, list(m.payload[:m.nof_bits]), F1C, 0xFFFF)
            assert r == 0 and u.alloc_type == ALLOC2 and u.raw[3] == DIST and u.raw[0] == riv_v
            assert u.tb[0].mcs_idx == mcs and u.tb[0].rv == -1 and u.raw[2] == (0 if ngap1 else 1)
            u.format, u.rnti = F1C, 0xFFFF
            r, g = _grant(c, u)
            want = OP.type2_prbs(nprb, riv_v, True, ngap1, fmt1c=True)
            if want is None:
                assert r != 0
                continue
            assert r == 0 and g.tb[0].tbs == OP.TBS_FORMAT1C[mcs] and g.tb[0].mod == 1  # QPSK
            for s in range(2):
                assert [n for n in range(nprb) if g.prb_idx[s][n]] == sorted(want[s])
