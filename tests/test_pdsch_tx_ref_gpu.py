"""The GPU transmitter's PDSCH symbols against the reference's own transmit building blocks compiled from
/root/reference (oracle/ref_pdsch_tx_harness.c: srsran_sequence_pdsch_apply_pack, srsran_mod_modulate_bytes,
srsran_layermap_type, srsran_precoding_type, composed as srsran_pdsch_encode does, pdsch.c:960-1112).
The coded bits come from the oracle encoder (pinned to the compiled turbocoder.c / rm_turbo.c by
test_sch*); the RE order is the reference's (pinned by tests/test_pdsch_map.py).  Two GPU entry points:
srsran_pdsch_encode (host grids) and the batched srsran_enb_dl_gpu_tx_batch (its device grid,
srsran_enb_dl_gpu_sf_symbols).  Tolerance 1e-6 absolute on unit-power symbols (float precoding)."""
import ctypes
import os
import sys

import numpy as np
import pytest

from synth import synth as SY

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MOD_OF_QM = {2: 1, 4: 2, 6: 3}  # srsran_mod_t
SCHEME_ID = {"port0": 0, "diversity": 1, "spatialmux": 2, "cdd": 3}  # srsran_tx_scheme_t

CASES = [  # (scheme, nof_prb, P, ntb, Qm, tbs, tti, cfi)
    ("cdd", 100, 2, 2, 6, 75376, 3, 1),
    ("cdd", 50, 2, 2, 4, 18336, 0, 2),
    ("diversity", 50, 2, 1, 4, 12216, 5, 2),
    ("diversity", 25, 4, 1, 2, 2216, 1, 3),
    ("port0", 15, 1, 1, 6, 5160, 7, 2),
]


@pytest.fixture(scope="module")
def env():
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    if not O.ref_available():  # on a HIP box the parity checker must be there: fail, never skip
        pytest.fail("oracle/_ref/libsrsref.so missing: the reference checker of this module was not built")
    L = ctypes.CDLL(O.REF_SO, mode=os.RTLD_LAZY)  # dft_precoding.c's FFTW plans stay unresolved, unused
    u32p = ctypes.POINTER(ctypes.c_uint32)
    L.ref_pdsch_tx_symbols.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint32, u32p, u32p,
                                       u32p, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                       ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.POINTER(ctypes.c_float)]
    L.ref_pdsch_tx_symbols.restype = ctypes.c_int
    L.ref_pdsch_tx_symbols_sc.argtypes = L.ref_pdsch_tx_symbols.argtypes[:-1] + [ctypes.c_float,
                                                                                 ctypes.POINTER(ctypes.c_float)]
    L.ref_pdsch_tx_symbols_sc.restype = ctypes.c_int
    import torch
    return torch, L, O.Oracle()


def ref_symbols(L, es, Qm, scheme, P, nl, rnti, sf_idx, cell_id, nre, scaling=1.0):
    ncw = len(es)
    stride = max(len(e) for e in es)
    buf = np.zeros((ncw, stride), np.uint8)
    for c, e in enumerate(es):
        buf[c, :len(e)] = e
    u = lambda v: (ctypes.c_uint32 * len(v))(*v)  # noqa: E731
    out = np.zeros((P, nre, 2), np.float32)
    r = L.ref_pdsch_tx_symbols_sc(ncw, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), stride,
                                  u([len(e) for e in es]), u([MOD_OF_QM[Qm]] * ncw), u(list(range(ncw))), rnti, sf_idx,
                                  cell_id, SCHEME_ID[scheme], P, nl, 0, nre, scaling,
                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    assert r == 0
    return out.view(np.complex64)[..., 0]


def coded_bits(ora, scheme, ntb, Qm, tbs, nre, pls):
    Nl = 2 if scheme == "diversity" else 1  # rate matching on Qm * Nl (sch.c:587-603)
    return [ora.dlsch_encode(tbs, Qm * Nl, 0, nre * Qm, pl) for pl in pls]


def rho_a(p_a, P):
    """apply_power_allocation's rho_a (pdsch.c:492): 10^(p_a / 20) x sqrt 2 with more than one port, in float"""
    return float(np.float32(float(np.float32(10.0) ** np.float32(p_a / 20.0)) * (1.0 if P == 1 else np.sqrt(2.0))))


@pytest.mark.parametrize("p_a", [0.0, -3.0])
@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}_{c[1]}prb_{c[2]}p_q{c[4]}_sf{c[6]}" for c in CASES])
def test_pdsch_encode_matches_reference_blocks(env, case, p_a):
    """srsran_pdsch_encode on host grids: every PDSCH RE equals the reference composition, precoded with the
    reference's rho_a (srsran_pdsch_encode applies it whatever power_scale says, pdsch.c:1057-1071)"""
    torch, L, ora = env
    from srsran_4g_amd import ue_dl as U
    scheme, nprb, P, ntb, Qm, tbs, tti, cfi = case
    cell_id, rnti = 29, 0x2B17
    mask = SY.pdsch_mask(nprb, P, cell_id, cfi, tti % 10)
    nre = int(mask.sum())
    rng = np.random.default_rng(tbs + 7 * tti)
    pls = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(ntb)]
    nl = P if scheme == "diversity" else ntb
    want = ref_symbols(L, coded_bits(ora, scheme, ntb, Qm, tbs, nre, pls), Qm, scheme, P, nl, rnti, tti % 10,
                       cell_id, nre, rho_a(p_a, P))
    cell = U.cell(nprb, P, cell_id)
    pd = U.Pdsch(cell, 1, enb=True)
    cfg = U.pdsch_cfg(nprb, nre, [tbs] * ntb, [Qm] * ntb, scheme=scheme, rnti=rnti)
    cfg.p_a = p_a
    grids = [np.zeros(mask.size, np.complex64) for _ in range(P)]
    ret, got = pd.encode(cfg, tti, cfi, pls, grids)
    pd.free()
    assert ret == 0
    for p in range(P):
        g = np.asarray(got[p]).reshape(mask.shape)
        np.testing.assert_allclose(g[mask], want[p], rtol=0, atol=1e-6)
        assert not np.any(g[~mask]), "REs outside the PDSCH written"


@pytest.mark.parametrize("case", CASES[:3], ids=[f"{c[0]}_{c[1]}prb_sf{c[6]}" for c in CASES[:3]])
def test_enb_tx_batch_grid_matches_reference_blocks(env, case):
    """the batched eNB transmitter: its device grid (srsran_enb_dl_gpu_sf_symbols) holds the reference
    composition on the PDSCH REs of every subframe of a batch"""
    torch, L, ora = env
    from srsran_4g_amd import enb_dl as E
    from srsran_4g_amd import ue_dl as U
    scheme, nprb, P, ntb, Qm, tbs, tti0, cfi = case
    cell_id, rnti = 41, 0x1D0C
    U.use_standard_symbol_size(True)
    N = SY.symbol_sz(nprb)
    nl = P if scheme == "diversity" else ntb
    cell = U.cell(nprb, P, cell_id)
    enb = E.EnbDl(cell)
    sfs, wants, masks, keep = [], [], [], []
    for j, tti in enumerate((tti0, tti0 + 1, tti0 + 5)):
        mask = SY.pdsch_mask(nprb, P, cell_id, cfi, tti % 10)
        nre = int(mask.sum())
        rng = np.random.default_rng(tbs + 13 * tti)
        pls = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(ntb)]
        d_pl = [torch.from_numpy(p).cuda() for p in pls]
        keep.append(d_pl)
        cfg = U.pdsch_cfg(nprb, nre, [tbs] * ntb, [Qm] * ntb, scheme=scheme, rnti=rnti)
        keep.append(cfg)
        sfs.append((tti, cfi, cfg, [p.data_ptr() for p in d_pl]))
        wants.append(ref_symbols(L, coded_bits(ora, scheme, ntb, Qm, tbs, nre, pls), Qm, scheme, P, nl, rnti,
                                 tti % 10, cell_id, nre))
        masks.append(mask)
    nsf = len(sfs)
    d_out = torch.zeros((nsf, P, 15 * N, 2), dtype=torch.float32, device="cuda")
    assert enb.tx_batch(sfs, d_out.data_ptr(), 1.0 / N) == 0
    torch.cuda.synchronize()
    ptr = enb.sf_symbols()
    assert ptr
    from srsran_4g_amd.sch import _memcpy_d2h
    sf_re = masks[0].size
    host = torch.empty(nsf * P * sf_re * 2, dtype=torch.float32)
    _memcpy_d2h(host, ptr, host.numel() * 4)
    enb.free()
    grid = host.numpy().view(np.complex64).reshape(nsf, P, sf_re)
    for b in range(nsf):
        for p in range(P):
            g = grid[b, p].reshape(masks[b].shape)
            np.testing.assert_allclose(g[masks[b]], wants[b][p], rtol=0, atol=1e-6)
