"""CPU restatement of srsUE's PDSCH receive chain composed from the oracle's pinned pieces
(TEST INFRASTRUCTURE ONLY -- the checker for the GPU chain; never imported by the product).

  srsran_ue_dl_decode_fft_estimate  ue_dl.c:349-364 -> ofdm_np.ofdm_rx + Oracle.chest_dl
  srsran_ue_dl_decode_pdsch         ue_dl.c:700-706 -> pdsch_decode below
  srsran_pdsch_decode               pdsch.c:788-958:
      srsran_pdsch_get              pdsch_np.re_table (symbols and estimates)
      apply_power_allocation        pdsch.c:485-521 (rho_b on CRS symbols, rho_a as scaling)
      srsran_predecoding_type       Oracle.predecode (MMSE with CSI), or the reference's compiled
                                    precoding.c (Reference.predecode, `pre`)
      codeword decode               pdsch.c:661-744: demod_s, sequence_pdsch_apply_s,
                                    csi_correction, srsran_dlsch_decode2 (Oracle.dlsch_decode);
                                    with llr8 the 8-bit forms (demod_b, apply_c, dlsch_decode8)
Parity: each piece is pinned to the reference (tests/test_phy_oracle.py, test_sch_oracle.py);
the OFDM stage is numpy (FFTW unavailable, 'parity unpinned' beyond round trips).
"""
import math

import numpy as np

import ofdm_np
import pdsch_np

SCHEME = {"port0": 0, "diversity": 1, "sm": 2, "cdd": 3}
MOD = {1: 0, 2: 1, 4: 2, 6: 3, 8: 4}
RHO_TABLE = ((1.0, 4.0 / 5, 3.0 / 5, 2.0 / 5), (5.0 / 4, 1.0, 3.0 / 4, 1.0 / 2))  # pdsch.c:44-46


def symbol_sz(nof_prb, standard=True):
    """srsran_symbol_sz (phy_common.c:340-385): standard rates = power-of-two sizes (1536 for 15 MHz);
    otherwise the reference's default 3/4 rates (384 / 768 / 1536 for 25 / 50 / 100 PRB)."""
    sizes = (512, 1024, 1536, 2048) if standard else (384, 768, 1024, 1536)
    for p, n in zip((6, 15, 25, 52, 79, 110), (128, 256) + sizes):
        if nof_prb <= p:
            return n
    raise ValueError(nof_prb)


def fft_estimate(ora, samples, nof_prb, cell_id, nports, tti, cfo=0.0, N=None, cp=0, tdd=None):
    """-> grids (nrx, 2*nsymb*12*nof_prb) complex64 (nsymb 7, or 6 with cp=1 extended), ce (nports, nrx, n)
    complex64, stats.  tdd = (sf_config, ss_config) of a TDD cell: a special subframe's CRS symbol counts
    (srsran_refsignal_cs_nof_symbols)."""
    N = N or symbol_sz(nof_prb)
    nre = 12 * nof_prb
    grids = []
    for x in samples:
        if cfo:  # srsran_cfo_correct: the reference's own phasor recurrence where _ref is built
            x = ofdm_np.ref_apply_cfo(x, cfo) if ofdm_np.ref_available() else ofdm_np.cfo(x, cfo)
        grids.append(ofdm_np.ofdm_rx(x, N, nre, ext=cp).astype(np.complex64))
    grids = np.stack(grids)
    nsym = (4, 2)
    if tdd and pdsch_np.tdd_type(tdd[0], tti % 10) == "S":
        import oracle as _o
        nsym = _o.crs_nsym(pdsch_np.TDD_SS_SYMBOLS[tdd[1]][0], cp)
    ce, st = ora.chest_dl(grids, nof_prb, cell_id, nports, tti % 10, N, cp=cp, nsym=nsym)
    return grids, ce, st


def pdsch_decode(ora, grids, ce, noise, nof_prb, cell_id, nports, tti, cfi, rnti, tbs, Qm, rv, scheme="cdd",
                 pmi=0, max_iterations=8, csi_enable=True, power_scale=False, p_a=0.0, p_b=0, prb_mask=None,
                 states=None, layers=None, cp=0, llr8=False, pre=None, tdd=None):
    """srsran_pdsch_decode for nof_tb = len(tbs) codewords (one layer each; layers=2 with one
    codeword: SM / CDD on two layers, pdsch.c:838-863 + layermap.c:138-147, 236-260).
    llr8: q->llr_is_8bit (pdsch.c:691-737, sch.c:409-428): demod_b, sequence_apply_c, the 8-bit CSI correction
    and decode_tb on the 8-bit decoders.  tdd = (sf_config, ss_config) of a TDD cell.
    pre: the object whose predecode() runs srsran_predecoding_type -- the oracle's exact-division restatement by
    default, or oracle.Reference() for the reference's own compiled precoding.c (its SIMD MMSE bodies use
    _mm256_rcp_ps, precoding.c:1123-1194 / simd.h:321-338, so it differs from the restatement in the last bits).
    Returns per codeword dict(ret, data, avg, llr)."""
    sf_idx = tti % 10
    lstart = cfi + (1 if nof_prb < 10 else 0)
    mask = np.ones((2, nof_prb), bool) if prb_mask is None else prb_mask
    if tdd:  # TDD: the grant's DwPTS symbols per slot and the TDD PSS / SSS holes (ra_dl.c:432-440, pdsch.c:90-107)
        tab = pdsch_np.re_table(nof_prb, nports, cell_id, mask, lstart, sf_idx, fdd=False, cp=cp,
                                nsl=pdsch_np.tdd_nof_symb_slot(tdd[0], tdd[1], sf_idx, cp))
    else:
        tab = pdsch_np.re_table(nof_prb, nports, cell_id, mask, lstart, sf_idx, cp=cp)
    idx = np.array([t[0] for t in tab], np.int64)
    crs = np.array([t[1] for t in tab], bool)
    y = grids[:, idx].astype(np.complex64)
    scaling = 1.0
    if power_scale:
        rho_a = np.float32(math.pow(10.0, p_a / 20.0) * (1.0 if nports == 1 else math.sqrt(2)))
        if rho_a != 0 and np.isfinite(rho_a):
            scaling = float(rho_a)
        rho_b = np.sqrt(np.float32(RHO_TABLE[0 if nports == 1 else 1][p_b]), dtype=np.float32)
        if rho_b != 0 and rho_b != 1:
            y[:, crs] = y[:, crs] * (np.float32(1) / rho_b)
    h = ce[:, :, idx]
    ntb = len(tbs)
    pre = pre or ora
    codebook = pmi if ntb == 1 else pmi + 1
    if scheme == "diversity":  # 1 codeword on nports layers, srsran_layerdemap_diversity (layermap.c:138-147)
        L = nports
        xl, csi = pre.predecode(1, y, h, L, codebook, scaling, noise)
        x = np.zeros((1, idx.size), np.complex64)  # 4 ports: a trailing half group stays 0
        for j in range(L):
            x[0, j:L * xl.shape[1]:L] = xl[j]
    elif layers == 2 and ntb == 1:  # predecode 2 layers; demap n/2 layer symbols each; CSI of layer 0
        xl, csi = pre.predecode(SCHEME[scheme], y, h, 2, codebook, scaling, noise)
        n = xl.shape[1]
        x = np.zeros((1, n), np.complex64)
        x[0, 0:2 * (n // 2):2], x[0, 1:2 * (n // 2):2] = xl[0, :n // 2], xl[1, :n // 2]
    else:
        x, csi = pre.predecode(SCHEME[scheme], y, h, ntb, codebook, scaling, noise)
    out = []
    for q in range(ntb):
        seed = ora.pdsch_seed(rnti, q, 2 * sf_idx, cell_id)
        if llr8:
            llr = demod = ora.demod_b(MOD[Qm[q]], x[q])
            llr = ora.sequence_apply_c(llr, seed)
            if csi_enable:
                llr = ora.csi_correction_b(MOD[Qm[q]], csi[q], llr)
        else:
            llr = demod = ora.demod_s(MOD[Qm[q]], x[q])
            llr = ora.sequence_apply_s(llr, seed)
            if csi_enable:
                llr = ora.csi_correction(MOD[Qm[q]], csi[q], llr)
        st = states[q] if states else None
        nl = 2 if (scheme == "diversity" or layers == 2) and ntb == 1 else 1  # Nl = 2 when layers != TBs (sch.c:587-590)
        dec = ora.dlsch_decode8 if llr8 else ora.dlsch_decode
        ret, data, noi, avg, state = dec(tbs[q], Qm[q] * nl, rv[q], llr, max_iterations, st)
        out.append(dict(ret=ret, data=data, avg=avg, llr=llr, state=state, nof_re=idx.size, sym=x[q], demod=demod))
    return out
