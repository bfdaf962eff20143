"""oracle/pusch.py -- TEST INFRASTRUCTURE ONLY: CPU checker of the PUSCH receive chain.

  dmrs(...)     refsignal_ul.c:95-358 restated (hopping tables, n_cs, u / v) around the reference's
                own srsran_zc_sequence_generate_lte (zc_sequence.c:286) and srsran_group_hopping_f_gh
                (phy_common.c:471), compiled into oracle/_ref
  chest(...)    chest_ul.c:298-433 in numpy, with the reference's srsran_chest_average_pilots /
                srsran_conv_same_cf (chest_common.c:97, convolution.c:182) doing the smoothing
  symbols(...)  pusch_get (pusch.c:48-105), srsran_predecoding_single (precoding.c:182-305) and
                srsran_dft_precoding (dft_precoding.c:114-126) with numpy's FFT standing in for FFTW
                (absent here: the DFT is parity-unpinned and compared within a tolerance)
  llrs(...)     the reference's srsran_demod_soft_demodulate_s + srsran_sequence_apply_s (compiled)
Never imported by the library: tests/ only.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SO = os.path.join(HERE, "_ref", "libsrsref.so")

N_DMRS_1 = (0, 2, 3, 4, 6, 8, 9, 10)  # refsignal_ul.c:42
N_DMRS_2 = (0, 6, 3, 4, 2, 8, 10, 9)  # refsignal_ul.c:39


def ref_available():
    return os.path.exists(REF_SO)


def nsymb_slot(cp):
    return 7 if cp == 0 else 6


def data_symbols(cp, shortened):
    """pusch_cp's symbol order (pusch.c:62-89)"""
    ns, lref = nsymb_slot(cp), (3 if cp == 0 else 2)
    out = []
    for slot in range(2):
        n_srs = 1 if (shortened and slot == 1) else 0
        out += [l + slot * ns for l in range(ns - n_srs) if l != lref]
    return out


def pusch_seed(rnti, nslot, cell_id):
    return ((rnti << 14) + ((nslot // 2) << 9) + cell_id) & 0xFFFFFFFF


class PuschOracle:
    def __init__(self):
        from oracle import Oracle, Reference
        self.ora = Oracle()
        self.ref = Reference()
        L = ctypes.CDLL(REF_SO, mode=os.RTLD_LAZY)
        L.srsran_zc_sequence_generate_lte.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float,
                                                      ctypes.c_uint32, ctypes.c_void_p]
        L.srsran_group_hopping_f_gh.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.srsran_chest_average_pilots.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                  ctypes.c_uint32, ctypes.c_uint32]
        self.L = L

    # ---- refsignal_ul.c ----
    def dmrs(self, cell_id, cp, cs_cfg, delta_ss, gh, sh, nof_prb, sf_idx, n_dmrs):
        nsym = nsymb_slot(cp)
        f_gh = np.zeros(20, np.uint32)
        self.L.srsran_group_hopping_f_gh(f_gh.ctypes.data, cell_id)
        c = self.ora.sequence_bits(((cell_id // 30) << 5) + ((cell_id % 30) + delta_ss) % 30, 8 * nsym * 20)
        r = np.zeros(24 * nof_prb, np.complex64)
        for ns in (2 * sf_idx, 2 * sf_idx + 1):
            n_prs = sum(int(c[8 * nsym * ns + i]) << i for i in range(8))
            n_cs = (N_DMRS_1[cs_cfg] + N_DMRS_2[n_dmrs] + n_prs) % 12
            alpha = float(np.float32(2 * np.pi * n_cs / 12))
            u = ((int(f_gh[ns]) if gh else 0) + cell_id % 30 + delta_ss) % 30
            v = int(c[ns]) if (nof_prb >= 6 and sh) else 0
            seg = np.zeros(12 * nof_prb, np.complex64)
            assert self.L.srsran_zc_sequence_generate_lte(u, v, alpha, nof_prb, seg.ctypes.data) == 0
            r[(ns % 2) * 12 * nof_prb:(ns % 2 + 1) * 12 * nof_prb] = seg
        return r

    # ---- chest_ul.c ----
    def chest(self, grid, nof_prb_cell, cp, L_prb, n_tilde, n_prb, r, meas_ta=False, smooth=True, w=0.3333,
              ce_in=None):
        """grid: (2 * nsym, 12 * nof_prb_cell) complex64 -> dict(ce grid, noise, cfo_hz, ta_us, rsrp, epre)"""
        nsym, M = nsymb_slot(cp), 12 * L_prb
        rx = np.stack([grid[(s + 1) * nsym - 4, n_tilde[s] * 12:n_tilde[s] * 12 + M] for s in (0, 1)]).astype(np.complex64)
        pe = (rx * np.conj(r.reshape(2, M))).astype(np.complex64)
        ce = np.zeros_like(grid) if ce_in is None else np.array(ce_in, np.complex64, copy=True)
        cfo = np.angle(np.sum(pe[0].astype(np.complex128) * np.conj(pe[1]))) / (2 * np.pi * 0.0005)
        ta = 0.0
        if meas_ta:
            for s in (0, 1):
                acc = np.sum(pe[s, 1:].astype(np.complex128) * np.conj(pe[s, :-1]))
                ta += np.float32(-np.angle(acc) / np.pi * 0.5) / 2
            ta = float(np.round(ta / 15e3 * 1e6 * 10) / 10) if ta != 0 else 0.0
        filt = np.array([w, 1 - 2 * w, w], np.float32)
        noise = 0.0
        avg = pe.copy()
        if smooth:
            for s in (0, 1):
                inp = np.ascontiguousarray(pe[s])
                out = np.zeros(M, np.complex64)
                self.L.srsran_chest_average_pilots(inp.ctypes.data, out.ctypes.data, filt.ctypes.data, M, 1, 3)
                avg[s] = out
            p = np.mean(np.abs(avg.astype(np.complex128) - pe) ** 2, axis=1)
            wf = np.float32(w)
            a = np.float32(7.419 * float(wf) * float(wf) + 0.1117 * float(wf) - 0.005387)
            noise = float((p[0] + p[1]) / 2 / (float(a) * 0.8))
        for s in (0, 1):
            for i in range(nsym):
                ce[s * nsym + i, n_prb[s] * 12:n_prb[s] * 12 + M] = avg[s]
        corr = np.mean(rx.astype(np.complex128))
        epre = float(np.mean(np.abs(rx.astype(np.complex128)) ** 2))
        rsrp = min(abs(corr) ** 2, epre)
        return dict(ce=ce, noise=noise, cfo_hz=float(cfo), ta_us=ta, rsrp=rsrp, epre=epre)

    # ---- pusch.c / precoding.c / dft_precoding.c ----
    def symbols(self, grid, ce, noise, cp, shortened, L_prb, n_tilde):
        nsym, M = nsymb_slot(cp), 12 * L_prb
        rows = data_symbols(cp, shortened)
        y = np.concatenate([grid[g, n_tilde[g // nsym] * 12:n_tilde[g // nsym] * 12 + M] for g in rows]).astype(np.complex128)
        h = np.concatenate([ce[g, n_tilde[g // nsym] * 12:n_tilde[g // nsym] * 12 + M] for g in rows]).astype(np.complex128)
        n = y.size
        den = np.abs(h) ** 2 + noise
        nvec = 8 * (n // 8)
        if noise <= 0:
            den[:nvec] = np.abs(h[:nvec]) ** 2
        z = (y * np.conj(h) / den).reshape(len(rows), M)
        d = np.fft.ifft(z, axis=1) * np.sqrt(M)
        return d.reshape(-1).astype(np.complex64)

    def llrs(self, d, mod, rnti, tti, cell_id):
        q = self.ref.demod_s(mod, d)
        return self.ref.sequence_apply_s(q, pusch_seed(rnti, 2 * (tti % 10), cell_id))
