"""Diagnostics for the UE DL control path on the GPU box (not a test)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa

import pdcch as P
from srsran_4g_amd import pdcch as PD
from srsran_4g_amd import ue_dl as U
from synth import synth as S

cid, tti, cfi, rnti, tbs = 1, 3, 2, 0x1234, 75376
rng = np.random.default_rng(42)
c = PD.cell(100, 2, cid)
bits = P.dci_pack_2a(100, PD.dci_size(c, P.FORMAT2A), (1 << 25) - 1, [(28, 1, 0), (28, 1, 0)], pid=1)
regs = PD.Regs(c)
nof_cce = regs.q.pdcch_nregs[cfi - 1] // 9
L, ncce = [loc for loc in PD.ue_locations(nof_cce, tti % 10, rnti) if loc[0] == 3][0]
print("nof_cce", nof_cce, "loc", L, ncce)
ctrl = P.Ref().ctrl_tx(100, 2, cid, tti, cfi, [(bits, L, ncce, rnti)])
pls = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(2)]
x, nre = S.pdsch_subframe(100, cid, 2, tti, cfi, rnti, tbs, 6, 0, pls, snr_db=30.0, rng=rng, pcfich=False,
                          ctrl=[ctrl[0], ctrl[1]])
U.use_standard_symbol_size(True)
ue = U.UeDl(U.cell(100, 2, cid), 2)
print("fft_estimate", ue.fft_estimate(x, tti, 0), "cfi", ue.last_cfi)
grids = ue.grids().reshape(2, 14, 1200)
ce = np.zeros((2, 2, 14, 1200), np.complex64)
for p in range(2):
    for r in range(2):
        ctypes.memmove(ce[p, r].ctypes.data, ue.q.chest_res.ce[p][r], 14 * 1200 * 8)
noise = ue.q.chest_res.noise_estimate
print("noise", noise, "ce sample", ce[0, 0, 0, :3], ce[1, 1, 5, 100:102])
ref = P.Ref()
rcfi, rcorr, rllr = ref.ctrl_rx(100, 2, cid, tti, grids, ce, noise)
print("ref cfi", rcfi, rcorr, "llr mean", np.abs(rllr).mean())
print("ref decode 2A", ref.pdcch_decode(tti, cfi, rllr, L, ncce, P.FORMAT2A)[2:], hex(rnti))
ctl = PD.Control(c, 2)
gcfi, gcorr, _ = ctl.pcfich(grids, ce, noise, tti)
gllr = ctl.pdcch_llr(grids, ce, noise, tti, cfi)
print("gpu cfi", gcfi, gcorr, "llr equal", np.array_equal(gllr, rllr))
out = ctl.decode(tti, cfi, [(L, ncce, P.FORMAT2A), (L, ncce, P.FORMAT1A)])
print("gpu decode", [(o[0], hex(o[2]), o[3]) for o in out], "payload ok", np.array_equal(out[0][1], bits))
dcis = ue.find_dl_dci(tti, cfi, rnti, tm=2)
print("find_dl_dci", len(dcis))
dcis = ue.find_dl_dci(tti, cfi, rnti, tm=2, common_ss=False)
print("find_dl_dci no common", len(dcis))
locs = PD.ue_locations(nof_cce, tti % 10, rnti)
fl = [(l, n, f) for (l, n) in locs for f in (P.FORMAT1A, P.FORMAT2A)]
out = ctl.decode(tti, cfi, fl)
print("batch", [(fl[i], o[0], hex(o[2]), round(o[3], 3)) for i, o in enumerate(out) if o[2] == rnti])
print("locs", locs)
