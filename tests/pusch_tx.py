"""Test-side PUSCH transmitter (36.211 5.3 / 5.5, 36.212 5.2.2): UL-SCH + UCI multiplexing by the
reference's own encoder (oracle/ref_uci_harness.c around uci.c), scrambling with the placeholder /
repetition rule of pusch.c:307-331, modulation, transform precoding (forward DFT / sqrt(M)),
resource mapping at n_prb_tilde with the DMRS of symbol 3 (2) of each slot, then a frequency-
selective channel constant over the subframe and AWGN.  Shared by tests/test_pusch_*.py."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oracle"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import pusch as OP  # noqa: E402  (oracle/pusch.py)
import uci as RU  # noqa: E402  (oracle/uci.py)
import uci_cases as UC  # noqa: E402
from synth.synth import modulate  # noqa: E402


def make_cfg(cell_prb, Qm, L, n_prb, tbs, nack=0, ri=0, cqi=None, cp=0, shortened=False, rnti=0x46, n_dmrs=0, rv=0,
             hop=None, softbuffer=None):
    nsymb = (12 if cp == 0 else 10) - (1 if shortened else 0)
    cfg = UC.make_cfg(Qm, L, nsymb, tbs, nack, ri, cqi, rv=rv, softbuffer=softbuffer)
    cfg.rnti = rnti
    cfg.grant.n_prb[0] = cfg.grant.n_prb[1] = n_prb
    cfg.grant.n_prb_tilde[0] = cfg.grant.n_prb_tilde[1] = n_prb if hop is None else hop
    cfg.grant.n_dmrs = n_dmrs
    cfg.enable_64qam = True
    cfg.max_nof_iterations = 8
    return cfg


def channel(ncell_re, rng, kind):
    k = np.arange(ncell_re)
    if kind == "flat":
        return np.full(ncell_re, 0.8 * np.exp(0.7j), np.complex128)
    if kind == "ideal":
        return np.ones(ncell_re, np.complex128)
    taps = (rng.standard_normal(3) + 1j * rng.standard_normal(3)) * np.array([0.8, 0.4, 0.2]) / np.sqrt(2)
    delays = np.array([0.0, 3.0, 7.0])
    return (taps[None, :] * np.exp(-2j * np.pi * k[:, None] * delays[None, :] / 2048.0)).sum(axis=1)


def pusch_subframe(po, cell_id, cell_prb, cp, cfg, dmrs_cfg, tti, rng, snr_db=30.0, kind="selective",
                   uci=None, payload=None, shortened=False):
    """-> (grid (2 nsym, 12 cell_prb) complex64, payload, uci value, H, sigma2)"""
    ref = RU.RefUci()
    Qm = {1: 2, 2: 4, 3: 6}[cfg.grant.tb.mod]
    tbs = cfg.grant.tb.tbs
    u = uci if uci is not None else UC.random_uci(cfg, rng)
    Qri, Qcqi, G = ref.tx_sizes(cfg, u)
    if payload is None:
        payload = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    e = po.ora.dlsch_encode(tbs, Qm, cfg.grant.tb.rv, G * Qm, payload) if tbs else np.zeros(0, np.uint8)
    types, _ = ref.tx(cfg, u, e)
    nb = types.size
    c = po.ora.sequence_bits(OP.pusch_seed(cfg.rnti, 2 * (tti % 10), cell_id), nb)
    t = np.asarray(types)
    s = np.where(t <= 1, t, 0).astype(np.uint8) ^ c
    s[t == RU.TYPE_PLACEHOLDER] = 1
    rep = np.nonzero((t == RU.TYPE_REPETITION) & (np.arange(nb) > 1))[0]
    s[rep] = s[rep - 1]
    x = modulate(s, Qm)
    L = cfg.grant.L_prb
    M = 12 * L
    nsym = OP.nsymb_slot(cp)
    grid = np.zeros((2 * nsym, 12 * cell_prb), np.complex128)
    rows = OP.data_symbols(cp, shortened)
    assert len(rows) * M == x.size
    for i, g in enumerate(rows):
        X = np.fft.fft(x[i * M:(i + 1) * M]) / np.sqrt(M)
        n0 = cfg.grant.n_prb_tilde[g // nsym] * 12
        grid[g, n0:n0 + M] = X
    r = po.dmrs(cell_id, cp, dmrs_cfg.cyclic_shift, dmrs_cfg.delta_ss, dmrs_cfg.group_hopping_en,
                dmrs_cfg.sequence_hopping_en, L, tti % 10, cfg.grant.n_dmrs)
    for sl in (0, 1):
        n0 = cfg.grant.n_prb_tilde[sl] * 12
        grid[(sl + 1) * nsym - 4, n0:n0 + M] = r[sl * M:(sl + 1) * M]
    H = channel(12 * cell_prb, rng, kind)
    grid = grid * H[None, :]
    sigma2 = 10 ** (-snr_db / 10)
    grid = grid + np.sqrt(sigma2 / 2) * (rng.standard_normal(grid.shape) + 1j * rng.standard_normal(grid.shape))
    return grid.astype(np.complex64), payload, u, H, sigma2
