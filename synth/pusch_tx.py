"""Synthetic PUSCH transmitter for the bench (no oracle, no reference): UL-SCH coding by
synth.dlsch_encode (the same turbo / rate matching chain), the UL channel interleaver of
synth/ulsch_tx.py, scrambling (36.211 5.3.1), modulation, transform precoding (forward DFT /
sqrt(M)), mapping at n_prb with the library's own DMRS, a frequency-selective channel and AWGN.
No UCI (the bench's PUSCH workload is data-only)."""
import numpy as np

from . import synth as SY
from .ulsch_tx import ulsch_interleave


def pusch_seed(rnti, nslot, cell_id):
    return ((rnti << 14) + ((nslot // 2) << 9) + cell_id) & 0xFFFFFFFF


def subframe(cell, dmrs_cfg, cell_prb, L, n_prb, tbs, Qm, tti, rnti, rng, snr_db=30.0, payload=None):
    """normal CP, 12 PUSCH symbols -> (grid (14, 12 cell_prb) complex64, payload)"""
    from srsran_4g_amd import pusch as P
    M, nsymb = 12 * L, 12
    G = M * nsymb * Qm
    if payload is None:
        payload = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    e = SY.dlsch_encode(tbs, Qm, 0, G, payload)
    q = ulsch_interleave(e.astype(np.int16), Qm, nsymb).astype(np.uint8)
    b = q ^ SY.gold(pusch_seed(rnti, 2 * (tti % 10), cell.id), G)
    x = SY.modulate(b, Qm)
    grid = np.zeros((14, 12 * cell_prb), np.complex128)
    rows = [l for l in range(14) if l not in (3, 10)]
    for i, g in enumerate(rows):
        grid[g, n_prb * 12:n_prb * 12 + M] = np.fft.fft(x[i * M:(i + 1) * M]) / np.sqrt(M)
    ret, r = P.dmrs(cell, dmrs_cfg, L, tti % 10, 0)
    assert ret == 0
    grid[3, n_prb * 12:n_prb * 12 + M] = r[:M]
    grid[10, n_prb * 12:n_prb * 12 + M] = r[M:]
    k = np.arange(12 * cell_prb)
    # a dominant path and two weaker random echoes: |H| stays within about [0.6, 1.4]
    taps = np.concatenate([[1.0], (rng.standard_normal(2) + 1j * rng.standard_normal(2)) * np.array([0.2, 0.1]) / np.sqrt(2)])
    H = (taps[None, :] * np.exp(-2j * np.pi * k[:, None] * np.array([0.0, 3.0, 7.0])[None, :] / 2048.0)).sum(axis=1)
    grid = grid * H[None, :]
    s2 = 10 ** (-snr_db / 10)
    grid = grid + np.sqrt(s2 / 2) * (rng.standard_normal(grid.shape) + 1j * rng.standard_normal(grid.shape))
    return grid.astype(np.complex64), payload
