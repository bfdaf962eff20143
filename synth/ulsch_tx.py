"""Synthetic UL-SCH transmit interleaver (tests and bench inputs; neither product nor oracle).

The channel interleaver of 36.212 5.2.2.8 as ulsch_interleave_qm2/4/6 (sch.c:684-852) apply it
without RI bits: the g bits are read in order, Qm at a time, and written to the column-major
position (i rows + j) Qm of row j, column i (rows = H' / N_symb), rows outer, columns inner.
An independent restatement of the transmit side: its composition with the oracle's
de-interleaver (restated from ulsch_interleave_gen, sch.c:661-682) is checked to be the identity.
"""
import numpy as np


def ulsch_interleave(g, Qm, nof_symb):
    g = np.asarray(g)
    H = g.size // Qm
    rows = H // nof_symb
    q = np.zeros_like(g)
    read = 0
    for j in range(rows):
        for i in range(nof_symb):
            k = (i * rows + j) * Qm
            q[k:k + Qm] = g[read:read + Qm]
            read += Qm
    return q
