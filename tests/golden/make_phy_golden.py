"""Generate tests/golden/phy_golden.npz from the reference's compiled pieces (oracle/_ref).

Run in the build container (where /root/reference exists and `make -C oracle` built oracle/_ref):
    python tests/golden/make_phy_golden.py
Inputs are seeded synthetic data; every OUTPUT below is the reference's:
  demod_m{mod}_*     srsran_demod_soft_demodulate_s (demod_soft.c:871-894), n symbols incl. an
                     SSE-block tail, mod 0..4 (BPSK .. 256QAM)
  seq_*              srsran_sequence_apply_s (sequence.c:507-561) for several seeds
  pdsch_seq_*        srsran_sequence_pdsch_apply_s (sequences.c:95-103)
  pre_s{scheme}_*    srsran_predecoding_type CSI variants (precoding.c:1866-1930); x and csi
  rm_k{idx}_rv{rv}_* srsran_rm_turbo_rx_lut (rm_turbo.c:390-483) into a pre-filled soft buffer
  tb_*               decode_tb over the reference's rm_turbo / turbodecoder / crc (ref_harness.c):
                     return value, payload bytes, average iterations, for clean and noisy TBs
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle"), ROOT]
from oracle import Reference  # noqa: E402
from synth import synth as S  # noqa: E402


def main():
    ref = Reference()
    rng = np.random.default_rng(0x601D)
    g = {}
    # soft demapping: amplitudes spanning the saturation range
    for mod in range(5):
        for n in (403, 4):
            sym = ((rng.standard_normal(n) + 1j * rng.standard_normal(n)) * 60.0).astype(np.complex64)
            sym[:3] = [0, 1e6 + 1e6j, -1e-3 - 7j]
            g[f"demod_m{mod}_n{n}_in"] = sym
            g[f"demod_m{mod}_n{n}_out"] = ref.demod_s(mod, sym)
    for i, seed in enumerate((0, 1, (0x1234 << 14) + (1 << 13) + (3 << 9) + 1, 0x7FFFFFFF)):
        x = rng.integers(-32768, 32768, 2011, dtype=np.int16)
        g[f"seq_{i}_seed"] = np.array([seed], np.uint32)
        g[f"seq_{i}_in"] = x
        g[f"seq_{i}_out"] = ref.sequence_apply_s(x, seed)
    for i, (rnti, q, ns, cell) in enumerate(((0x1234, 0, 2, 1), (0x4601, 1, 18, 503), (65535, 1, 0, 0))):
        x = rng.integers(-32768, 32768, 1507, dtype=np.int16)
        g[f"pdsch_seq_{i}_args"] = np.array([rnti, q, ns, cell], np.uint32)
        g[f"pdsch_seq_{i}_in"] = x
        g[f"pdsch_seq_{i}_out"] = ref.sequence_pdsch_apply_s(x, rnti, q, ns, cell)
    # predecoding (CSI variants, as the PDSCH calls them): even n (the reference CDD tail overruns on odd n)
    for scheme, nrx, nports, nl, cb in ((0, 2, 1, 1, 0), (1, 2, 2, 2, 0), (3, 2, 2, 2, 0), (2, 2, 2, 2, 1),
                                        (2, 2, 2, 2, 2), (2, 2, 2, 2, 0)):
        n = 600
        y = ((rng.standard_normal((nrx, n)) + 1j * rng.standard_normal((nrx, n))) * 0.7).astype(np.complex64)
        h = (rng.standard_normal((nports, nrx, n)) + 1j * rng.standard_normal((nports, nrx, n))).astype(np.complex64)
        x, csi = ref.predecode(scheme, y, h, nl, cb, 1.0, 0.05)
        p = f"pre_s{scheme}_cb{cb}_"
        g[p + "args"] = np.array([scheme, nrx, nports, nl, cb], np.int32)
        g[p + "y"], g[p + "h"], g[p + "x"], g[p + "csi"] = y, h, x, csi
    # rate de-matching with HARQ combining into a non-zero soft buffer
    for idx in (0, 60, 140, 187):  # (rv 0 and 2; the largest size with rv 2 only)
        K = [k for k in _cb_sizes()][idx]
        for rv in ((2,) if idx == 187 else (0, 2)):
            N = 3 * K + 12
            E = N + N // 3
            e = rng.integers(-30000, 30000, E, dtype=np.int16)
            nsb = 16 if (K % 16 == 0 and K > 800) else 8 if (K % 8 == 0 and K > 400) else 0
            sblen = 3 * (K + 32) + 12 if nsb else N
            sb0 = rng.integers(-30000, 30000, sblen, dtype=np.int16)
            p = f"rm_k{idx}_rv{rv}_"
            g[p + "e"], g[p + "sb0"] = e, sb0
            g[p + "out"] = ref.rm_turbo_rx(idx, rv, e, sb0)
    # DL-SCH decode_tb: a clean TB and a noisy one (CB CRC failures, early-stop spread)
    for i, (tbs, qm, sigma) in enumerate(((12960, 4, 0.2), (12960, 4, 0.75), (1544, 2, 0.5))):
        G = qm * ((3 * tbs) // (2 * qm) + 11)
        tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        e = S.dlsch_encode(tbs, qm, 0, G, tb).astype(np.float32) * 2 - 1
        llr = np.trunc(100 * (e + rng.standard_normal(G).astype(np.float32) * sigma)).astype(np.int16)
        ret, data, noi, avg, _ = ref.dlsch_decode(tbs, qm, 0, llr, 8)
        p = f"tb_{i}_"
        g[p + "args"] = np.array([tbs, qm, 0, 8], np.int32)
        g[p + "llr"] = llr
        g[p + "ret"] = np.array([ret], np.int32)
        g[p + "data"] = data
        g[p + "avg"] = np.array([avg], np.float32)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "phy_golden.npz")
    np.savez_compressed(out, **g)
    print(f"wrote {len(g)} arrays to {out} ({os.path.getsize(out)} bytes)")


def _cb_sizes():
    from oracle import CB_SIZES
    return CB_SIZES


if __name__ == "__main__":
    main()
