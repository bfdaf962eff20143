"""Synthetic NR DL-SCH / UL-SCH transmitter (tests and bench inputs; neither product nor oracle).

The 38.212 transmit chain the reference's sch_nr_encode runs (sch_nr.c:410-550): TB CRC (CRC24A, or
CRC16 for TBS <= 3824), segmentation (product's srsran_sch_nr_fill_tb_info), CB CRC24B when C > 1,
filler bits, LDPC encoding (synth/ldpc_tx.py, first 2Z bits punctured), bit selection from k0 over the
circular buffer of Ncb bits skipping the fillers, and the row/column bit interleaver (ldpc_rm.c:173-201,
348-362).  Pinned against the compiled reference encoder in tests/test_nr_sch_host.py.
"""
import numpy as np

from synth.ldpc_tx import encode as ldpc_encode

CRC24A, CRC24B, CRC16 = 0x1864CFB, 0x1800063, 0x11021
BASEK0 = ((0, 0), (17, 13), (33, 25), (56, 43))
_tables = {}


def _table(poly, order):
    key = (poly, order)
    if key not in _tables:
        t = np.zeros(256, np.uint32)
        mask = (1 << order) - 1
        for b in range(256):
            c = b << (order - 8)
            for _ in range(8):
                c = ((c << 1) ^ poly) if c & (1 << (order - 1)) else (c << 1)
            t[b] = c & mask
        _tables[key] = t
    return _tables[key]


def crc_bytes(data, poly, order):
    """Zero-init MSB-first CRC over whole bytes (srsran_crc_checksum_byte)."""
    t = _table(poly, order)
    c = 0
    mask = (1 << order) - 1
    for b in np.asarray(data, np.uint8).tolist():
        c = ((c << 8) & mask) ^ int(t[((c >> (order - 8)) ^ b) & 0xFF])
    return c


def crc_bits(bits, poly, order):
    """CRC over an unpacked bit vector (srsran_crc_checksum on bits)."""
    bits = np.asarray(bits, np.uint8)
    n = bits.size - bits.size % 8
    c = crc_bytes(np.packbits(bits[:n]), poly, order)
    for b in bits[n:].tolist():
        top = ((c >> (order - 1)) & 1) ^ b
        c = ((c << 1) & ((1 << order) - 1)) ^ (poly & ((1 << order) - 1) if top else 0)
    return c


def _unpack(v, n):
    return np.array([(v >> (n - 1 - i)) & 1 for i in range(n)], np.uint8)


def rm_params(t, rv):
    N = t.Z * (66 if t.bg == 0 else 50)
    if N <= t.Nref:
        return t.Z * BASEK0[rv & 3][t.bg], N
    return t.Z * ((BASEK0[rv & 3][t.bg] * t.Nref) // N), t.Nref


def cb_E(t, r):
    """sch_nr_get_E (sch_nr.c:178-189)."""
    qn = t.Nl * t.Qm
    if r <= t.Cp - (t.G // qn) % t.Cp - 1:
        return qn * (t.G // (qn * t.Cp))
    return qn * -(-t.G // (qn * t.Cp))


class NrCodeblocks:
    """Encoded circular buffers of one TB (computed once, rate matched per redundancy version)."""

    def __init__(self, t, payload, pcm=None):
        self.t = t
        Kp, Kr, L_cb, L_tb, C, Z = t.Kp, t.Kr, t.L_cb, t.L_tb, t.C, t.Z
        payload = np.asarray(payload, np.uint8)
        assert payload.size == t.A // 8
        tb_crc = crc_bytes(payload, CRC24A if L_tb == 24 else CRC16, L_tb)
        bits = np.concatenate([np.unpackbits(payload), _unpack(tb_crc, L_tb)])
        cb_len = Kp - L_cb
        msgs = np.zeros((C, Kr), np.uint8)
        for r in range(C):
            seg = bits[r * cb_len:(r + 1) * cb_len]
            msgs[r, :cb_len] = seg
            if L_cb:
                msgs[r, cb_len:Kp] = _unpack(crc_bits(seg, CRC24B, 24), 24)
        self.cw = ldpc_encode(t.bg, Z, msgs.reshape(C, -1) if C > 1 else msgs[0], pcm)
        self.cw = self.cw.reshape(C, -1)[:, 2 * Z:]
        self.filler = (Kp - 2 * Z, Kr - 2 * Z)

    def rate_match(self, rv):
        t = self.t
        k0, Ncb = rm_params(t, rv)
        f0, f1 = self.filler
        idx = np.array([i for i in range(Ncb) if not (f0 <= i < f1)], np.int64)
        pos0 = int(np.searchsorted(idx, k0))  # first non-filler position at or after k0
        out = []
        for r in range(t.C):
            E = cb_E(t, r)
            order = np.roll(idx, -pos0)
            sel = self.cw[r][order[np.arange(E) % order.size]]
            Qm = t.Qm
            if Qm > 1:  # output[i + j Qm] = sel[i cols + j]
                sel = sel.reshape(Qm, E // Qm).T.reshape(-1)
            out.append(sel)
        return np.concatenate(out).astype(np.uint8)


def aligned_tbs(n_re, R, Qm, Nl):
    """Largest multiple of 8 <= N_info whose code blocks are equal, byte-aligned (as 38.214 5.1.3.2 sizes are)."""
    from srsran_4g_amd import sch_nr as S

    tbs = max(24, 8 * (int(n_re * R * Qm * Nl) // 8))
    while True:
        s = S.cbsegm_ldpc(S.select_basegraph(tbs, R), tbs)
        if s["C"] == 1 or (tbs + s["L_tb"]) % (8 * s["C"]) == 0:
            return tbs
        tbs -= 8


def bpsk_llrs(rng, e, snr, amp=10.0):
    """Bits as +-1 with AWGN at `snr` dB, int8 LLRs clip(round(amp y)) (bit 1 -> negative)."""
    x = 1.0 - 2.0 * np.asarray(e, np.float64)
    y = x + 10 ** (-snr / 20) * rng.standard_normal(x.shape)
    return np.clip(np.round(amp * y), -127, 127).astype(np.int8)


def encode_tb(t, payload, rv, pcm=None):
    return NrCodeblocks(t, payload, pcm).rate_match(rv)
