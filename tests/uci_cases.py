"""Shared UCI-on-PUSCH test cases (tests/test_uci_host.py, tests/test_uci_gpu.py): PUSCH
configurations with HARQ-ACK / RI / CQI and the reference transmitter's soft bits for them."""
import numpy as np

from srsran_4g_amd import sch as S

# (name, Qm, L_prb, N_symb, tbs, n_ack, ri_len, cqi) -- cqi: None or (type, dict of cqi cfg fields)
WB = S.SRSRAN_CQI_TYPE_WIDEBAND
SB_UE = S.SRSRAN_CQI_TYPE_SUBBAND_UE
SB_DIFF = S.SRSRAN_CQI_TYPE_SUBBAND_UE_DIFF
HL = S.SRSRAN_CQI_TYPE_SUBBAND_HL
CASES = [
    ("ack1_qpsk", 2, 6, 12, 1544, 1, 0, None),
    ("ack2_ri1_wb_16qam", 4, 25, 12, 11064, 2, 1, (WB, dict(pmi_present=True))),
    ("ack4_ri2_hl_64qam_srs", 6, 50, 11, 30576, 4, 2, (HL, dict(N=13, pmi_present=True))),
    ("ri1_sbdiff_qpsk", 2, 10, 12, 2600, 0, 1, (SB_DIFF, dict(L=3))),
    ("ack10_hl_rank2_16qam", 4, 20, 12, 7992, 10, 0, (HL, dict(N=9, pmi_present=True, rank_is_not_one=True))),
    ("ack3_ri1_extcp_qpsk", 2, 8, 10, 1736, 3, 1, (WB, dict())),
    ("ack2_ri2_extcp9_16qam", 4, 12, 9, 3624, 2, 2, (SB_UE, dict(subband_label_2_bits=True))),
    ("uci_only_hl_ri", 2, 4, 12, 0, 1, 1, (HL, dict(N=6, pmi_present=True))),
    ("uci_only_wb", 4, 2, 12, 0, 2, 0, (WB, dict(pmi_present=True, four_antenna_ports=True))),
    ("ack1_256qam", 8, 10, 12, 6200, 1, 1, (WB, dict(pmi_present=True, rank_is_not_one=True))),
    ("cqi_long_only", 6, 30, 12, 18336, 0, 0, (HL, dict(N=12))),
]


def make_cfg(Qm, L, nsymb, tbs, nack, ri_len, cqi, I=(9, 6, 8), rv=0, softbuffer=None):
    """srsran_pusch_cfg_t for L PRBs x N_symb, offsets I = (I_cqi, I_ri, I_ack)"""
    cfg = S.srsran_pusch_cfg_t()
    tb = cfg.grant.tb
    tb.mod = S.MOD_FROM_QM[Qm]
    tb.tbs = tbs
    tb.rv = rv
    tb.nof_bits = L * 12 * nsymb * Qm
    tb.enabled = True
    cfg.grant.L_prb = L
    cfg.grant.nof_symb = nsymb
    cfg.grant.nof_re = L * 12 * nsymb
    cfg.uci_offset.I_offset_cqi, cfg.uci_offset.I_offset_ri, cfg.uci_offset.I_offset_ack = I
    cfg.uci_cfg.ack[0].nof_acks = nack
    cfg.uci_cfg.cqi.ri_len = ri_len
    if cqi is not None:
        cfg.uci_cfg.cqi.data_enable = True
        cfg.uci_cfg.cqi.type = cqi[0]
        for k, v in cqi[1].items():
            setattr(cfg.uci_cfg.cqi, k, v)
    if softbuffer is not None:
        cfg.softbuffers.rx = __import__("ctypes").pointer(softbuffer.s)
    return cfg


def random_uci(cfg, rng):
    """random HARQ-ACK / RI / CQI values fitting the configuration"""
    u = S.srsran_uci_value_t()
    for i in range(cfg.uci_cfg.ack[0].nof_acks):
        u.ack.ack_value[i] = int(rng.integers(0, 2))
    # one RI bit carries the rank (the reference's transmitter keeps ri[1] = 0)
    u.ri = int(rng.integers(0, 2)) if cfg.uci_cfg.cqi.ri_len else 0
    c = cfg.uci_cfg.cqi
    if c.data_enable:
        t = c.type
        if t == WB:
            u.cqi.wideband.wideband_cqi = int(rng.integers(0, 16))
            u.cqi.wideband.spatial_diff_cqi = int(rng.integers(0, 8))
            u.cqi.wideband.pmi = int(rng.integers(0, 16 if c.four_antenna_ports else 2 if c.rank_is_not_one else 4))
        elif t == SB_UE:
            u.cqi.subband_ue.subband_cqi = int(rng.integers(0, 16))
            u.cqi.subband_ue.subband_label = int(rng.integers(0, 4 if c.subband_label_2_bits else 2))
        elif t == SB_DIFF:
            u.cqi.subband_ue_diff.wideband_cqi = int(rng.integers(0, 16))
            u.cqi.subband_ue_diff.subband_diff_cqi = int(rng.integers(0, 1 << c.L))
        else:
            u.cqi.subband_hl.wideband_cqi_cw0 = int(rng.integers(0, 16))
            u.cqi.subband_hl.subband_diff_cqi_cw0 = int(rng.integers(0, 1 << (2 * c.N)))
            u.cqi.subband_hl.wideband_cqi_cw1 = int(rng.integers(0, 16))
            u.cqi.subband_hl.subband_diff_cqi_cw1 = int(rng.integers(0, 1 << (2 * c.N)))
            u.cqi.subband_hl.pmi = int(rng.integers(0, 16 if c.four_antenna_ports else 2 if c.rank_is_not_one else 4))
    if c.data_enable and c.type == HL and c.ri_len:
        # the UE reports CQI for the rank it signals; without a TB the reference sizes RI / ACK from
        # the rank-1 report on receive (sch.c:1040-1044) but from the real one on transmit, so keep rank 1
        if cfg.grant.tb.tbs == 0:
            u.ri = 0
        c.rank_is_not_one = bool(u.ri)
    return u


def cqi_fields(cfg, v):
    """the CQI value fields the configuration carries, as a tuple"""
    c, t = cfg.uci_cfg.cqi, cfg.uci_cfg.cqi.type
    if t == WB:
        return (v.wideband.wideband_cqi, v.wideband.spatial_diff_cqi if (c.pmi_present and c.rank_is_not_one) else 0,
                v.wideband.pmi if c.pmi_present else 0)
    if t == SB_UE:
        return (v.subband_ue.subband_cqi, v.subband_ue.subband_label)
    if t == SB_DIFF:
        return (v.subband_ue_diff.wideband_cqi, v.subband_ue_diff.subband_diff_cqi)
    two = c.rank_is_not_one
    return (v.subband_hl.wideband_cqi_cw0, v.subband_hl.subband_diff_cqi_cw0,
            v.subband_hl.wideband_cqi_cw1 if two else 0, v.subband_hl.subband_diff_cqi_cw1 if two else 0,
            v.subband_hl.pmi if c.pmi_present else 0)
