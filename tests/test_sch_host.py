"""CPU tests of the DL-SCH host logic in the product library (no GPU needed).

srsran_cbsegm / cbsize / cbindex and the CRC utilities are host code of
srsran_4g_amd/csrc/sch_api.cpp (cbsegm.c:62-151, crc.c:69-195); they are checked
against the oracle (itself pinned to the reference, tests/test_sch_oracle.py).
Every device entry point must fail loudly without a HIP device.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import LTE_CRC24A, LTE_CRC24B, Oracle
from srsran_4g_amd import sch as S


@pytest.fixture(scope="module")
def ora():
    return Oracle()


def test_cbsize_table():
    from srsran_4g_amd.tdec import CB_SIZES
    L = S.lib()
    assert [L.srsran_cbsegm_cbsize(i) for i in range(188)] == list(CB_SIZES)
    assert L.srsran_cbsegm_cbsize(188) == -1
    for K in (40, 41, 6144, 6145, 528, 520):
        idx = L.srsran_cbsegm_cbindex(K)
        exp = next((i for i, k in enumerate(CB_SIZES) if k >= K), -1)
        assert idx == exp
        assert L.srsran_cbsegm_cbsize_isvalid(K) == (K in CB_SIZES)


def test_cbsegm_matches_oracle(ora):
    fields = ("C", "K1", "K2", "K1_idx", "K2_idx", "C1", "C2", "F")
    for tbs in list(range(0, 400000, 8))[::37] + [75376, 97896, 6120, 6200, 40, 16, 20, 391656, 500000]:
        rc, s = S.cbsegm(tbs)
        orc, o = ora.cbsegm(tbs)
        assert rc == orc, tbs
        if rc == 0:
            assert all(getattr(s, f) == o[f] for f in fields), (tbs, {f: getattr(s, f) for f in fields}, o)


def test_crc_host_matches_oracle(ora):
    rng = np.random.default_rng(1)
    for n in (8, 64, 6144, 75400):
        d = rng.integers(0, 256, n // 8 + 3, dtype=np.uint8)
        for p in (LTE_CRC24A, LTE_CRC24B):
            assert S.crc_checksum_byte(p, d, n) == ora.crc_byte(p, 24, d, n)
    # attach then match (crc.c:165-185)
    c = S.srsran_crc_t()
    L = S.lib()
    L.srsran_crc_init(ctypes.byref(c), LTE_CRC24A, 24)
    d = np.zeros(103, np.uint8)
    d[:100] = rng.integers(0, 256, 100, dtype=np.uint8)
    L.srsran_crc_attach_byte(ctypes.byref(c), d.ctypes.data_as(S._u8p), 800)
    assert L.srsran_crc_match_byte(ctypes.byref(c), d.ctypes.data_as(S._u8p), 800)
    d[5] ^= 1
    assert not L.srsran_crc_match_byte(ctypes.byref(c), d.ctypes.data_as(S._u8p), 800)


def test_mod_bits():
    L = S.lib()
    assert [L.srsran_mod_bits_x_symbol(m) for m in range(6)] == [1, 2, 4, 6, 8, 0]


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_device_entry_points_fail_without_gpu():
    L = S.lib()
    sb = S.srsran_softbuffer_rx_t()
    assert L.srsran_softbuffer_rx_init(ctypes.byref(sb), 100) != 0
    q = S.srsran_sch_t()
    assert L.srsran_sch_init(ctypes.byref(q)) != 0
    e = np.zeros(300, np.int16)
    out = np.zeros(S.SOFTBUFFER_SIZE, np.int16)
    assert L.srsran_rm_turbo_rx_lut(e.ctypes.data_as(S._i16p), out.ctypes.data_as(S._i16p), 300, 0, 0) != 0
    assert not out.any()


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors must match include/srsran_sch.h as compiled by a C compiler."""
    import os
    import subprocess
    src = tmp_path / "l.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "srsran_sch.h"\nint main(){printf("%zu %zu %zu %zu %zu '
        '%zu %zu %zu %zu %zu %zu\\n", sizeof(srsran_cbsegm_t), sizeof(srsran_crc_t), sizeof(srsran_softbuffer_rx_t),'
        ' sizeof(srsran_ra_tb_t), sizeof(srsran_pdsch_grant_t), sizeof(srsran_pdsch_cfg_t), sizeof(srsran_sch_t),'
        ' sizeof(srsran_dlsch_gpu_tb_t), offsetof(srsran_pdsch_cfg_t, softbuffers), offsetof(srsran_sch_t, gpu),'
        ' offsetof(srsran_pdsch_grant_t, nof_layers));}\n')
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.check_call(["gcc", "-I", inc, str(src), "-o", str(tmp_path / "l")])
    got = [int(x) for x in subprocess.check_output([str(tmp_path / "l")]).split()]
    exp = [ctypes.sizeof(t) for t in (S.srsran_cbsegm_t, S.srsran_crc_t, S.srsran_softbuffer_rx_t, S.srsran_ra_tb_t,
                                      S.srsran_pdsch_grant_t, S.srsran_pdsch_cfg_t, S.srsran_sch_t,
                                      S.srsran_dlsch_gpu_tb_t)]
    exp += [S.srsran_pdsch_cfg_t.softbuffers.offset, S.srsran_sch_t.gpu.offset,
            S.srsran_pdsch_grant_t.nof_layers.offset]
    assert got == exp
