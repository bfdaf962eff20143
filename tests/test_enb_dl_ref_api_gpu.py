"""The reference-named eNB DL object (include/srsran_enb_dl.h section enb_dl.h, enb_dl.h:101-124) as srsENB and
lib/test/phy/phy_dl_test.c:152-196 drive it, one subframe at a time: srsran_enb_dl_put_base ->
srsran_enb_dl_put_pdcch_dl -> srsran_ra_dl_dci_to_grant -> srsran_enb_dl_put_pdsch -> srsran_enb_dl_gen_signal.

* Through ctypes: the time samples in out_buffer equal the batched transmitter's (srsran_enb_dl_gpu_tx_batch, whose
  control REs are pinned to the reference's own pcfich.c / pdcch.c / regs.c by test_enb_ctrl_gpu.py and PDSCH REs to
  the reference's composition by test_pdsch_tx_ref_gpu.py) for the same subframe, with the reference's PDSCH scaling
  rho_a (pdsch.c:492, 1057-1071); the GPU UE finds the DCI and decodes the PDSCH (power_scale on, as phy_dl_test).
* A C99 program written like phy_dl_test.c's work_enb, compiled here against include/ and linked against the
  in-tree libsrsran_4g_amd.so, runs the same sequence; the UE decodes its samples."""
import ctypes
import os
import subprocess
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F1, F1A, F2A = 1, 2, 7
TM1, TM2, TM3 = 0, 1, 2

CASES = [  # (nof_prb, ports, tm, format, mcs, tti, cfi)
    (100, 2, TM3, F2A, 27, 3, 1),
    (50, 2, TM2, F1, 18, 5, 2),
    (25, 1, TM1, F1A, 12, 0, 3),
    (15, 4, TM2, F1, 10, 7, 2),
]


@pytest.fixture(scope="module")
def env():
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.fail("no HIP device on a GPU test run")
    import torch
    return torch


def _dci(PD, U, cell, nprb, fmt, mcs, tti, cfi, rnti, nof_cce):
    d = PD.srsran_dci_dl_t()
    d.rnti, d.format, d.pid = rnti, fmt, 2
    if fmt == F1A:
        d.alloc_type = 2
        d.raw[0] = U.lib().srsran_ra_type2_to_riv(nprb, 0, nprb)
        d.raw[1] = d.raw[2] = d.raw[3] = 0
    else:
        d.alloc_type = 0
        d.raw[0] = (1 << int(np.ceil(nprb / U.lib().srsran_ra_type0_P(nprb)))) - 1
    for i in range(2 if fmt == F2A else 1):
        d.tb[i].mcs_idx, d.tb[i].rv, d.tb[i].ndi, d.tb[i].cw_idx = mcs, 0, True, i
    locs = [loc for loc in PD.ue_locations(nof_cce, tti % 10, rnti) if (1 << loc[0]) <= nof_cce]
    d.location.L, d.location.ncce = max(locs)
    return d


def _ue_decode(U, S, cell, P, rx, tti, cfi, rnti, tm, fmt, pls, grant):
    ue = U.UeDl(cell, rx.shape[0])
    try:
        assert ue.fft_estimate(list(rx), tti, 0) == 0 and ue.last_cfi == cfi
        dcis = ue.find_dl_dci(tti, cfi, rnti, tm=tm)
        assert len(dcis) == 1 and dcis[0].format == fmt and dcis[0].rnti == rnti
        r, g = ue.dci_to_grant(dcis[0], tti, cfi, tm=tm)
        assert r == 0 and g.nof_tb == len(pls) and g.nof_re == grant.nof_re
        qm_of = {m: q for q, m in S.MOD_FROM_QM.items()}
        sbs = [S.SoftbufferRx(nof_prb=cell.nof_prb) for _ in pls]
        ucfg = U.pdsch_cfg(cell.nof_prb, g.nof_re, [g.tb[i].tbs for i in range(len(pls))],
                           [qm_of[g.tb[i].mod] for i in range(len(pls))], rnti=rnti, softbuffers=sbs,
                           scheme={F2A: "cdd", F1: "diversity" if P > 1 else "port0",
                                   F1A: "diversity" if P > 1 else "port0"}[fmt], nof_ports=P,
                           power_scale=True, p_a=0.0)
        ucfg.grant = g
        ret, res = ue.decode_pdsch(ucfg, tti, cfi)
        assert ret == 0
        for i, pl in enumerate(pls):
            assert res[i][0] and np.array_equal(res[i][1][:len(pl)], pl), i
        for sb in sbs:
            sb.free()
    finally:
        ue.free()


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}prb_{c[1]}p_tm{c[2] + 1}_sf{c[5]}" for c in CASES])
def test_reference_api_equals_batch_and_decodes(env, case):
    torch = env
    from srsran_4g_amd import enb_dl as E
    from srsran_4g_amd import pdcch as PD
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import ue_dl as U
    nprb, P, tm, fmt, mcs, tti, cfi = case
    cell_id, rnti = 301, 0x3C11
    U.use_standard_symbol_size(True)
    cell = U.cell(nprb, P, cell_id)
    N = U.lib().srsran_symbol_sz(nprb)
    out = [np.zeros(15 * N, np.complex64) for _ in range(P)]
    enb = E.EnbDlRef(cell, out)
    try:
        nof_cce = enb.q.pdcch.nof_cce[cfi - 1]
        regs = PD.Regs(cell)
        assert nof_cce == regs.q.pdcch_nregs[cfi - 1] // 9  # the object's PDCCH locations are the cell's
        regs.free()
        assert enb.is_common(3, 0) == False  # dl_sf not set yet: no CFI, nothing is common (enb_dl.c:384-390)
        d = _dci(PD, U, cell, nprb, fmt, mcs, tti, cfi, rnti, nof_cce)
        r, grant = PD.dci_to_grant(cell, d, tti, cfi, tm)
        assert r == 0
        ntb = grant.nof_tb
        rng = np.random.default_rng(nprb + tti)
        pls = [rng.integers(0, 256, grant.tb[i].tbs // 8, dtype=np.uint8) for i in range(ntb)]
        qm_of = {m: q for q, m in S.MOD_FROM_QM.items()}
        cfg = U.pdsch_cfg(nprb, grant.nof_re, [grant.tb[i].tbs for i in range(ntb)],
                          [qm_of[grant.tb[i].mod] for i in range(ntb)], rnti=rnti, power_scale=True, p_a=0.0)
        cfg.grant = grant
        sf = U.sf_cfg(tti, cfi)
        enb.put_base(sf)
        assert enb.is_common(2, 0) and not enb.is_common(2, 1)
        assert enb.put_pdcch_dl(U.srsran_dci_cfg_t(), d) == 0
        assert enb.put_pdsch(cfg, pls) == 0
        enb.gen_signal()
        got = np.stack(out)
        grid = [enb.sf_symbols(p, 14 * 12 * nprb) for p in range(P)]
    finally:
        enb.free()
    # the same subframe through the batch, with the reference's rho_a
    r, msg = PD.pack_pdsch(cell, d)
    assert r == 0
    b = E.EnbDl(cell)
    d_pl = [torch.from_numpy(p).cuda() for p in pls]
    d_tx = torch.zeros((1, P, 15 * N, 2), dtype=torch.float32, device="cuda")
    rho = float(np.float32(np.sqrt(2.0))) if P > 1 else 1.0
    assert b.tx_batch([(tti, cfi, cfg, [p.data_ptr() for p in d_pl], (True, [msg]))], d_tx.data_ptr(),
                      pdsch_scaling=rho) == 0
    torch.cuda.synchronize()
    want = d_tx.cpu().numpy().view(np.complex64)[0, :, :, 0]
    b.free()
    assert np.array_equal(got, want)
    assert any(np.abs(g).max() > 0 for g in grid)
    # the UE: channel [[1, 1], [1, -1]] (2 ports, phy_dl_test.c:568-583) / identity (1) / two rows (4), 30 dB
    H = {1: np.ones((1, 1)), 2: np.array([[1, 1], [1, -1]]), 4: np.array([[1, 1, 1, 1], [1, -1, 1, -1]])}[P]
    rx = (H.astype(np.complex64) @ got).astype(np.complex64)
    sigma = np.sqrt(np.mean(np.abs(rx) ** 2) / 10 ** 3.0 / 2)
    rng = np.random.default_rng(99)
    rx = (rx + sigma * (rng.standard_normal(rx.shape) + 1j * rng.standard_normal(rx.shape))).astype(np.complex64)
    _ue_decode(U, S, cell, P, rx, tti, cfi, rnti, tm, fmt, pls, grant)


C_CALLER = r'''
/* work_enb of lib/test/phy/phy_dl_test.c:152-196, over libsrsran_4g_amd.so: one subframe, its samples and payload
 * to argv[1] ([P][sf_len] cf_t, then the payload bytes) */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "srsran_enb_dl.h"

int main(int argc, char** argv)
{
  srsran_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.nof_prb = 50; cell.nof_ports = 2; cell.id = 77; cell.cp = SRSRAN_CP_NORM;
  cell.phich_length = SRSRAN_PHICH_NORM; cell.phich_resources = SRSRAN_PHICH_R_1;
  const uint32_t sf_len = 15 * (uint32_t)srsran_symbol_sz(cell.nof_prb);
  cf_t* out[SRSRAN_MAX_PORTS] = {NULL};
  for (int p = 0; p < SRSRAN_MAX_PORTS; p++) {
    out[p] = calloc(sf_len, sizeof(cf_t));
  }
  srsran_enb_dl_t* enb_dl = malloc(sizeof(srsran_enb_dl_t));
  if (srsran_enb_dl_init(enb_dl, out, cell.nof_prb) || srsran_enb_dl_set_cell(enb_dl, cell)) {
    fprintf(stderr, "init\n");
    return 1;
  }
  srsran_dl_sf_cfg_t dl_sf;
  memset(&dl_sf, 0, sizeof(dl_sf));
  dl_sf.tti = 3;
  dl_sf.cfi = 2;
  const uint16_t rnti = 0x1234;
  srsran_dci_dl_t dci;
  memset(&dci, 0, sizeof(dci));
  dci.rnti = rnti; dci.format = SRSRAN_DCI_FORMAT1; dci.alloc_type = SRSRAN_RA_ALLOC_TYPE0; dci.pid = 1;
  dci.type0_alloc.rbg_bitmask = 0x1ffff;  /* 17 RBGs of 3 PRB: the whole 50-PRB cell */
  dci.tb[0].mcs_idx = 16; dci.tb[0].ndi = true; dci.tb[0].rv = 0; dci.tb[0].cw_idx = 0;
  srsran_dci_location_t locs[SRSRAN_MAX_CANDIDATES_UE];
  uint32_t n = srsran_pdcch_ue_locations(&enb_dl->pdcch, &dl_sf, locs, SRSRAN_MAX_CANDIDATES_UE, rnti);
  if (n == 0) {
    return 2;
  }
  dci.location = locs[n - 1];
  srsran_dci_cfg_t dci_cfg;
  memset(&dci_cfg, 0, sizeof(dci_cfg));

  srsran_enb_dl_put_base(enb_dl, &dl_sf);
  if (srsran_enb_dl_put_pdcch_dl(enb_dl, &dci_cfg, &dci)) {
    return 3;
  }
  srsran_pdsch_cfg_t pdsch_cfg;
  memset(&pdsch_cfg, 0, sizeof(pdsch_cfg));
  if (srsran_ra_dl_dci_to_grant(&cell, &dl_sf, SRSRAN_TM2, false, &dci, &pdsch_cfg.grant)) {
    return 4;
  }
  pdsch_cfg.power_scale = true;
  pdsch_cfg.p_a         = 0.0f;
  pdsch_cfg.p_b         = 1;
  pdsch_cfg.rnti        = rnti;
  const uint32_t nbytes = (uint32_t)pdsch_cfg.grant.tb[0].tbs / 8;
  uint8_t* data_tx[SRSRAN_MAX_CODEWORDS] = {malloc(nbytes), NULL};
  for (uint32_t i = 0; i < nbytes; i++) {
    data_tx[0][i] = (uint8_t)((i * 37 + 11) & 0xff);
  }
  if (srsran_enb_dl_put_pdsch(enb_dl, &pdsch_cfg, data_tx) < 0) {
    return 5;
  }
  srsran_enb_dl_gen_signal(enb_dl);
  FILE* f = fopen(argv[1], "wb");
  for (uint32_t p = 0; p < cell.nof_ports; p++) {
    fwrite(out[p], sizeof(cf_t), sf_len, f);
  }
  fwrite(data_tx[0], 1, nbytes, f);
  fclose(f);
  printf("%u %u\n", sf_len, nbytes);
  srsran_enb_dl_free(enb_dl);
  free(enb_dl);
  free(data_tx[0]);
  for (int p = 0; p < SRSRAN_MAX_PORTS; p++) {
    free(out[p]);
  }
  return 0;
}
'''


def test_c99_caller_like_phy_dl_test(env):
    from srsran_4g_amd import pdcch as PD
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import tdec
    from srsran_4g_amd import ue_dl as U
    libdir = os.path.dirname(tdec.LIB_PATH)
    with tempfile.TemporaryDirectory() as d:
        src, exe, dat = os.path.join(d, "enb.c"), os.path.join(d, "enb"), os.path.join(d, "sf.bin")
        open(src, "w").write(C_CALLER)
        r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), src, "-o", exe,
                            "-L", libdir, "-lsrsran_4g_amd", "-Wl,-rpath," + libdir, "-lm"],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]
        r = subprocess.run([exe, dat], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
        sf_len, nbytes = map(int, r.stdout.split())
        raw = open(dat, "rb").read()
    x = np.frombuffer(raw[:2 * sf_len * 8], np.complex64).reshape(2, sf_len)
    pl = np.frombuffer(raw[2 * sf_len * 8:], np.uint8)
    assert len(pl) == nbytes and np.array_equal(pl, (np.arange(nbytes) * 37 + 11) & 0xff)
    U.use_standard_symbol_size(False)  # the C caller used the library's default (the reference's) symbol size
    try:
        cell = U.cell(50, 2, 77)
        rx = (np.array([[1, 1], [1, -1]], np.complex64) @ x).astype(np.complex64)
        d = PD.srsran_dci_dl_t()
        d.rnti, d.format, d.alloc_type = 0x1234, F1, 0
        d.raw[0] = 0x1ffff
        d.tb[0].mcs_idx, d.tb[0].ndi, d.tb[0].cw_idx = 16, True, 0
        r, grant = PD.dci_to_grant(cell, d, 3, 2, TM2)
        assert r == 0 and grant.tb[0].tbs // 8 == nbytes
        _ue_decode(U, S, cell, 2, rx, 3, 2, 0x1234, TM2, F1, [pl], grant)
    finally:
        U.use_standard_symbol_size(True)
