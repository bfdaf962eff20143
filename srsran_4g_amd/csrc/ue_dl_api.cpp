// srsran_4g_amd/csrc/ue_dl_api.cpp -- the PDSCH slice of srsran_ue_dl_t (include/srsran_ue_dl.h).
//
// Host-synchronous: srsran_ue_dl_init / set_cell / decode_fft_estimate(_noguru) / decode_pdsch
// (ue_dl.c:67-180, 349-384, 700-706) over the GPU OFDM, channel estimator and PDSCH objects.
// Batched: srsran_ue_dl_gpu_decode_batch chains, on one stream and without host round trips,
//   OFDM (CFO rotation fused)  ->  CRS estimation of every subframe  ->  PDSCH decode batch.
// Control channels (ue_dl.c:315-347, 386-698): decode_fft_estimate decodes the PCFICH (sets sf->cfi)
// and extracts the PDCCH LLRs on the GPU; srsran_ue_dl_find_dl_dci blind-searches them, every
// candidate of the search spaces in one launch.  The batch path takes the CFI from its caller.
#include <hip/hip_runtime.h>

#include <cmath>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/srsran_pdcch.h"
#include "chest_kernel.h"
#include "pdsch_internal.h"
#include "stage_copy.h"
#include "stage_timing.h"
#include "../../include/srsran_ue_dl.h"

namespace {

constexpr int kStageRing = 3;  // batches whose sf-index upload may be in flight (a ring, as the PDSCH / SCH staging)

struct UeDlGpu {
  srsran_amd::StreamHandoff ho;  // stream of the previous batch (d_grid / d_ce / d_res shared between batches)
  hipEvent_t staged[kStageRing] = {};  // the estimator launch that reads the slot's subframe indices finished
  uint32_t   ring_next          = 0;
  // subframe indices, kStageRing slots of cap entries, in pinned coherent host memory that the estimator
  // reads in place (d_sf: its device alias) -- no upload, which in the stream cost a copy launch and ~20 us
  // of GPU idle per batch (gpurun_out r04j rocprof trace)
  uint32_t*  h_sf   = nullptr;
  uint32_t*  d_sf   = nullptr;
  float2*    d_grid = nullptr;
  float2*    d_ce   = nullptr;
  float*     d_res  = nullptr;
  uint32_t   cap    = 0;  // subframes
  bool       cap_full = false;  // d_ce sized for full-grid (INTERPOLATE) estimates
  // control channels (srsran_ue_dl_t::regs / pcfich / pdcch of the reference)
  srsran_regs_t         regs{};
  srsran_pcfich_t       pcfich{};
  srsran_pdcch_t        pdcch{};
  bool                  ctrl_init = false;  // objects allocated (<= 2 rx antennas)
  bool                  ctrl_cell = false;  // tables built for the current cell
  srsran_dci_location_t allocated[SRSRAN_MAX_DCI_MSG];
  uint32_t              nof_allocated = 0;
  srsran_dci_msg_t      pending_ul[SRSRAN_MAX_DCI_MSG];
  uint32_t              nof_pending_ul = 0;
  // PHICH m_i of the PDCCH's REG tables (ue_dl.c:263-273): `regs` has m_i = 1 (FDD), regs_mi the
  // tables of m_i = 0 and 2 for srsran_ue_dl_set_mi_manual; a TDD cell with the extended PHICH duration also has
  // regs_ext, the tables of m_i = 1, 0, 2 whose PHICH keeps to two symbols (subframes 1 and 6, ue_dl.c:59-64, 198)
  srsran_regs_t        regs_mi[2]{};
  srsran_regs_t        regs_ext[3]{};
  bool                 ext_tables = false;
  bool                 mi_auto    = true;
  uint32_t             mi_manual  = 1;
  const srsran_regs_t* regs_set   = nullptr;  // the tables the PDCCH object holds
};

// 36.213 Table 6.9-1: PHICH m_i per TDD uplink-downlink configuration and subframe (ue_dl.c:50-57)
const uint8_t kMiTdd[7][10] = {{2, 1, 0, 0, 0, 2, 1, 0, 0, 0}, {0, 1, 0, 0, 1, 0, 1, 0, 0, 1},
                               {0, 0, 0, 1, 0, 0, 0, 0, 1, 0}, {1, 0, 0, 0, 0, 0, 0, 0, 1, 1},
                               {0, 0, 0, 0, 0, 0, 0, 0, 1, 1}, {0, 0, 0, 0, 0, 0, 0, 0, 1, 0},
                               {1, 1, 0, 0, 0, 1, 1, 0, 0, 1}};

// set_mi_value (ue_dl.c:296-313): the PDCCH works on the REG tables of the selected m_i (MI_VALUE: 1 for FDD, the
// table above for TDD)
void select_mi(UeDlGpu* g, const srsran_cell_t& cell, const srsran_dl_sf_cfg_t* sf)
{
  const uint32_t auto_mi = cell.frame_type == SRSRAN_FDD || sf->tdd_config.sf_config >= 7
                               ? 1u
                               : kMiTdd[sf->tdd_config.sf_config][sf->tti % 10];
  const uint32_t mi      = g->mi_auto ? auto_mi : g->mi_manual;
  // MI_IDX: + 3 (the two-symbol PHICH tables) for a TDD cell with the extended duration in subframes 1 and 6; the
  // manual choice never adds it (ue_dl.c:308-311)
  const bool           ext = g->mi_auto && g->ext_tables && (sf->tti % 10 == 1 || sf->tti % 10 == 6);
  const uint32_t       i   = mi == 1 ? 0 : mi == 0 ? 1 : 2;  // mi_reg_idx_inv
  srsran_regs_t* const t   = ext ? &g->regs_ext[i] : i == 0 ? &g->regs : &g->regs_mi[i - 1];
  if (t != g->regs_set) {
    srsran_pdcch_set_regs(&g->pdcch, t);
    g->regs_set = t;
  }
}

bool grow(srsran_ue_dl_t* q, UeDlGpu* g, uint32_t nsf, bool full)
{
  if (g->cap >= nsf && (g->cap_full || !full)) {
    return true;
  }
  hipDeviceSynchronize();
  hipHostFree(g->h_sf);
  hipFree(g->d_grid);
  hipFree(g->d_ce);
  hipFree(g->d_res);
  g->h_sf = nullptr, g->d_sf = nullptr, g->d_grid = nullptr, g->d_ce = nullptr, g->d_res = nullptr;
  g->cap             = 0;
  const size_t nre   = 12 * (size_t)q->cell.nof_prb;
  const size_t nrx   = q->nof_rx_antennas;
  const size_t ports = q->cell.nof_ports;
  if (hipHostMalloc((void**)&g->h_sf, kStageRing * nsf * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&g->d_sf, g->h_sf, 0) != hipSuccess ||
      hipMalloc((void**)&g->d_grid, nsf * nrx * 14 * nre * sizeof(float2)) != hipSuccess ||
      hipMalloc((void**)&g->d_ce, nsf * ports * nrx * nre * (full ? 14 : 1) * sizeof(float2)) != hipSuccess ||
      hipMalloc((void**)&g->d_res, nsf * 4 * sizeof(float)) != hipSuccess) {
    return false;
  }
  g->cap      = nsf;
  g->cap_full = full;
  return true;
}



}  // namespace

extern "C" {

int srsran_ue_dl_init(srsran_ue_dl_t* q, cf_t* input[SRSRAN_MAX_PORTS], uint32_t max_prb, uint32_t nof_rx_antennas)
{
  if (!q || nof_rx_antennas == 0 || nof_rx_antennas > SRSRAN_MAX_PORTS || max_prb == 0 || max_prb > SRSRAN_MAX_PRB) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(q, 0, sizeof(*q));
  q->nof_rx_antennas = nof_rx_antennas;
  for (int j = 0; j < SRSRAN_MAX_PORTS; j++) {
    q->sf_symbols[j] = (cf_t*)calloc((size_t)14 * 12 * max_prb, sizeof(cf_t));
    if (!q->sf_symbols[j]) {
      srsran_ue_dl_free(q);
      return SRSRAN_ERROR;
    }
  }
  srsran_ofdm_cfg_t ofdm_cfg;  // ue_dl.c:88-98
  memset(&ofdm_cfg, 0, sizeof(ofdm_cfg));
  ofdm_cfg.nof_prb          = max_prb;
  ofdm_cfg.cp               = SRSRAN_CP_NORM;
  ofdm_cfg.rx_window_offset = 0.0f;
  ofdm_cfg.normalize        = false;
  ofdm_cfg.sf_type          = SRSRAN_SF_NORM;
  for (uint32_t i = 0; i < nof_rx_antennas; i++) {
    ofdm_cfg.in_buffer  = input ? input[i] : nullptr;
    ofdm_cfg.out_buffer = q->sf_symbols[i];
    if (srsran_ofdm_rx_init_cfg(&q->fft[i], &ofdm_cfg)) {
      fprintf(stderr, "[srsran_ue_dl] Error initiating FFT\n");
      srsran_ue_dl_free(q);
      return SRSRAN_ERROR;
    }
  }
  ofdm_cfg.in_buffer  = input ? input[0] : nullptr;  // ue_dl.c:104-111: the MBSFN transform reads antenna 0 only
  ofdm_cfg.out_buffer = q->sf_symbols[0];
  ofdm_cfg.sf_type    = SRSRAN_SF_MBSFN;
  if (srsran_ofdm_rx_init_cfg(&q->fft_mbsfn, &ofdm_cfg)) {
    fprintf(stderr, "[srsran_ue_dl] Error initiating FFT for MBSFN subframes\n");
    srsran_ue_dl_free(q);
    return SRSRAN_ERROR;
  }
  srsran_ofdm_set_non_mbsfn_region(&q->fft_mbsfn, 2);
  if (srsran_chest_dl_init(&q->chest, max_prb, nof_rx_antennas) || srsran_chest_dl_res_init(&q->chest_res, max_prb) ||
      srsran_pdsch_init_ue(&q->pdsch, max_prb, nof_rx_antennas)) {
    fprintf(stderr, "[srsran_ue_dl] Error initiating channel estimator / PDSCH\n");
    srsran_ue_dl_free(q);
    return SRSRAN_ERROR;
  }
  UeDlGpu* g = new UeDlGpu();
  q->gpu     = g;
  for (hipEvent_t& e : g->staged) {
    if (srsran_amd::ring_event_create(&e) != hipSuccess) {
      srsran_ue_dl_free(q);
      return SRSRAN_ERROR;
    }
  }
  if (nof_rx_antennas <= 2) {
    if (srsran_pcfich_init(&g->pcfich, nof_rx_antennas) || srsran_pdcch_init_ue(&g->pdcch, max_prb, nof_rx_antennas)) {
      srsran_ue_dl_free(q);
      return SRSRAN_ERROR;
    }
    g->ctrl_init = true;
  }
  return SRSRAN_SUCCESS;
}

void srsran_ue_dl_free(srsran_ue_dl_t* q)
{
  if (!q) {
    return;
  }
  UeDlGpu* g = (UeDlGpu*)q->gpu;
  if (g) {
    hipDeviceSynchronize();
    hipHostFree(g->h_sf);
    hipFree(g->d_grid);
    hipFree(g->d_ce);
    hipFree(g->d_res);
    for (hipEvent_t e : g->staged) {
      if (e) {
        hipEventDestroy(e);
      }
    }
    if (g->ctrl_init) {
      srsran_pcfich_free(&g->pcfich);
      srsran_pdcch_free(&g->pdcch);
    }
    srsran_regs_free(&g->regs);
    srsran_regs_free(&g->regs_mi[0]);
    srsran_regs_free(&g->regs_mi[1]);
    for (auto& r : g->regs_ext) {
      srsran_regs_free(&r);
    }
    srsran_amd::handoff_free(g->ho);
    delete g;
  }
  for (int j = 0; j < SRSRAN_MAX_PORTS; j++) {
    if (q->fft[j].gpu) {
      srsran_ofdm_rx_free(&q->fft[j]);
    }
    free(q->sf_symbols[j]);
  }
  if (q->fft_mbsfn.gpu) {
    srsran_ofdm_rx_free(&q->fft_mbsfn);
  }
  if (q->chest.gpu) {
    srsran_chest_dl_free(&q->chest);
  }
  srsran_chest_dl_res_free(&q->chest_res);
  if (q->pdsch.gpu) {
    srsran_pdsch_free(&q->pdsch);
  }
  memset(q, 0, sizeof(*q));
}

int srsran_ue_dl_set_cell(srsran_ue_dl_t* q, srsran_cell_t cell)
{
  if (!q || !q->gpu || cell.nof_prb == 0 || cell.nof_prb > SRSRAN_MAX_PRB) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  for (uint32_t i = 0; i < q->nof_rx_antennas; i++) {
    if (srsran_ofdm_rx_set_prb(&q->fft[i], cell.cp, cell.nof_prb)) {
      fprintf(stderr, "[srsran_ue_dl] Error setting FFT sampling frequency\n");
      return SRSRAN_ERROR;
    }
  }
  if (srsran_ofdm_rx_set_prb(&q->fft_mbsfn, SRSRAN_CP_EXT, cell.nof_prb)) {  // ue_dl.c:218-221
    fprintf(stderr, "[srsran_ue_dl] Error resizing MBSFN FFT\n");
    return SRSRAN_ERROR;
  }
  if (srsran_chest_dl_set_cell(&q->chest, cell) || srsran_pdsch_set_cell(&q->pdsch, cell)) {
    return SRSRAN_ERROR;
  }
  UeDlGpu* g = (UeDlGpu*)q->gpu;
  q->cell    = cell;
  g->cap     = 0;  // buffer shapes depend on the cell
  // control channels: 1, 2 or 4 ports, normal or extended PHICH duration (others: PDSCH only, CFI from the caller);
  // the REG tables of ue_dl.c:190-203 (SRSRAN_MI_NOF_REGS: 1 FDD, 6 TDD -- the m_i = 0 / 2 ones kept for FDD too,
  // srsran_ue_dl_set_mi_manual; the two-symbol PHICH ones only where MI_IDX can select them)
  srsran_regs_free(&g->regs);
  srsran_regs_free(&g->regs_mi[0]);
  srsran_regs_free(&g->regs_mi[1]);
  for (auto& r : g->regs_ext) {
    srsran_regs_free(&r);
  }
  g->ext_tables = cell.frame_type == SRSRAN_TDD && cell.phich_length == SRSRAN_PHICH_EXT;
  g->ctrl_cell  = g->ctrl_init && (cell.nof_ports == 1 || cell.nof_ports == 2 || cell.nof_ports == 4) &&
                 srsran_regs_init(&g->regs, cell) == SRSRAN_SUCCESS &&
                 srsran_regs_init_opts(&g->regs_mi[0], cell, 0, false) == SRSRAN_SUCCESS &&
                 srsran_regs_init_opts(&g->regs_mi[1], cell, 2, false) == SRSRAN_SUCCESS &&
                 (!g->ext_tables || (srsran_regs_init_opts(&g->regs_ext[0], cell, 1, true) == SRSRAN_SUCCESS &&
                                     srsran_regs_init_opts(&g->regs_ext[1], cell, 0, true) == SRSRAN_SUCCESS &&
                                     srsran_regs_init_opts(&g->regs_ext[2], cell, 2, true) == SRSRAN_SUCCESS)) &&
                 srsran_pcfich_set_cell(&g->pcfich, &g->regs, cell) == SRSRAN_SUCCESS &&
                 srsran_pdcch_set_cell(&g->pdcch, &g->regs, cell) == SRSRAN_SUCCESS;
  g->regs_set = &g->regs;
  g->nof_pending_ul = 0;  // ue_dl.c:189
  hipDeviceSynchronize();
  hipHostFree(g->h_sf);
  hipFree(g->d_grid);
  hipFree(g->d_ce);
  hipFree(g->d_res);
  g->h_sf = nullptr, g->d_sf = nullptr, g->d_grid = nullptr, g->d_ce = nullptr, g->d_res = nullptr;
  return SRSRAN_SUCCESS;
}

static int fft_estimate(srsran_ue_dl_t* q, srsran_dl_sf_cfg_t* sf, srsran_ue_dl_cfg_t* cfg, cf_t* input[])
{
  if (!q || !q->gpu || !sf || !cfg) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (sf->sf_type == SRSRAN_SF_MBSFN) {
    // ue_dl.c:353-356 / 373-376: fft_mbsfn, configured on antenna 0's buffers, runs once per antenna (the same
    // transform each time; its _ng form ignores the arguments, ofdm.c:576-578): the other antennas' grids keep the
    // previous subframe
    if (!q->fft_mbsfn.cfg.in_buffer) {
      fprintf(stderr, "[srsran_ue_dl] MBSFN subframes need the input buffers given to srsran_ue_dl_init\n");
      return SRSRAN_ERROR;
    }
    srsran_ofdm_rx_sf(&q->fft_mbsfn);
  } else if (sf->sf_type != SRSRAN_SF_NORM) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  } else {
    for (uint32_t j = 0; j < q->nof_rx_antennas; j++) {
      if (input) {
        srsran_ofdm_rx_sf_ng(&q->fft[j], input[j], q->sf_symbols[j]);
      } else {
        srsran_ofdm_rx_sf(&q->fft[j]);
      }
    }
  }
  if (srsran_chest_dl_estimate_cfg(&q->chest, sf, &cfg->chest_cfg, q->sf_symbols, &q->chest_res)) {
    return SRSRAN_ERROR;
  }
  // estimate_pdcch_pcfich (ue_dl.c:315-347): PCFICH -> sf->cfi, then the PDCCH LLRs
  UeDlGpu* g = (UeDlGpu*)q->gpu;
  if (!g->ctrl_cell) {
    return sf->cfi >= 1 && sf->cfi <= 3 ? SRSRAN_SUCCESS : SRSRAN_ERROR;  // CFI from the caller
  }
  float corr = 0;
  select_mi(g, q->cell, sf);
  if (srsran_pcfich_decode(&g->pcfich, sf, &q->chest_res, q->sf_symbols, &corr) < 0) {
    fprintf(stderr, "[srsran_ue_dl] Error decoding PCFICH\n");
    return SRSRAN_ERROR;
  }
  if (q->cell.frame_type == SRSRAN_TDD && (sf->tti % 10 == 1 || sf->tti % 10 == 6) && sf->cfi == 3) {
    sf->cfi = 2;  // ue_dl.c:331-334: at most 2 control symbols in the special subframes' DwPTS
  }
  if (srsran_pdcch_extract_llr(&g->pdcch, sf, &q->chest_res, q->sf_symbols)) {
    fprintf(stderr, "[srsran_ue_dl] Error extracting PDCCH LLRs\n");
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

int srsran_ue_dl_decode_fft_estimate(srsran_ue_dl_t* q, srsran_dl_sf_cfg_t* sf, srsran_ue_dl_cfg_t* cfg)
{
  return fft_estimate(q, sf, cfg, nullptr);
}

int srsran_ue_dl_decode_fft_estimate_noguru(srsran_ue_dl_t*     q,
                                            srsran_dl_sf_cfg_t* sf,
                                            srsran_ue_dl_cfg_t* cfg,
                                            cf_t*               input[SRSRAN_MAX_PORTS])
{
  if (!input) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  return fft_estimate(q, sf, cfg, input);
}

int srsran_ue_dl_decode_pdsch(srsran_ue_dl_t*     q,
                              srsran_dl_sf_cfg_t* sf,
                              srsran_pdsch_cfg_t* pdsch_cfg,
                              srsran_pdsch_res_t  data[SRSRAN_MAX_CODEWORDS])
{
  if (!q) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  return srsran_pdsch_decode(&q->pdsch, sf, pdsch_cfg, &q->chest_res, q->sf_symbols, data);
}

// the batch over cf_t samples (d16 null) or int16 I/Q ones converted x scale in the OFDM load
static int decode_batch(srsran_ue_dl_t*              q,
                        srsran_ue_dl_cfg_t*          cfg,
                        uint32_t                     nof_sf,
                        const srsran_ue_dl_gpu_sf_t* sfs,
                        const cf_t*                  d_samples,
                        const int16_t*               d16,
                        float                        scale,
                        float                        cfo,
                        int32_t*                     d_result,
                        float*                       d_avg_noi,
                        void*                        stream)
{
  if (!q || !q->gpu || !cfg || (nof_sf && (!sfs || (!d_samples && !d16) || !d_result || !d_avg_noi))) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_sf == 0) {
    return 0;
  }
  srsran_amd::HostScope whole(srsran_amd::HP_UE_DL);
  srsran_amd::HostScope front(srsran_amd::HP_FRONT);
  UeDlGpu*    g    = (UeDlGpu*)q->gpu;
  hipStream_t s    = (hipStream_t)stream;
  const bool  full = cfg->chest_cfg.estimator_alg == SRSRAN_ESTIMATOR_ALG_INTERPOLATE;  // every symbol its own row
  // one TDD frame configuration per batch (the estimator takes one); compared field by field (the struct has
  // padding) and only in a TDD cell (an FDD caller may leave the field unset)
  for (uint32_t b = 1; q->cell.frame_type == SRSRAN_TDD && b < nof_sf; b++) {
    const srsran_tdd_config_t &t = sfs[b].tdd_config, &t0 = sfs[0].tdd_config;
    if (t.configured != t0.configured || t.sf_config != t0.sf_config || t.ss_config != t0.ss_config) {
      fprintf(stderr, "[srsran_ue_dl] batch: subframes with different TDD configurations\n");
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
  }
  srsran_chest_dl_gpu_set_tdd_config(&q->chest, sfs[0].tdd_config);
  if (!srsran_amd::chest_batch_cfg_supported(&q->chest, &cfg->chest_cfg, full)) {  // before any batch is staged
    return SRSRAN_ERROR;
  }
  if (!grow(q, g, nof_sf, full)) {
    return SRSRAN_ERROR;
  }
  const size_t nre = 12 * (size_t)q->cell.nof_prb, nrx = q->nof_rx_antennas, np = q->cell.nof_ports;
  const size_t rows = 2 * SRSRAN_CP_NSYMB(q->cell.cp);  // grid symbols per subframe
  std::vector<srsran_pdsch_gpu_sf_t> ps(nof_sf);
  for (uint32_t b = 0; b < nof_sf; b++) {
    srsran_pdsch_gpu_sf_t& f = ps[b];
    memset(&f, 0, sizeof(f));
    f.cfg     = sfs[b].pdsch_cfg;
    f.tti     = sfs[b].tti;
    f.cfi     = sfs[b].cfi;
    f.d_grid  = (const cf_t*)(g->d_grid + b * nrx * rows * nre);
    f.d_ce    = (const cf_t*)(g->d_ce + b * np * nrx * nre * (full ? rows : 1));
    f.ce_full = full ? 1 : 0;
    f.d_noise = g->d_res + 4 * b;
    for (int t = 0; t < SRSRAN_MAX_CODEWORDS; t++) {
      f.d_payload[t] = sfs[b].d_payload[t];
      f.new_data[t]  = sfs[b].new_data[t];
    }
  }
  // the estimator launch (after the OFDM launch), with the batch's staging copies fused in when given
  auto estimate = [&](const srsran_amd::CopyJobs* jobs) -> int {
    if (nof_sf <= (uint32_t)srsran_amd::CHEST_INLINE_SF) {  // the indices travel in the estimator's launch arguments
      uint8_t h_sf[srsran_amd::CHEST_INLINE_SF];
      for (uint32_t b = 0; b < nof_sf; b++) {
        h_sf[b] = (uint8_t)(sfs[b].tti % 10);
      }
      if (srsran_amd::chest_dl_gpu_estimate_batch_inline(&q->chest, &cfg->chest_cfg, h_sf, jobs, nof_sf, (const cf_t*)g->d_grid,
                                                         nrx * rows * nre, (cf_t*)g->d_ce,
                                                         np * nrx * nre * (full ? rows : 1), full ? 1 : 0, g->d_res,
                                                         stream)) {
        return SRSRAN_ERROR;
      }
    } else {  // larger batches: a ring slot of pinned memory the estimator reads in place
      for (uint32_t i = 0; jobs && i < jobs->n; i++) {  // (the copies then go on their own, first)
        if (srsran_amd::stage_copy_job(jobs->job[i], s) != hipSuccess) {
          return SRSRAN_ERROR;
        }
      }
      const uint32_t slot = g->ring_next;
      g->ring_next        = (slot + 1) % kStageRing;
      if (hipEventSynchronize(g->staged[slot]) != hipSuccess) {
        return SRSRAN_ERROR;
      }
      uint32_t* h_sf = g->h_sf + (size_t)slot * g->cap;
      uint32_t* d_sf = g->d_sf + (size_t)slot * g->cap;
      for (uint32_t b = 0; b < nof_sf; b++) {
        h_sf[b] = sfs[b].tti % 10;
      }
      if (srsran_chest_dl_gpu_estimate_batch_cfg(&q->chest, &cfg->chest_cfg, d_sf, nof_sf, (const cf_t*)g->d_grid,
                                                 nrx * rows * nre, (cf_t*)g->d_ce, np * nrx * nre * (full ? rows : 1),
                                                 full ? 1 : 0, g->d_res, stream)) {
        return SRSRAN_ERROR;
      }
      hipEventRecord(g->staged[slot], s);  // h_sf of this slot is free again once the estimator has run
    }
    return SRSRAN_SUCCESS;
  };
  // The PDSCH / DL-SCH batch first, with its launches deferred (stage_copy.h): its descriptors depend on the
  // configuration only, so they are built and staged now, their copies ride in the estimator's launch below (no
  // copy kernels in the chain) and the predecoder ... TB launches are replayed after it.
  front.stop();
  // (one DL-SCH group only: TBs with different iteration limits go through several DL-SCH batches, whose staging
  // ring could come round within one deferred call -- such batches launch in line)
  bool     one_limit = true;
  uint32_t lim       = q->pdsch.dl_sch.max_iterations;
  for (uint32_t b = 0; b < nof_sf && one_limit; b++) {
    const uint32_t m = sfs[b].pdsch_cfg ? sfs[b].pdsch_cfg->max_nof_iterations : 0;
    const uint32_t l = m ? m : lim;
    one_limit        = b == 0 || l == lim;
    lim              = l;
  }
  if (srsran_amd::stage_side_copy() || !one_limit) {  // in line: OFDM, estimator, then the PDSCH batch
    if (srsran_amd::handoff(g->ho, s) != hipSuccess ||
        (d16 ? srsran_ofdm_rx_gpu_sc16(&q->fft[0], d16, scale, (cf_t*)g->d_grid, (uint32_t)nrx, nof_sf, cfo, stream)
                : srsran_ofdm_rx_gpu(&q->fft[0], d_samples, (cf_t*)g->d_grid, (uint32_t)nrx, nof_sf, cfo, stream)) ||
        estimate(nullptr) != SRSRAN_SUCCESS) {
      return SRSRAN_ERROR;
    }
    return srsran_pdsch_gpu_decode_batch(&q->pdsch, nof_sf, ps.data(), d_result, d_avg_noi, stream);
  }
  srsran_amd::LaunchRecorder rec;
  srsran_amd::launch_recorder() = &rec;
  const int ret = srsran_pdsch_gpu_decode_batch(&q->pdsch, nof_sf, ps.data(), d_result, d_avg_noi, stream);
  srsran_amd::launch_recorder() = nullptr;
  // staged slots must see their copies run whatever happens next, or their fences never come
  auto copies_alone = [&] {
    for (const srsran_amd::CopyJob& j : rec.jobs) {
      srsran_amd::stage_copy_job(j, s);
    }
  };
  if (ret < 0) {
    copies_alone();
    return ret;
  }
  srsran_amd::HostScope front2(srsran_amd::HP_FRONT);
  srsran_amd::CopyJobs js{};
  bool                 copies_ok = true;
  for (size_t i = 0; i < rec.jobs.size(); i++) {
    if (i < (size_t)srsran_amd::kMaxFusedJobs) {
      js.job[js.n++] = rec.jobs[i];
    } else {  // beyond the fused ones: on their own (every one, even after a failure: their fences must come)
      copies_ok = srsran_amd::stage_copy_job(rec.jobs[i], s) == hipSuccess && copies_ok;
    }
  }
  if (!copies_ok || srsran_amd::handoff(g->ho, s) != hipSuccess ||
      (d16 ? srsran_ofdm_rx_gpu_sc16(&q->fft[0], d16, scale, (cf_t*)g->d_grid, (uint32_t)nrx, nof_sf, cfo, stream)
                : srsran_ofdm_rx_gpu(&q->fft[0], d_samples, (cf_t*)g->d_grid, (uint32_t)nrx, nof_sf, cfo, stream)) ||
      estimate(&js) != SRSRAN_SUCCESS) {
    for (uint32_t i = 0; i < js.n; i++) {  // the fused ones did not run: their fences must come as well
      srsran_amd::stage_copy_job(js.job[i], s);
    }
    return SRSRAN_ERROR;
  }
  front2.stop();
  for (auto& launch : rec.launches) {  // the deferred PDSCH / DL-SCH launches, in their order
    if (launch() != hipSuccess) {
      return SRSRAN_ERROR;
    }
  }
  return ret;
}

int srsran_ue_dl_gpu_decode_batch(srsran_ue_dl_t*              q,
                                  srsran_ue_dl_cfg_t*          cfg,
                                  uint32_t                     nof_sf,
                                  const srsran_ue_dl_gpu_sf_t* sfs,
                                  const cf_t*                  d_samples,
                                  float                        cfo,
                                  int32_t*                     d_result,
                                  float*                       d_avg_noi,
                                  void*                        stream)
{
  if (nof_sf && !d_samples) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  return decode_batch(q, cfg, nof_sf, sfs, d_samples, nullptr, 1.0f, cfo, d_result, d_avg_noi, stream);
}

int srsran_gpu_worker_stream_create(void** stream)
{
  if (!stream) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  hipStream_t s = nullptr;
  if (srsran_amd::own_queue_stream(&s) != hipSuccess) {
    *stream = nullptr;
    return SRSRAN_ERROR;
  }
  *stream = s;
  return SRSRAN_SUCCESS;
}

void srsran_gpu_worker_stream_free(void* stream)
{
  if (stream) {
    hipStreamSynchronize((hipStream_t)stream);
    hipStreamDestroy((hipStream_t)stream);
  }
}

int srsran_ue_dl_gpu_decode_batch_sc16(srsran_ue_dl_t*              q,
                                       srsran_ue_dl_cfg_t*          cfg,
                                       uint32_t                     nof_sf,
                                       const srsran_ue_dl_gpu_sf_t* sfs,
                                       const int16_t*               d_samples,
                                       float                        scale,
                                       float                        cfo,
                                       int32_t*                     d_result,
                                       float*                       d_avg_noi,
                                       void*                        stream)
{
  if ((nof_sf && !d_samples) || !std::isfinite(scale)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  return decode_batch(q, cfg, nof_sf, sfs, nullptr, d_samples, scale, cfo, d_result, d_avg_noi, stream);
}

// ---------------- DCI blind search (ue_dl.c:386-689) ----------------
namespace {

const srsran_dci_format_t kUeFormats[8][2] = {
    {SRSRAN_DCI_FORMAT1A, SRSRAN_DCI_FORMAT1},  {SRSRAN_DCI_FORMAT1A, SRSRAN_DCI_FORMAT1},
    {SRSRAN_DCI_FORMAT1A, SRSRAN_DCI_FORMAT2A}, {SRSRAN_DCI_FORMAT1A, SRSRAN_DCI_FORMAT2},
    {SRSRAN_DCI_FORMAT1A, SRSRAN_DCI_FORMAT1D}, {SRSRAN_DCI_FORMAT1A, SRSRAN_DCI_FORMAT1B},
    {SRSRAN_DCI_FORMAT1A, SRSRAN_DCI_FORMAT1},  {SRSRAN_DCI_FORMAT1A, SRSRAN_DCI_FORMAT2B}};
const srsran_dci_format_t kCommonFormats[2] = {SRSRAN_DCI_FORMAT1A, SRSRAN_DCI_FORMAT1C};

struct SearchSpace {
  srsran_dci_location_t loc[SRSRAN_MAX_CANDIDATES];
  uint32_t              nof_locations = 0;
  srsran_dci_format_t   formats[2];
  uint32_t              nof_formats = 0;
  srsran_dci_cfg_t      cfg{};
  bool                  common = false;
};

bool find_dci(const srsran_dci_msg_t* msgs, uint32_t n, const srsran_dci_msg_t& m)
{
  for (uint32_t k = 0; k < n; k++) {
    if (msgs[k].nof_bits == m.nof_bits && memcmp(msgs[k].payload, m.payload, m.nof_bits) == 0) {
      return true;
    }
  }
  return false;
}

bool allocated(const UeDlGpu* g, const srsran_dci_location_t& l)
{
  for (uint32_t i = 0; i < g->nof_allocated; i++) {
    const uint32_t L = g->allocated[i].L, n = g->allocated[i].ncce;  // as ue_dl.c:402-414 (L, not 2^L)
    if ((n <= l.ncce && l.ncce < n + L) || (l.ncce <= n && n < l.ncce + l.L)) {
      return true;
    }
  }
  return false;
}

}  // namespace

int srsran_ue_dl_find_dl_dci(srsran_ue_dl_t*     q,
                             srsran_dl_sf_cfg_t* sf,
                             srsran_ue_dl_cfg_t* dl_cfg,
                             uint16_t            rnti,
                             srsran_dci_dl_t     dci_dl[SRSRAN_MAX_DCI_MSG])
{
  if (!q || !q->gpu || !sf || !dl_cfg || !dci_dl) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  UeDlGpu* g = (UeDlGpu*)q->gpu;
  if (!g->ctrl_cell || sf->cfi < 1 || sf->cfi > 3 || g->pdcch.llr_cfi != sf->cfi) {
    fprintf(stderr, "[srsran_ue_dl] find_dl_dci: no PDCCH LLRs for this subframe (decode_fft_estimate first)\n");
    return SRSRAN_ERROR;
  }
  g->nof_pending_ul = 0;
  g->nof_allocated  = 0;
  if (!rnti) {
    return 0;
  }
  // search spaces in the reference's order: C-RNTI -> UE-specific then (dci_common_ss) common with
  // format 1A; SI / P / RA-RNTI -> common with formats 1A, 1C (ue_dl.c:604-651)
  std::vector<SearchSpace> ss;
  SearchSpace              common;
  common.cfg = dl_cfg->cfg.dci;
  srsran_dci_cfg_set_common_ss(&common.cfg);
  common.common        = true;
  common.nof_locations = srsran_pdcch_common_locations(&g->pdcch, common.loc, SRSRAN_MAX_CANDIDATES_COM, sf->cfi);
  const bool crnti     = !(rnti == SRSRAN_SIRNTI || rnti == SRSRAN_PRNTI || SRSRAN_RNTI_ISRAR(rnti));
  if (crnti) {
    if (dl_cfg->cfg.tm > SRSRAN_TM8) {
      return SRSRAN_ERROR;
    }
    SearchSpace ue;
    ue.cfg           = dl_cfg->cfg.dci;
    ue.nof_locations = srsran_pdcch_ue_locations(&g->pdcch, sf, ue.loc, SRSRAN_MAX_CANDIDATES_UE, rnti);
    ue.nof_formats   = 2;
    ue.formats[0]    = kUeFormats[dl_cfg->cfg.tm][0];
    ue.formats[1]    = kUeFormats[dl_cfg->cfg.tm][1];
    ss.push_back(ue);
    if (dl_cfg->cfg.dci_common_ss) {
      common.nof_formats = 1;
      common.formats[0]  = SRSRAN_DCI_FORMAT1A;
      ss.push_back(common);
    }
  } else {
    common.nof_formats = 2;
    common.formats[0]  = kCommonFormats[0];
    common.formats[1]  = kCommonFormats[1];
    ss.push_back(common);
  }
  // every (location, format) of every search space decoded in one launch, then the sequential
  // selection of dci_blind_search on the results
  std::vector<srsran_dci_msg_t> cand;
  std::vector<float>            corr;
  std::vector<int>              fmt_ok;
  for (const SearchSpace& s : ss) {
    for (uint32_t l = 0; l < s.nof_locations; l++) {
      for (uint32_t f = 0; f < s.nof_formats; f++) {
        srsran_dci_msg_t m;
        memset(&m, 0, sizeof(m));
        m.location = s.loc[l];
        m.format   = s.formats[f];
        cand.push_back(m);
      }
    }
  }
  // formats the library cannot size (1B / 1D) are decoded as nothing found
  std::vector<srsran_dci_msg_t> dec;
  std::vector<uint32_t>         dec_of(cand.size(), UINT32_MAX);
  size_t                        ci = 0;
  for (const SearchSpace& s : ss) {
    for (uint32_t l = 0; l < s.nof_locations; l++) {
      for (uint32_t f = 0; f < s.nof_formats; f++, ci++) {
        srsran_dci_cfg_t c = s.cfg;
        if (srsran_dci_format_sizeof(&q->cell, sf, &c, cand[ci].format) > 0) {
          dec_of[ci] = (uint32_t)dec.size();
          dec.push_back(cand[ci]);
        }
      }
    }
  }
  corr.assign(dec.size(), 0.0f);
  // the two search spaces use different DCI configurations: decode each space's candidates with its own
  {
    size_t first = 0;
    ci           = 0;
    for (const SearchSpace& s : ss) {
      size_t n = 0;
      for (uint32_t l = 0; l < s.nof_locations; l++) {
        for (uint32_t f = 0; f < s.nof_formats; f++, ci++) {
          n += dec_of[ci] != UINT32_MAX;
        }
      }
      srsran_dci_cfg_t c = s.cfg;
      if (n && srsran_pdcch_gpu_decode_msgs(&g->pdcch, sf, &c, dec.data() + first, (uint32_t)n, corr.data() + first)) {
        return SRSRAN_ERROR;
      }
      first += n;
    }
  }
  srsran_dci_msg_t msgs[SRSRAN_MAX_DCI_MSG];
  uint32_t         nof_msg = 0;
  ci                       = 0;
  for (const SearchSpace& s : ss) {
    uint32_t nof_dci = 0;
    srsran_dci_msg_t* out = msgs + nof_msg;
    const size_t ci0 = ci;
    ci += (size_t)s.nof_locations * s.nof_formats;
    for (uint32_t l = 0; l < s.nof_locations; l++) {
      const size_t cl = ci0 + (size_t)l * s.nof_formats;
      if (nof_msg + nof_dci >= SRSRAN_MAX_DCI_MSG) {
        break;
      }
      if (allocated(g, s.loc[l])) {
        continue;
      }
      for (uint32_t f = 0; f < s.nof_formats; f++) {
        const uint32_t d = dec_of[cl + f];
        if (d == UINT32_MAX) {
          continue;
        }
        srsran_dci_msg_t m = dec[d];
        if (m.rnti != rnti || m.nof_bits == 0) {
          continue;
        }
        if (!std::isnormal(corr[d]) || corr[d] < 0.5f) {
          continue;
        }
        if (dl_cfg->cfg.dci_common_ss && (dl_cfg->cfg.dci.multiple_csi_request_enabled || dl_cfg->cfg.dci.srs_request_enabled) &&
            srsran_location_find_location(common.loc, common.nof_locations, &m.location)) {
          srsran_dci_cfg_t c = dl_cfg->cfg.dci;
          srsran_dci_cfg_set_common_ss(&c);
          if (m.nof_bits == srsran_dci_format_sizeof(&q->cell, sf, &c, SRSRAN_DCI_FORMAT1A)) {
            m.format = m.payload[0] ? SRSRAN_DCI_FORMAT1A : SRSRAN_DCI_FORMAT0;
          }
        }
        if (m.format == SRSRAN_DCI_FORMAT0) {
          if (g->nof_pending_ul < SRSRAN_MAX_DCI_MSG && !find_dci(g->pending_ul, g->nof_pending_ul, m)) {
            g->pending_ul[g->nof_pending_ul++] = m;
          }
        } else if (!find_dci(out, nof_dci, m) && !find_dci(g->pending_ul, g->nof_pending_ul, m)) {
          if (g->nof_allocated < SRSRAN_MAX_DCI_MSG) {
            g->allocated[g->nof_allocated++] = m.location;
          }
          out[nof_dci++] = m;
          break;
        }
      }
    }
    nof_msg += nof_dci;
  }
  for (uint32_t i = 0; i < nof_msg; i++) {
    if (srsran_dci_msg_unpack_pdsch(&q->cell, sf, &dl_cfg->cfg.dci, &msgs[i], &dci_dl[i])) {
      fprintf(stderr, "[srsran_ue_dl] Unpacking DL DCI\n");
      return SRSRAN_ERROR;
    }
  }
  return (int)nof_msg;
}

int srsran_ue_dl_find_ul_dci(srsran_ue_dl_t*     q,
                             srsran_dl_sf_cfg_t* sf,
                             srsran_ue_dl_cfg_t* dl_cfg,
                             uint16_t            rnti,
                             srsran_dci_ul_t     dci_ul[SRSRAN_MAX_DCI_MSG])
{
  if (!q || !q->gpu || !dl_cfg || !dci_ul) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (!rnti) {
    return 0;
  }
  // the format 0 messages the last find_dl_dci set aside; the list is consumed
  UeDlGpu*         g = (UeDlGpu*)q->gpu;
  const uint32_t   n = std::min<uint32_t>(SRSRAN_MAX_DCI_MSG, g->nof_pending_ul);
  srsran_dci_msg_t msgs[SRSRAN_MAX_DCI_MSG];
  memcpy(msgs, g->pending_ul, n * sizeof(srsran_dci_msg_t));
  g->nof_pending_ul = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (srsran_dci_msg_unpack_pusch(&q->cell, sf, &dl_cfg->cfg.dci, &msgs[i], &dci_ul[i])) {
      fprintf(stderr, "[srsran_ue_dl] Unpacking UL DCI\n");
      return SRSRAN_ERROR;
    }
  }
  return (int)n;
}

void srsran_ue_dl_set_mi_auto(srsran_ue_dl_t* q)
{
  if (q && q->gpu) {
    ((UeDlGpu*)q->gpu)->mi_auto = true;
  }
}

void srsran_ue_dl_set_mi_manual(srsran_ue_dl_t* q, uint32_t mi_idx)
{
  if (q && q->gpu && mi_idx <= 2) {
    UeDlGpu* g   = (UeDlGpu*)q->gpu;
    g->mi_auto   = false;
    g->mi_manual = mi_idx;
  }
}

int srsran_ue_dl_set_mbsfn_area_id(srsran_ue_dl_t* q, uint16_t mbsfn_area_id)  // ue_dl.c:277-294 (PMCH: not provided)
{
  if (!q) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (srsran_chest_dl_set_mbsfn_area_id(&q->chest, mbsfn_area_id)) {
    fprintf(stderr, "[srsran_ue_dl] Error setting MBSFN area ID\n");
    return SRSRAN_ERROR;
  }
  q->current_mbsfn_area_id = mbsfn_area_id;
  return SRSRAN_SUCCESS;
}

void srsran_ue_dl_set_non_mbsfn_region(srsran_ue_dl_t* q, uint8_t non_mbsfn_region_length)  // ue_dl.c:258-261
{
  if (q) {
    srsran_ofdm_set_non_mbsfn_region(&q->fft_mbsfn, non_mbsfn_region_length);
  }
}

int srsran_ue_dl_dci_to_pdsch_grant(srsran_ue_dl_t*       q,
                                    srsran_dl_sf_cfg_t*   sf,
                                    srsran_ue_dl_cfg_t*   cfg,
                                    srsran_dci_dl_t*      dci,
                                    srsran_pdsch_grant_t* grant)
{
  if (!q || !cfg) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  return srsran_ra_dl_dci_to_grant(&q->cell, sf, cfg->cfg.tm, cfg->cfg.pdsch.use_tbs_index_alt, dci, grant);
}

}  // extern "C"
