// srsran_4g_amd/csrc/ue_dl_api.cpp -- the PDSCH slice of srsran_ue_dl_t (include/srsran_ue_dl.h).
//
// Host-synchronous: srsran_ue_dl_init / set_cell / decode_fft_estimate(_noguru) / decode_pdsch
// (ue_dl.c:67-180, 349-384, 700-706) over the GPU OFDM, channel estimator and PDSCH objects.
// Batched: srsran_ue_dl_gpu_decode_batch chains, on one stream and without host round trips,
//   OFDM (CFO rotation fused)  ->  CRS estimation of every subframe  ->  PDSCH decode batch.
// PCFICH / PDCCH / PHICH / PMCH are not part of this path: the CFI comes from sf->cfi.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/srsran_ue_dl.h"

namespace {

struct UeDlGpu {
  hipEvent_t staged = nullptr;  // sf-index upload finished
  uint32_t*  h_sf   = nullptr;  // pinned
  uint32_t*  d_sf   = nullptr;
  float2*    d_grid = nullptr;
  float2*    d_ce   = nullptr;
  float*     d_res  = nullptr;
  uint32_t   cap    = 0;  // subframes
};

bool grow(srsran_ue_dl_t* q, UeDlGpu* g, uint32_t nsf)
{
  if (g->cap >= nsf) {
    return true;
  }
  hipDeviceSynchronize();
  hipHostFree(g->h_sf);
  hipFree(g->d_sf);
  hipFree(g->d_grid);
  hipFree(g->d_ce);
  hipFree(g->d_res);
  g->h_sf = nullptr, g->d_sf = nullptr, g->d_grid = nullptr, g->d_ce = nullptr, g->d_res = nullptr;
  g->cap             = 0;
  const size_t nre   = 12 * (size_t)q->cell.nof_prb;
  const size_t nrx   = q->nof_rx_antennas;
  const size_t ports = q->cell.nof_ports;
  if (hipHostMalloc((void**)&g->h_sf, nsf * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc((void**)&g->d_sf, nsf * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc((void**)&g->d_grid, nsf * nrx * 14 * nre * sizeof(float2)) != hipSuccess ||
      hipMalloc((void**)&g->d_ce, nsf * ports * nrx * nre * sizeof(float2)) != hipSuccess ||
      hipMalloc((void**)&g->d_res, nsf * 4 * sizeof(float)) != hipSuccess) {
    return false;
  }
  g->cap = nsf;
  return true;
}

bool srsue_chest_cfg(const srsran_chest_dl_cfg_t& c)
{
  return c.estimator_alg == SRSRAN_ESTIMATOR_ALG_AVERAGE && c.noise_alg == SRSRAN_NOISE_ALG_REFS &&
         c.filter_type == SRSRAN_CHEST_FILTER_GAUSS && c.filter_coef[0] == 4.0f && c.filter_coef[1] == 1.0f &&
         !c.sync_error_enable && !c.rsrp_neighbour;
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
  if (srsran_chest_dl_init(&q->chest, max_prb, nof_rx_antennas) || srsran_chest_dl_res_init(&q->chest_res, max_prb) ||
      srsran_pdsch_init_ue(&q->pdsch, max_prb, nof_rx_antennas)) {
    fprintf(stderr, "[srsran_ue_dl] Error initiating channel estimator / PDSCH\n");
    srsran_ue_dl_free(q);
    return SRSRAN_ERROR;
  }
  UeDlGpu* g = new UeDlGpu();
  q->gpu     = g;
  if (hipEventCreateWithFlags(&g->staged, hipEventDisableTiming) != hipSuccess) {
    srsran_ue_dl_free(q);
    return SRSRAN_ERROR;
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
    hipFree(g->d_sf);
    hipFree(g->d_grid);
    hipFree(g->d_ce);
    hipFree(g->d_res);
    if (g->staged) {
      hipEventDestroy(g->staged);
    }
    delete g;
  }
  for (int j = 0; j < SRSRAN_MAX_PORTS; j++) {
    if (q->fft[j].gpu) {
      srsran_ofdm_rx_free(&q->fft[j]);
    }
    free(q->sf_symbols[j]);
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
  if (srsran_chest_dl_set_cell(&q->chest, cell) || srsran_pdsch_set_cell(&q->pdsch, cell)) {
    return SRSRAN_ERROR;
  }
  UeDlGpu* g = (UeDlGpu*)q->gpu;
  q->cell    = cell;
  g->cap     = 0;  // buffer shapes depend on the cell
  hipDeviceSynchronize();
  hipHostFree(g->h_sf);
  hipFree(g->d_sf);
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
  if (sf->sf_type != SRSRAN_SF_NORM) {
    fprintf(stderr, "[srsran_ue_dl] MBSFN subframes are not provided\n");
    return SRSRAN_ERROR;
  }
  for (uint32_t j = 0; j < q->nof_rx_antennas; j++) {
    if (input) {
      srsran_ofdm_rx_sf_ng(&q->fft[j], input[j], q->sf_symbols[j]);
    } else {
      srsran_ofdm_rx_sf(&q->fft[j]);
    }
  }
  if (srsran_chest_dl_estimate_cfg(&q->chest, sf, &cfg->chest_cfg, q->sf_symbols, &q->chest_res)) {
    return SRSRAN_ERROR;
  }
  // PCFICH is not decoded here: sf->cfi is the caller's (estimate_pdcch_pcfich, ue_dl.c:310-347)
  return sf->cfi >= 1 && sf->cfi <= 3 ? SRSRAN_SUCCESS : SRSRAN_ERROR;
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
  if (!q || !q->gpu || !cfg || (nof_sf && (!sfs || !d_samples || !d_result || !d_avg_noi))) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_sf == 0) {
    return 0;
  }
  if (!srsue_chest_cfg(cfg->chest_cfg)) {
    fprintf(stderr, "[srsran_ue_dl] the batch path runs srsUE's default channel estimator configuration only\n");
    return SRSRAN_ERROR;
  }
  UeDlGpu*    g = (UeDlGpu*)q->gpu;
  hipStream_t s = (hipStream_t)stream;
  if (!grow(q, g, nof_sf) || hipEventSynchronize(g->staged) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  for (uint32_t b = 0; b < nof_sf; b++) {
    g->h_sf[b] = sfs[b].tti % 10;
  }
  hipMemcpyAsync(g->d_sf, g->h_sf, nof_sf * sizeof(uint32_t), hipMemcpyHostToDevice, s);
  hipEventRecord(g->staged, s);
  const size_t nre = 12 * (size_t)q->cell.nof_prb, nrx = q->nof_rx_antennas, np = q->cell.nof_ports;
  if (srsran_ofdm_rx_gpu(&q->fft[0], d_samples, (cf_t*)g->d_grid, (uint32_t)nrx, nof_sf, cfo, stream) ||
      srsran_chest_dl_gpu_estimate_batch(&q->chest, g->d_sf, nof_sf, (const cf_t*)g->d_grid, nrx * 14 * nre,
                                         (cf_t*)g->d_ce, np * nrx * nre, g->d_res, stream)) {
    return SRSRAN_ERROR;
  }
  std::vector<srsran_pdsch_gpu_sf_t> ps(nof_sf);
  for (uint32_t b = 0; b < nof_sf; b++) {
    srsran_pdsch_gpu_sf_t& f = ps[b];
    memset(&f, 0, sizeof(f));
    f.cfg     = sfs[b].pdsch_cfg;
    f.tti     = sfs[b].tti;
    f.cfi     = sfs[b].cfi;
    f.d_grid  = (const cf_t*)(g->d_grid + b * nrx * 14 * nre);
    f.d_ce    = (const cf_t*)(g->d_ce + b * np * nrx * nre);
    f.ce_full = 0;
    f.d_noise = g->d_res + 4 * b;
    for (int t = 0; t < SRSRAN_MAX_CODEWORDS; t++) {
      f.d_payload[t] = sfs[b].d_payload[t];
      f.new_data[t]  = sfs[b].new_data[t];
    }
  }
  return srsran_pdsch_gpu_decode_batch(&q->pdsch, nof_sf, ps.data(), d_result, d_avg_noi, stream);
}

}  // extern "C"
