// srsran_4g_amd/csrc/enb_dl_api.cpp -- eNB downlink transmit of PDSCH subframes on the GPU
// (include/srsran_enb_dl.h): DL-SCH encoding (srsran_dlsch_gpu_encode_batch), CRS, scrambling +
// modulation + precoding + RE mapping (llr_kernel.hip: pdsch_tx_kernel, crs_put_kernel) and the
// OFDM modulator (ofdm_kernel.hip: ofdm_tx_kernel).  enb_dl.c:300-470, pdsch.c:1015-1120.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/srsran_enb_dl.h"
#include "llr_kernel.h"
#include "pdsch_internal.h"

using namespace srsran_amd;

namespace {

struct EnbDlGpu {
  srsran_sch_t  sch{};
  srsran_ofdm_t ofdm{};
  uint32_t      N = 0, sf_len = 0;
  float2*       d_grid = nullptr;  // [sf][port][2 nsymb][nre]
  size_t        grid_cap = 0;
  uint8_t*      d_e = nullptr;     // packed e bits of every codeword
  size_t        e_cap = 0;
  uint32_t*     d_idx = nullptr;   // RE tables of every subframe
  size_t        idx_cap = 0;
  PdschTx*      d_items = nullptr;
  size_t        items_cap = 0;
  uint32_t*     d_sfidx = nullptr;
  size_t        sfidx_cap = 0;
  // RE tables on the device, keyed by (PRB allocation, symbols a slot, first symbol, subframe): built
  // once, not re-uploaded every batch
  std::unordered_map<std::string, std::pair<uint32_t*, uint32_t>> tabs;
};

constexpr size_t kTabCache = 512;  // RE tables kept on the device

// Called once before a batch looks up its tables: when the batch could push the cache past its bound,
// the cache is emptied here (after the device is idle), never in the middle of the batch, so every
// table a batch has looked up stays allocated until its launches have run.
void tab_evict(EnbDlGpu* g, uint32_t nof_sf)
{
  if (g->tabs.size() + nof_sf > kTabCache) {
    hipDeviceSynchronize();
    for (auto& kv : g->tabs) {
      hipFree(kv.second.first);
    }
    g->tabs.clear();
  }
}

// (device table, RE count) of a grant, built and cached on first use; {nullptr, 0} on failure
std::pair<uint32_t*, uint32_t> get_tab(EnbDlGpu* g, const srsran_cell_t& cell, const srsran_pdsch_grant_t& gr,
                                       uint32_t lstart, uint32_t sf_idx)
{
  std::string key;
  key.reserve(2 * cell.nof_prb + 8);
  for (uint32_t s = 0; s < 2; s++) {
    for (uint32_t n = 0; n < cell.nof_prb; n++) {
      key.push_back(gr.prb_idx[s][n] ? '1' : '0');
    }
    key.push_back((char)gr.nof_symb_slot[s]);
  }
  key.push_back((char)lstart);
  key.push_back((char)sf_idx);
  auto it = g->tabs.find(key);
  if (it != g->tabs.end()) {
    return it->second;
  }
  const std::vector<uint32_t> t = pdsch_re_table(cell, gr, lstart, sf_idx);
  uint32_t*                   d = nullptr;
  if (hipMalloc((void**)&d, std::max<size_t>(t.size(), 1) * sizeof(uint32_t)) != hipSuccess ||
      hipMemcpy(d, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
    hipFree(d);
    return {nullptr, 0};
  }
  return g->tabs[key] = std::make_pair(d, (uint32_t)t.size());
}

bool grow(void** p, size_t* cap, size_t need)
{
  if (need <= *cap) {
    return true;
  }
  hipFree(*p);
  *p   = nullptr;
  *cap = 0;
  if (hipMalloc(p, need) != hipSuccess) {
    return false;
  }
  *cap = need;
  return true;
}

}  // namespace

extern "C" {

int srsran_enb_dl_gpu_init(srsran_enb_dl_gpu_t* q, srsran_cell_t cell)
{
  if (!q || cell.nof_prb < 6 || cell.nof_prb > SRSRAN_MAX_PRB || cell.nof_ports == 0 || cell.nof_ports == 3 ||
      cell.nof_ports > 4 ||
      (cell.cp != SRSRAN_CP_NORM && cell.cp != SRSRAN_CP_EXT)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(q, 0, sizeof(*q));
  q->cell       = cell;
  EnbDlGpu* g   = new EnbDlGpu();
  q->gpu        = g;
  srsran_ofdm_cfg_t oc;
  memset(&oc, 0, sizeof(oc));
  oc.nof_prb   = cell.nof_prb;
  oc.cp        = cell.cp;
  oc.normalize = false;  // enb_dl.c:158
  if (srsran_sch_init(&g->sch) != SRSRAN_SUCCESS || srsran_ofdm_tx_init_cfg(&g->ofdm, &oc) != SRSRAN_SUCCESS) {
    srsran_enb_dl_gpu_free(q);
    return SRSRAN_ERROR;
  }
  g->N      = g->ofdm.cfg.symbol_sz;
  g->sf_len = g->ofdm.sf_sz;
  return SRSRAN_SUCCESS;
}

void srsran_enb_dl_gpu_free(srsran_enb_dl_gpu_t* q)
{
  if (!q) {
    return;
  }
  EnbDlGpu* g = (EnbDlGpu*)q->gpu;
  if (g) {
    hipDeviceSynchronize();
    srsran_sch_free(&g->sch);
    srsran_ofdm_tx_free(&g->ofdm);
    hipFree(g->d_grid);
    hipFree(g->d_e);
    hipFree(g->d_idx);
    hipFree(g->d_items);
    hipFree(g->d_sfidx);
    for (auto& kv : g->tabs) {
      hipFree(kv.second.first);
    }
    delete g;
  }
  memset(q, 0, sizeof(*q));
}

int srsran_enb_dl_gpu_tx_batch(srsran_enb_dl_gpu_t*          q,
                               uint32_t                      nof_sf,
                               const srsran_enb_dl_gpu_sf_t* sfs,
                               cf_t*                         d_samples,
                               float                         scale,
                               void*                         stream)
{
  if (!q || !q->gpu || (nof_sf && (!sfs || !d_samples))) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_sf == 0) {
    return SRSRAN_SUCCESS;
  }
  EnbDlGpu*           g     = (EnbDlGpu*)q->gpu;
  hipStream_t         st    = (hipStream_t)stream;
  const srsran_cell_t& cell = q->cell;
  const uint32_t      P     = cell.nof_ports, nre_sf = SRSRAN_SF_LEN_RE(cell.nof_prb, cell.cp);
  std::vector<std::pair<uint32_t*, uint32_t>> tables(nof_sf);
  std::vector<PdschTx>               items(nof_sf);
  std::vector<srsran_dlsch_gpu_enc_t> enc;
  std::vector<size_t>                 e_off;
  std::vector<uint32_t>               sfidx(nof_sf);
  size_t                              e_tot = 0;
  uint32_t                            max_nre = 0;
  tab_evict(g, nof_sf);
  for (uint32_t b = 0; b < nof_sf; b++) {
    const srsran_enb_dl_gpu_sf_t& s   = sfs[b];
    const srsran_pdsch_cfg_t*     cfg = s.cfg;
    if (!cfg || s.cfi < 1 || s.cfi > 3) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    const srsran_pdsch_grant_t& gr = cfg->grant;
    int                         scheme;
    if (gr.tx_scheme == SRSRAN_TXSCHEME_PORT0 && P == 1 && gr.nof_tb == 1) {
      scheme = 0;
    } else if (gr.tx_scheme == SRSRAN_TXSCHEME_DIVERSITY && P == 2 && gr.nof_tb == 1) {
      scheme = 1;
    } else if (gr.tx_scheme == SRSRAN_TXSCHEME_DIVERSITY && P == 4 && gr.nof_tb == 1) {
      scheme = 4;
    } else if (gr.tx_scheme == SRSRAN_TXSCHEME_CDD && P == 2 && gr.nof_tb == 2 && gr.nof_layers == 2) {
      scheme = 3;
    } else {
      fprintf(stderr, "[srsran_enb_dl] transmission scheme %d with %u ports / %u TBs is not provided\n",
              (int)gr.tx_scheme, P, gr.nof_tb);
      return SRSRAN_ERROR;
    }
    sfidx[b]  = s.tti % 10;
    const uint32_t lstart = s.cfi + (cell.nof_prb < 10 ? 1 : 0);  // SRSRAN_NOF_CTRL_SYMBOLS
    tables[b] = get_tab(g, cell, gr, lstart, sfidx[b]);
    if (!tables[b].first) {
      return SRSRAN_ERROR;
    }
    const uint32_t nre = tables[b].second;
    max_nre            = std::max(max_nre, nre);
    PdschTx& it        = items[b];
    memset(&it, 0, sizeof(it));
    it.nre       = nre;
    it.scheme    = scheme;
    it.scaling   = 1.0f;
    // scaling * M_SQRT1_2 (2 ports); scaling /= M_SQRT2 (4 ports, precoding.c:1962)
    it.div_scale = scheme == 4 ? (float)(1.0f / 1.41421356237309504880) : (float)(1.0 * 0.70710678118654752440);
    uint32_t cw = 0;
    for (uint32_t t = 0; t < SRSRAN_MAX_CODEWORDS; t++) {
      const srsran_ra_tb_t& tb = gr.tb[t];
      if (!tb.enabled) {
        continue;
      }
      const uint32_t Qm = srsran_mod_bits_x_symbol(tb.mod), Nl = gr.nof_layers != gr.nof_tb ? 2 : 1;
      if (!s.d_data[t] || Qm == 0 || tb.nof_bits != nre * Qm * (scheme == 1 ? 1 : 1) || tb.tbs <= 0 || cw >= 2) {
        fprintf(stderr, "[srsran_enb_dl] TB %u: nof_bits %u does not match %u REs x Qm %u\n", t, tb.nof_bits, nre, Qm);
        return SRSRAN_ERROR_INVALID_INPUTS;
      }
      e_off.push_back(e_tot);
      enc.push_back({(uint32_t)tb.tbs, Qm * Nl, (uint32_t)tb.rv, tb.nof_bits, s.d_data[t], nullptr});
      it.seed[cw] = pdsch_seed(cfg->rnti, (int)tb.cw_idx, 2 * sfidx[b], cell.id);
      it.mod[cw]  = (int)tb.mod;
      e_tot += ((tb.nof_bits + 7) / 8 + 15) & ~(size_t)15;
      cw++;
    }
    if ((scheme == 3) != (cw == 2)) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
  }
  const size_t grid_bytes = (size_t)nof_sf * P * nre_sf * sizeof(float2);
  if (!grow((void**)&g->d_grid, &g->grid_cap, grid_bytes) || !grow((void**)&g->d_e, &g->e_cap, e_tot + 16) ||
      !grow((void**)&g->d_items, &g->items_cap, nof_sf * sizeof(PdschTx)) ||
      !grow((void**)&g->d_sfidx, &g->sfidx_cap, nof_sf * sizeof(uint32_t))) {
    return SRSRAN_ERROR;
  }
  // device pointers of the codewords, tables and grids
  size_t k = 0;
  for (uint32_t b = 0; b < nof_sf; b++) {
    PdschTx& it = items[b];
    it.idx      = tables[b].first;
    for (uint32_t p = 0; p < P; p++) {
      it.grid[p] = g->d_grid + ((size_t)b * P + p) * nre_sf;
    }
    const uint32_t ncw = it.scheme == 3 ? 2 : 1;
    for (uint32_t c = 0; c < ncw; c++, k++) {
      enc[k].d_e_bits = g->d_e + e_off[k];
      it.e[c]         = g->d_e + e_off[k];
    }
  }
  if (srsran_dlsch_gpu_encode_batch(&g->sch, (uint32_t)enc.size(), enc.data(), st) != SRSRAN_SUCCESS ||
      hipMemsetAsync(g->d_grid, 0, grid_bytes, st) != hipSuccess ||
      hipMemcpyAsync(g->d_items, items.data(), nof_sf * sizeof(PdschTx), hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(g->d_sfidx, sfidx.data(), nof_sf * sizeof(uint32_t), hipMemcpyHostToDevice, st) != hipSuccess ||
      crs_put_launch(g->d_grid, cell.nof_prb, cell.id, P, SRSRAN_CP_NSYMB(cell.cp), g->d_sfidx, nof_sf, st) != hipSuccess ||
      pdsch_tx_launch(g->d_items, nof_sf, max_nre, st) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  const float sc = scale > 0.0f ? scale : 0.05f / sqrtf((float)cell.nof_prb);  // enb_dl_get_norm_factor
  return srsran_ofdm_tx_gpu(&g->ofdm, (const cf_t*)g->d_grid, d_samples, P, nof_sf, sc, st);
}

}  // extern "C"
