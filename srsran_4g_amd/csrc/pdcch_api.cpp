// srsran_4g_amd/csrc/pdcch_api.cpp -- REG mapping, PCFICH and PDCCH objects (include/srsran_pdcch.h).
//
// Host: the REG tables (regs.c:706-783 REG numbering, :367-392 PCFICH, :183-290 PHICH groups,
// :48-115 PDCCH interleaving + cyclic shift) become RE index lists per channel and CFI, uploaded
// once per cell; search spaces (pdcch.c:176-272); Gold sequences (sequence.c LTE_pr, 36.211 7.2).
// GPU (pdcch_kernel.hip): RE gather + predecoding, demodulation / descrambling, CFI correlation,
// and every PDCCH candidate of a search in one launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/srsran_pdcch.h"
#include "eq_kernel.h"
#include "pdcch_kernel.h"

using namespace srsran_amd;

namespace {

// ---------------- Gold sequence (36.211 7.2; sequence.c:48-102) ----------------
void gold_bits(uint32_t c_init, uint32_t len, std::vector<uint32_t>& words)
{
  words.assign((len + 31) / 32, 0u);
  uint32_t x1 = 1, x2 = c_init & 0x7fffffffu;  // 31-bit registers, bit n = x(n)
  for (uint32_t n = 0; n < 1600 + len; n++) {
    if (n >= 1600) {
      const uint32_t c = (x1 ^ x2) & 1u;
      words[(n - 1600) >> 5] |= c << ((n - 1600) & 31);
    }
    const uint32_t f1 = ((x1 >> 3) ^ x1) & 1u;
    const uint32_t f2 = ((x2 >> 3) ^ (x2 >> 2) ^ (x2 >> 1) ^ x2) & 1u;
    x1                = (x1 >> 1) | (f1 << 30);
    x2                = (x2 >> 1) | (f2 << 30);
  }
}

// ---------------- REG tables (regs.c) ----------------
struct Reg {
  uint32_t l, k0, k[4];
  bool     assigned;
};

int regs_per_symbol(uint32_t l, uint32_t nof_ports, srsran_cp_t cp)  // regs_num_x_symbol, regs.c:587-617
{
  switch (l) {
    case 0:
      return 2;
    case 1:
      return nof_ports == 4 ? 2 : 3;
    case 3:  // extended CP: the CRS of ports 0 / 1 sit in symbol 3 (36.211 6.10.1.2)
      return cp == SRSRAN_CP_NORM ? 3 : 2;
    default:
      return 3;
  }
}

void reg_init(Reg& r, uint32_t l, uint32_t nreg, uint32_t base, int maxreg, uint32_t vo)  // regs.c:518-559
{
  r.l        = l;
  r.assigned = false;
  if (maxreg == 2) {  // two CRS REs in the 6 subcarriers of the REG (at vo and vo + 3)
    r.k0  = base + nreg * 6;
    int j = 0;
    for (uint32_t i = 0; i < 6; i++) {
      if (i != vo && i != vo + 3) {
        r.k[j++] = r.k0 + i;
      }
    }
  } else {
    r.k0 = base + nreg * 4;
    for (uint32_t i = 0; i < 4; i++) {
      r.k[i] = r.k0 + i;
    }
  }
}

int build_regs(srsran_regs_t* h, uint32_t phich_mi, bool mbsfn_or_sf1_6)
{
  const srsran_cell_t& c     = h->cell;
  const uint32_t       nprb  = c.nof_prb;
  const uint32_t       nctrl = nprb <= 10 ? 4 : 3;
  const uint32_t       vo    = c.id % 3;
  h->max_ctrl_symbols        = nctrl;
  int      n[4];
  uint32_t nof_regs = 0;
  for (uint32_t i = 0; i < nctrl; i++) {
    n[i] = regs_per_symbol(i, c.nof_ports, c.cp);
    nof_regs += nprb * n[i];
  }
  // REGs sorted by PRB, then the frequency-first interleaving of regs.c:747-770
  std::vector<Reg> regs(nof_regs);
  uint32_t         j[4] = {0, 0, 0, 0};
  uint32_t         k = 0, i = 0, prb = 0, jmax = 0;
  while (k < nof_regs) {
    if (n[i] == 3 || (n[i] == 2 && jmax != 1)) {
      reg_init(regs[k], i, j[i], prb * 12, n[i], vo);
      j[i]++;
      k++;
    }
    if (++i == nctrl) {
      i = 0;
      jmax++;
    }
    if (jmax == 3) {
      prb++;
      j[0] = j[1] = j[2] = j[3] = 0;
      jmax                      = 0;
    }
  }
  auto find = [&](uint32_t kk, uint32_t l) -> Reg* {
    for (Reg& r : regs) {
      if (r.l == l && r.k0 == kk) {
        return &r;
      }
    }
    return nullptr;
  };
  // PCFICH (36.211 6.7.4)
  const uint32_t nre   = nprb * 12;
  const uint32_t k_hat = 6 * (c.id % (2 * nprb));
  for (uint32_t q = 0; q < 4; q++) {
    Reg* r = find((k_hat + (q * nprb / 2) * 6) % nre, 0);
    if (!r || r->assigned) {
      return SRSRAN_ERROR;
    }
    r->assigned = true;
    for (int e = 0; e < 4; e++) {
      h->pcfich_re[4 * q + e] = r->k[e] + r->l * nre;
    }
  }
  // PHICH (36.211 6.9.3, regs.c:249-350): m' mapping units of 3 REGs; normal duration in symbol 0, extended
  // duration in symbols 0-2 (li = i), or in symbols 0-1 of MBSFN / TDD subframe 1 and 6 (li = (m'/2 + i + 1) mod 2)
  float ng = 0;
  switch (h->phich_res) {
    case SRSRAN_PHICH_R_1_6:
      ng = 1.0f / 6;
      break;
    case SRSRAN_PHICH_R_1_2:
      ng = 1.0f / 2;
      break;
    case SRSRAN_PHICH_R_1:
      ng = 1;
      break;
    case SRSRAN_PHICH_R_2:
      ng = 2;
      break;
  }
  h->ngroups_phich_m1 = (uint32_t)(int)ceilf(ng * ((float)nprb / 8));
  h->ngroups_phich    = phich_mi * h->ngroups_phich_m1;
  if (h->ngroups_phich) {
    const bool        ext = h->phich_len == SRSRAN_PHICH_EXT;
    std::vector<Reg*> lr[3];  // free REGs of symbols 0-2, lowest frequency first
    for (Reg& r : regs) {
      if (r.l < 3 && !r.assigned) {
        lr[r.l].push_back(&r);
      }
    }
    uint32_t n[3];
    for (int l = 0; l < 3; l++) {
      n[l] = (uint32_t)lr[l].size();
    }
    for (uint32_t mi = 0; mi < h->ngroups_phich; mi++) {
      for (uint32_t q = 0; q < 3; q++) {
        const uint32_t li = !ext ? 0 : mbsfn_or_sf1_6 ? (mi / 2 + q + 1) % 2 : q;
        if (n[li] == 0 || (ext && mbsfn_or_sf1_6 && n[1] == 0)) {
          return SRSRAN_ERROR;
        }
        const uint32_t ni = ((c.id * n[li] / (ext && mbsfn_or_sf1_6 ? n[1] : n[0])) + mi + q * n[li] / 3) % n[li];
        lr[li][ni]->assigned = true;
      }
    }
  }
  // PDCCH per CFI (36.211 6.8.5): sub-block interleaving of the free REGs, cyclic shift by the cell id
  static const uint8_t PERM[32] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                   0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};
  for (uint32_t cfi = 0; cfi < 3; cfi++) {
    const uint32_t    nsym = nprb <= 10 ? cfi + 2 : cfi + 1;
    std::vector<Reg*> tmp;
    for (Reg& r : regs) {
      if (r.l < nsym && !r.assigned) {
        tmp.push_back(&r);
      }
    }
    const uint32_t    m      = (uint32_t)tmp.size();
    const int         nrows  = (int)((m - 1) / 32 + 1);
    const int         ndummy = std::max(0, 32 * nrows - (int)m);
    std::vector<Reg*> out(m, nullptr);
    uint32_t          kk = 0;
    for (int jj = 0; jj < 32; jj++) {
      for (int ii = 0; ii < nrows; ii++) {
        if (ii * 32 + PERM[jj] >= ndummy) {
          const uint32_t mm = ii * 32 + PERM[jj] - ndummy;
          const uint32_t kp = kk < c.id ? (m + kk - (c.id % m)) % m : (kk - c.id) % m;
          out[mm]           = tmp[kp];
          kk++;
        }
      }
    }
    h->pdcch_nregs[cfi] = (m / 9) * 9;
    h->pdcch_re[cfi]    = (uint32_t*)malloc(4 * (size_t)std::max(1u, h->pdcch_nregs[cfi]) * sizeof(uint32_t));
    if (!h->pdcch_re[cfi]) {
      return SRSRAN_ERROR;
    }
    for (uint32_t r = 0; r < h->pdcch_nregs[cfi]; r++) {
      for (int e = 0; e < 4; e++) {
        h->pdcch_re[cfi][4 * r + e] = out[r]->k[e] + out[r]->l * nre;
      }
    }
  }
  return SRSRAN_SUCCESS;
}

// ---------------- device state ----------------
struct CtrlGpu {
  hipStream_t  stream   = nullptr;
  float2*      d_grid   = nullptr;  // nrx x rows x nre
  float2*      d_ce     = nullptr;  // ports x nrx x rows x nre
  float2*      d_x      = nullptr;  // equalised symbols (codeword order)
  float*       d_csi    = nullptr;  // predecoder CSI scratch (1-port MMSE)
  uint32_t*    d_idx    = nullptr;  // PCFICH: 16; PDCCH: 3 tables
  uint32_t     idx_off[3] = {0, 0, 0};
  uint32_t*    d_seq    = nullptr;  // 10 subframes x seq_words
  uint32_t     seq_words = 0;
  float*       d_llr    = nullptr;  // PDCCH: 72 * max_cce; PCFICH: data_f
  uint32_t*    d_cfi    = nullptr;
  float*       d_corr   = nullptr;
  PdcchCand*   d_cand   = nullptr;
  PdcchCandOut* d_out   = nullptr;
  PdcchCandOut* h_out   = nullptr;  // pinned
  uint32_t     cand_cap = 0;
  uint32_t     rows = 0, nre = 0, nrx = 0, ports = 0;
};

void ctrl_free(CtrlGpu* g)
{
  if (!g) {
    return;
  }
  if (g->stream) {
    hipStreamSynchronize(g->stream);
    hipStreamDestroy(g->stream);
  }
  hipFree(g->d_grid);
  hipFree(g->d_ce);
  hipFree(g->d_x);
  hipFree(g->d_csi);
  hipFree(g->d_idx);
  hipFree(g->d_seq);
  hipFree(g->d_llr);
  hipFree(g->d_cfi);
  hipFree(g->d_corr);
  hipFree(g->d_cand);
  hipFree(g->d_out);
  hipHostFree(g->h_out);
  delete g;
}

CtrlGpu* ctrl_new(uint32_t max_prb, uint32_t nof_rx)
{
  CtrlGpu* g   = new CtrlGpu();
  const size_t nre = 12 * (size_t)max_prb;
  g->nrx       = nof_rx;
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void**)&g->d_grid, nof_rx * 4 * nre * sizeof(float2)) != hipSuccess ||
      hipMalloc((void**)&g->d_ce, 4 * nof_rx * 4 * nre * sizeof(float2)) != hipSuccess ||
      hipMalloc((void**)&g->d_x, 4 * nre * sizeof(float2)) != hipSuccess ||
      hipMalloc((void**)&g->d_csi, 2 * 4 * nre * sizeof(float)) != hipSuccess ||
      hipMalloc((void**)&g->d_idx, (16 + 3 * 4 * nre) * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc((void**)&g->d_seq, 10 * ((72 * 100 + 31) / 32) * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc((void**)&g->d_llr, 72 * 100 * sizeof(float)) != hipSuccess ||
      hipMalloc((void**)&g->d_cfi, sizeof(uint32_t)) != hipSuccess ||
      hipMalloc((void**)&g->d_corr, sizeof(float)) != hipSuccess) {
    ctrl_free(g);
    return nullptr;
  }
  return g;
}

// uploads the control rows of the host grids and estimates (the reference's host-side objects)
int ctrl_upload(CtrlGpu* g, const srsran_cell_t& cell, uint32_t rows, cf_t* sf_symbols[], srsran_chest_dl_res_t* ch)
{
  const size_t nre = 12 * (size_t)cell.nof_prb, n = rows * nre;
  g->rows = rows, g->nre = (uint32_t)nre, g->ports = cell.nof_ports;
  for (uint32_t r = 0; r < g->nrx; r++) {
    if (!sf_symbols[r] || hipMemcpyAsync(g->d_grid + r * n, sf_symbols[r], n * sizeof(float2), hipMemcpyHostToDevice,
                                         g->stream) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    for (uint32_t p = 0; p < cell.nof_ports; p++) {
      if (!ch->ce[p][r] || hipMemcpyAsync(g->d_ce + (p * g->nrx + r) * n, ch->ce[p][r], n * sizeof(float2),
                                          hipMemcpyHostToDevice, g->stream) != hipSuccess) {
        return SRSRAN_ERROR;
      }
    }
  }
  return SRSRAN_SUCCESS;
}

// gather + predecode n REs of table idx into g->d_x (codeword order)
int ctrl_equalise(CtrlGpu* g, const uint32_t* d_idx, uint32_t n, float noise)
{
  const size_t plane = (size_t)g->rows * g->nre;
  if (g->ports == 2) {
    CtrlEqArgs a{};
    for (uint32_t r = 0; r < g->nrx && r < 2; r++) {
      a.y[r] = g->d_grid + r * plane;
      for (int p = 0; p < 2; p++) {
        a.h[p][r] = g->d_ce + (p * g->nrx + r) * plane;
      }
    }
    a.idx         = d_idx;
    a.d           = g->d_x;
    a.n           = n;
    a.sse_symbols = n > 32 ? 4 * (n / 4) : 0;
    a.nrx         = (int)std::min(g->nrx, 2u);
    return ctrl_diversity_launch(a, g->stream) == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
  }
  if (g->ports == 4) {  // srsran_predecoding_diversity_multi without CSI + srsran_layerdemap_diversity
    PredArgs a{};
    for (uint32_t r = 0; r < g->nrx && r < 4; r++) {
      a.y[r] = g->d_grid + r * plane;
      for (int p = 0; p < 4; p++) {
        a.h[p][r] = g->d_ce + (p * g->nrx + r) * plane;
      }
    }
    a.x[0]       = g->d_x;
    a.scheme     = 4;
    a.nrx        = (int)std::min(g->nrx, 4u);
    a.n          = n;
    a.norm       = 1.0f;  // scaling
    a.idx        = d_idx;
    a.rho_b_inv  = 1.0f;
    a.interleave = 1;
    return predecode_launch(a, g->stream) == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
  }
  if (g->ports != 1) {
    fprintf(stderr, "[srsran_pdcch] %u ports: 1, 2 or 4 are provided\n", g->ports);
    return SRSRAN_ERROR;
  }
  PredArgs a{};
  for (uint32_t r = 0; r < g->nrx && r < 4; r++) {
    a.y[r]    = g->d_grid + r * plane;
    a.h[0][r] = g->d_ce + r * plane;
  }
  a.x[0]      = g->d_x;
  a.csi[0]    = g->d_csi;
  a.csi[1]    = g->d_csi + n;
  a.scheme    = 0;
  a.nrx       = (int)g->nrx;
  a.n         = n;
  a.norm      = 1.0f;
  a.noise     = noise;
  a.idx       = d_idx;
  a.rho_b_inv = 1.0f;
  return predecode_launch(a, g->stream) == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

bool valid_cell(const srsran_cell_t& c)
{
  return c.nof_prb >= 6 && c.nof_prb <= SRSRAN_MAX_PRB && (c.nof_ports == 1 || c.nof_ports == 2 || c.nof_ports == 4) &&
         (c.cp == SRSRAN_CP_NORM || c.cp == SRSRAN_CP_EXT) && c.id < 504;
}

}  // namespace

extern "C" {

// ---------------- regs ----------------
int srsran_regs_init(srsran_regs_t* h, srsran_cell_t cell)
{
  return srsran_regs_init_opts(h, cell, 1, false);
}

int srsran_regs_init_opts(srsran_regs_t* h, srsran_cell_t cell, uint32_t phich_mi, bool mbsfn_or_sf1_6_tdd)
{
  if (!h || !valid_cell(cell)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(h, 0, sizeof(*h));
  h->cell      = cell;
  h->phich_res = cell.phich_resources;
  h->phich_len = cell.phich_length;
  h->phich_mi  = phich_mi;
  if (build_regs(h, phich_mi, mbsfn_or_sf1_6_tdd)) {
    srsran_regs_free(h);
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

void srsran_regs_free(srsran_regs_t* h)
{
  if (!h) {
    return;
  }
  for (int c = 0; c < 3; c++) {
    free(h->pdcch_re[c]);
  }
  memset(h, 0, sizeof(*h));
}

int srsran_regs_pdcch_nregs(srsran_regs_t* h, uint32_t cfi)
{
  return h && cfi >= 1 && cfi <= 3 ? (int)h->pdcch_nregs[cfi - 1] : SRSRAN_ERROR;
}

int srsran_regs_pdcch_ncce(srsran_regs_t* h, uint32_t cfi)
{
  const int n = srsran_regs_pdcch_nregs(h, cfi);
  return n > 0 ? n / 9 : SRSRAN_ERROR;
}

uint32_t srsran_regs_pcfich_nregs(srsran_regs_t* h) { return h ? 4 : 0; }
uint32_t srsran_regs_phich_ngroups(srsran_regs_t* h) { return h ? h->ngroups_phich : 0; }
uint32_t srsran_regs_phich_ngroups_m1(srsran_regs_t* h) { return h ? h->ngroups_phich_m1 : 0; }

// ---------------- PCFICH ----------------
int srsran_pcfich_init(srsran_pcfich_t* q, uint32_t nof_rx_antennas)
{
  if (!q || nof_rx_antennas == 0 || nof_rx_antennas > 2) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(q, 0, sizeof(*q));
  q->nof_rx_antennas = nof_rx_antennas;
  q->nof_symbols     = PCFICH_RE;
  int dev            = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  q->gpu = ctrl_new(SRSRAN_MAX_PRB, nof_rx_antennas);
  return q->gpu ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

void srsran_pcfich_free(srsran_pcfich_t* q)
{
  if (q) {
    ctrl_free((CtrlGpu*)q->gpu);
    memset(q, 0, sizeof(*q));
  }
}

int srsran_pcfich_set_cell(srsran_pcfich_t* q, srsran_regs_t* regs, srsran_cell_t cell)
{
  if (!q || !q->gpu || !regs || !valid_cell(cell)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  CtrlGpu* g = (CtrlGpu*)q->gpu;
  q->regs    = regs;
  q->cell    = cell;
  std::vector<uint32_t> seq(10);
  for (uint32_t sf = 0; sf < 10; sf++) {  // srsran_sequence_pcfich (sequences.c:38-41)
    std::vector<uint32_t> w;
    gold_bits((sf + 1) * (2 * cell.id + 1) * 512 + cell.id, 32, w);
    seq[sf] = w[0];
  }
  if (hipMemcpyAsync(g->d_seq, seq.data(), 10 * sizeof(uint32_t), hipMemcpyHostToDevice, g->stream) != hipSuccess ||
      hipMemcpyAsync(g->d_idx, regs->pcfich_re, 16 * sizeof(uint32_t), hipMemcpyHostToDevice, g->stream) !=
          hipSuccess ||
      hipStreamSynchronize(g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

int srsran_pcfich_decode(srsran_pcfich_t* q, srsran_dl_sf_cfg_t* sf, srsran_chest_dl_res_t* channel,
                         cf_t* sf_symbols[SRSRAN_MAX_PORTS], float* corr_result)
{
  if (!q || !q->gpu || !sf || !channel || !sf_symbols || !q->regs) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  CtrlGpu* g = (CtrlGpu*)q->gpu;
  uint32_t cfi = 0;
  float    corr = 0;
  if (ctrl_upload(g, q->cell, 1, sf_symbols, channel) ||
      ctrl_equalise(g, g->d_idx, PCFICH_RE, channel->noise_estimate) ||
      pcfich_launch(g->d_x, g->d_seq + sf->tti % 10, g->d_llr, g->d_cfi, g->d_corr, g->stream) != hipSuccess ||
      hipMemcpyAsync(&cfi, g->d_cfi, sizeof(cfi), hipMemcpyDeviceToHost, g->stream) != hipSuccess ||
      hipMemcpyAsync(&corr, g->d_corr, sizeof(corr), hipMemcpyDeviceToHost, g->stream) != hipSuccess ||
      hipMemcpyAsync(q->data_f, g->d_llr, sizeof(q->data_f), hipMemcpyDeviceToHost, g->stream) != hipSuccess ||
      hipStreamSynchronize(g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  sf->cfi = cfi;
  if (corr_result) {
    *corr_result = corr;
  }
  return 1;
}

float srsran_pcfich_cfi_decode(srsran_pcfich_t* q, uint32_t* cfi)
{
  static const uint32_t words[3] = {0xB6DB6DB6u, 0x6DB6DB6Du, 0xDB6DB6DBu};
  float                 best     = 0;
  int                   idx      = 0;
  for (int c = 0; c < 3; c++) {
    float acc = 0;
    for (int i = 0; i < 32; i++) {
      acc += (((words[c] >> i) & 1u) ? 1.0f : -1.0f) * q->data_f[i];
    }
    if (acc > best) {
      best = acc;
      idx  = c;
    }
  }
  if (cfi) {
    *cfi = (uint32_t)idx + 1;
  }
  return best;
}

// ---------------- PDCCH ----------------
int srsran_pdcch_init_ue(srsran_pdcch_t* q, uint32_t max_prb, uint32_t nof_rx_antennas)
{
  if (!q || nof_rx_antennas == 0 || nof_rx_antennas > 2 || max_prb == 0 || max_prb > SRSRAN_MAX_PRB) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(q, 0, sizeof(*q));
  q->nof_rx_antennas = nof_rx_antennas;
  q->is_ue           = true;
  q->max_bits        = max_prb * 3 * 12 * 2;
  q->gpu             = ctrl_new(max_prb, nof_rx_antennas);
  return q->gpu ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

void srsran_pdcch_free(srsran_pdcch_t* q)
{
  if (q) {
    ctrl_free((CtrlGpu*)q->gpu);
    memset(q, 0, sizeof(*q));
  }
}

void srsran_pdcch_set_regs(srsran_pdcch_t* q, srsran_regs_t* regs)
{
  if (!q || !q->gpu || !regs) {
    return;
  }
  CtrlGpu* g = (CtrlGpu*)q->gpu;
  q->regs    = regs;
  uint32_t off = 16;
  for (int c = 0; c < 3; c++) {
    q->nof_regs[c] = (regs->pdcch_nregs[c] / 9) * 9;
    q->nof_cce[c]  = q->nof_regs[c] / 9;
    g->idx_off[c]  = off;
    hipMemcpyAsync(g->d_idx + off, regs->pdcch_re[c], 4 * (size_t)q->nof_regs[c] * sizeof(uint32_t),
                   hipMemcpyHostToDevice, g->stream);
    off += 4 * q->nof_regs[c];
  }
  q->max_bits = q->nof_cce[2] * 72;
  hipStreamSynchronize(g->stream);
}

int srsran_pdcch_set_cell(srsran_pdcch_t* q, srsran_regs_t* regs, srsran_cell_t cell)
{
  if (!q || !q->gpu || !regs || !valid_cell(cell)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  q->cell = cell;
  srsran_pdcch_set_regs(q, regs);
  CtrlGpu*       g     = (CtrlGpu*)q->gpu;
  const uint32_t nbits = 8 * regs->pdcch_nregs[2];  // sequence for the largest control region (pdcch.c:160-169)
  g->seq_words         = (nbits + 31) / 32;
  std::vector<uint32_t> all;
  for (uint32_t sf = 0; sf < 10; sf++) {  // srsran_sequence_pdcch (sequences.c:54-57)
    std::vector<uint32_t> w;
    gold_bits(sf * 512 + cell.id, nbits, w);
    all.insert(all.end(), w.begin(), w.end());
  }
  if (hipMemcpyAsync(g->d_seq, all.data(), all.size() * sizeof(uint32_t), hipMemcpyHostToDevice, g->stream) !=
          hipSuccess ||
      hipStreamSynchronize(g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

float srsran_pdcch_coderate(uint32_t nof_bits, uint32_t l)
{
  return (float)(nof_bits + 16) / (2 * ((1 << l) * 9));
}

int srsran_pdcch_extract_llr(srsran_pdcch_t* q, srsran_dl_sf_cfg_t* sf, srsran_chest_dl_res_t* channel,
                             cf_t* sf_symbols[SRSRAN_MAX_PORTS])
{
  if (!q || !q->gpu || !sf || sf->cfi < 1 || sf->cfi > 3 || !channel || !sf_symbols) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  CtrlGpu*       g     = (CtrlGpu*)q->gpu;
  const uint32_t ebits = 72 * q->nof_cce[sf->cfi - 1];
  const uint32_t rows  = q->cell.nof_prb <= 10 ? sf->cfi + 1 : sf->cfi;
  if (ctrl_upload(g, q->cell, rows, sf_symbols, channel) ||
      ctrl_equalise(g, g->d_idx + g->idx_off[sf->cfi - 1], ebits / 2, channel->noise_estimate / 2) ||
      pdcch_llr_launch(g->d_x, ebits, g->d_seq + (sf->tti % 10) * g->seq_words, g->d_llr, g->stream) != hipSuccess ||
      hipStreamSynchronize(g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  q->llr_cfi = sf->cfi;
  return SRSRAN_SUCCESS;
}

int srsran_pdcch_get_llr(srsran_pdcch_t* q, float* llr, uint32_t max)
{
  if (!q || !q->gpu || !llr || q->llr_cfi < 1) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  CtrlGpu*       g = (CtrlGpu*)q->gpu;
  const uint32_t n = std::min(max, 72 * q->nof_cce[q->llr_cfi - 1]);
  if (hipMemcpyAsync(llr, g->d_llr, n * sizeof(float), hipMemcpyDeviceToHost, g->stream) != hipSuccess ||
      hipStreamSynchronize(g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  return (int)n;
}

int srsran_pdcch_set_llr(srsran_pdcch_t* q, uint32_t cfi, const float* llr, uint32_t n)
{
  if (!q || !q->gpu || !llr || cfi < 1 || cfi > 3 || n != 72 * q->nof_cce[cfi - 1]) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  CtrlGpu* g = (CtrlGpu*)q->gpu;
  if (hipMemcpyAsync(g->d_llr, llr, n * sizeof(float), hipMemcpyHostToDevice, g->stream) != hipSuccess ||
      hipStreamSynchronize(g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  q->llr_cfi = cfi;
  return SRSRAN_SUCCESS;
}

int srsran_pdcch_gpu_decode_msgs(srsran_pdcch_t* q, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* dci_cfg,
                                 srsran_dci_msg_t* msgs, uint32_t nof_msg, float* corr)
{
  if (!q || !q->gpu || !sf || (nof_msg && !msgs) || sf->cfi < 1 || sf->cfi > 3 || q->llr_cfi != sf->cfi) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_msg == 0) {
    return SRSRAN_SUCCESS;
  }
  CtrlGpu*                g = (CtrlGpu*)q->gpu;
  std::vector<PdcchCand> c(nof_msg);
  const uint32_t         ncce = q->nof_cce[sf->cfi - 1];
  for (uint32_t i = 0; i < nof_msg; i++) {
    srsran_dci_msg_t& m = msgs[i];
    if (!srsran_dci_location_isvalid(&m.location) || m.location.ncce + (1u << m.location.L) > ncce) {
      fprintf(stderr, "[srsran_pdcch] invalid location: nCCE %u, L %u, CCEs %u\n", m.location.ncce, m.location.L, ncce);
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    const uint32_t nb = srsran_dci_format_sizeof(&q->cell, sf, dci_cfg, m.format);
    if (nb == 0 || nb > SRSRAN_DCI_MAX_BITS - 16) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    c[i] = {m.location.L, m.location.ncce, nb};
  }
  if (nof_msg > g->cand_cap) {
    hipFree(g->d_cand);
    hipFree(g->d_out);
    hipHostFree(g->h_out);
    g->d_cand = nullptr, g->d_out = nullptr, g->h_out = nullptr, g->cand_cap = 0;
    if (hipMalloc((void**)&g->d_cand, nof_msg * sizeof(PdcchCand)) != hipSuccess ||
        hipMalloc((void**)&g->d_out, nof_msg * sizeof(PdcchCandOut)) != hipSuccess ||
        hipHostMalloc((void**)&g->h_out, nof_msg * sizeof(PdcchCandOut)) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    g->cand_cap = nof_msg;
  }
  if (hipMemcpyAsync(g->d_cand, c.data(), nof_msg * sizeof(PdcchCand), hipMemcpyHostToDevice, g->stream) !=
          hipSuccess ||
      pdcch_cand_launch(g->d_llr, g->d_cand, nof_msg, g->d_out, g->stream) != hipSuccess ||
      hipMemcpyAsync(g->h_out, g->d_out, nof_msg * sizeof(PdcchCandOut), hipMemcpyDeviceToHost, g->stream) !=
          hipSuccess ||
      hipStreamSynchronize(g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  for (uint32_t i = 0; i < nof_msg; i++) {  // srsran_pdcch_decode_msg's updates (pdcch.c:368-398)
    const PdcchCandOut& o = g->h_out[i];
    srsran_dci_msg_t&   m = msgs[i];
    if (corr) {
      corr[i] = o.corr;
    }
    if (o.nof_bits == 0) {
      continue;  // mean |LLR| below 0.3: msg untouched
    }
    memcpy(m.payload, o.payload, o.nof_bits);
    m.rnti     = o.crc_rem;
    m.nof_bits = o.nof_bits;
    if (m.format == SRSRAN_DCI_FORMAT0 || m.format == SRSRAN_DCI_FORMAT1A) {
      m.format = m.payload[dci_cfg && dci_cfg->cif_enabled ? 3 : 0] == 0 ? SRSRAN_DCI_FORMAT0 : SRSRAN_DCI_FORMAT1A;
    }
  }
  return SRSRAN_SUCCESS;
}

int srsran_pdcch_decode_msg(srsran_pdcch_t* q, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* dci_cfg, srsran_dci_msg_t* msg)
{
  return srsran_pdcch_gpu_decode_msgs(q, sf, dci_cfg, msg, 1, nullptr);
}

float srsran_pdcch_msg_corr(srsran_pdcch_t* q, srsran_dci_msg_t* msg)
{
  // the correlation is produced with the decode (the re-encoding runs in the candidate kernel);
  // a standalone call re-decodes the message's location
  if (!q || !msg || q->llr_cfi < 1) {
    return 0.0f;
  }
  srsran_dl_sf_cfg_t sf;
  memset(&sf, 0, sizeof(sf));
  sf.cfi               = q->llr_cfi;
  srsran_dci_msg_t tmp = *msg;
  float            c   = 0.0f;
  return srsran_pdcch_gpu_decode_msgs(q, &sf, nullptr, &tmp, 1, &c) == SRSRAN_SUCCESS ? c : 0.0f;
}

uint32_t srsran_pdcch_ue_locations_ncce_L(uint32_t nof_cce, srsran_dci_location_t* c, uint32_t max_candidates,
                                          uint32_t sf_idx, uint16_t rnti, int Ls)
{
  static const uint32_t nof_candidates[4] = {6, 6, 2, 2};
  uint32_t              Yk                = rnti;
  for (uint32_t m = 0; m < sf_idx + 1; m++) {
    Yk = (39827 * Yk) % 65537;
  }
  uint32_t k = 0;
  for (int l = 0; l <= 3; l++) {
    const uint32_t L = 1u << l;
    if (Ls >= 0 && Ls != (int)L) {
      continue;
    }
    for (uint32_t i = 0; i < nof_candidates[l]; i++) {
      if (nof_cce < L) {
        continue;
      }
      const uint32_t ncce  = L * ((Yk + i) % (nof_cce / L));
      bool           valid = k < max_candidates && ncce + L <= nof_cce;
      for (uint32_t j = 0; j < k && valid; j++) {
        valid = c[j].L != (uint32_t)l || c[j].ncce != ncce;
      }
      if (valid) {
        c[k].L    = (uint32_t)l;
        c[k].ncce = ncce;
        k++;
      }
    }
  }
  return k;
}

uint32_t srsran_pdcch_ue_locations_ncce(uint32_t nof_cce, srsran_dci_location_t* c, uint32_t max_candidates,
                                        uint32_t sf_idx, uint16_t rnti)
{
  return srsran_pdcch_ue_locations_ncce_L(nof_cce, c, max_candidates, sf_idx, rnti, -1);
}

uint32_t srsran_pdcch_ue_locations(srsran_pdcch_t* q, srsran_dl_sf_cfg_t* sf, srsran_dci_location_t* c,
                                   uint32_t max_candidates, uint16_t rnti)
{
  const uint32_t ncce = sf->cfi >= 1 && sf->cfi <= 3 ? q->nof_cce[sf->cfi - 1] : 0;
  return srsran_pdcch_ue_locations_ncce(ncce, c, max_candidates, sf->tti % 10, rnti);
}

uint32_t srsran_pdcch_common_locations_ncce(uint32_t nof_cce, srsran_dci_location_t* c, uint32_t max_candidates)
{
  uint32_t k = 0;
  for (uint32_t l = 2; l <= 3; l++) {
    const uint32_t L = 1u << l;
    for (uint32_t i = 0; i < std::min(nof_cce, 16u) / L; i++) {
      const uint32_t ncce = L * i;
      if (k < max_candidates && ncce + L <= nof_cce) {
        c[k].L    = l;
        c[k].ncce = ncce;
        k++;
      }
    }
  }
  return k;
}

uint32_t srsran_pdcch_common_locations(srsran_pdcch_t* q, srsran_dci_location_t* c, uint32_t max_candidates,
                                       uint32_t cfi)
{
  return srsran_pdcch_common_locations_ncce(cfi >= 1 && cfi <= 3 ? q->nof_cce[cfi - 1] : 0, c, max_candidates);
}

}  // extern "C"
