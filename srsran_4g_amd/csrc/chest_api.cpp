// srsran_4g_amd/csrc/chest_api.cpp -- C-ABI host side of the DL channel estimator.
//
// include/srsran_ue_dl.h: srsran_chest_dl_{init,free,set_cell,res_init,res_free,estimate,
// estimate_cfg} (chest_dl.c:68-1027) plus the device entry point.  The CRS of every subframe
// (refsignal_dl.c:65-119, 36.211 6.10.1.1) is generated once per cell on the host and kept in
// HBM; estimation itself runs in chest_kernel.hip.  No CPU fallback.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "../../include/srsran_ue_dl.h"
#include "chest_kernel.h"
#include "pdsch_internal.h"
#include "ofdm_kernel.h"

using namespace srsran_amd;

namespace {

// phy_common.c:31-35: non-standard (3/4) sampling rates unless built with FORCE_STANDARD_RATE;
// srsUE and the reference tests opt in with srsran_use_standard_symbol_size(true).
bool g_standard_rates = false;

// LTE Gold sequence c(n), n = 0..len-1 (36.211 7.2, Nc = 1600)
void gold(uint32_t c_init, uint8_t* c, uint32_t len)
{
  uint32_t x1 = 1, x2 = c_init & 0x7FFFFFFFu;
  auto     s1 = [](uint32_t s) { return (s >> 1) ^ (((s ^ (s >> 3)) & 1u) << 30); };
  auto     s2 = [](uint32_t s) { return (s >> 1) ^ (((s ^ (s >> 1) ^ (s >> 2) ^ (s >> 3)) & 1u) << 30); };
  for (int n = 0; n < 1600; n++) {
    x1 = s1(x1);
    x2 = s2(x2);
  }
  for (uint32_t n = 0; n < len; n++) {
    c[n] = (uint8_t)((x1 ^ x2) & 1u);
    x1   = s1(x1);
    x2   = s2(x2);
  }
}

struct ChestGpu {
  hipStream_t stream  = nullptr;
  float2*     pilots  = nullptr;  // [sf][pp][4 * CHEST_MAX_NREF]
  float2*     grid    = nullptr;  // host-synchronous path scratch
  float2*     ce      = nullptr;
  float*      stats   = nullptr;  // [rx][port][8]
  float*      bstats  = nullptr;  // batch path: [sf][CHEST_STATS_PER_SF]
  float*      bsync   = nullptr;  // batch path, sync correction: [sf][CHEST_SYNC_PER_SF] phase sums
  float*      bserr   = nullptr;  // batch path, sync correction: [sf][rx * 4 + port] sync errors
  uint32_t    bstats_cap = 0;
  uint32_t    max_prb = 0;
  uint32_t    nrx     = 0;
  float       filter[8];
  uint32_t    filter_len = 0;
  float2*     pss     = nullptr;  // the cell's 62 PSS values (noise PSS)
  float*      noise   = nullptr;  // device q->noise_estimate [4][4]: host-sync upload / batch state; [16]: the batch
                                  // path's kept CFO (the last subframe with its own estimate)
  float*      sync    = nullptr;  // correct_sync_error sums [4 rx][4 port][10]
  float2*     tab     = nullptr;  // sync correction phasor table (12 * max_prb)
  float       sync_err[SRSRAN_MAX_PORTS][SRSRAN_MAX_PORTS] = {};  // q->sync_err (chest_dl.c:776)
  srsran_tdd_config_t tdd{};  // the batch estimators' TDD frame configuration (srsran_chest_dl_gpu_set_tdd_config)
  // MBSFN reference signals per area (q->mbsfn_refs, chest_dl.c:263-278): host tables [10 sf][3][6 nof_prb], the
  // one of area mbsfn_loaded on the device
  std::map<uint16_t, std::vector<float2>> mbsfn;
  float2* d_mbsfn      = nullptr;
  int     mbsfn_loaded = -1;
};

// srsran_refsignal_mbsfn_gen_seq (refsignal_dl.c:382-422): for every subframe and MBSFN symbol l (grid symbols
// 2 / 6 / 10, l' = 2 / 0 / 4 of slots 2 sf, 2 sf + 1, 2 sf + 1), c_init = 2^9 (7 (ns + 1) + l' + 1)(2 N_MBSFN + 1) +
// N_MBSFN and r(m') = (1 - 2 c(2m')) / sqrt 2 + j (1 - 2 c(2m' + 1)) / sqrt 2 at m' = m + 3 (110 - N_RB)
std::vector<float2> mbsfn_pilots(const srsran_cell_t& cell, uint32_t area)
{
  const uint32_t       N = cell.nof_prb;
  std::vector<float2>  t(10 * 18 * (size_t)N);
  std::vector<uint8_t> c(20 * 110);
  const float          a = (float)0.70710678118654752440;
  for (uint32_t sf = 0; sf < 10; sf++) {
    for (uint32_t l = 0; l < 3; l++) {
      const uint32_t lp = (2 + 4 * l) % 6, slot = l ? 2 * sf + 1 : 2 * sf;
      gold(512 * (7 * (slot + 1) + lp + 1) * (2 * area + 1) + area, c.data(), 20 * 110);
      for (uint32_t i = 0; i < 6 * N; i++) {
        const uint32_t mp = i + 3 * (110 - N);
        t[(sf * 3 + l) * 6 * N + i] = make_float2((1 - 2 * (float)c[2 * mp]) * a, (1 - 2 * (float)c[2 * mp + 1]) * a);
      }
    }
  }
  return t;
}

// srsran_refsignal_cs_nof_symbols (refsignal_dl.c:169-226) of a TDD special subframe: the CRS symbols of ports 0 / 1
// (port23 = false) or 2 / 3 that fall in its DwPTS
uint32_t special_crs_nsym(const srsran_tdd_config_t& tdd, srsran_cp_t cp, bool port23)
{
  const uint32_t n = srsran_sfidx_tdd_nof_dw(tdd);
  const bool     norm = cp == SRSRAN_CP_NORM;
  if (n >= (norm ? 12u : 10u)) {
    return port23 ? 2 : 4;
  } else if (n >= (norm ? 9u : 8u)) {
    return port23 ? 2 : 3;
  } else if (n >= (norm ? 5u : 4u)) {
    return port23 ? 1 : 2;
  }
  return 1;
}

// the special subframes of a TDD cell and their CRS symbol counts into the estimator's arguments (FDD cells and an
// unconfigured TDD configuration: none, as srsran_refsignal_cs_nof_symbols)
void tdd_args(const srsran_cell_t& cell, const srsran_tdd_config_t& tdd, ChestArgs& a)
{
  a.special_mask = 0;
  a.ss_nsym[0]   = 4;
  a.ss_nsym[1]   = 2;
  if (cell.frame_type != SRSRAN_TDD || !tdd.configured) {
    return;
  }
  for (uint32_t i = 0; i < 10; i++) {
    if (srsran_sfidx_tdd_type(tdd, i) == SRSRAN_TDD_SF_S) {
      a.special_mask |= 1u << i;
    }
  }
  a.ss_nsym[0] = special_crs_nsym(tdd, cell.cp, false);
  a.ss_nsym[1] = special_crs_nsym(tdd, cell.cp, true);
}

// INTERPOLATE in a special subframe whose DwPTS holds 2 CRS symbols of ports 0 / 1 (or 2-3 with extended CP): the
// reference's time interpolation reads estimate rows of the CRS symbols beyond the DwPTS, which it did not write in
// this call (chest_dl.c:520-546: left from an earlier subframe), so no result can equal it
bool tdd_interp_ok(const srsran_cell_t& cell, const srsran_tdd_config_t& tdd, const srsran_chest_dl_cfg_t* cfg)
{
  if (!cfg || cfg->estimator_alg != SRSRAN_ESTIMATOR_ALG_INTERPOLATE || cell.frame_type != SRSRAN_TDD ||
      !tdd.configured) {
    return true;
  }
  const uint32_t n = special_crs_nsym(tdd, cell.cp, false);
  return cell.cp == SRSRAN_CP_NORM ? n != 2 : (n == 1 || n == 4);
}

// srsran_pss_generate (pss.c:341-368): the argument in double, cosf / sinf of its float
void pss_generate(uint32_t N_id_2, float2* sig)
{
  const float root[3] = {25.0f, 29.0f, 34.0f};
  for (int i = 0; i < 62; i++) {
    const double v   = i < 31 ? ((float)i * ((float)i + 1.0)) : (((float)i + 2.0) * ((float)i + 1.0));
    const float  arg = (float)((float)-1 * M_PI * root[N_id_2] * v / 63.0);
    sig[i]           = make_float2(cosf(arg), sinf(arg));
  }
}

// the estimator options a call may use (chest_dl.c:655-745), the host-synchronous and the batch estimators alike
bool cfg_supported(const srsran_chest_dl_cfg_t* cfg)
{
  if (!cfg) {
    return true;
  }
  const bool est   = cfg->estimator_alg == SRSRAN_ESTIMATOR_ALG_AVERAGE || cfg->estimator_alg == SRSRAN_ESTIMATOR_ALG_INTERPOLATE;
  const bool noise = cfg->noise_alg == SRSRAN_NOISE_ALG_REFS || cfg->noise_alg == SRSRAN_NOISE_ALG_PSS ||
                     cfg->noise_alg == SRSRAN_NOISE_ALG_EMPTY;
  const bool filt  = cfg->filter_type == SRSRAN_CHEST_FILTER_TRIANGLE || cfg->filter_type == SRSRAN_CHEST_FILTER_NONE ||
                     (cfg->filter_type == SRSRAN_CHEST_FILTER_GAUSS && cfg->filter_coef[0] <= 7);
  return est && noise && filt && !cfg->rsrp_neighbour;
}

constexpr size_t kPilotsPerSf = 2 * 4 * CHEST_MAX_NREF;  // float2 per subframe (both port pairs)

uint32_t gauss(float* f, uint32_t order, float std_dev)  // chest_common.c:70-95
{
  const uint32_t len = order + 1;
  const int      c   = (int)(len - 1) / 2;
  for (uint32_t i = 0; i < len; i++) {
    f[i] = expf(-powf((float)((int)i - c), 2) / (2.0f * powf(std_dev, 2)));
  }
  float s = 0;
  for (uint32_t i = 0; i < len; i++) {
    s += f[i];
  }
  if (!std::isnormal(s)) {
    return 0;
  }
  for (uint32_t i = 0; i < len; i++) {
    f[i] *= 1.0f / s;
  }
  return len;
}

// the filter of chest_interpolate_noise_est (chest_dl.c:700-717) into the launch arguments: GAUSS with coefficients
// (order, stddev) or automatic (coef[0] <= 0: order 4, stddev 200 x noise, computed in the kernel), TRIANGLE
// {w, 1 - 2w, w} with w = coef[0] (srsran_chest_set_smooth_filter3_coeff), NONE (no smoothing)
void set_filter(const srsran_chest_dl_cfg_t* cfg, ChestArgs& a)
{
  a.filter_auto = a.filter_none = 0;
  if (cfg->filter_type == SRSRAN_CHEST_FILTER_TRIANGLE) {
    a.filter[0] = a.filter[2] = cfg->filter_coef[0];
    a.filter[1]  = 1 - 2 * cfg->filter_coef[0];
    a.filter_len = 3;
  } else if (cfg->filter_type == SRSRAN_CHEST_FILTER_NONE) {
    a.filter_none = 1;
  } else if (cfg->filter_coef[0] <= 0) {
    a.filter_auto = 1;
  } else {
    a.filter_len = gauss(a.filter, (uint32_t)cfg->filter_coef[0], cfg->filter_coef[1]);
  }
}

}  // namespace

extern "C" {

int srsran_symbol_sz_power2(uint32_t nof_prb)
{
  if (nof_prb <= 6) {
    return 128;
  } else if (nof_prb <= 15) {
    return 256;
  } else if (nof_prb <= 25) {
    return 512;
  } else if (nof_prb <= 52) {
    return 1024;
  } else if (nof_prb <= 79) {
    return 1536;
  } else if (nof_prb <= 110) {
    return 2048;
  }
  return -1;
}

int srsran_symbol_sz(uint32_t nof_prb)
{
  if (nof_prb == 0 || nof_prb > 110) {
    return SRSRAN_ERROR;
  }
  if (g_standard_rates) {
    return srsran_symbol_sz_power2(nof_prb);
  }
  return nof_prb <= 6 ? 128 : nof_prb <= 15 ? 256 : nof_prb <= 25 ? 384 : nof_prb <= 52 ? 768 : nof_prb <= 79 ? 1024 : 1536;
}

void srsran_use_standard_symbol_size(bool enabled) { g_standard_rates = enabled; }

bool srsran_symbol_size_is_standard(void) { return g_standard_rates; }

int srsran_sampling_freq_hz(uint32_t nof_prb)
{
  const int n = srsran_symbol_sz(nof_prb);
  return n < 0 ? SRSRAN_ERROR : 15000 * n;
}

int srsran_nof_prb(uint32_t symbol_sz)  // phy_common.c:387-430
{
  static const uint32_t kStd[6] = {128, 256, 512, 1024, 1536, 2048};
  static const uint32_t kNon[6] = {128, 256, 384, 768, 1024, 1536};
  static const int      kPrb[6] = {6, 15, 25, 50, 75, 100};
  const uint32_t*       t       = g_standard_rates ? kStd : kNon;
  for (int i = 0; i < 6; i++) {
    if (t[i] == symbol_sz) {
      return kPrb[i];
    }
  }
  return SRSRAN_ERROR;
}

bool srsran_symbol_sz_isvalid(uint32_t symbol_sz) { return srsran_nof_prb(symbol_sz) > 0; }  // phy_common.c:421-437

// ---------------- TDD frame structure (phy_common.c:92-182; 36.211 Tables 4.2-1 / 4.2-2) ----------------
srsran_tdd_sf_t srsran_sfidx_tdd_type(srsran_tdd_config_t tdd_config, uint32_t sf_idx)
{
  static const char kPattern[SRSRAN_MAX_TDD_SF_CONFIGS][11] = {"DSUUUDSUUU", "DSUUDDSUUD", "DSUDDDSUDD", "DSUUUDDDDD",
                                                               "DSUUDDDDDD", "DSUDDDDDDD", "DSUUUDSUUD"};
  if (tdd_config.sf_config < SRSRAN_MAX_TDD_SF_CONFIGS && sf_idx < 10 && tdd_config.configured) {
    const char c = kPattern[tdd_config.sf_config][sf_idx];
    return c == 'D' ? SRSRAN_TDD_SF_D : c == 'U' ? SRSRAN_TDD_SF_U : SRSRAN_TDD_SF_S;
  }
  return SRSRAN_TDD_SF_D;
}

// DwPTS / GP / UpPTS symbols of the special subframe configurations
static const uint8_t kTddSsSymbols[SRSRAN_MAX_TDD_SS_CONFIGS][3] = {{3, 10, 1}, {9, 4, 1},  {10, 3, 1}, {11, 2, 1},
                                                                    {12, 1, 1}, {3, 9, 2},  {9, 3, 2},  {10, 2, 2},
                                                                    {11, 1, 1}, {6, 6, 2}};

uint32_t srsran_sfidx_tdd_nof_dw(srsran_tdd_config_t c)
{
  return c.ss_config < SRSRAN_MAX_TDD_SS_CONFIGS ? kTddSsSymbols[c.ss_config][0] : 0;
}

uint32_t srsran_sfidx_tdd_nof_gp(srsran_tdd_config_t c)
{
  return c.ss_config < SRSRAN_MAX_TDD_SS_CONFIGS ? kTddSsSymbols[c.ss_config][1] : 0;
}

uint32_t srsran_sfidx_tdd_nof_up(srsran_tdd_config_t c)
{
  return c.ss_config < SRSRAN_MAX_TDD_SS_CONFIGS ? kTddSsSymbols[c.ss_config][2] : 0;
}

uint32_t srsran_tdd_nof_harq(srsran_tdd_config_t c)
{
  static const uint32_t n[SRSRAN_MAX_TDD_SF_CONFIGS] = {7, 4, 2, 3, 2, 1, 6};
  return c.sf_config < SRSRAN_MAX_TDD_SF_CONFIGS ? n[c.sf_config] : 0;
}

uint32_t srsran_sfidx_tdd_nof_dw_slot(srsran_tdd_config_t c, uint32_t slot, srsran_cp_t cp)
{
  const uint32_t n = srsran_sfidx_tdd_nof_dw(c), ns = SRSRAN_CP_NSYMB(cp);
  if (n < ns) {
    return slot == 1 ? 0 : n;
  }
  return slot == 1 ? n - ns : ns;
}

int srsran_chest_dl_init(srsran_chest_dl_t* q, uint32_t max_prb, uint32_t nof_rx_antennas)
{
  if (!q || max_prb == 0 || max_prb > 110 || nof_rx_antennas == 0 || nof_rx_antennas > SRSRAN_MAX_PORTS) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(q, 0, sizeof(*q));
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    fprintf(stderr, "[srsran_chest_dl] no HIP device available\n");
    return SRSRAN_ERROR;
  }
  ChestGpu* g     = new ChestGpu();
  g->max_prb      = max_prb;
  g->nrx          = nof_rx_antennas;
  const size_t sf = 14 * 12 * (size_t)max_prb;
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void**)&g->pilots, 10 * kPilotsPerSf * sizeof(float2)) != hipSuccess ||
      hipMalloc((void**)&g->grid, nof_rx_antennas * sf * sizeof(float2)) != hipSuccess ||
      hipMalloc((void**)&g->ce, SRSRAN_MAX_PORTS * nof_rx_antennas * sf * sizeof(float2)) != hipSuccess ||
      hipMalloc((void**)&g->stats, SRSRAN_MAX_PORTS * SRSRAN_MAX_PORTS * 8 * sizeof(float)) != hipSuccess ||
      hipMalloc((void**)&g->pss, 62 * sizeof(float2)) != hipSuccess ||
      hipMalloc((void**)&g->noise, 17 * sizeof(float)) != hipSuccess || hipMemset(g->noise, 0, 17 * sizeof(float)) ||
      hipMalloc((void**)&g->sync, 16 * 10 * sizeof(float)) != hipSuccess ||
      hipMalloc((void**)&g->tab, 12 * (size_t)max_prb * sizeof(float2)) != hipSuccess ||
      hipMalloc((void**)&g->d_mbsfn, 10 * 18 * (size_t)max_prb * sizeof(float2)) != hipSuccess) {
    q->gpu = g;
    srsran_chest_dl_free(q);
    return SRSRAN_ERROR;
  }
  q->gpu             = g;
  q->nof_rx_antennas = nof_rx_antennas;
  return SRSRAN_SUCCESS;
}

void srsran_chest_dl_free(srsran_chest_dl_t* q)
{
  if (!q) {
    return;
  }
  ChestGpu* g = (ChestGpu*)q->gpu;
  if (g) {
    if (g->stream) {
      hipStreamSynchronize(g->stream);
      hipStreamDestroy(g->stream);
    }
    hipFree(g->pilots);
    hipFree(g->grid);
    hipFree(g->ce);
    hipFree(g->stats);
    hipFree(g->bstats);
    hipFree(g->bsync);
    hipFree(g->bserr);
    hipFree(g->pss);
    hipFree(g->noise);
    hipFree(g->sync);
    hipFree(g->tab);
    hipFree(g->d_mbsfn);
    delete g;
  }
  memset(q, 0, sizeof(*q));
}

int srsran_chest_dl_set_cell(srsran_chest_dl_t* q, srsran_cell_t cell)
{
  if (!q || !q->gpu || cell.nof_prb == 0 || cell.nof_prb > ((ChestGpu*)q->gpu)->max_prb || cell.id >= 504 ||
      (cell.nof_ports != 1 && cell.nof_ports != 2 && cell.nof_ports != 4)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (cell.cp != SRSRAN_CP_NORM && cell.cp != SRSRAN_CP_EXT) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  ChestGpu* g = (ChestGpu*)q->gpu;
  q->cell     = cell;
  const uint32_t nsymb = SRSRAN_CP_NSYMB(cell.cp), N_cp = cell.cp == SRSRAN_CP_NORM ? 1 : 0;
  // refsignal_dl.c:65-119: per slot ns, CRS symbol l' of port pair pp, c_init as 36.211 6.10.1.1
  std::vector<float2> h(10 * kPilotsPerSf, make_float2(0.f, 0.f));
  std::vector<uint8_t> c(4 * 110);
  const float          a = (float)0.70710678118654752440;
  for (uint32_t ns = 0; ns < 20; ns++) {
    for (uint32_t pp = 0; pp < 2; pp++) {
      const uint32_t nsym_slot = pp == 0 ? 2 : 1;
      for (uint32_t l = 0; l < nsym_slot; l++) {
        const uint32_t lp     = pp == 0 ? (l ? nsymb - 3 : 0) : 1;  // srsran_refsignal_cs_nsymbol
        const uint32_t c_init = 1024 * (7 * (ns + 1) + lp + 1) * (2 * cell.id + 1) + 2 * cell.id + N_cp;
        gold(c_init, c.data(), 4 * 110);
        float2* dst = &h[(ns / 2) * kPilotsPerSf + pp * 4 * CHEST_MAX_NREF +
                         2 * cell.nof_prb * ((ns % 2) * nsym_slot + l)];
        for (uint32_t i = 0; i < 2 * cell.nof_prb; i++) {
          const uint32_t mp = i + 110 - cell.nof_prb;
          dst[i]            = make_float2((1 - 2 * (float)c[2 * mp]) * a, (1 - 2 * (float)c[2 * mp + 1]) * a);
        }
      }
    }
  }
  float2 pss[62];
  pss_generate(cell.id % 3, pss);  // chest_dl.c:291
  if (hipMemcpy(g->pilots, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(g->pss, pss, sizeof(pss), hipMemcpyHostToDevice) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  g->filter_len = gauss(g->filter, 4, 1.0f);
  g->mbsfn_loaded = -1;
  return SRSRAN_SUCCESS;
}

int srsran_chest_dl_set_mbsfn_area_id(srsran_chest_dl_t* q, uint16_t mbsfn_area_id)
{
  if (!q || !q->gpu || mbsfn_area_id >= 256 || q->cell.nof_prb == 0) {  // SRSRAN_MAX_MBSFN_AREA_IDS
    return SRSRAN_ERROR;
  }
  ChestGpu* g = (ChestGpu*)q->gpu;
  if (!g->mbsfn.count(mbsfn_area_id)) {  // generated once per area, with the cell of that moment (chest_dl.c:266-273)
    g->mbsfn[mbsfn_area_id] = mbsfn_pilots(q->cell, mbsfn_area_id);
  }
  return SRSRAN_SUCCESS;
}

int srsran_chest_dl_res_init(srsran_chest_dl_res_t* q, uint32_t max_prb)
{
  if (!q) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(q, 0, sizeof(*q));
  q->nof_re = 14 * 12 * max_prb;
  for (int p = 0; p < SRSRAN_MAX_PORTS; p++) {
    for (int r = 0; r < SRSRAN_MAX_PORTS; r++) {
      q->ce[p][r] = (cf_t*)calloc(q->nof_re, sizeof(cf_t));
      if (!q->ce[p][r]) {
        return SRSRAN_ERROR;
      }
    }
  }
  return SRSRAN_SUCCESS;
}

void srsran_chest_dl_res_free(srsran_chest_dl_res_t* q)
{
  if (!q) {
    return;
  }
  for (int p = 0; p < SRSRAN_MAX_PORTS; p++) {
    for (int r = 0; r < SRSRAN_MAX_PORTS; r++) {
      free(q->ce[p][r]);
    }
  }
  memset(q, 0, sizeof(*q));
}

static int chest_enqueue(srsran_chest_dl_t* q, uint32_t tti, const float2* d_grid, float2* d_ce, int full,
                         hipStream_t s, const srsran_chest_dl_cfg_t* cfg = nullptr,
                         const srsran_tdd_config_t* tdd = nullptr)
{
  ChestGpu* g = (ChestGpu*)q->gpu;
  ChestArgs a{};
  tdd_args(q->cell, tdd ? *tdd : g->tdd, a);
  a.grid       = d_grid;
  a.pilots     = g->pilots + (tti % 10) * kPilotsPerSf;
  a.ce         = d_ce;
  a.stats      = g->stats;
  a.nof_prb    = q->cell.nof_prb;
  a.cell_id    = q->cell.id;
  a.nports     = q->cell.nof_ports;
  a.nrx        = q->nof_rx_antennas;
  a.nsymb      = SRSRAN_CP_NSYMB(q->cell.cp);
  a.ce_stride  = (full ? 2 * a.nsymb : 1) * 12 * q->cell.nof_prb;
  a.full_grid  = full ? 1 : 0;
  a.filter_len = g->filter_len;
  memcpy(a.filter, g->filter, sizeof(a.filter));
  a.sf_index = tti % 10;
  a.pss      = g->pss;
  a.noise_in = g->noise;
  if (cfg) {
    set_filter(cfg, a);
    a.estimator = cfg->estimator_alg == SRSRAN_ESTIMATOR_ALG_INTERPOLATE ? 1 : 0;
    a.noise_alg = (uint32_t)cfg->noise_alg;
    if (a.estimator == 1 && !full) {
      return SRSRAN_ERROR;  // every symbol has its own estimate
    }
  }
  return chest_launch(a, s) == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

// correct_sync_error (chest_dl.c:750-804) of the host-synchronous path on the uploaded grids g->grid: the pilot
// phase sums on the device, the reference's scalar arithmetic here, and where the error exceeds 0.05 samples
// every row of that rx grid rotated on the device by srsran_vec_apply_cfo's phasors (then copied back to the
// caller's buffer, which the reference corrects in place)
static int correct_sync_error(srsran_chest_dl_t* q, uint32_t tti, const srsran_tdd_config_t& tdd,
                              cf_t* input[SRSRAN_MAX_PORTS])
{
  ChestGpu*      g   = (ChestGpu*)q->gpu;
  const uint32_t nre = 12 * q->cell.nof_prb, rows = 2 * SRSRAN_CP_NSYMB(q->cell.cp), np = q->cell.nof_ports;
  ChestArgs      a{};
  tdd_args(q->cell, tdd, a);
  a.sf_index = tti % 10;
  a.grid    = g->grid;
  a.pilots  = g->pilots + (tti % 10) * kPilotsPerSf;
  a.nof_prb = q->cell.nof_prb;
  a.cell_id = q->cell.id;
  a.nports  = np;
  a.nrx     = q->nof_rx_antennas;
  a.nsymb   = SRSRAN_CP_NSYMB(q->cell.cp);
  float sums[16 * 10];
  if (chest_sync_sums_launch(a, g->sync, g->stream) != hipSuccess ||
      hipMemcpyAsync(sums, g->sync, sizeof(sums), hipMemcpyDeviceToHost, g->stream) != hipSuccess ||
      hipStreamSynchronize(g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  const int sz = srsran_symbol_sz(q->cell.nof_prb);
  for (uint32_t rx = 0; rx < q->nof_rx_antennas; rx++) {
    float pwr_sum = 0.0f, sync_err = 0.0f;
    for (uint32_t port = 0; port < np; port++) {
      const float*   o    = sums + (rx * 4 + port) * 10;
      const uint32_t nsym = chest_crs_nsym(a, tti % 10, port), npilots = nsym * 2 * q->cell.nof_prb;
      const float    k    = (float)sz / 6.0f;
      float          sum  = 0.0f;
      for (uint32_t l = 0; l < nsym; l++) {  // srsran_vec_estimate_frequency: -cargf(sum) * M_1_PI * 0.5f
        const float f = (float)(-atan2f(o[2 * l + 1], o[2 * l]) * M_1_PI * 0.5f);
        sum += f * k;
      }
      const float pwr            = o[8] / (float)npilots;  // srsran_vec_avg_power_cf
      g->sync_err[rx][port]      = sum / (float)nsym;
      if (!std::isinf(sum) && !std::isnan(sum) && !std::isinf(pwr) && !std::isnan(pwr)) {
        sync_err += g->sync_err[rx][port] * pwr;
        pwr_sum += pwr;
      }
    }
    if (std::isnormal(pwr_sum)) {
      sync_err /= pwr_sum;
    }
    if (std::isnormal(sync_err) && fabsf(sync_err) > 0.05f) {
      float c, sn;
      cfo_phasor(sync_err / (float)sz, &c, &sn);
      float2* grid = g->grid + (size_t)rx * rows * nre;
      if (cfo_table_launch(c, sn, g->tab, nre, g->stream) != hipSuccess ||
          grid_rotate_launch(grid, g->tab, nre, rows, g->stream) != hipSuccess ||
          hipMemcpyAsync(input[rx], grid, (size_t)rows * nre * sizeof(cf_t), hipMemcpyDeviceToHost, g->stream) !=
              hipSuccess) {
        return SRSRAN_ERROR;
      }
    }
  }
  return SRSRAN_SUCCESS;
}

// fill_res (chest_dl.c:962-986) from the per (rx, port) statistics
static void fill_res(srsran_chest_dl_t* q, const float* st, srsran_chest_dl_res_t* res, bool update_cfo)
{
  const uint32_t np = q->cell.nof_ports, nrx = q->nof_rx_antennas;
  float          n  = 0;
  for (uint32_t rx = 0; rx < nrx; rx++) {
    float s = 0;
    for (uint32_t p = 0; p < np; p++) {
      const float* v          = st + (rx * np + p) * 8;
      q->noise_estimate[rx][p] = v[0];
      q->rsrp[rx][p]           = v[1];
      q->rssi[rx][p]           = v[2];
      s += v[0];
    }
    n += s / (float)np;
  }
  // chest_estimate_cfo: the last (rx, port) pair with 4 CRS symbols wins (chest_dl.c:655)
  for (int idx = (int)(nrx * np) - 1; update_cfo && idx >= 0; idx--) {
    const uint32_t p = (uint32_t)idx % np;
    if (p < 2) {
      const float* v  = st + idx * 8;
      const float  sz = (float)srsran_symbol_sz(q->cell.nof_prb);
      const float  ng = (float)(int)ceilf(144.0f * sz / 2048.0f);
      q->cfo          = -atan2f(v[4], v[3]) * sz / ((float)SRSRAN_CP_NSYMB(q->cell.cp) * (sz + ng)) / 2 / (float)M_PI;
      break;
    }
  }
  if (!res) {
    return;
  }
  res->noise_estimate     = n / (float)nrx;
  res->noise_estimate_dbm = 10.0f * log10f(res->noise_estimate) + 30.0f;
  res->cfo                = q->cfo;
  float rsrp_max          = -1e9f;
  for (uint32_t p = 0; p < np; p++) {
    float s = 0;
    for (uint32_t rx = 0; rx < nrx; rx++) {
      s += q->rsrp[rx][p];
    }
    s /= (float)nrx;
    res->rsrp_port_dbm[p] = 10.0f * log10f(s) + 30.0f;
    rsrp_max              = s > rsrp_max ? s : rsrp_max;
    for (uint32_t rx = 0; rx < nrx; rx++) {
      res->snr_ant_port_db[rx][p]   = 10.0f * log10f(q->rsrp[rx][p] / q->noise_estimate[rx][p]);
      res->rsrp_ant_port_dbm[rx][p] = 10.0f * log10f(q->rsrp[rx][p]) + 30.0f;
      res->rsrq_ant_port_db[rx][p]  = 10.0f * log10f(q->cell.nof_prb * q->rsrp[rx][p] / q->rssi[rx][p]);
    }
  }
  res->rsrp     = rsrp_max;
  res->rsrp_dbm = 10.0f * log10f(rsrp_max) + 30.0f;
  float rsrq = 0, rssi = 0;
  for (uint32_t rx = 0; rx < nrx; rx++) {
    rsrq += q->cell.nof_prb * q->rsrp[rx][0] / q->rssi[rx][0];
    rssi += 4 * q->rssi[rx][0] / q->cell.nof_prb / SRSRAN_NRE;
  }
  res->rsrq     = rsrq / (float)nrx;
  res->rsrq_db  = 10.0f * log10f(res->rsrq);
  res->rssi_dbm = 10.0f * log10f(rssi / (float)nrx) + 30.0f;
  res->snr_db   = 10.0f * log10f(res->rsrp / res->noise_estimate);
  res->sync_error = ((ChestGpu*)q->gpu)->sync_err[0][0];  // the channel used for synchronisation (chest_dl.c:974)
}

// srsran_chest_dl_estimate_cfg of an MBSFN subframe (chest_dl.c:1005-1026 with estimate_port_mbsfn, 836-865)
static int estimate_mbsfn(srsran_chest_dl_t*     q,
                          srsran_dl_sf_cfg_t*    sf,
                          srsran_chest_dl_cfg_t* cfg,
                          cf_t*                  input[SRSRAN_MAX_PORTS],
                          srsran_chest_dl_res_t* res)
{
  ChestGpu*      g   = (ChestGpu*)q->gpu;
  const uint32_t sfi = sf->tti % 10, nrx = q->nof_rx_antennas, np = q->cell.nof_ports, N = q->cell.nof_prb;
  const auto     it  = g->mbsfn.find(cfg->mbsfn_area_id);
  if (it == g->mbsfn.end() || it->second.size() != 10 * 18 * (size_t)N) {
    fprintf(stderr, "[srsran_chest_dl] MBSFN area id=%u not initialized for this cell (srsran_chest_dl_set_mbsfn_area_id)\n",
            (unsigned)cfg->mbsfn_area_id);
    return SRSRAN_ERROR;
  }
  if (cfg->estimator_alg != SRSRAN_ESTIMATOR_ALG_INTERPOLATE || np > 2 || sfi == 0 || sfi == 5) {
    // AVERAGE: the reference interpolates from estimate rows it did not write (chest_dl.c:511-521, 719-721); ports
    // 2 / 3: their CRS row is 1, yet the time interpolation starts from row 0 (518); subframes 0 / 5 are never MBSFN
    fprintf(stderr, "[srsran_chest_dl] MBSFN subframes: INTERPOLATE, ports 0 / 1 and subframes other than 0 / 5 only\n");
    return SRSRAN_ERROR;
  }
  const uint32_t nsf = 2 * SRSRAN_CP_NSYMB(q->cell.cp) * 12 * N, nrows12 = 12 * 12 * N;
  for (uint32_t rx = 0; rx < nrx; rx++) {
    hipMemcpyAsync(g->grid + rx * nsf, input[rx], nsf * sizeof(cf_t), hipMemcpyHostToDevice, g->stream);
  }
  if (cfg->sync_error_enable) {  // chest_dl.c:1007-1009 runs for MBSFN subframes too, on the CRS layout
    if (correct_sync_error(q, sf->tti, sf->tdd_config, input)) {
      return SRSRAN_ERROR;
    }
  } else {
    memset(g->sync_err, 0, sizeof(g->sync_err));
  }
  if (g->mbsfn_loaded != (int)cfg->mbsfn_area_id) {
    hipMemcpyAsync(g->d_mbsfn, it->second.data(), it->second.size() * sizeof(float2), hipMemcpyHostToDevice,
                   g->stream);
    g->mbsfn_loaded = cfg->mbsfn_area_id;
  }
  float kept[16] = {};
  for (uint32_t rx = 0; rx < nrx; rx++) {
    for (uint32_t p = 0; p < np; p++) {
      kept[rx * 4 + p] = q->noise_estimate[rx][p];
    }
  }
  hipMemcpyAsync(g->noise, kept, sizeof(kept), hipMemcpyHostToDevice, g->stream);
  ChestArgs a{};
  a.grid         = g->grid;
  a.pilots       = g->pilots + sfi * kPilotsPerSf;
  a.mbsfn_pilots = g->d_mbsfn + (size_t)sfi * 18 * N;
  a.ce           = g->ce;
  a.stats        = g->stats;
  a.nof_prb      = N;
  a.cell_id      = q->cell.id;
  a.nports       = np;
  a.nrx          = nrx;
  a.nsymb        = SRSRAN_CP_NSYMB(q->cell.cp);
  a.ce_stride    = nsf;
  a.full_grid    = 1;
  a.estimator    = 1;
  a.noise_alg    = (uint32_t)cfg->noise_alg;
  a.noise_in     = g->noise;
  a.sf_index     = sfi;
  set_filter(cfg, a);
  if (chest_mbsfn_launch(a, g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  for (uint32_t p = 0; p < np; p++) {
    for (uint32_t rx = 0; rx < nrx; rx++) {  // rows 0..11 (the rest of res->ce is left as it was)
      hipMemcpyAsync(res->ce[p][rx], g->ce + (p * nrx + rx) * nsf, nrows12 * sizeof(cf_t), hipMemcpyDeviceToHost,
                     g->stream);
    }
  }
  float st[SRSRAN_MAX_PORTS * SRSRAN_MAX_PORTS * 8];
  hipMemcpyAsync(st, g->stats, nrx * np * 8 * sizeof(float), hipMemcpyDeviceToHost, g->stream);
  if (hipStreamSynchronize(g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  for (uint32_t rx = 0; rx < nrx; rx++) {  // RSRP / RSSI are not measured in MBSFN subframes: q keeps them
    for (uint32_t p = 0; p < np; p++) {
      st[(rx * np + p) * 8 + 1] = q->rsrp[rx][p];
      st[(rx * np + p) * 8 + 2] = q->rssi[rx][p];
    }
  }
  fill_res(q, st, res, false);  // no CFO estimate either (chest_dl.c:655)
  return SRSRAN_SUCCESS;
}

int srsran_chest_dl_estimate_cfg(srsran_chest_dl_t*     q,
                                 srsran_dl_sf_cfg_t*    sf,
                                 srsran_chest_dl_cfg_t* cfg,
                                 cf_t*                  input[SRSRAN_MAX_PORTS],
                                 srsran_chest_dl_res_t* res)
{
  if (!q || !q->gpu || !sf || !cfg || !input || !res || q->cell.nof_prb == 0) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if ((sf->sf_type != SRSRAN_SF_NORM && sf->sf_type != SRSRAN_SF_MBSFN) || !cfg_supported(cfg)) {
    fprintf(stderr, "[srsran_chest_dl] the WIENER estimator, Gauss filter orders above 7 and rsrp_neighbour are not "
                    "provided\n");
    return SRSRAN_ERROR;
  }
  if (sf->sf_type == SRSRAN_SF_MBSFN) {
    return estimate_mbsfn(q, sf, cfg, input, res);
  }
  if (!tdd_interp_ok(q->cell, sf->tdd_config, cfg)) {
    fprintf(stderr, "[srsran_chest_dl] INTERPOLATE in TDD special subframes with 2 CRS symbols (3 with extended CP): "
                    "the reference interpolates towards rows it did not estimate\n");
    return SRSRAN_ERROR;
  }
  ChestGpu*      g   = (ChestGpu*)q->gpu;
  const uint32_t nsf = 2 * SRSRAN_CP_NSYMB(q->cell.cp) * 12 * q->cell.nof_prb, nrx = q->nof_rx_antennas,
                 np  = q->cell.nof_ports;
  for (uint32_t rx = 0; rx < nrx; rx++) {
    hipMemcpyAsync(g->grid + rx * nsf, input[rx], nsf * sizeof(cf_t), hipMemcpyHostToDevice, g->stream);
  }
  if (cfg->sync_error_enable) {
    if (correct_sync_error(q, sf->tti, sf->tdd_config, input)) {
      return SRSRAN_ERROR;
    }
  } else {
    memset(g->sync_err, 0, sizeof(g->sync_err));
  }
  float kept[16] = {};  // q->noise_estimate: the automatic filter's / PSS / EMPTY input
  for (uint32_t rx = 0; rx < nrx; rx++) {
    for (uint32_t p = 0; p < np; p++) {
      kept[rx * 4 + p] = q->noise_estimate[rx][p];
    }
  }
  hipMemcpyAsync(g->noise, kept, sizeof(kept), hipMemcpyHostToDevice, g->stream);
  if (chest_enqueue(q, sf->tti, g->grid, g->ce, 1, g->stream, cfg, &sf->tdd_config)) {
    return SRSRAN_ERROR;
  }
  for (uint32_t p = 0; p < np; p++) {
    for (uint32_t rx = 0; rx < nrx; rx++) {
      hipMemcpyAsync(res->ce[p][rx], g->ce + (p * nrx + rx) * nsf, nsf * sizeof(cf_t), hipMemcpyDeviceToHost,
                     g->stream);
    }
  }
  float st[SRSRAN_MAX_PORTS * SRSRAN_MAX_PORTS * 8];
  hipMemcpyAsync(st, g->stats, nrx * np * 8 * sizeof(float), hipMemcpyDeviceToHost, g->stream);
  if (hipStreamSynchronize(g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  // chest_estimate_cfo sizes its pilots by the FDD count (chest_dl.c:626): in a special subframe with fewer CRS
  // symbols it reads pilot estimates of an earlier subframe; q->cfo is kept from the last full subframe instead
  ChestArgs ta{};
  tdd_args(q->cell, sf->tdd_config, ta);
  const bool full_crs = chest_crs_nsym(ta, sf->tti % 10, 0) == 4;
  fill_res(q, st, res, full_crs && cfg->cfo_estimate_enable && ((1u << (sf->tti % 10)) & cfg->cfo_estimate_sf_mask));
  return SRSRAN_SUCCESS;
}

int srsran_chest_dl_estimate(srsran_chest_dl_t* q, srsran_dl_sf_cfg_t* sf, cf_t* input[SRSRAN_MAX_PORTS],
                             srsran_chest_dl_res_t* res)
{
  srsran_chest_dl_cfg_t cfg;
  memset(&cfg, 0, sizeof(cfg));  // AVERAGE, REFS, GAUSS with automatic coefficients (chest_dl.c:999-1007)
  return srsran_chest_dl_estimate_cfg(q, sf, &cfg, input, res);
}

}  // extern "C"

extern "C" int srsran_chest_dl_gpu_set_tdd_config(srsran_chest_dl_t* q, srsran_tdd_config_t tdd_config)
{
  if (!q || !q->gpu) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  ((ChestGpu*)q->gpu)->tdd = tdd_config;
  return SRSRAN_SUCCESS;
}

extern "C" int srsran_chest_dl_gpu_estimate(srsran_chest_dl_t* q,
                                            uint32_t           tti,
                                            const cf_t*        d_grid,
                                            cf_t*              d_ce,
                                            int                full_grid,
                                            float*             d_res,
                                            void*              stream)
{
  if (!q || !q->gpu || !d_grid || !d_ce || q->cell.nof_prb == 0) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  hipStream_t s = (hipStream_t)stream;
  if (chest_enqueue(q, tti, (const float2*)d_grid, (float2*)d_ce, full_grid, s)) {
    return SRSRAN_ERROR;
  }
  if (d_res) {
    ChestGpu* g = (ChestGpu*)q->gpu;
    chest_finalize_launch(g->stats, q->cell.nof_ports, q->nof_rx_antennas, q->cell.nof_prb,
                          (float)srsran_symbol_sz(q->cell.nof_prb), SRSRAN_CP_NSYMB(q->cell.cp), d_res, 1, s,
                          g->noise + 16);
  }
  return hipGetLastError() == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

/* added: nsf subframes in one launch.  d_sf_idx[b] = tti % 10 of subframe b (device);
 * d_grid + b * grid_sf_stride: nof_rx grids; d_ce + b * ce_sf_stride: [port][rx] rows of 12 * nof_prb
 * (the AVERAGE estimate); d_res + 4 * b: noise_estimate, rsrp, rssi, cfo. */
extern "C" int srsran_chest_dl_gpu_estimate_batch(srsran_chest_dl_t* q,
                                                  const uint32_t*    d_sf_idx,
                                                  uint32_t           nsf,
                                                  const cf_t*        d_grid,
                                                  size_t             grid_sf_stride,
                                                  cf_t*              d_ce,
                                                  size_t             ce_sf_stride,
                                                  float*             d_res,
                                                  void*              stream)
{
  return srsran_chest_dl_gpu_estimate_batch_cfg(q, nullptr, d_sf_idx, nsf, d_grid, grid_sf_stride, d_ce, ce_sf_stride,
                                                0, d_res, stream);
}

namespace srsran_amd {
bool chest_batch_cfg_supported(const srsran_chest_dl_t* q, const srsran_chest_dl_cfg_t* cfg, int full_grid)
{
  if (q && q->gpu && !tdd_interp_ok(q->cell, ((const ChestGpu*)q->gpu)->tdd, cfg)) {
    fprintf(stderr, "[srsran_chest_dl] batch: INTERPOLATE in TDD special subframes with 2 CRS symbols (3 with extended "
                    "CP) is not provided\n");
    return false;
  }
  if (!cfg_supported(cfg) || (cfg && cfg->estimator_alg == SRSRAN_ESTIMATOR_ALG_INTERPOLATE && !full_grid)) {
    fprintf(stderr, "[srsran_chest_dl] batch: configuration not provided (WIENER, TRIANGLE / NONE filters, filter "
                    "orders above 7, rsrp_neighbour, or INTERPOLATE without full grids)\n");
    return false;
  }
  return true;
}
}  // namespace srsran_amd

namespace {
// srsran_chest_dl_gpu_estimate_batch_cfg with the subframe indices from d_sf_idx (device) or h_sf (host, carried in
// the launch arguments, nsf <= CHEST_INLINE_SF)
int estimate_batch(srsran_chest_dl_t*           q,
                   const srsran_chest_dl_cfg_t* cfg,
                   const uint32_t*              d_sf_idx,
                   const uint8_t*               h_sf,
                   const srsran_amd::CopyJobs*  jobs,
                   uint32_t                     nsf,
                   const cf_t*                  d_grid,
                   size_t                       grid_sf_stride,
                   cf_t*                        d_ce,
                   size_t                       ce_sf_stride,
                   int                          full_grid,
                   float*                       d_res,
                   void*                        stream)
{
  if (!q || !q->gpu || (!d_sf_idx && !h_sf) || !d_grid || !d_ce || !d_res || q->cell.nof_prb == 0 ||
      (h_sf && nsf > (uint32_t)srsran_amd::CHEST_INLINE_SF)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (!srsran_amd::chest_batch_cfg_supported(q, cfg, full_grid)) {
    return SRSRAN_ERROR;
  }
  ChestGpu* g = (ChestGpu*)q->gpu;
  if (nsf > g->bstats_cap) {
    hipStreamSynchronize((hipStream_t)stream);  // the previous batch may still use them
    hipFree(g->bstats);
    hipFree(g->bsync);
    hipFree(g->bserr);
    g->bstats = g->bsync = g->bserr = nullptr;
    g->bstats_cap = 0;
    if (hipMalloc((void**)&g->bstats, nsf * CHEST_STATS_PER_SF * sizeof(float)) != hipSuccess ||
        hipMalloc((void**)&g->bsync, nsf * CHEST_SYNC_PER_SF * sizeof(float)) != hipSuccess ||
        hipMalloc((void**)&g->bserr, nsf * 16 * sizeof(float)) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    g->bstats_cap = nsf;
  }
  hipStream_t s = (hipStream_t)stream;
  ChestArgs   a{};
  tdd_args(q->cell, g->tdd, a);
  a.grid           = (const float2*)d_grid;
  a.pilots         = g->pilots;
  a.sf_idx         = d_sf_idx;
  if (h_sf) {
    a.sf_idx = nullptr;
    a.sf_inl = 1;
    memcpy(a.sf_inline, h_sf, nsf);
  }
  if (jobs) {
    a.jobs = *jobs;
  }
  a.grid_sf_stride = grid_sf_stride;
  a.ce             = (float2*)d_ce;
  a.ce_sf_stride   = ce_sf_stride;
  a.stats          = g->bstats;
  a.nof_prb        = q->cell.nof_prb;
  a.cell_id        = q->cell.id;
  a.nports         = q->cell.nof_ports;
  a.nrx            = q->nof_rx_antennas;
  a.nsymb          = SRSRAN_CP_NSYMB(q->cell.cp);
  a.ce_stride      = (full_grid ? 2 * a.nsymb : 1) * 12 * q->cell.nof_prb;
  a.full_grid      = full_grid ? 1 : 0;
  a.filter_len     = g->filter_len;
  memcpy(a.filter, g->filter, sizeof(a.filter));
  a.pss      = g->pss;
  a.noise_in = g->noise;  // the state before the batch (REFS: unused)
  if (cfg) {
    set_filter(cfg, a);
    a.estimator = cfg->estimator_alg == SRSRAN_ESTIMATOR_ALG_INTERPOLATE ? 1 : 0;
    a.noise_alg = (uint32_t)cfg->noise_alg;
  }
  const float sz = (float)srsran_symbol_sz(q->cell.nof_prb);
  if (cfg && cfg->sync_error_enable) {  // correct_sync_error on every subframe's grids first, in place (the reference
    // corrects its input buffer, chest_dl.c:795-803)
    if (chest_sync_sums_launch(a, g->bsync, s, nsf) != hipSuccess ||
        chest_sync_apply_launch(a, g->bsync, g->bserr, (float2*)d_grid, sz, nsf, s) != hipSuccess) {
      return SRSRAN_ERROR;
    }
  }
  if (a.noise_alg == 0) {  // REFS: the stats reduced by a small second launch (an in-kernel last-workgroup
    // reduction needed device-scope fences, whose L2 write-backs cost more than the launch: r04p stamps)
    return chest_launch(a, s, nsf) == hipSuccess &&
                   chest_finalize_launch(g->bstats, q->cell.nof_ports, q->nof_rx_antennas, q->cell.nof_prb, sz, a.nsymb,
                                         d_res, nsf, s, g->noise + 16) == hipSuccess
               ? SRSRAN_SUCCESS
               : SRSRAN_ERROR;
  }
  if (!a.filter_auto) {  // PSS / EMPTY with a fixed filter: the kept estimates carried in one pass after the launch
    if (chest_launch(a, s, nsf) != hipSuccess ||
        chest_finalize_kept_launch(g->bstats, q->cell.nof_ports, q->nof_rx_antennas, q->cell.nof_prb, sz, a.nsymb,
                                   g->noise, d_res, nsf, s, g->noise + 16) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    return SRSRAN_SUCCESS;
  }
  // PSS / EMPTY with the automatic filter: a subframe's filter width comes from the estimate kept after the last
  // subframe 0 / 5 before it (chest_dl.c:703-707, 731-745), so the batch runs in segments that each end at a subframe
  // 0 / 5 -- every subframe of a segment filters with the state from before it, whose last subframe then renews it
  // (with device-side subframe indices the host cannot see where they fall: one subframe a segment)
  for (uint32_t start = 0; start < nsf;) {
    uint32_t n = 1;
    if (h_sf) {
      while (start + n - 1 < nsf - 1 && h_sf[start + n - 1] != 0 && h_sf[start + n - 1] != 5) {
        n++;
      }
    }
    ChestArgs sa = a;
    sa.grid      = a.grid + start * grid_sf_stride;
    sa.ce        = a.ce + start * ce_sf_stride;
    sa.stats     = g->bstats + (size_t)start * CHEST_STATS_PER_SF;
    if (h_sf) {
      memcpy(sa.sf_inline, h_sf + start, n);
    } else {
      sa.sf_idx = d_sf_idx + start;
    }
    if (start > 0) {
      sa.jobs.n = 0;  // the staging copies ride in the first launch only
    }
    if (chest_launch(sa, s, n) != hipSuccess ||
        chest_finalize_kept_launch(sa.stats, q->cell.nof_ports, q->nof_rx_antennas, q->cell.nof_prb, sz, a.nsymb,
                                   g->noise, d_res + 4 * start, n, s, g->noise + 16) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    start += n;
  }
  return SRSRAN_SUCCESS;
}
}  // namespace

extern "C" int srsran_chest_dl_gpu_estimate_batch_cfg(srsran_chest_dl_t*           q,
                                                      const srsran_chest_dl_cfg_t* cfg,
                                                      const uint32_t*              d_sf_idx,
                                                      uint32_t                     nsf,
                                                      const cf_t*                  d_grid,
                                                      size_t                       grid_sf_stride,
                                                      cf_t*                        d_ce,
                                                      size_t                       ce_sf_stride,
                                                      int                          full_grid,
                                                      float*                       d_res,
                                                      void*                        stream)
{
  if (!d_sf_idx) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  return estimate_batch(q, cfg, d_sf_idx, nullptr, nullptr, nsf, d_grid, grid_sf_stride, d_ce, ce_sf_stride, full_grid,
                        d_res, stream);
}

// Diagnostic build only (lib/stamps/, tools/chest_stamps.py): chest_kernel workgroups write their phase clock
// stamps to d_buf ([workgroup][16] u64) from now on; SRSRAN_ERROR in the product build
extern "C" int srsran_chest_dl_gpu_debug_set_stamps(void* d_buf)
{
  return srsran_amd::chest_set_stamps(d_buf) == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

namespace srsran_amd {
int chest_dl_gpu_estimate_batch_inline(srsran_chest_dl_t*           q,
                                       const srsran_chest_dl_cfg_t* cfg,
                                       const uint8_t*               h_sf,
                                       const CopyJobs*              jobs,
                                       uint32_t                     nsf,
                                       const cf_t*                  d_grid,
                                       size_t                       grid_sf_stride,
                                       cf_t*                        d_ce,
                                       size_t                       ce_sf_stride,
                                       int                          full_grid,
                                       float*                       d_res,
                                       void*                        stream)
{
  return estimate_batch(q, cfg, nullptr, h_sf, jobs, nsf, d_grid, grid_sf_stride, d_ce, ce_sf_stride, full_grid, d_res,
                        stream);
}
}  // namespace srsran_amd
