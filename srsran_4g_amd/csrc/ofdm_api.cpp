// srsran_4g_amd/csrc/ofdm_api.cpp -- C-ABI host side of the OFDM receiver and CFO correction.
//
// include/srsran_ue_dl.h: srsran_ofdm_rx_{init_cfg,set_prb,free,sf,sf_ng}, srsran_ofdm_set_normalize
// (ofdm.c:38-563) and srsran_cfo_{init,free,resize,set_tol,correct} (cfo.c:36-107), plus the
// batched device entry point.  The transforms run in ofdm_kernel.hip; no FFTW, no CPU fallback.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "../../include/srsran_ue_dl.h"
#include "stage_copy.h"
#include "devkey.h"
#include "ofdm_kernel.h"

using namespace srsran_amd;

namespace {

std::mutex                    g_tw_mu;
std::map<std::pair<int, uint32_t>, float2*> g_tw;  // per (device, FFT size): exp(-2 pi i m / N)

const float2* twiddles(uint32_t N)
{
  std::lock_guard<std::mutex> lk(g_tw_mu);
  const auto                  key = std::make_pair(cur_dev(), N);
  auto                        it  = g_tw.find(key);
  if (it != g_tw.end()) {
    return it->second;
  }
  std::vector<float2> h(N);
  for (uint32_t m = 0; m < N; m++) {
    const double ang = -2.0 * M_PI * (double)m / (double)N;
    h[m]             = make_float2((float)cos(ang), (float)sin(ang));
  }
  float2* d = nullptr;
  if (hipMalloc((void**)&d, N * sizeof(float2)) != hipSuccess ||
      hipMemcpy(d, h.data(), N * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) {
    return nullptr;
  }
  g_tw[key] = d;
  return d;
}

// srsran_vec_apply_cfo's phasor table for one (frequency, length), rebuilt on the launch stream only when the
// frequency changes (the reference recomputes it every call: SRSRAN_CFO_USE_EXP_TABLE is 0, cfo.c:33)
struct CfoTab {
  float2*    d     = nullptr;
  size_t     cap   = 0;
  uint32_t   bits  = 0;  // the float's bit pattern
  uint32_t   len   = 0;
  bool       valid = false;
  hipEvent_t used  = nullptr;  // the last launch that read d
  hipEvent_t built = nullptr;  // the launch that wrote d
  hipStream_t built_on = nullptr;
};

bool grow(void** p, size_t* cap, size_t need);

const float2* cfo_table(CfoTab& t, float f, uint32_t len, hipStream_t s)
{
  uint32_t bits;
  memcpy(&bits, &f, 4);
  if (t.valid && t.bits == bits && t.len == len) {
    if (t.built_on != s) {  // built on another stream: this launch must not read it before it is written
      hipStreamWaitEvent(s, t.built, 0);
    }
    return t.d;
  }
  if ((!t.used && srsran_amd::ring_event_create(&t.used) != hipSuccess) ||
      (!t.built && srsran_amd::ring_event_create(&t.built) != hipSuccess)) {
    return nullptr;
  }
  if (t.valid) {
    hipStreamWaitEvent(s, t.used, 0);  // a launch on another stream may still read the old table
  }
  if (len * sizeof(float2) > t.cap) {
    hipEventSynchronize(t.used);
    if (!grow((void**)&t.d, &t.cap, len * sizeof(float2))) {
      return nullptr;
    }
  }
  float c, sn;
  cfo_phasor(f, &c, &sn);
  if (cfo_table_launch(c, sn, t.d, len, s) != hipSuccess) {
    t.valid = false;
    return nullptr;
  }
  hipEventRecord(t.built, s);
  t.built_on = s;
  t.bits  = bits;
  t.len   = len;
  t.valid = true;
  return t.d;
}

void cfo_table_free(CfoTab& t)
{
  hipFree(t.d);
  if (t.used) {
    hipEventDestroy(t.used);
  }
  if (t.built) {
    hipEventDestroy(t.built);
  }
  t = CfoTab();
}

uint32_t cp_len(uint32_t c, uint32_t N) { return (uint32_t)ceilf((float)c * (float)N / 2048.0f); }  // SRSRAN_CP_LEN

struct OfdmGpu {
  hipStream_t stream = nullptr;
  float2*     d_in   = nullptr;
  float2*     d_out  = nullptr;
  size_t      in_cap = 0, out_cap = 0;
  OfdmArgs    proto{};
  CfoTab      cfo;
  bool        mbsfn = false;  // cfg.sf_type == SRSRAN_SF_MBSFN (ofdm.c:219-225)
  uint32_t    non_mbsfn_region = 2;
};

// slot 0 of an MBSFN subframe (ofdm_rx_slot_mbsfn, ofdm.c:522-535): the first `nr` symbols with the normal cyclic
// prefixes, the guard SRSRAN_NON_MBSFN_REGION_GUARD_LENGTH (phy_common.h:166-169) before symbol nr, extended cyclic
// prefixes after it -- the sample offset of each of the SRSRAN_CP_NSYMB(SRSRAN_CP_EXT) symbols
void mbsfn_offsets(uint32_t N, uint32_t nr, uint32_t* off)
{
  const uint32_t cpn0 = cp_len(160, N), cpn = cp_len(144, N), cpe = cp_len(512, N);
  uint32_t       pos  = 0;
  for (uint32_t i = 0; i < 6; i++) {
    if (i == nr) {
      pos += nr == 1 ? cpe - cpn0 : 2 * cpe - cpn0 - cpn;
    }
    pos += i >= nr ? cpe : (i == 0 ? cpn0 : cpn);
    off[i] = pos;
    pos += N;
  }
}

bool grow(void** p, size_t* cap, size_t need)
{
  if (*cap >= need) {
    return true;
  }
  hipFree(*p);
  *p = nullptr;
  if (hipMalloc(p, need) != hipSuccess) {
    *cap = 0;
    return false;
  }
  *cap = need;
  return true;
}

int configure(srsran_ofdm_t* q, uint32_t nof_prb, uint32_t symbol_sz)
{
  OfdmGpu* g = (OfdmGpu*)q->gpu;
  if (nof_prb == 0 || nof_prb > q->max_prb) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  const uint32_t N = symbol_sz ? symbol_sz : (uint32_t)srsran_symbol_sz(nof_prb);
  OfdmArgs       a{};
  a.nstages = ofdm_plan(N, a.radix, a.ns_magic);
  if ((int)N <= 0 || N > OFDM_MAX_N || a.nstages <= 0 || 12 * nof_prb > N) {
    fprintf(stderr, "[srsran_ofdm] unsupported symbol size %u\n", N);
    return SRSRAN_ERROR;
  }
  a.tw = twiddles(N);
  if (!a.tw) {
    return SRSRAN_ERROR;
  }
  const bool ext   = q->cfg.cp == SRSRAN_CP_EXT;
  a.N              = N;
  a.nsymb          = ext ? 6 : 7;                      // SRSRAN_CP_NSYMB
  a.cp0            = cp_len(ext ? 512 : 160, N);       // SRSRAN_CP_EXT_LEN / SRSRAN_CP_NORM_0_LEN
  a.cp             = cp_len(ext ? 512 : 144, N);       // SRSRAN_CP_EXT_LEN / SRSRAN_CP_NORM_LEN
  a.nre            = 12 * nof_prb;
  a.sf_len         = 2 * (a.nsymb * N + a.cp0 + (a.nsymb - 1) * a.cp);
  a.nrx            = 1;
  a.norm           = q->cfg.normalize ? 1.0f / sqrtf((float)N) : 1.0f;
  if (g->mbsfn) {
    a.mbsfn = 1;
    mbsfn_offsets(N, g->non_mbsfn_region, a.mbsfn_off);
  }
  g->proto         = a;
  q->cfg.nof_prb   = nof_prb;
  q->cfg.symbol_sz = N;
  q->nof_symbols   = a.nsymb;
  q->nof_re        = a.nre;
  q->slot_sz       = a.sf_len / 2;
  q->sf_sz         = a.sf_len;
  return SRSRAN_SUCCESS;
}

int run(srsran_ofdm_t* q, const float2* d_in, float2* d_out, uint32_t nrx, uint32_t nsf, float cfo, hipStream_t s)
{
  OfdmGpu* g = (OfdmGpu*)q->gpu;
  OfdmArgs a = g->proto;
  if (a.mbsfn && a.nsymb != 6) {  // MBSFN layouts are extended-CP ones (see srsran_ofdm_rx_sf_ng)
    return SRSRAN_ERROR;
  }
  a.in       = d_in;
  a.out      = d_out;
  a.nrx      = nrx;
  a.cfo_tab  = nullptr;
  if (cfo != 0.0f) {  // a zero frequency multiplies every sample by exactly 1 in the reference
    a.cfo_tab = cfo_table(g->cfo, cfo, a.sf_len, s);
    if (!a.cfo_tab) {
      return SRSRAN_ERROR;
    }
  }
  if (ofdm_rx_launch(a, nsf, s) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  if (a.cfo_tab) {
    hipEventRecord(g->cfo.used, s);
  }
  return SRSRAN_SUCCESS;
}

}  // namespace

extern "C" {

int srsran_ofdm_rx_init_cfg(srsran_ofdm_t* q, srsran_ofdm_cfg_t* cfg)
{
  if (!q || !cfg || cfg->nof_prb == 0 || cfg->nof_prb > 110) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if ((cfg->cp != SRSRAN_CP_NORM && cfg->cp != SRSRAN_CP_EXT) ||
      (cfg->sf_type != SRSRAN_SF_NORM && cfg->sf_type != SRSRAN_SF_MBSFN) ||
      std::isnormal(cfg->freq_shift_f) ||
      std::isnormal(cfg->rx_window_offset) || std::isnormal(cfg->phase_compensation_hz) || cfg->keep_dc) {
    fprintf(stderr, "[srsran_ofdm] only the srsran_ue_dl receiver configuration is provided\n");
    return SRSRAN_ERROR;
  }
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    fprintf(stderr, "[srsran_ofdm] no HIP device available\n");
    return SRSRAN_ERROR;
  }
  memset(q, 0, sizeof(*q));
  q->cfg     = *cfg;
  q->max_prb = cfg->nof_prb;
  OfdmGpu* g = new OfdmGpu();
  q->gpu     = g;
  g->mbsfn   = cfg->sf_type == SRSRAN_SF_MBSFN;  // non-MBSFN region 2 by default (ofdm.c:222)
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
    srsran_ofdm_rx_free(q);
    return SRSRAN_ERROR;
  }
  const int ret = configure(q, cfg->nof_prb, cfg->symbol_sz);
  if (ret) {
    srsran_ofdm_rx_free(q);
  }
  return ret;
}

int srsran_ofdm_rx_set_prb(srsran_ofdm_t* q, srsran_cp_t cp, uint32_t nof_prb)
{
  if (!q || !q->gpu) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (cp != SRSRAN_CP_NORM && cp != SRSRAN_CP_EXT) {
    return SRSRAN_ERROR;
  }
  q->cfg.cp = cp;
  return configure(q, nof_prb, 0);
}

void srsran_ofdm_rx_free(srsran_ofdm_t* q)
{
  if (!q) {
    return;
  }
  OfdmGpu* g = (OfdmGpu*)q->gpu;
  if (g) {
    if (g->stream) {
      hipStreamSynchronize(g->stream);
      hipStreamDestroy(g->stream);
    }
    hipFree(g->d_in);
    hipFree(g->d_out);
    cfo_table_free(g->cfo);
    delete g;
  }
  memset(q, 0, sizeof(*q));
}

void srsran_ofdm_set_normalize(srsran_ofdm_t* q, bool normalize_enable)
{
  if (q && q->gpu) {
    q->cfg.normalize             = normalize_enable;
    ((OfdmGpu*)q->gpu)->proto.norm = normalize_enable ? 1.0f / sqrtf((float)q->cfg.symbol_sz) : 1.0f;
  }
}

void srsran_ofdm_set_non_mbsfn_region(srsran_ofdm_t* q, uint8_t non_mbsfn_region)
{
  if (q && q->gpu) {
    OfdmGpu* g          = (OfdmGpu*)q->gpu;
    g->non_mbsfn_region = non_mbsfn_region;
    if (g->mbsfn) {
      mbsfn_offsets(g->proto.N, non_mbsfn_region, g->proto.mbsfn_off);
    }
  }
}

int srsran_ofdm_rx_init_mbsfn(srsran_ofdm_t* q, srsran_cp_t cp, cf_t* in_buffer, cf_t* out_buffer, uint32_t max_prb)
{
  srsran_ofdm_cfg_t cfg;  // ofdm.c:285-297
  memset(&cfg, 0, sizeof(cfg));
  cfg.cp         = cp;
  cfg.in_buffer  = in_buffer;
  cfg.out_buffer = out_buffer;
  cfg.nof_prb    = max_prb;
  cfg.sf_type    = SRSRAN_SF_MBSFN;
  return srsran_ofdm_rx_init_cfg(q, &cfg);
}

void srsran_ofdm_rx_sf_ng(srsran_ofdm_t* q, cf_t* input, cf_t* output)
{
  if (!q || !q->gpu) {
    return;
  }
  OfdmGpu* g = (OfdmGpu*)q->gpu;
  if (g->mbsfn) {
    // ofdm.c:576-578: an MBSFN object transforms its configured buffers whatever the arguments say; slot 0 has the
    // extended-CP symbol count (nof_symbols_mbsfn), slot 1 the object's own layout -- provided for extended CP, the
    // configuration srsran_ue_dl gives it (ue_dl.c:218)
    input  = q->cfg.in_buffer;
    output = q->cfg.out_buffer;
    if (q->cfg.cp != SRSRAN_CP_EXT) {
      fprintf(stderr, "[srsran_ofdm] MBSFN subframes with a normal-CP object are not provided\n");
      return;
    }
  }
  if (!input || !output) {
    return;
  }
  const size_t ni = q->sf_sz, no = 2 * q->nof_symbols * (size_t)q->nof_re;
  if (!grow((void**)&g->d_in, &g->in_cap, ni * sizeof(cf_t)) || !grow((void**)&g->d_out, &g->out_cap, no * sizeof(cf_t))) {
    return;
  }
  hipMemcpyAsync(g->d_in, input, ni * sizeof(cf_t), hipMemcpyHostToDevice, g->stream);
  if (run(q, g->d_in, g->d_out, 1, 1, 0.0f, g->stream) == SRSRAN_SUCCESS) {
    hipMemcpyAsync(output, g->d_out, no * sizeof(cf_t), hipMemcpyDeviceToHost, g->stream);
  }
  hipStreamSynchronize(g->stream);
}

void srsran_ofdm_rx_sf(srsran_ofdm_t* q)
{
  if (q) {
    srsran_ofdm_rx_sf_ng(q, q->cfg.in_buffer, q->cfg.out_buffer);
  }
}

int srsran_ofdm_rx_gpu(srsran_ofdm_t* q, const cf_t* d_in, cf_t* d_out, uint32_t nof_rx, uint32_t nof_sf, float cfo,
                       void* stream)
{
  if (!q || !q->gpu || !d_in || !d_out || nof_rx == 0) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_sf == 0) {
    return SRSRAN_SUCCESS;
  }
  return run(q, (const float2*)d_in, (float2*)d_out, nof_rx, nof_sf, cfo, (hipStream_t)stream);
}

// ---------------- cfo.c ----------------
struct CfoGpu {
  hipStream_t stream = nullptr;
  float2*     d      = nullptr;
  size_t      cap    = 0;
  CfoTab      tab;
};

int srsran_cfo_init(srsran_cfo_t* h, uint32_t nsamples)
{
  if (!h) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(h, 0, sizeof(*h));
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    fprintf(stderr, "[srsran_cfo] no HIP device available\n");
    return SRSRAN_ERROR;
  }
  CfoGpu* g = new CfoGpu();
  h->gpu    = g;
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess ||
      !grow((void**)&g->d, &g->cap, 2 * (size_t)(nsamples ? nsamples : 1) * sizeof(float2))) {
    srsran_cfo_free(h);
    return SRSRAN_ERROR;
  }
  h->nsamples    = nsamples;
  h->max_samples = nsamples;
  h->tol         = 0.0f;
  return SRSRAN_SUCCESS;
}

void srsran_cfo_free(srsran_cfo_t* h)
{
  if (!h) {
    return;
  }
  CfoGpu* g = (CfoGpu*)h->gpu;
  if (g) {
    if (g->stream) {
      hipStreamSynchronize(g->stream);
      hipStreamDestroy(g->stream);
    }
    hipFree(g->d);
    cfo_table_free(g->tab);
    delete g;
  }
  memset(h, 0, sizeof(*h));
}

int srsran_cfo_resize(srsran_cfo_t* h, uint32_t samples)
{
  if (!h || !h->gpu || samples > h->max_samples) {
    return SRSRAN_ERROR;
  }
  h->nsamples = samples;
  return SRSRAN_SUCCESS;
}

void srsran_cfo_set_tol(srsran_cfo_t* h, float tol)
{
  if (h) {
    h->tol = tol;
  }
}

void srsran_cfo_correct(srsran_cfo_t* h, const cf_t* input, cf_t* output, float freq)
{
  if (!h || !h->gpu || !input || !output || h->nsamples == 0) {
    return;
  }
  CfoGpu*      g = (CfoGpu*)h->gpu;
  const size_t n = h->nsamples;
  hipMemcpyAsync(g->d, input, n * sizeof(cf_t), hipMemcpyHostToDevice, g->stream);
  const float2* tab = cfo_table(g->tab, freq, (uint32_t)n, g->stream);
  if (tab && cfo_launch(g->d, g->d + n, tab, (uint32_t)n, g->stream) == hipSuccess) {
    hipEventRecord(g->tab.used, g->stream);
    hipMemcpyAsync(output, g->d + n, n * sizeof(cf_t), hipMemcpyDeviceToHost, g->stream);
  }
  hipStreamSynchronize(g->stream);
  h->last_freq = freq;
}


// ---------------- modulator (ofdm.c:585-690), srsran_enb_dl's configuration ----------------
int srsran_ofdm_tx_init_cfg(srsran_ofdm_t* q, srsran_ofdm_cfg_t* cfg)
{
  return srsran_ofdm_rx_init_cfg(q, cfg);  // same plan, twiddles and object; the direction is per call
}

void srsran_ofdm_tx_free(srsran_ofdm_t* q) { srsran_ofdm_rx_free(q); }

int srsran_ofdm_tx_gpu(srsran_ofdm_t* q, const cf_t* d_in, cf_t* d_out, uint32_t nof_ports, uint32_t nof_sf, float scale,
                       void* stream)
{
  if (!q || !q->gpu || !d_in || !d_out || nof_ports == 0 || nof_ports > 4 || nof_sf == 0) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  OfdmArgs a = ((OfdmGpu*)q->gpu)->proto;  // proto.norm = 1 / sqrt(N) when normalising, else 1
  a.in       = (const float2*)d_in;
  a.out      = (float2*)d_out;
  a.nrx      = nof_ports;
  a.norm     = a.norm * scale;
  return ofdm_tx_launch(a, nof_sf, (hipStream_t)stream) == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

void srsran_ofdm_tx_sf(srsran_ofdm_t* q)
{
  if (!q || !q->gpu || !q->cfg.in_buffer || !q->cfg.out_buffer) {
    return;
  }
  OfdmGpu*     g  = (OfdmGpu*)q->gpu;
  const size_t ni = 2 * q->nof_symbols * (size_t)q->nof_re, no = q->sf_sz;
  if (!grow((void**)&g->d_in, &g->in_cap, ni * sizeof(cf_t)) || !grow((void**)&g->d_out, &g->out_cap, no * sizeof(cf_t))) {
    return;
  }
  hipMemcpyAsync(g->d_in, q->cfg.in_buffer, ni * sizeof(cf_t), hipMemcpyHostToDevice, g->stream);
  if (srsran_ofdm_tx_gpu(q, (const cf_t*)g->d_in, (cf_t*)g->d_out, 1, 1, 1.0f, g->stream) == SRSRAN_SUCCESS) {
    hipMemcpyAsync(q->cfg.out_buffer, g->d_out, no * sizeof(cf_t), hipMemcpyDeviceToHost, g->stream);
  }
  hipStreamSynchronize(g->stream);
}

}  // extern "C"
