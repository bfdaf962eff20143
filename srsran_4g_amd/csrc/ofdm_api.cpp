// srsran_4g_amd/csrc/ofdm_api.cpp -- C-ABI host side of the OFDM receiver and CFO correction.
//
// include/srsran_ue_dl.h: srsran_ofdm_rx_{init_cfg,set_prb,free,sf,sf_ng}, srsran_ofdm_set_normalize
// (ofdm.c:38-563) and srsran_cfo_{init,free,resize,set_tol,correct} (cfo.c:36-107), plus the
// batched device entry point.  The transforms run in ofdm_kernel.hip; no FFTW, no CPU fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
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
  // srsran_ofdm_cfg_t options (ofdm.c:151-157, 228-233, 357-449), tables on the device (config time only, as the
  // reference's "shall not be called during run-time")
  bool        dc_skip  = true;     // the DFT plan's dc flag (srsran_dft_plan_set_dc): the DC bin carries nothing
  uint32_t    win_n    = 0;        // window_offset_n
  float2*     d_wo     = nullptr;  // window_offset_buffer [N]
  size_t      wo_cap   = 0;
  float2*     d_ph     = nullptr;  // [0, 2 nsymb): RX conj(phase_compensation), [2 nsymb, 4 nsymb): TX phase_compensation
  size_t      ph_cap   = 0;
  bool        ph_on    = false;
  float2*     d_shift  = nullptr;  // shift_buffer [sf_sz]
  size_t      shift_cap = 0;
  float2*     d_comb   = nullptr;  // a CFO table times shift_buffer (srsran_ofdm_rx_gpu with both)
  size_t      comb_cap = 0;
  bool        shift_on = false;
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

bool upload(float2** d, size_t* cap, const std::vector<float2>& h)
{
  return grow((void**)d, cap, h.size() * sizeof(float2)) &&
         hipMemcpy(*d, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice) == hipSuccess;
}

// each symbol's cyclic prefix length, as SRSRAN_CP_LEN_NORM(i % nsymb) / SRSRAN_CP_LEN_EXT
uint32_t sym_cp(const OfdmArgs& a, uint32_t i) { return i % a.nsymb == 0 ? a.cp0 : a.cp; }

// window_offset_buffer (ofdm.c:156-158): cexpf(I M_PI 2 n i / N), the argument in double, the exponential in float
int build_window(OfdmGpu* g)
{
  if (g->win_n == 0) {
    return SRSRAN_SUCCESS;
  }
  const uint32_t      N = g->proto.N;
  std::vector<float2> h(N);
  for (uint32_t i = 0; i < N; i++) {
    const float y = (float)(M_PI * 2.0 * (double)(float)g->win_n * (double)(float)i / (double)(float)N);
    h[i]          = make_float2(cosf(y), sinf(y));
  }
  return upload(&g->d_wo, &g->wo_cap, h) ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

// srsran_ofdm_set_freq_shift's shift_buffer (ofdm.c:432-443): per symbol, t over its cyclic prefix and body,
// cexpf(I 2 M_PI (t - cplen) f / N)
int build_shift(OfdmGpu* g, float f)
{
  const OfdmArgs&     a = g->proto;
  std::vector<float2> h(a.sf_len);
  size_t              n = 0;
  for (uint32_t l = 0; l < 2 * a.nsymb; l++) {
    const uint32_t cpl = sym_cp(a, l);
    for (uint32_t t = 0; t < a.N + cpl; t++) {
      const float y = (float)(2.0 * M_PI * (double)((float)t - (float)cpl) * (double)f / (double)a.N);
      h[n++]        = make_float2(cosf(y), sinf(y));
    }
  }
  return upload(&g->d_shift, &g->shift_cap, h) ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

// srsran_ofdm_set_phase_compensation's phasors (ofdm.c:380-406): symbol l starts at t = (samples up to the end of
// its cyclic prefix) / (N x 15 kHz); phase -2 pi f t in double, cexp cast to float -- the receiver multiplies by the
// conjugate, the modulator by the phasor
int build_phase(OfdmGpu* g, double f)
{
  const OfdmArgs&     a = g->proto;
  const double        srate = (double)a.N * 15e3;
  std::vector<float2> h(4 * a.nsymb);
  uint32_t            count = 0;
  for (uint32_t l = 0; l < 2 * a.nsymb; l++) {
    count += sym_cp(a, l);
    const double ph = -2.0 * M_PI * f * ((double)count / srate);
    const float  c = (float)cos(ph), sn = (float)sin(ph);
    h[l]               = make_float2(c, -sn);
    h[2 * a.nsymb + l] = make_float2(c, sn);
    count += a.N;
  }
  return upload(&g->d_ph, &g->ph_cap, h) ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

// the option tables of the current size (configure, srsran_ofdm_set_*)
int build_options(srsran_ofdm_t* q)
{
  OfdmGpu* g = (OfdmGpu*)q->gpu;
  if (build_window(g) || (g->shift_on && build_shift(g, q->cfg.freq_shift_f)) ||
      (g->ph_on && build_phase(g, q->cfg.phase_compensation_hz))) {
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
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
  if (g->win_n > a.cp) {  // a window reaching before the cyclic prefix: outside the subframe's samples
    fprintf(stderr, "[srsran_ofdm] rx_window_offset of %u samples exceeds the cyclic prefix (%u)\n", g->win_n, a.cp);
    return SRSRAN_ERROR;
  }
  a.win            = g->win_n;
  a.dc0            = g->dc_skip ? 0 : 1;
  g->proto         = a;
  q->cfg.nof_prb   = nof_prb;
  q->cfg.symbol_sz = N;
  q->nof_symbols   = a.nsymb;
  q->nof_re        = a.nre;
  q->slot_sz       = a.sf_len / 2;
  q->sf_sz         = a.sf_len;
  return build_options(q);
}

// shift: apply the frequency shift's samples product in the transform (srsran_ofdm_rx_gpu; the host calls apply it to
// the input buffer first, as the reference does)
int run(srsran_ofdm_t* q, const float2* d_in, float2* d_out, uint32_t nrx, uint32_t nsf, float cfo, hipStream_t s,
        bool shift = true, const short2* d_in16 = nullptr, float scale = 1.0f)
{
  OfdmGpu* g = (OfdmGpu*)q->gpu;
  OfdmArgs a = g->proto;
  if (a.mbsfn && a.nsymb != 6) {  // MBSFN layouts are extended-CP ones (see srsran_ofdm_rx_sf_ng)
    return SRSRAN_ERROR;
  }
  a.in16     = d_in16;
  a.in_scale = scale;
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
  const bool used_cfo = a.cfo_tab != nullptr;
  if (shift && g->shift_on) {  // srsran_ofdm_rx_sf's input product by shift_buffer (ofdm.c:553-555)
    if (a.cfo_tab) {         // after the CFO correction: one table, their product
      if (!grow((void**)&g->d_comb, &g->comb_cap, a.sf_len * sizeof(float2)) ||
          cfo_launch(a.cfo_tab, g->d_comb, g->d_shift, a.sf_len, s) != hipSuccess) {
        return SRSRAN_ERROR;
      }
      a.cfo_tab = g->d_comb;
    } else {
      a.cfo_tab = g->d_shift;
    }
  }
  if (ofdm_rx_launch(a, nsf, s) != hipSuccess ||
      ofdm_rx_post_launch(d_out, nsf * nrx * 2 * a.nsymb, a, a.win ? g->d_wo : nullptr, g->ph_on ? g->d_ph : nullptr,
                          s) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  if (used_cfo) {
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
      (cfg->sf_type != SRSRAN_SF_NORM && cfg->sf_type != SRSRAN_SF_MBSFN)) {
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
  // options (ofdm.c:64-65, 151-157, 228-236): the window offset clamped to [0, 100] and written back to the caller's
  // configuration, window_offset_n = round(cp2 x offset) from the second symbol's cyclic prefix (the receiver's only;
  // the modulator never reads it); the shift and the DC flag; phase compensation set by its setter
  const uint32_t N0 = cfg->symbol_sz ? cfg->symbol_sz : (uint32_t)std::max(srsran_symbol_sz(cfg->nof_prb), 0);
  if (std::isnormal(cfg->rx_window_offset)) {
    cfg->rx_window_offset = std::min(100.0f, std::max(0.0f, cfg->rx_window_offset));
    g->win_n = (uint32_t)roundf((float)cp_len(cfg->cp == SRSRAN_CP_EXT ? 512 : 144, N0) * cfg->rx_window_offset);
  }
  q->cfg.rx_window_offset      = cfg->rx_window_offset;
  q->cfg.phase_compensation_hz = 0.0;
  g->shift_on                  = std::isnormal(cfg->freq_shift_f);
  g->dc_skip                   = !cfg->keep_dc && !g->shift_on;
  int ret = configure(q, cfg->nof_prb, cfg->symbol_sz);
  if (ret == SRSRAN_SUCCESS) {
    ret = srsran_ofdm_set_phase_compensation(q, cfg->phase_compensation_hz);
  }
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
  // ofdm.c:341-347 through ofdm_init_mbsfn_: a configuration of cp and nof_prb alone -- the window offset kept, the
  // shift rebuilt for the new size, the DC flag from that configuration's keep_dc (false) and the shift, and phase
  // compensation set to its 0 Hz (off)
  OfdmGpu* g = (OfdmGpu*)q->gpu;
  q->cfg.cp  = cp;
  g->dc_skip = !g->shift_on;
  g->ph_on   = false;
  q->cfg.phase_compensation_hz = 0.0;
  return configure(q, nof_prb, 0);
}

int srsran_ofdm_set_freq_shift(srsran_ofdm_t* q, float freq_shift)
{
  if (!q || !q->gpu) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  OfdmGpu* g          = (OfdmGpu*)q->gpu;
  q->cfg.freq_shift_f = freq_shift;
  g->shift_on         = std::isnormal(freq_shift);
  g->dc_skip          = !g->shift_on;  // ofdm.c:427, 446: DC removed without a shift, kept with one
  g->proto.dc0        = g->dc_skip ? 0 : 1;
  return g->shift_on ? build_shift(g, freq_shift) : SRSRAN_SUCCESS;
}

int srsran_ofdm_set_phase_compensation(srsran_ofdm_t* q, double center_freq_hz)
{
  if (!q || !q->gpu) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  OfdmGpu* g = (OfdmGpu*)q->gpu;
  if (q->cfg.phase_compensation_hz == center_freq_hz) {  // ofdm.c:364-367
    return SRSRAN_SUCCESS;
  }
  q->cfg.phase_compensation_hz = center_freq_hz;
  g->ph_on                     = std::isnormal(center_freq_hz);
  return g->ph_on ? build_phase(g, center_freq_hz) : SRSRAN_SUCCESS;
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
    hipFree(g->d_wo);
    hipFree(g->d_ph);
    hipFree(g->d_shift);
    hipFree(g->d_comb);
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
  if (g->shift_on) {  // ofdm.c:569-571: the input buffer itself multiplied by shift_buffer
    if (cfo_launch(g->d_in, g->d_in, g->d_shift, (uint32_t)ni, g->stream) != hipSuccess) {
      hipStreamSynchronize(g->stream);
      return;
    }
    hipMemcpyAsync(input, g->d_in, ni * sizeof(cf_t), hipMemcpyDeviceToHost, g->stream);
  }
  if (run(q, g->d_in, g->d_out, 1, 1, 0.0f, g->stream, false) == SRSRAN_SUCCESS) {
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

int srsran_ofdm_rx_gpu_sc16(srsran_ofdm_t* q, const int16_t* d_in, float scale, cf_t* d_out, uint32_t nof_rx,
                            uint32_t nof_sf, float cfo, void* stream)
{
  if (!q || !q->gpu || !d_in || !d_out || nof_rx == 0 || !std::isfinite(scale)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_sf == 0) {
    return SRSRAN_SUCCESS;
  }
  return run(q, nullptr, (float2*)d_out, nof_rx, nof_sf, cfo, (hipStream_t)stream, true, (const short2*)d_in, scale);
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
  OfdmGpu* g = (OfdmGpu*)q->gpu;
  if (g->mbsfn) {
    fprintf(stderr, "[srsran_ofdm] MBSFN modulation is not provided\n");
    return SRSRAN_ERROR;
  }
  OfdmArgs a = g->proto;  // proto.norm = 1 / sqrt(N) when normalising, else 1
  a.in       = (const float2*)d_in;
  a.out      = (float2*)d_out;
  a.nrx      = nof_ports;
  a.norm     = a.norm * scale;
  if (ofdm_tx_launch(a, nof_sf, (hipStream_t)stream) != hipSuccess ||
      ofdm_tx_post_launch((float2*)d_out, nof_sf * nof_ports, a, g->ph_on ? g->d_ph + 2 * a.nsymb : nullptr,
                          g->shift_on ? g->d_shift : nullptr, (hipStream_t)stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
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
