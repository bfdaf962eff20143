// srsran_4g_amd/csrc/phch_api.cpp -- C-ABI host side of the PDSCH LLR stages (include/srsran_phch.h).
//
// Host-synchronous drop-ins for srsran_demod_soft_demodulate_s (demod_soft.c:871-894),
// srsran_sequence_apply_s (sequence.c:507-561) and srsran_sequence_pdsch_apply_s
// (sequences.c:95-103), plus the fused device entry point.  No CPU fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <mutex>

#include "../../include/srsran_phch.h"
#include "devkey.h"
#include "eq_kernel.h"
#include "llr_kernel.h"
#include "pdsch_internal.h"

using namespace srsran_amd;

namespace {

std::mutex g_mu;
struct Ctx {  // host-synchronous stage APIs: one stream + scratch per device
  hipStream_t stream = nullptr;
  void*       d_a    = nullptr;
  size_t      a_cap  = 0;
  void*       d_b    = nullptr;
  size_t      b_cap  = 0;
};
std::map<int, Ctx> g_ctxs;

bool grow(void** p, size_t* cap, size_t need)
{
  if (*cap >= need) {
    return true;
  }
  hipFree(*p);
  *p = nullptr;
  need = std::max(need, (size_t)4096);
  if (hipMalloc(p, need) != hipSuccess) {
    *cap = 0;
    return false;
  }
  *cap = need;
  return true;
}

bool ctx_ready(Ctx& g_ctx)
{
  if (g_ctx.stream) {
    return true;
  }
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    fprintf(stderr, "[srsran_phch] no HIP device available\n");
    return false;
  }
  return hipStreamCreateWithFlags(&g_ctx.stream, hipStreamNonBlocking) == hipSuccess;
}

}  // namespace

namespace srsran_amd {

// srsran_predecoding_type's dispatch (precoding.c:1866-1930) for the MMSE CSI predecoders
// provided here; fills the scheme-dependent norm.  Returns false for unsupported shapes.
bool pred_setup(PredArgs& a, int nrx, int nports, int nlayers, int codebook, int type, float scaling)
{
  a.nrx      = nrx;
  a.codebook = codebook;
  switch (type) {
    case SRSRAN_TXSCHEME_PORT0:
      if (nports != 1 || nlayers != 1 || nrx < 1 || nrx > 4) {
        return false;
      }
      a.scheme = 0;
      a.norm   = 1.0f / scaling;  // precoding.c:319
      return true;
    case SRSRAN_TXSCHEME_DIVERSITY:
      if ((nports != 2 && nports != 4) || nlayers != nports || nrx < 1 || nrx > 4) {
        return false;
      }
      a.scheme = nports == 2 ? 1 : 4;
      a.norm   = scaling;  // hh *= scaling (precoding.c:695, 741-744)
      return true;
    case SRSRAN_TXSCHEME_CDD:
      if (nports != 2 || nrx != 2 || nlayers != 2) {
        return false;
      }
      a.scheme = 3;
      a.norm   = 2.0f / scaling;  // precoding.c:1052
      return true;
    case SRSRAN_TXSCHEME_SPATIALMUX:
      if (nports != 2 || nrx != 2 || nlayers != 2 || codebook < 0 || codebook > 2) {
        return false;
      }
      a.scheme = 2;
      a.norm   = codebook == 0 ? (float)1.41421356237309504880 / scaling : 2.0f / scaling;  // precoding.c:1451-1458
      return true;
    default:
      return false;
  }
}

uint32_t pdsch_seed(uint16_t rnti, int q, uint32_t nslot, uint32_t cell_id)
{
  return ((uint32_t)rnti << 14) + ((uint32_t)q << 13) + ((nslot / 2) << 9) + cell_id;  // sequences.c:62-65
}

}  // namespace srsran_amd

extern "C" {

int srsran_demod_soft_demodulate_s(srsran_mod_t modulation, const cf_t* symbols, short* llr, int nsymbols)
{
  const uint32_t q = srsran_mod_bits_x_symbol(modulation);
  if (q == 0 || nsymbols < 0 || (nsymbols && (!symbols || !llr))) {
    fprintf(stderr, "[srsran_demod_soft] Invalid modulation %d\n", (int)modulation);
    return -1;
  }
  if (nsymbols == 0) {
    return 0;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  Ctx&                        g_ctx = g_ctxs[cur_dev()];
  if (!ctx_ready(g_ctx) || !grow(&g_ctx.d_a, &g_ctx.a_cap, (size_t)nsymbols * sizeof(cf_t)) ||
      !grow(&g_ctx.d_b, &g_ctx.b_cap, (size_t)nsymbols * q * sizeof(int16_t))) {
    return -1;
  }
  hipMemcpyAsync(g_ctx.d_a, symbols, (size_t)nsymbols * sizeof(cf_t), hipMemcpyHostToDevice, g_ctx.stream);
  if (llr_launch((int)modulation, (const float*)g_ctx.d_a, (uint32_t)nsymbols, 0, 0, 0, nullptr, nullptr,
                 (int16_t*)g_ctx.d_b, g_ctx.stream) != hipSuccess) {
    return -1;
  }
  hipMemcpyAsync(llr, g_ctx.d_b, (size_t)nsymbols * q * sizeof(int16_t), hipMemcpyDeviceToHost, g_ctx.stream);
  return hipStreamSynchronize(g_ctx.stream) == hipSuccess ? 0 : -1;
}

void srsran_sequence_apply_s(const int16_t* in, int16_t* out, uint32_t length, uint32_t seed)
{
  if (length == 0 || !in || !out) {
    return;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  Ctx&                        g_ctx = g_ctxs[cur_dev()];
  const size_t bytes = (size_t)length * sizeof(int16_t);
  if (!ctx_ready(g_ctx) || !grow(&g_ctx.d_a, &g_ctx.a_cap, bytes) || !grow(&g_ctx.d_b, &g_ctx.b_cap, bytes)) {
    return;
  }
  hipMemcpyAsync(g_ctx.d_a, in, bytes, hipMemcpyHostToDevice, g_ctx.stream);
  if (seq_apply_launch((const int16_t*)g_ctx.d_a, (int16_t*)g_ctx.d_b, length, seed, g_ctx.stream) != hipSuccess) {
    fprintf(stderr, "[srsran_sequence] launch failed\n");
    return;
  }
  hipMemcpyAsync(out, g_ctx.d_b, bytes, hipMemcpyDeviceToHost, g_ctx.stream);
  hipStreamSynchronize(g_ctx.stream);
}

void srsran_sequence_pdsch_apply_s(const int16_t* in,
                                   int16_t*       out,
                                   uint16_t       rnti,
                                   int            q,
                                   uint32_t       nslot,
                                   uint32_t       cell_id,
                                   uint32_t       len)
{
  srsran_sequence_apply_s(in, out, len, pdsch_seed(rnti, q, nslot, cell_id));
}

int srsran_predecoding_type(cf_t*              y[4],
                            cf_t*              h[4][4],
                            cf_t*              x[4],
                            float*             csi[2],
                            int                nof_rxant,
                            int                nof_ports,
                            int                nof_layers,
                            int                codebook_idx,
                            int                nof_symbols,
                            srsran_tx_scheme_t type,
                            float              scaling,
                            float              noise_estimate)
{
  PredArgs a{};
  if (nof_ports > 4 || nof_layers > 4 || nof_symbols < 0 ||
      !pred_setup(a, nof_rxant, nof_ports, nof_layers, codebook_idx, (int)type, scaling)) {
    fprintf(stderr, "[srsran_predecoding] unsupported: scheme %d, %d ports, %d rx, %d layers\n", (int)type,
            nof_ports, nof_rxant, nof_layers);
    return SRSRAN_ERROR;
  }
  if (nof_symbols == 0) {
    return SRSRAN_SUCCESS;
  }
  const size_t n   = (size_t)nof_symbols;
  const size_t nin = (size_t)nof_rxant * (1 + nof_ports);  // y + h
  const size_t nout = (size_t)nof_layers;
  std::lock_guard<std::mutex> lk(g_mu);
  Ctx&                        g_ctx = g_ctxs[cur_dev()];
  if (!ctx_ready(g_ctx) || !grow(&g_ctx.d_a, &g_ctx.a_cap, nin * n * sizeof(cf_t)) ||
      !grow(&g_ctx.d_b, &g_ctx.b_cap, nout * n * (sizeof(cf_t) + sizeof(float)))) {
    return SRSRAN_ERROR;
  }
  cf_t*  dy  = (cf_t*)g_ctx.d_a;
  cf_t*  dh  = dy + (size_t)nof_rxant * n;
  cf_t*  dx  = (cf_t*)g_ctx.d_b;
  float* dcs = (float*)(dx + nout * n);
  for (int r = 0; r < nof_rxant; r++) {
    hipMemcpyAsync(dy + r * n, y[r], n * sizeof(cf_t), hipMemcpyHostToDevice, g_ctx.stream);
    a.y[r] = (const float2*)(dy + r * n);
    for (int p = 0; p < nof_ports; p++) {
      cf_t* d = dh + ((size_t)p * nof_rxant + r) * n;
      hipMemcpyAsync(d, h[p][r], n * sizeof(cf_t), hipMemcpyHostToDevice, g_ctx.stream);
      a.h[p][r] = (const float2*)d;
    }
  }
  for (int l = 0; l < nof_layers; l++) {
    a.x[l] = (float2*)(dx + l * n);
  }
  a.csi[0]  = dcs;
  a.csi[1]  = dcs + n;
  a.csi_max = nullptr;
  a.n       = (uint32_t)n;
  a.noise   = noise_estimate;
  if (predecode_launch(a, g_ctx.stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  // diversity: n/2 (2 ports) or m_ap (4 ports) symbols per layer, one CSI row; REs of an unpaired
  // last RE / half group are not written (precoding.c:674, 715)
  const bool   txd = a.scheme == 1 || a.scheme == 4;
  const size_t xn  = a.scheme == 1 ? n / 2 : a.scheme == 4 ? ((n % 4) ? (n >= 2 ? (n - 2) / 4 : 0) : n / 4) : n;
  for (int l = 0; l < nof_layers; l++) {
    hipMemcpyAsync(x[l], dx + l * n, xn * sizeof(cf_t), hipMemcpyDeviceToHost, g_ctx.stream);
    if (csi && l < (txd ? 1 : 2) && csi[l]) {
      hipMemcpyAsync(csi[l], dcs + l * n, (txd ? (size_t)nof_layers * xn : n) * sizeof(float), hipMemcpyDeviceToHost,
                     g_ctx.stream);
    }
  }
  if (hipStreamSynchronize(g_ctx.stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  // the reference's return values: single_csi -> nof_symbols, diversity_csi -> pairs, 2x2 MMSE -> 0
  return a.scheme == 0 ? (int)n : txd ? (int)xn : SRSRAN_SUCCESS;
}

int srsran_predecoding_gpu(const cf_t* const  d_y[4],
                           const cf_t* const  d_h[4][4],
                           cf_t* const        d_x[4],
                           float* const       d_csi[2],
                           float*             d_csi_max,
                           int                nof_rxant,
                           int                nof_ports,
                           int                nof_layers,
                           int                codebook_idx,
                           int                nof_symbols,
                           srsran_tx_scheme_t type,
                           float              scaling,
                           float              noise_estimate,
                           void*              stream)
{
  PredArgs a{};
  if (!d_y || !d_h || !d_x || !d_csi || nof_symbols < 0 ||
      !pred_setup(a, nof_rxant, nof_ports, nof_layers, codebook_idx, (int)type, scaling)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  for (int r = 0; r < nof_rxant; r++) {
    a.y[r] = (const float2*)d_y[r];
    for (int p = 0; p < nof_ports; p++) {
      a.h[p][r] = (const float2*)d_h[p][r];
    }
  }
  for (int l = 0; l < nof_layers; l++) {
    a.x[l] = (float2*)d_x[l];
  }
  a.csi[0]  = d_csi[0];
  a.csi[1]  = d_csi[1];
  a.csi_max = (uint32_t*)d_csi_max;
  a.n       = (uint32_t)nof_symbols;
  a.noise   = noise_estimate;
  return predecode_launch(a, (hipStream_t)stream) == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

int srsran_pdsch_gpu_llr(srsran_mod_t modulation,
                         const cf_t*  d_symbols,
                         uint32_t     nsymbols,
                         int          scramble,
                         uint32_t     seed,
                         const float* d_csi,
                         const float* d_csi_max,
                         int16_t*     d_llr,
                         void*        stream)
{
  if (srsran_mod_bits_x_symbol(modulation) == 0 || (nsymbols && (!d_symbols || !d_llr)) || (d_csi && !d_csi_max)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  return llr_launch((int)modulation, (const float*)d_symbols, nsymbols, scramble, seed, 0, d_csi, d_csi_max, d_llr,
                    (hipStream_t)stream) == hipSuccess
             ? SRSRAN_SUCCESS
             : SRSRAN_ERROR;
}

}  // extern "C"
