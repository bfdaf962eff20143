// srsran_4g_amd/csrc/phch_api.cpp -- C-ABI host side of the PDSCH LLR stages (include/srsran_phch.h).
//
// Host-synchronous drop-ins for srsran_demod_soft_demodulate_s (demod_soft.c:871-894),
// srsran_sequence_apply_s (sequence.c:507-561) and srsran_sequence_pdsch_apply_s
// (sequences.c:95-103), plus the fused device entry point.  No CPU fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <mutex>

#include "../../include/srsran_phch.h"
#include "llr_kernel.h"

using namespace srsran_amd;

namespace {

std::mutex g_mu;
struct Ctx {
  hipStream_t stream = nullptr;
  void*       d_a    = nullptr;
  size_t      a_cap  = 0;
  void*       d_b    = nullptr;
  size_t      b_cap  = 0;
} g_ctx;

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

bool ctx_ready()
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

uint32_t pdsch_seed(uint16_t rnti, int q, uint32_t nslot, uint32_t cell_id)
{
  return ((uint32_t)rnti << 14) + ((uint32_t)q << 13) + ((nslot / 2) << 9) + cell_id;  // sequences.c:62-65
}

}  // namespace

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
  if (!ctx_ready() || !grow(&g_ctx.d_a, &g_ctx.a_cap, (size_t)nsymbols * sizeof(cf_t)) ||
      !grow(&g_ctx.d_b, &g_ctx.b_cap, (size_t)nsymbols * q * sizeof(int16_t))) {
    return -1;
  }
  hipMemcpyAsync(g_ctx.d_a, symbols, (size_t)nsymbols * sizeof(cf_t), hipMemcpyHostToDevice, g_ctx.stream);
  if (llr_launch((int)modulation, (const float*)g_ctx.d_a, (uint32_t)nsymbols, 0, 0, 0, (int16_t*)g_ctx.d_b,
                 g_ctx.stream) != hipSuccess) {
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
  const size_t bytes = (size_t)length * sizeof(int16_t);
  if (!ctx_ready() || !grow(&g_ctx.d_a, &g_ctx.a_cap, bytes) || !grow(&g_ctx.d_b, &g_ctx.b_cap, bytes)) {
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

int srsran_pdsch_gpu_llr(srsran_mod_t modulation,
                         const cf_t*  d_symbols,
                         uint32_t     nsymbols,
                         int          scramble,
                         uint32_t     seed,
                         int16_t*     d_llr,
                         void*        stream)
{
  if (srsran_mod_bits_x_symbol(modulation) == 0 || (nsymbols && (!d_symbols || !d_llr))) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  return llr_launch((int)modulation, (const float*)d_symbols, nsymbols, scramble, seed, 0, d_llr,
                    (hipStream_t)stream) == hipSuccess
             ? SRSRAN_SUCCESS
             : SRSRAN_ERROR;
}

}  // extern "C"
