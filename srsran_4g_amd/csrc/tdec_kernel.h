// srsran_4g_amd/csrc/tdec_kernel.h -- launch interface of the HIP turbo decoder.
#ifndef SRSRAN_AMD_TDEC_KERNEL_H
#define SRSRAN_AMD_TDEC_KERNEL_H
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace srsran_amd {

static constexpr int TDEC_W       = 32;  // beta checkpoint window (must match the kernel)
static constexpr int TDEC_OVERLAP = 40;  // sliding-window training length

struct TdecArgs {
  const short*    in;        // ncb code blocks, in_stride int16 apart (device)
  uint32_t        in_stride;
  int             layout_sb; // 0: natural 3K+12, 1: rm_turbo sub-block layout
  uint32_t        K;
  uint32_t        ncb;
  int             n_start;   // first half-iteration index to run
  int             n_end;     // one past the last half-iteration index
  uint8_t*        out;       // ncb * K/8 hard-decision bytes (device)
  const uint16_t* tfwd;      // slot of pi(n(q))    (device, K entries, q order)
  const uint16_t* trev;      // slot of pi^-1(n(q)) (device, K entries, q order)
  const uint16_t* tfwd_nat;  // slot of pi(n)       (device, K entries, natural order)
  const uint16_t* trev_nat;  // slot of pi^-1(n)    (device, K entries, natural order)
  short*          state;     // optional ncb * 2 * xyw saved LLR/AUX state (device) or nullptr
  uint32_t        L;         // sub-block length (K for the generic decoder)
  uint32_t        Ls;        // LDS slot stride per sub-block
  uint32_t        xyw;       // LDS words per code block
  uint32_t        M;         // beta checkpoints per sub-block
  uint32_t        magicL;    // ceil(2^32 / L)
  uint32_t        dbg;       // profiling ablation only (SRSRAN_TDEC_ABLATE): bit0 skip prepare, bit1 skip MAP
};

hipError_t tdec_launch(int nsb, const TdecArgs& a, hipStream_t stream);
size_t     tdec_lds_bytes(int nsb, int xyw, int M);

}  // namespace srsran_amd
#endif
