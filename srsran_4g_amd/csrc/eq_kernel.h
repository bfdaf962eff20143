// srsran_4g_amd/csrc/eq_kernel.h -- MIMO predecoding (MMSE equalisation) with CSI.
#ifndef SRSRAN_AMD_EQ_KERNEL_H
#define SRSRAN_AMD_EQ_KERNEL_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsran_amd {

struct PredArgs {
  const float2* y[4];     // [rx] received REs
  const float2* h[4][4];  // [port][rx] channel estimates
  float2*       x[4];     // [layer] equalised symbols
  float*        csi[2];   // [layer] CSI (srsran_predecoding_*_csi)
  uint32_t*     csi_max;  // optional [layer] running max of csi (float bits, csi >= 0)
  int           scheme;   // 0 PORT0, 2 SPATIALMUX, 3 CDD
  int           nrx;
  int           codebook;
  uint32_t      n;
  float         norm;
  float         noise;
};

hipError_t predecode_launch(const PredArgs& a, hipStream_t stream);

}  // namespace srsran_amd
#endif
