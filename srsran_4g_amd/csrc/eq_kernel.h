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
  int           scheme;   // 0 PORT0, 1 DIVERSITY (n = REs, n/2 pairs), 2 SPATIALMUX, 3 CDD, 4 DIVERSITY on 4 ports
                          // (n/4 SFBC + FSTD groups)
  int           nrx;
  int           codebook;
  uint32_t      n;
  float         norm;
  float         noise;
  // ---- fused PDSCH extraction (srsran_pdsch_get, pdsch.c:838-853); all optional ----
  const uint32_t* idx;       // RE k reads grid index idx[k] & 0x7fffffff (nullptr: k itself)
  uint32_t        ce_row;    // > 0: h[p][r] is one AVERAGE row, indexed by (grid index % ce_row)
  const float*    noise_ptr; // device noise estimate (overrides `noise`)
  float           rho_b_inv; // y scale on CRS-bearing symbols (bit 31 of idx), 1 = none
  int             interleave; // DIVERSITY: write the codeword (layer-demapped) into x[0]; 2: SM / CDD
                              // with one codeword on 2 layers: d[2k + l] = x_l[k], k < n / 2, into x[0]
  int             pairs;      // csi_max_batch_launch only: idx lists (estimate index | RE parity << 31) pairs, the
                              // distinct (subcarrier, parity) of an AVERAGE estimate's REs -- their CSI values are the
                              // REs' own, so their maximum is the REs' maximum
};

hipError_t predecode_launch(const PredArgs& a, hipStream_t stream);
// nitems descriptors (device array), all with the same scheme; max_n = largest n
hipError_t predecode_batch_launch(const PredArgs* d_items, uint32_t nitems, int scheme, uint32_t max_n,
                                  hipStream_t stream);
// the same items' per-layer CSI maxima only (into csi_max; PORT0, SM, CDD): the pre-pass of the fused predecode +
// LLR path, which needs every codeword's maximum before its first LLR is scaled (pdsch.c:530)
hipError_t csi_max_batch_launch(const PredArgs* d_items, uint32_t nitems, int scheme, uint32_t max_n, hipStream_t stream);

}  // namespace srsran_amd
#endif
