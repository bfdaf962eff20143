// srsran_4g_amd/csrc/pusch_kernel.h -- launch interface of the PUSCH receive kernels: UL channel
// estimation from the DMRS (chest_ul.c:298-433) and equalisation + SC-FDMA transform de-precoding
// (pusch.c:392-416, dft_precoding.c:114-126).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsran_amd {

static constexpr uint32_t PUSCH_MAX_M      = 1200;  // 12 * 100 PRB
static constexpr uint32_t PUSCH_MAX_STAGES = 8;

struct ChestUlOut {
  float noise;      // noise_estimate (0 without smoothing)
  float cfo_hz;
  float ta_us;
  float rsrp;       // min(|mean pilot|^2, epre)
  float epre;       // mean pilot power
  float data_pow;   // sum |y|^2 over the PUSCH data REs (meas_epre_en), summed by the eq kernel
};

// One UE / PUSCH allocation.  Grids are one subframe of the cell: nsym_sf symbols x ncell_re REs.
struct PuschUe {
  const float2* grid;      // received subframe grid
  const float2* dmrs;      // 2 * M pregenerated DMRS values (slot 0, slot 1)
  float2*       ce;        // channel estimate grid (written by the chest kernel, read by the eq kernel)
  float2*       sym;       // nof_symb * M de-precoded symbols
  ChestUlOut*   out;
  uint32_t      ncell_re;  // 12 * cell nof_prb
  uint32_t      M;         // 12 * L_prb
  uint32_t      nsym_slot; // 7 normal CP / 6 extended
  uint32_t      n_tilde[2];// first PRB read per slot (pusch_get / dmrs_pusch_get: n_prb_tilde)
  uint32_t      n_prb[2];  // first PRB of the estimate per slot (chest_ul: grant.n_prb)
  uint32_t      nof_symb;  // PUSCH data symbols
  uint8_t       data_sym[14];   // grid symbol of data symbol l
  uint8_t       radix[PUSCH_MAX_STAGES];  // inverse-DFT plan, radices 4 / 2 / 3 / 5
  uint32_t      nstages;
  float         filt[3];   // smoothing filter (filter_len 3), or all 0 with smooth = 0
  int32_t       smooth;    // smooth_filter_len == 3
  int32_t       meas_ta;
  double        noise_div; // a * 0.8 of estimate_noise_pilots (chest_ul.c:220-225), or 1
  float         noise;     // noise estimate for the equaliser (noise_dev = 0)
  int32_t       noise_dev; // 1: the equaliser reads out->noise (written by the chest kernel)
  float         dft_norm;  // 1 / sqrt(M)
};

// chest_ul_estimate for nue UEs (device descriptor array): one workgroup per UE
hipError_t chest_ul_launch(const PuschUe* d_ues, uint32_t nue, hipStream_t stream);
// predecoding_single + inverse DFT of every data symbol: grid (14, nue)
hipError_t pusch_eq_idft_launch(const PuschUe* d_ues, uint32_t nue, hipStream_t stream);

}  // namespace srsran_amd
