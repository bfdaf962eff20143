// srsran_4g_amd/csrc/stage_timing.h -- optional HIP-event timing of every kernel launch, per
// pipeline stage (include/srsran_amd_prof.h).  Disabled: one relaxed atomic load per launch.
#ifndef SRSRAN_AMD_STAGE_TIMING_H
#define SRSRAN_AMD_STAGE_TIMING_H
#include <hip/hip_runtime.h>

namespace srsran_amd {

enum Stage { ST_OFDM = 0, ST_CHEST, ST_PRED, ST_LLR, ST_RM, ST_TDEC, ST_TB, ST_NR_RM, ST_LDPC, ST_NR_TB, ST_CHEST_UL, ST_PUSCH_EQ, ST_COUNT };

// Records a start event on construction and a stop event on destruction (same stream).
class StageScope {
public:
  StageScope(int stage, hipStream_t stream);
  ~StageScope();

private:
  int         stage_;
  hipStream_t stream_;
  hipEvent_t  e0_ = nullptr;
  int         dev_ = 0;
};

}  // namespace srsran_amd
#endif
