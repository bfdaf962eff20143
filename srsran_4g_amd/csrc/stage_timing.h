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

// Host-side phases of the batch APIs (wall clock on the calling thread), to split the enqueue cost
// of a batch between descriptor building, staging waits and launches (srsran_amd_host_timing_*).
enum HostPhase {
  HP_UE_DL = 0,     // srsran_ue_dl_gpu_decode_batch, whole call
  HP_FRONT,         // OFDM + channel estimation enqueue
  HP_PDSCH_DESC,    // predecoder / LLR descriptors (RE tables, seeds)
  HP_PDSCH_WAIT,    // wait for the previous batch's descriptor upload
  HP_PDSCH_LAUNCH,  // descriptor upload + predecode / LLR launches
  HP_SCH_DESC,      // DL-SCH: segmentation, de-matching and turbo descriptors
  HP_SCH_WAIT,      // wait for the previous batch's descriptor upload
  HP_SCH_LAUNCH,    // descriptor upload + de-matching / turbo / TB launches
  HP_COUNT
};

class HostScope {
public:
  explicit HostScope(int phase);
  ~HostScope() { stop(); }
  void stop();  // ends the phase early (idempotent)

private:
  int     phase_;
  int64_t t0_ = -1;
};

}  // namespace srsran_amd
#endif
