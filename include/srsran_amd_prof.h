/*
 * include/srsran_amd_prof.h -- added diagnostics: HIP-event timing of the GPU pipeline's kernel
 * launches per stage (no counterpart in the reference).  Stages: 0 OFDM, 1 channel estimation,
 * 2 predecoding, 3 demap/descramble/CSI, 4 rate dematching, 5 turbo decoding, 6 TB CRC / output,
 * 7 NR LDPC rate de-matching, 8 LDPC decoding, 9 NR TB assembly / CRC, 10 UL channel estimation,
 * 11 PUSCH equalisation + transform de-precoding.
 */
#ifndef SRSRAN_AMD_PROF_H
#define SRSRAN_AMD_PROF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRSRAN_AMD_NOF_STAGES 12

/* start (non-zero) or stop recording; clears the accumulators */
void srsran_amd_timing_enable(int enable);
/* waits for the recorded launches, returns per-stage total ms and launch counts, clears them */
int srsran_amd_timing_read(float ms[SRSRAN_AMD_NOF_STAGES], uint32_t launches[SRSRAN_AMD_NOF_STAGES]);
/* the kernel name of a stage (as rocprofv3 reports it, without template arguments) */
const char* srsran_amd_stage_name(int stage);

/* Host-side phases of the batch APIs (wall clock of the calling thread, microseconds): 0 the whole
 * srsran_ue_dl_gpu_decode_batch call, 1 OFDM + estimation enqueue, 2 PDSCH descriptors, 3 wait for the
 * previous PDSCH descriptor upload, 4 PDSCH upload + launches, 5 DL-SCH descriptors, 6 wait for the
 * previous DL-SCH descriptor upload, 7 DL-SCH upload + launches. */
#define SRSRAN_AMD_NOF_HOST_PHASES 8
/* start (non-zero) or stop recording; clears the accumulators */
void srsran_amd_host_timing_enable(int enable);
/* per-phase total microseconds and call counts since the last read; clears them */
int srsran_amd_host_timing_read(double us[SRSRAN_AMD_NOF_HOST_PHASES], uint32_t calls[SRSRAN_AMD_NOF_HOST_PHASES]);
const char* srsran_amd_host_phase_name(int phase);

#ifdef __cplusplus
}
#endif
#endif
