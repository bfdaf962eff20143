/*
 * include/srsran_tdec.h -- drop-in C API of the MI355X turbo decoder.
 *
 * Replaces the reference interface lib/include/srsran/phy/fec/turbo/turbodecoder.h
 * (srsRAN_4G, paths relative to /root/reference/lib).  Same function names, argument
 * meaning and return conventions; the decoding runs on the GPU through HIP.  Every
 * entry point is a plain C symbol with plain pointers and sizes.
 *
 * Semantics are those of the reference AUTO 16-bit decoder of an AVX2 build
 * (turbodecoder.c:381-408): generic decoder for K <= 400, 8-sub-block window for
 * 408..800, 16-sub-block window for K >= 816.  Results (hard bits, CRC outcome)
 * are bit-identical to the reference on the same int16 LLRs.
 *
 * Input layout: by default the input is the sub-block ("SB") layout written by
 * srsran_rm_turbo_rx_lut for window decoders (SRSRAN_TDEC_EXPECT_INPUT_SB,
 * turbodecoder.h:47); srsran_tdec_force_not_sb() selects the natural 3K+12 layout.
 */
#ifndef SRSRAN_AMD_TDEC_H
#define SRSRAN_AMD_TDEC_H

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* lib/include/srsran/config.h:56-63 */
#ifndef SRSRAN_SUCCESS
#define SRSRAN_SUCCESS 0
#define SRSRAN_ERROR -1
#define SRSRAN_ERROR_INVALID_INPUTS -2
#endif

/* turbodecoder.h:26-33 */
#define SRSRAN_TCOD_RATE 3
#define SRSRAN_TCOD_TOTALTAIL 12
#define SRSRAN_TCOD_MAX_LEN_CB 6144
#define SRSRAN_TDEC_EXPECT_INPUT_SB 1
#define SRSRAN_NOF_TC_CB_SIZES 188

/* turbodecoder_impl.h:26-36 */
typedef enum {
  SRSRAN_TDEC_AUTO = 0,
  SRSRAN_TDEC_GENERIC,
  SRSRAN_TDEC_SSE,
  SRSRAN_TDEC_SSE_WINDOW,
  SRSRAN_TDEC_NEON_WINDOW,
  SRSRAN_TDEC_AVX_WINDOW,
  SRSRAN_TDEC_SSE8_WINDOW,
  SRSRAN_TDEC_AVX8_WINDOW,
  SRSRAN_TDEC_NOF_IMP
} srsran_tdec_impl_type_t;

/*
 * turbodecoder.h:63-95.  Callers own the struct (stack/static) as in the
 * reference; the fields callers read are kept with the same names.  The CPU
 * scratch buffers and per-implementation tables of the reference are replaced by
 * one opaque device context.
 */
typedef struct {
  uint32_t                max_long_cb;
  bool                    force_not_sb;
  srsran_tdec_impl_type_t dec_type;
  uint32_t                current_long_cb;
  int                     current_cbidx;
  int                     n_iter;
  void*                   gpu; /* opaque: HIP stream, device buffers, saved decoder state */
} srsran_tdec_t;

/* turbodecoder.c:129-132 */
int srsran_tdec_init(srsran_tdec_t* h, uint32_t max_long_cb);
/* turbodecoder.c:151-317.  Supported: AUTO, GENERIC, SSE_WINDOW, AVX_WINDOW. */
int srsran_tdec_init_manual(srsran_tdec_t* h, uint32_t max_long_cb, srsran_tdec_impl_type_t dec_type);
/* turbodecoder.c:319-363 */
void srsran_tdec_free(srsran_tdec_t* h);
/* turbodecoder.c:365-368 */
void srsran_tdec_force_not_sb(srsran_tdec_t* h);
/* turbodecoder.c:510-525 */
int srsran_tdec_new_cb(srsran_tdec_t* h, uint32_t long_cb);
/* turbodecoder.c:579-582 */
int srsran_tdec_get_nof_iterations(srsran_tdec_t* h);
/* turbodecoder.c:381-393 / 410-424 (AVX2 build) */
uint32_t srsran_tdec_autoimp_get_subblocks(uint32_t long_cb);
uint32_t srsran_tdec_autoimp_get_subblocks_8bit(uint32_t long_cb);
/* turbodecoder.c:527-533: one half-iteration, then hard decision into output (K/8 bytes). */
void srsran_tdec_iteration(srsran_tdec_t* h, int16_t* input, uint8_t* output);
/* turbodecoder.c:536-549: nof_iterations half-iterations, then hard decision. */
int srsran_tdec_run_all(srsran_tdec_t* h, int16_t* input, uint8_t* output, uint32_t nof_iterations, uint32_t long_cb);
/* turbodecoder.c:551-577 (AUTO, tdec_iteration_8 at :455-483): int8 LLRs; K > 2048 on the AVX2 8-bit
 * window decoder (32 sub-blocks), 800 < K <= 2048 on the SSE 8-bit window decoder (16), smaller K (and a
 * manually selected 16-bit decoder) on the 16-bit decoders after widening (convert_8_to_16).  Input layout
 * as srsran_tdec_run_all: sub-block (3 (K + 32) + 12) unless srsran_tdec_force_not_sb or K <= 400. */
void srsran_tdec_iteration_8bit(srsran_tdec_t* h, int8_t* input, uint8_t* output);
int  srsran_tdec_run_all_8bit(srsran_tdec_t* h, int8_t* input, uint8_t* output, uint32_t nof_iterations, uint32_t long_cb);

/* ---------------- batch extensions (new names; no reference counterpart) -----
 * srsran_tdec_gpu_run_batch_8bit: srsran_tdec_run_all_8bit over nof_cb device-resident int8 code blocks
 * (in_stride bytes apart) on a HIP stream (NULL = the null stream); layout_sb as srsran_tdec_gpu_run_batch;
 * decisions to d_output (nof_cb x K/8 bytes).  Asynchronous. */
int srsran_tdec_gpu_run_batch_8bit(uint32_t      long_cb,
                                   const int8_t* d_input,
                                   uint32_t      in_stride,
                                   int           layout_sb,
                                   uint8_t*      d_output,
                                   uint32_t      nof_cb,
                                   uint32_t      nof_iterations,
                                   void*         stream);
/* ---------------- */

/*
 * Decode nof_cb code blocks of the same size with srsran_tdec_run_all semantics.
 * Host buffers: input = nof_cb blocks in_stride int16 apart (layout as selected on h),
 * output = nof_cb * long_cb/8 bytes.  Synchronous.
 */
int srsran_tdec_run_all_batch(srsran_tdec_t* h,
                              const int16_t* input,
                              uint32_t       in_stride,
                              uint8_t*       output,
                              uint32_t       nof_cb,
                              uint32_t       nof_iterations,
                              uint32_t       long_cb);

/*
 * Device-resident batch: input/output are device pointers, work is enqueued on
 * `stream` (a hipStream_t, NULL = default stream) and the call returns without
 * synchronising.  layout_sb selects the rm_turbo sub-block layout (ignored for
 * K <= 400, which is always natural as in the reference).
 */
int srsran_tdec_gpu_run_batch(uint32_t       long_cb,
                              const int16_t* d_input,
                              uint32_t       in_stride,
                              int            layout_sb,
                              uint8_t*       d_output,
                              uint32_t       nof_cb,
                              uint32_t       nof_iterations,
                              void*          stream);

/*
 * Device-resident multi-size batch: nof_groups groups, group g = nof_cb[g] code
 * blocks of size long_cb[g] at d_input[g] (in_stride[g] int16 apart) -> d_output[g].
 * Groups are decoded concurrently on internal streams that fork from and join
 * back into `stream` (no host synchronisation).  This is the shape of a DL-SCH
 * transport block (K+ / K- code blocks, cbsegm.c:62-117) and of many TBs at once.
 */
int srsran_tdec_gpu_run_multi(uint32_t              nof_groups,
                              const uint32_t*       long_cb,
                              const int16_t* const* d_input,
                              const uint32_t*       in_stride,
                              int                   layout_sb,
                              uint8_t* const*       d_output,
                              const uint32_t*       nof_cb,
                              uint32_t              nof_iterations,
                              void*                 stream);

/* 1 if a HIP device is usable, 0 otherwise (no kernel is launched). */
int srsran_tdec_gpu_available(void);

/* Name of the decoder kernel used for long_cb (for profiling reports), or NULL. */
const char* srsran_tdec_gpu_kernel_name(uint32_t long_cb);

/* Name of the kernel a batch of nof_cb blocks of long_cb on the SB layout runs under the current
   thresholds below, for profiling reports. */
const char* srsran_tdec_gpu_kernel_name_batch(uint32_t long_cb, uint32_t nof_cb);

/* Name of the last turbo-decoder kernel the calling thread launched (any API: plain, multi-size,
   DL-SCH / UL-SCH batches), "" before the first, as rocprofv3 reports it. */
const char* srsran_tdec_gpu_last_kernel(void);

/* Blocks per launch (or per fused class launch) from which the 16-sub-block class runs the lane-pair
   decoder (default 512: below it the quad decoder fills the chip better).  Process-wide. */
void     srsran_tdec_gpu_set_pair_threshold(uint32_t nof_cb);
uint32_t srsran_tdec_gpu_get_pair_threshold(void);
/* Blocks per launch (or per fused class launch) from which a decoder class runs its single-lane decoder
   (one lane per sub-block / block, 64 lanes a wave: the throughput mapping) instead of the lane pair /
   quad decoder.  nof_subblocks: 16 (default 1024), 8 (default 4096) or 0 = the generic class K <= 400
   (default UINT32_MAX, i.e. never: its quad decoder is faster at every batch size measured).
   Process-wide. */
void     srsran_tdec_gpu_set_class_single_threshold(uint32_t nof_subblocks, uint32_t nof_cb);
uint32_t srsran_tdec_gpu_get_class_single_threshold(uint32_t nof_subblocks);
/* Shorthands: the 16- and 8-sub-block classes together (get: the 16 class), the generic class. */
void     srsran_tdec_gpu_set_single_threshold(uint32_t nof_cb);
uint32_t srsran_tdec_gpu_get_single_threshold(void);
void     srsran_tdec_gpu_set_generic_single_threshold(uint32_t nof_cb);
/* Single-lane launches whose block sizes are all <= k run the build with 8-step windows (fewer
   registers: two or three waves per SIMD where LDS allows; twice the checkpoints in LDS).  Process-wide. */
void     srsran_tdec_gpu_set_w8_max_k(uint32_t k);
uint32_t srsran_tdec_gpu_get_w8_max_k(void);
/* In a fused multi-size launch (srsran_tdec_gpu_run_multi) of the 16-sub-block single-lane class, the
   sizes up to k (at least the w8_max_k above) form their own launch on the 8-step-window build
   (default 1536; 0 = no cut beyond w8_max_k).  Process-wide. */
void     srsran_tdec_gpu_set_w8_fused_max_k(uint32_t k);
uint32_t srsran_tdec_gpu_get_w8_fused_max_k(void);
uint32_t srsran_tdec_gpu_get_generic_single_threshold(void);

#ifdef __cplusplus
}
#endif
#endif /* SRSRAN_AMD_TDEC_H */
