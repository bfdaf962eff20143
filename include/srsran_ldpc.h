/*
 * include/srsran_ldpc.h -- drop-in C API of the MI355X NR LDPC decoder.
 *
 * Replaces the reference interfaces (srsRAN_4G, paths relative to /root/reference/lib):
 *   include/srsran/phy/fec/ldpc/base_graph.h:38-113    srsran_basegraph_t, create_compact_pcm, BG sizes
 *   include/srsran/phy/fec/ldpc/ldpc_decoder.h:37-180  srsran_ldpc_decoder_{type_t,args_t,t},
 *                                                      srsran_ldpc_decoder_{init,free,decode_f,decode_s,
 *                                                      decode_c,decode_crc_c}
 * Same names, argument meaning and return values (ldpc_decoder.c:44-95, 552-685): decode_c returns
 * max_nof_iter, decode_crc_c the number of iterations run until the CRC matched or 0 when it never
 * did, and -1 on error.  The decoding runs on the GPU through HIP; the host-side calls are
 * synchronous like the reference.
 *
 * Arithmetic: bit-identical to the reference's 8-bit layered decoders --
 *   SRSRAN_LDPC_DECODER_C                           ldpc_dec_c.c   (c2v scaling m * (int)(100 s) / 100)
 *   SRSRAN_LDPC_DECODER_C_AVX2, SRSRAN_LDPC_DECODER_C_AVX512
 *                                                   ldpc_dec_c_avx2*.c / _avx512*.c
 *                                                   (scaling (m * (uint16)((s + 2^-16) 65535)) >> 16)
 *   SRSRAN_LDPC_DECODER_S                           ldpc_dec_s.c   (16-bit LLRs, 15-bit messages, decode_s)
 * Not provided on the GPU (init returns SRSRAN_ERROR): the float (F) decoder and the flooded
 * schedules (*_FLOOD), neither of which srsRAN selects by default (sch_nr.c:290-300).
 *
 * Added: srsran_ldpc_decoder_gpu_decode_batch(), an asynchronous batch entry point over device
 * buffers on the caller's HIP stream.
 */
#ifndef SRSRAN_AMD_LDPC_H
#define SRSRAN_AMD_LDPC_H

#include <stdbool.h>
#include <stdint.h>

#include "srsran_sch.h" /* srsran_crc_t */

#ifdef __cplusplus
extern "C" {
#endif

/* base_graph.h:44-67 */
#define SRSRAN_LDPC_BG1_MAX_LEN_CB 8448
#define SRSRAN_LDPC_BG2_MAX_LEN_CB 3840
#define SRSRAN_LDPC_MAX_LEN_CB SRSRAN_LDPC_BG1_MAX_LEN_CB
#define BG1Nfull 68
#define BG1N 66
#define BG1M 46
#define BG1K 22
#define BG2Nfull 52
#define BG2N 50
#define BG2M 42
#define BG2K 10
#define MAX_CNCT 20
#define NOF_LIFTSIZE 8
#define MAX_LIFTSIZE 384
#define VOID_LIFTSIZE 255
#define NO_CNCT 0xFFFF

/* base_graph.h:70-73 */
typedef enum {
  BG1 = 0,
  BG2,
} srsran_basegraph_t;

/* base_graph.h:96: compact PCM (shift mod ls, NO_CNCT where unconnected) and per-row column lists */
int create_compact_pcm(uint16_t* pcm, int8_t (*positions)[MAX_CNCT], srsran_basegraph_t bg, uint16_t ls);

/* ldpc_decoder.h:38-50 */
typedef enum {
  SRSRAN_LDPC_DECODER_F = 0,
  SRSRAN_LDPC_DECODER_S,
  SRSRAN_LDPC_DECODER_C,
  SRSRAN_LDPC_DECODER_C_FLOOD,
  SRSRAN_LDPC_DECODER_C_AVX2,
  SRSRAN_LDPC_DECODER_C_AVX2_FLOOD,
  SRSRAN_LDPC_DECODER_C_AVX512,
  SRSRAN_LDPC_DECODER_C_AVX512_FLOOD,
} srsran_ldpc_decoder_type_t;

/* ldpc_decoder.h:55-61 */
typedef struct {
  srsran_ldpc_decoder_type_t type;
  srsran_basegraph_t         bg;
  uint16_t                   ls;
  float                      scaling_fctr;
  uint32_t                   max_nof_iter; /* 0 -> 10 (ldpc_decoder.c:42) */
} srsran_ldpc_decoder_args_t;

/* ldpc_decoder.h:66-100: same fields; `ptr` holds the GPU context (stream, device tables). */
typedef struct {
  void*              ptr;
  srsran_basegraph_t bg;
  uint16_t           ls;
  uint32_t           max_nof_iter;
  uint8_t            bgN;
  uint16_t           liftN;
  uint8_t            bgM;
  uint16_t           liftM;
  uint8_t            bgK;
  uint16_t           liftK;
  uint16_t*          pcm;
  int8_t (*var_indices)[MAX_CNCT];
  float scaling_fctr;
  void (*free)(void*);
  int (*decode_f)(void*, const float*, uint8_t*, uint32_t, srsran_crc_t*);
  int (*decode_s)(void*, const int16_t*, uint8_t*, uint32_t, srsran_crc_t*);
  int (*decode_c)(void*, const int8_t*, uint8_t*, uint32_t, srsran_crc_t*);
} srsran_ldpc_decoder_t;

int  srsran_ldpc_decoder_init(srsran_ldpc_decoder_t* q, const srsran_ldpc_decoder_args_t* args); /* ldpc_decoder.c:552 */
void srsran_ldpc_decoder_free(srsran_ldpc_decoder_t* q);                                          /* ldpc_decoder.c:650 */
int  srsran_ldpc_decoder_decode_f(srsran_ldpc_decoder_t* q, const float* llrs, uint8_t* message, uint32_t cdwd_rm_length);
int  srsran_ldpc_decoder_decode_s(srsran_ldpc_decoder_t* q, const int16_t* llrs, uint8_t* message, uint32_t cdwd_rm_length);
int  srsran_ldpc_decoder_decode_c(srsran_ldpc_decoder_t* q, const int8_t* llrs, uint8_t* message, uint32_t cdwd_rm_length);
int  srsran_ldpc_decoder_decode_crc_c(srsran_ldpc_decoder_t* q,
                                      const int8_t*          llrs,
                                      uint8_t*               message,
                                      uint32_t               cdwd_rm_length,
                                      srsran_crc_t*          crc);

/*
 * Added batch entry point (asynchronous on `stream`, a hipStream_t; NULL = default stream).
 *   d_llrs     nof_cw x (liftN - 2 ls) int8 LLRs, llr_stride bytes apart (device)
 *   d_message  nof_cw x liftK bytes (one bit per byte, as decode_c) or, packed != 0, liftK / 8
 *              MSB-first bytes (liftK % 8 == 0), message_stride bytes apart (device)
 *   crc        NULL: run max_nof_iter iterations; else CRC early stop per codeword (decode_crc_c)
 *   d_ret      optional nof_cw bytes: the value decode_crc_c / decode_c would return (device)
 */
int srsran_ldpc_decoder_gpu_decode_batch(srsran_ldpc_decoder_t* q,
                                         const int8_t*          d_llrs,
                                         uint32_t               llr_stride,
                                         uint32_t               nof_cw,
                                         uint32_t               cdwd_rm_length,
                                         const srsran_crc_t*    crc,
                                         uint8_t*               d_message,
                                         uint32_t               message_stride,
                                         int                    packed,
                                         uint8_t*               d_ret,
                                         void*                  stream);

/* Same for a SRSRAN_LDPC_DECODER_S decoder: int16 LLRs, llr_stride in int16 elements. */
int srsran_ldpc_decoder_gpu_decode_batch_s(srsran_ldpc_decoder_t* q,
                                           const int16_t*         d_llrs,
                                           uint32_t               llr_stride,
                                           uint32_t               nof_cw,
                                           uint32_t               cdwd_rm_length,
                                           const srsran_crc_t*    crc,
                                           uint8_t*               d_message,
                                           uint32_t               message_stride,
                                           int                    packed,
                                           uint8_t*               d_ret,
                                           void*                  stream);

#ifdef __cplusplus
}
#endif
#endif
