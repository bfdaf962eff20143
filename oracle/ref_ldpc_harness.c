/*
 * oracle/ref_ldpc_harness.c -- drives the reference NR LDPC decoder / encoder compiled from
 * /root/reference (TEST INFRASTRUCTURE ONLY; built into oracle/_ref/ by oracle/Makefile).
 *
 * The reference sources lib/src/phy/fec/ldpc/{ldpc_decoder.c, ldpc_dec_*.c, ldpc_encoder.c,
 * ldpc_enc_*.c, base_graph.c} compile as they are; this file only gives ctypes a flat entry
 * point (init -> decode -> free) so the tests never mirror the reference's structs.
 */
#include <stdint.h>
#include <string.h>

#include "srsran/phy/fec/crc.h"
#include "srsran/phy/fec/ldpc/ldpc_decoder.h"
#include "srsran/phy/fec/ldpc/ldpc_encoder.h"

/* type: srsran_ldpc_decoder_type_t; llr_bits 8 / 16; crc_order 0 = no early stop */
int ref_ldpc_decode(int         type,
                    int         bg,
                    int         ls,
                    float       scaling_fctr,
                    int         max_iter,
                    const void* llrs,
                    int         llr_bits,
                    uint32_t    cdwd_rm_length,
                    uint32_t    crc_poly,
                    int         crc_order,
                    uint8_t*    message)
{
  srsran_ldpc_decoder_args_t args = {};
  args.type                       = (srsran_ldpc_decoder_type_t)type;
  args.bg                         = (srsran_basegraph_t)bg;
  args.ls                         = (uint16_t)ls;
  args.scaling_fctr               = scaling_fctr;
  args.max_nof_iter               = (uint32_t)max_iter;
  srsran_ldpc_decoder_t q;
  if (srsran_ldpc_decoder_init(&q, &args) != 0) {
    return -100;
  }
  srsran_crc_t crc;
  memset(&crc, 0, sizeof(crc));
  if (crc_order > 0 && srsran_crc_init(&crc, crc_poly, crc_order) != 0) {
    srsran_ldpc_decoder_free(&q);
    return -101;
  }
  int r;
  if (llr_bits == 16) {
    r = srsran_ldpc_decoder_decode_s(&q, (const int16_t*)llrs, message, cdwd_rm_length);
  } else if (crc_order > 0) {
    r = srsran_ldpc_decoder_decode_crc_c(&q, (const int8_t*)llrs, message, cdwd_rm_length, &crc);
  } else {
    r = srsran_ldpc_decoder_decode_c(&q, (const int8_t*)llrs, message, cdwd_rm_length);
  }
  srsran_ldpc_decoder_free(&q);
  return r;
}

/* output = codeword without the 2*ls punctured bits (liftN - 2*ls bits) */
int ref_ldpc_encode(int bg, int ls, const uint8_t* msg, uint8_t* cw)
{
  srsran_ldpc_encoder_t q;
  if (srsran_ldpc_encoder_init(&q, SRSRAN_LDPC_ENCODER_C, (srsran_basegraph_t)bg, (uint16_t)ls) != 0) {
    return -100;
  }
  const int r = srsran_ldpc_encoder_encode(&q, msg, cw, q.liftK);
  srsran_ldpc_encoder_free(&q);
  return r;
}

/* n codewords (llr_stride bytes apart) through one decoder object, as a CPU throughput sample */
int ref_ldpc_decode_many(int type, int bg, int ls, float scaling_fctr, int max_iter, const int8_t* llrs,
                         uint32_t llr_stride, int n, uint8_t* messages)
{
  srsran_ldpc_decoder_args_t args = {};
  args.type                       = (srsran_ldpc_decoder_type_t)type;
  args.bg                         = (srsran_basegraph_t)bg;
  args.ls                         = (uint16_t)ls;
  args.scaling_fctr               = scaling_fctr;
  args.max_nof_iter               = (uint32_t)max_iter;
  srsran_ldpc_decoder_t q;
  if (srsran_ldpc_decoder_init(&q, &args) != 0) {
    return -100;
  }
  const uint32_t len = q.liftN - 2 * q.ls;
  for (int i = 0; i < n; i++) {
    srsran_ldpc_decoder_decode_c(&q, llrs + (size_t)i * llr_stride, messages + (size_t)i * q.liftK, len);
  }
  srsran_ldpc_decoder_free(&q);
  return 0;
}
