/* oracle/tdec_oracle.h -- CPU restatement of the srsRAN turbo decoder (test infrastructure only). */
#ifndef ORACLE_TDEC_H
#define ORACLE_TDEC_H
#include <stdint.h>

int      oracle_cb_index(uint32_t K);
uint32_t oracle_cb_size(int idx);
uint32_t oracle_nof_subblocks(uint32_t K);
int      oracle_qpp(uint32_t K, uint16_t* fwd, uint16_t* rev);

/* Decode one CB: nof_iterations half-iterations, hard decision MSB-first (K/8 bytes).
 * trace (optional, nof_iterations*K int16): decoder output after each half-iteration,
 * natural order (dec2 output is de-interleaved, i.e. app1). */
int oracle_tdec_run(uint32_t K, const int16_t* input, int layout_sb, uint32_t nof_iterations, uint8_t* output, int16_t* trace);
int oracle_tdec_run_batch(uint32_t K,
                          const int16_t* input,
                          uint32_t       in_stride,
                          int            layout_sb,
                          uint32_t       nof_iterations,
                          uint8_t*       output,
                          uint32_t       nof_cb);

uint32_t oracle_nof_subblocks_8bit(uint32_t K);
/* 8-bit window decoder (nsb 16 / 32 classes), SB layout input; trace: nof_iterations * K int8, natural order */
int oracle_tdec8_run(uint32_t K, const int8_t* in, uint32_t nof_iterations, uint8_t* output, int8_t* trace);

int oracle_tcod_encode(uint32_t K, const uint8_t* bits, uint8_t* out);
int oracle_natural_to_sb(uint32_t K, const int16_t* in, int16_t* out);
#endif
