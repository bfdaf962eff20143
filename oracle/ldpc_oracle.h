/* oracle/ldpc_oracle.h -- CPU restatement of the NR LDPC decoder / encoder (test infrastructure only). */
#ifndef ORACLE_LDPC_H
#define ORACLE_LDPC_H
#include <stdint.h>

/* scaling arithmetic of the check-to-variable magnitudes */
#define ORACLE_LDPC_SCALE_C 0    /* m * (int)(s * 100) / 100        (ldpc_dec_c.c:149, 232; ldpc_dec_s.c) */
#define ORACLE_LDPC_SCALE_SIMD 1 /* (m * (uint16)((s + 2^-16) * 65535)) >> 16  (ldpc_dec_c_avx2.c:148, 520-531) */

int oracle_ldpc_ls_index(int ls);
int oracle_ldpc_pcm(int bg, int ls, uint16_t* pcm, int8_t* positions);
int oracle_ldpc_encode(int bg, int ls, const uint8_t* msg, uint8_t* cw);
int oracle_ldpc_decode_c(int            bg,
                         int            ls,
                         int            scale_mode,
                         float          scaling_fctr,
                         int            max_iter,
                         const int8_t*  llrs,
                         uint32_t       cdwd_rm_length,
                         uint32_t       crc_poly,
                         int            crc_order,
                         uint8_t*       message);
int oracle_ldpc_decode_s(int            bg,
                         int            ls,
                         float          scaling_fctr,
                         int            max_iter,
                         const int16_t* llrs,
                         uint32_t       cdwd_rm_length,
                         uint32_t       crc_poly,
                         int            crc_order,
                         uint8_t*       message);
#endif
