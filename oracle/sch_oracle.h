/* oracle/sch_oracle.h -- CPU restatement of the DL-SCH receive pieces (test infrastructure only). */
#ifndef ORACLE_SCH_H
#define ORACLE_SCH_H
#include <stdint.h>

typedef struct {
  uint32_t F, C, K1, K2, K1_idx, K2_idx, C1, C2, tbs;
} oracle_cbsegm_t;

void     oracle_crc_table(uint32_t poly, int order, uint32_t table[256]);
uint32_t oracle_crc_checksum_byte(uint32_t poly, int order, const uint8_t* data, uint32_t nbits);
uint32_t oracle_crc_bits(uint32_t poly, int order, const uint8_t* bits, uint32_t nbits);
int      oracle_cbsegm(uint32_t tbs, oracle_cbsegm_t* s);
int      oracle_rm_rx_table(uint32_t K, uint32_t rv, int layout_sb, uint16_t* table);
int      oracle_rm_turbo_rx(uint32_t K, uint32_t rv, int layout_sb, const int16_t* in, uint32_t E, int16_t* softbuf);
int      oracle_rm_turbo_tx(uint32_t K, uint32_t rv, const uint8_t* coded, uint32_t E, uint8_t* out);
int      oracle_dlsch_decode_tb(uint32_t       tbs,
                                uint32_t       Qm,
                                uint32_t       rv,
                                uint32_t       nof_e_bits,
                                const int16_t* e_bits,
                                uint32_t       max_iterations,
                                int16_t*       softbuf,
                                uint32_t       softbuf_stride,
                                uint8_t*       cb_crc,
                                uint8_t*       cb_data,
                                uint32_t       cb_data_stride,
                                uint8_t*       data,
                                uint32_t*      cb_noi_out,
                                float*         avg_iterations);
int      oracle_dlsch_decode_tb8(uint32_t tbs, uint32_t Qm, uint32_t rv, uint32_t nof_e_bits, const int8_t* e_bits,
                                 uint32_t max_iterations, int16_t* softbuf, uint32_t softbuf_stride, uint8_t* cb_crc,
                                 uint8_t* cb_data, uint32_t cb_data_stride, uint8_t* data, uint32_t* cb_noi_out,
                                 float* avg_iterations);
int      oracle_dlsch_encode_tb(uint32_t tbs, uint32_t Qm, uint32_t rv, uint32_t nof_e_bits, const uint8_t* tb_bytes,
                                uint8_t* e_bits);
int      oracle_dlsch_encode_tb_x(uint32_t tbs, uint32_t Qm, uint32_t rv, uint32_t nof_e_bits, const uint8_t* tb_bytes,
                                  uint8_t* e_bits, uint32_t tb_crc_xor);
#endif
