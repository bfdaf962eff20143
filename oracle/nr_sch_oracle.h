/* oracle/nr_sch_oracle.h -- CPU restatement of the NR SCH receive path (test infrastructure only). */
#ifndef ORACLE_NR_SCH_H
#define ORACLE_NR_SCH_H
#include <stdint.h>

typedef struct {
  uint32_t tbs, L_tb, L_cb, C, K, Z;
} oracle_nr_cbsegm_t;

typedef struct {
  int      bg;
  uint32_t Qm, G, A, L_tb, L_cb, B, Bp, Kp, Kr, F, Nref, Z, Nl, C;
} oracle_nr_tb_info_t;

int      oracle_nr_cbsegm(int bg, uint32_t tbs, oracle_nr_cbsegm_t* s);
int      oracle_nr_select_bg(uint32_t tbs, double R);
uint32_t oracle_nr_Nref(uint32_t nof_prb, int mcs_table_256qam, uint32_t max_mimo_layers);
int      oracle_nr_tb_info(uint32_t tbs, double R, uint32_t Qm, uint32_t G, uint32_t Nl, int lbrm, uint32_t nof_prb,
                           int mcs_table_256qam, oracle_nr_tb_info_t* t);
uint32_t oracle_nr_E(const oracle_nr_tb_info_t* t, uint32_t j);
int      oracle_ldpc_rm_rx_c(const int8_t* in, int8_t* out, uint32_t E, uint32_t F, int bg, uint32_t ls, uint32_t rv,
                             uint32_t Qm, uint32_t Nref);
int      oracle_nr_sch_decode(const oracle_nr_tb_info_t* t, uint32_t rv, const int8_t* e_bits, float scaling,
                              int max_iter, int8_t* softbuf, uint32_t softbuf_stride, uint8_t* cb_crc, uint8_t* cb_data,
                              uint32_t cb_data_stride, uint8_t* payload, int* tb_crc, float* avg_iter);
#endif
