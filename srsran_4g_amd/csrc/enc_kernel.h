// srsran_4g_amd/csrc/enc_kernel.h -- launch interface of the DL-SCH transmit kernels (sch.c:240-359:
// TB CRC, code block CRC, turbo encoding (turbocoder.c), rate matching (rm_turbo.c:345-388)).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsran_amd {

struct EncTb {
  const uint8_t* data;     // payload, tbs / 8 bytes (device)
  uint32_t*      crc;      // out: TB CRC24A (device)
  uint8_t*       e_bits;   // unpacked e bits of the TB (device scratch), nof_e_bits
  uint8_t*       packed;   // out: packed e bits, MSB first (device)
  uint32_t       nbytes;   // tbs / 8
  uint32_t       nof_e_bits;
};

struct EncCb {
  const uint8_t*  data;    // the TB payload (device)
  const uint32_t* tb_crc;  // its TB CRC24A (device)
  uint8_t*        e;       // first unpacked e bit of this code block
  const uint16_t* fwd;     // rate-matching read-out table (rm_fwd_table), period N
  uint32_t        tb_bytes;
  uint32_t        rp;      // first bit of the code block in (payload || TB CRC)
  uint32_t        rlen;    // bits taken from there (K - 24 with a CB CRC, else K)
  uint32_t        K, f1, f2, N, E;
  uint32_t        cb_crc;  // 1: CRC24B appended (C > 1)
};

// TB CRC24A of every TB: one wave per TB
hipError_t enc_tb_crc_launch(const EncTb* d_tbs, uint32_t ntb, hipStream_t stream);
// every code block: CRC24B, turbo encoding, rate matching into the TB's unpacked e bits
hipError_t enc_cb_launch(const EncCb* d_cbs, uint32_t ncb, hipStream_t stream);
// unpacked -> packed e bits, per TB; max_bytes = largest ceil(nof_e_bits / 8)
hipError_t enc_pack_launch(const EncTb* d_tbs, uint32_t ntb, uint32_t max_bytes, hipStream_t stream);

constexpr uint8_t kTxNull = 100;  // SRSRAN_TX_NULL (turbocoder.h:40-42): a filler bit

// srsran_tcod_encode of one code block: K unpacked bits (device) -> 3 K + 12 unpacked bits (device)
hipError_t tcod_launch(const uint8_t* d_in, uint8_t* d_out, uint32_t K, uint32_t f1, uint32_t f2, hipStream_t stream);

// srsran_rm_turbo_tx_lut of one code block (device buffers; tables from tx_api.cpp)
struct RmTxLut {
  const uint8_t*  sys;     // packed systematic stream, K + 4 bits (rv 0)
  const uint8_t*  par;     // packed parity streams, 2 (K + 4) bits (rv 0)
  const uint16_t* tsys;    // w bit i <- sys bit tsys[i], i < K + 4
  const uint16_t* tpar;    // w bit K + 4 + i <- par bit tpar[i], i < 2 (K + 4)
  uint8_t*        w_buff;  // the circular buffer, 3 K + 12 bits packed (written for rv 0, read otherwise)
  uint8_t*        output;  // packed output
  uint32_t        K, rv, r_ptr, out_len, w_offset, zero_tail;
};
hipError_t rm_tx_lut_launch(const RmTxLut& a, hipStream_t stream);

}  // namespace srsran_amd
