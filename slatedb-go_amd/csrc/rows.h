// v0 row decode against a decoded block held in LDS or memory (row.go:191-261), shared by the
// wave-per-block decoder (decode.hip) and the parse/materialize decoder (decode_lpb3.hip).
#pragma once
#include "common.h"

namespace slate {

// ---------------------------------------------------------------- v0 rows
// row.go:191-261 against firstKey of length fk (fk < 0: firstKey == nil).
__device__ inline void decode_row(const uint8_t* data, uint32_t data_len, uint32_t off, int fk, slate_row& r,
                                  uint32_t* suffix_len_out) {
  r.row_off = off;
  r.key_prefix_len = 0;
  r.key_suffix_len = 0;
  r.value_len = 0;
  r.flags = 0;
  r.meta_len = 0;
  const uint8_t* p = data + off;
  uint32_t n = data_len - off;
  *suffix_len_out = 0;
  if (n >= 4) {
    r.key_prefix_len = ld_be16(p);
    r.key_suffix_len = ld_be16(p + 2);
  }
  if (n < 13) { r.status = SLATE_E_ROW_TOO_SHORT; return; }
  uint16_t pl = r.key_prefix_len, sl = r.key_suffix_len;
  if (pl > uint16_t(fk < 0 ? 0 : fk)) { r.status = SLATE_E_ROW_PREFIX; return; }
  uint32_t o = 4;
  if (n - o < sl) { r.status = SLATE_E_ROW_SUFFIX; return; }
  o += sl;
  if (n - o < 9) { r.status = SLATE_E_ROW_PANIC; return; }
  uint8_t flags = p[o + 8];
  o += 9;
  if (flags & 2) {
    if (n - o < 8) { r.status = SLATE_E_ROW_EXPIRE; return; }
    o += 8;
  }
  if (flags & 4) {
    if (n - o < 8) { r.status = SLATE_E_ROW_CREATE; return; }
    o += 8;
  }
  if ((flags & 1) == 0) {
    if (n - o < 4) { r.status = SLATE_E_ROW_VALUE_LEN; return; }
    uint32_t vl = ld_be32(p + o);
    o += 4;
    if (n - o < vl) { r.status = SLATE_E_ROW_VALUE; return; }
    r.value_len = vl;
  }
  r.flags = flags & 7;
  r.meta_len = uint8_t(o - 4 - sl);
  r.status = SLATE_OK;
  *suffix_len_out = sl;
}

}  // namespace slate
