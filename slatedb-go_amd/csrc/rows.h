// v0 row decode against a decoded block held in LDS or memory (row.go:191-261), shared by the
// wave-per-block decoder (decode.hip) and the parse/materialize decoder (decode_lpb3.hip).
#pragma once
#include "common.h"
#include "kernels.h"

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


__device__ inline void write_meta(slate_block_meta* m, const slate_block_meta& v, int lane) {
  if (lane == 0) *m = v;
}

// block.Decode's structure checks (block.go:95-131) and the row descriptors of a decoded block
// held in LDS (buf, n bytes), then block b's meta; one wave.  Shared by the wave-per-block
// decoder (decode.hip) and the CodecZstd fast path (zstd_fast.hip).
__device__ inline void block_finish(const DecodeArgs& a, uint32_t b, const uint8_t* buf, uint32_t n, int lane,
                                    slate_block_meta m) {
  if (n < 2) {
    m.status = SLATE_E_BLOCK_UNCOMP_SMALL;
    write_meta(&a.meta[b], m, lane);
    return;
  }
  uint32_t cnt = ld_be16(buf + n - 2);
  int64_t osi = int64_t(n) - 2 - 2 * int64_t(cnt);
  if (osi <= 0) {
    m.status = SLATE_E_BLOCK_INDEX_OFFSET;
    m.detail = int32_t(osi);
    write_meta(&a.meta[b], m, lane);
    return;
  }
  uint16_t osi16 = uint16_t(osi);
  uint32_t bad = 0xFFFFFFFFu;  // first offset index exceeding uint16(offsetStartIndex)
  for (uint32_t i = lane; i < cnt; i += kWave) {
    if (ld_be16(buf + osi + 2 * i) > osi16 && i < bad) bad = i;
  }
  for (int o = 32; o >= 1; o >>= 1) bad = min(bad, uint32_t(__shfl_xor(int(bad), o, 64)));
  if (bad != 0xFFFFFFFFu) {
    m.status = SLATE_E_BLOCK_OFFSET_BOUNDS;
    m.aux = uint16_t(bad);
    m.detail = ld_be16(buf + osi + 2 * bad);
    write_meta(&a.meta[b], m, lane);
    return;
  }
  m.data_len = uint32_t(osi);
  m.n_rows = uint16_t(cnt);
  if (cnt == 0) {
    m.status = SLATE_E_BLOCK_NO_OFFSETS;
    write_meta(&a.meta[b], m, lane);
    return;
  }
  // FirstKey quirk (block.go:130-131): uint16 arithmetic, panics out of range
  {
    uint32_t off0 = ld_be16(buf + osi);
    if (uint64_t(osi) - off0 < 2) {
      m.status = SLATE_E_BLOCK_FIRSTKEY_PANIC;
      write_meta(&a.meta[b], m, lane);
      return;
    }
    uint16_t kl = ld_be16(buf + off0);
    uint16_t lo = uint16_t(off0 + 2), hi = uint16_t(off0 + 2 + kl);
    if (lo > hi || hi > n) {
      m.status = SLATE_E_BLOCK_FIRSTKEY_PANIC;
      write_meta(&a.meta[b], m, lane);
      return;
    }
    m.aux = kl;
  }
  // ---- row descriptors
  uint64_t rb = a.row_base[b];
  uint32_t rcap = uint32_t(min(uint64_t(0xFFFFFFFFu), a.row_base[b + 1] - rb));
  uint32_t nr = cnt;
  if (nr > rcap) {
    nr = rcap;
    m.flags |= SLATE_BLKF_ROWS_TRUNCATED;
  }
  int fk = -1;
  {
    slate_row r0;
    uint32_t sl0;
    decode_row(buf, uint32_t(osi), ld_be16(buf + osi), -1, r0, &sl0);
    if (r0.status == SLATE_OK) fk = int(sl0);
  }
  slate_row* grows = a.rows + rb;
  if (dbg_bits(a) & 4) nr = 0;
  for (uint32_t i = lane; i < nr; i += kWave) {
    slate_row r;
    uint32_t sl;
    decode_row(buf, uint32_t(osi), ld_be16(buf + osi + 2 * i), i == 0 ? -1 : fk, r, &sl);
    grows[i] = r;
  }
  write_meta(&a.meta[b], m, lane);
}

}  // namespace slate
