#include "flatbuf.h"

#include <cstring>

#include "common.h"

namespace slate {

// Host CRC for the ~80-byte info footer (flatbuf.go:62-124 framing); block and filter CRCs run
// on the GPU, the CodecNone index's on the host (crc32_host16).
static const CrcTables kHostCrc = CrcTables();
uint32_t crc32_host(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) c = kHostCrc.t[0][(c ^ p[i]) & 0xff] ^ (c >> 8);
  return ~c;
}

// Slicing-by-16 on the host, for the CodecNone index's CRC (~12 MB at configs[2]), taken on the
// builder's index thread beside the blocks' copy-back instead of through the GPU after it.
namespace {
struct HostCrc16 {
  uint32_t t[16][256];
  HostCrc16() {
    for (uint32_t i = 0; i < 256; i++) t[0][i] = kHostCrc.t[0][i];
    for (uint32_t i = 0; i < 256; i++)
      for (int s = 1; s < 16; s++) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};
const HostCrc16 kHost16;
}  // namespace
uint32_t crc32_host16(const uint8_t* p, size_t n) {
  const auto& t = kHost16.t;
  uint32_t c = 0xFFFFFFFFu;
  for (; n >= 16; p += 16, n -= 16) {
    uint32_t w[4];
    memcpy(w, p, 16);  // (little-endian host)
    const uint32_t x = c ^ w[0];
    c = t[15][x & 0xff] ^ t[14][(x >> 8) & 0xff] ^ t[13][(x >> 16) & 0xff] ^ t[12][x >> 24] ^
        t[11][w[1] & 0xff] ^ t[10][(w[1] >> 8) & 0xff] ^ t[9][(w[1] >> 16) & 0xff] ^ t[8][w[1] >> 24] ^
        t[7][w[2] & 0xff] ^ t[6][(w[2] >> 8) & 0xff] ^ t[5][(w[2] >> 16) & 0xff] ^ t[4][w[2] >> 24] ^
        t[3][w[3] & 0xff] ^ t[2][(w[3] >> 8) & 0xff] ^ t[1][(w[3] >> 16) & 0xff] ^ t[0][w[3] >> 24];
  }
  for (; n; p++, n--) c = t[0][(c ^ *p) & 0xff] ^ (c >> 8);
  return ~c;
}

FbBuilder::FbBuilder(size_t reserve) : buf_(reserve), head_(reserve) {}

void FbBuilder::grow() {
  size_t old = buf_.size();
  size_t nl = old ? old * 2 : 1;
  std::vector<uint8_t> nb(nl);
  if (old) memcpy(nb.data() + (nl - old), buf_.data(), old);
  buf_.swap(nb);
  head_ += nl - old;
}

// builder.go Prep: pad so that `size` is aligned after `additional` bytes.
void FbBuilder::prep(int size, int additional) {
  if (size > minalign_) minalign_ = size;
  size_t used = buf_.size() - head_;
  int align = int((~(used + size_t(additional))) + 1) & (size - 1);
  while (long(head_) <= long(align + size + additional)) grow();
  for (int i = 0; i < align; i++) place_byte(0);
}

void FbBuilder::place_u32(uint32_t v) {
  head_ -= 4;
  for (int i = 0; i < 4; i++) buf_[head_ + i] = uint8_t(v >> (8 * i));
}

void FbBuilder::prepend_u64(uint64_t v) {
  prep(8, 0);
  head_ -= 8;
  for (int i = 0; i < 8; i++) buf_[head_ + i] = uint8_t(v >> (8 * i));
}

void FbBuilder::prepend_i8(int8_t v) {
  prep(1, 0);
  place_byte(uint8_t(v));
}

void FbBuilder::prepend_u16(uint16_t v) {
  prep(2, 0);
  head_ -= 2;
  buf_[head_] = uint8_t(v);
  buf_[head_ + 1] = uint8_t(v >> 8);
}

void FbBuilder::prepend_uoffset(uint32_t off) {
  prep(4, 0);
  place_u32(offset() - off + 4);
}

void FbBuilder::prepend_soffset(int32_t off) {
  prep(4, 0);
  place_u32(uint32_t(int32_t(offset()) - off + 4));
}

void FbBuilder::start_object(int numfields) {
  vtable_.assign(size_t(numfields), 0);
  object_end_ = offset();
}

// builder.go WriteVtable: trailing-zero trim, newest-first dedup comparing field
// entries only (both-zero entries match), else write the vtable.
uint32_t FbBuilder::end_object() {
  prepend_soffset(0);
  uint32_t obj = offset();
  while (!vtable_.empty() && vtable_.back() == 0) vtable_.pop_back();
  uint32_t existing = 0;
  for (size_t k = vtables_.size(); k-- > 0;) {
    uint32_t vt2off = vtables_[k];
    size_t start = buf_.size() - vt2off;
    uint16_t vlen = uint16_t(buf_[start] | (buf_[start + 1] << 8));
    size_t nfields = (size_t(vlen) - 4) / 2;
    if (nfields != vtable_.size()) continue;
    bool eq = true;
    for (size_t f = 0; f < nfields && eq; f++) {
      uint16_t x = uint16_t(buf_[start + 4 + 2 * f] | (buf_[start + 5 + 2 * f] << 8));
      if (x == 0 && vtable_[f] == 0) continue;
      if (int32_t(x) != int32_t(obj) - int32_t(vtable_[f])) eq = false;
    }
    if (eq) {
      existing = vt2off;
      break;
    }
  }
  if (existing == 0) {
    for (size_t f = vtable_.size(); f-- > 0;) prepend_u16(uint16_t(vtable_[f] ? obj - vtable_[f] : 0));
    prepend_u16(uint16_t(obj - object_end_));
    prepend_u16(uint16_t((vtable_.size() + 2) * 2));
    size_t obj_start = buf_.size() - obj;
    int32_t v = int32_t(offset()) - int32_t(obj);
    for (int q = 0; q < 4; q++) buf_[obj_start + q] = uint8_t(uint32_t(v) >> (8 * q));
    vtables_.push_back(offset());
  } else {
    head_ = buf_.size() - obj;
    int32_t v = int32_t(existing) - int32_t(obj);
    for (int q = 0; q < 4; q++) buf_[head_ + q] = uint8_t(uint32_t(v) >> (8 * q));
  }
  vtable_.clear();
  return obj;
}

uint32_t FbBuilder::start_vector(int elem, int n, int align) {
  prep(4, elem * n);
  prep(align, elem * n);
  return offset();
}

uint32_t FbBuilder::end_vector(uint32_t n) {
  place_u32(n);
  return offset();
}

uint32_t FbBuilder::create_byte_string(const uint8_t* s, size_t n) {
  prep(4, int(n + 1));
  place_byte(0);
  head_ -= n;
  if (n) memcpy(buf_.data() + head_, s, n);
  return end_vector(uint32_t(n));
}

uint32_t FbBuilder::create_byte_vector(const uint8_t* s, size_t n) {
  prep(4, int(n));
  head_ -= n;
  if (n) memcpy(buf_.data() + head_, s, n);
  return end_vector(uint32_t(n));
}

void FbBuilder::finish(uint32_t root) {
  prep(minalign_, 4);
  prepend_uoffset(root);
}

std::vector<uint8_t> fb_encode_info(const InfoFields& info) {
  FbBuilder b(256 + info.first_key.size());
  uint32_t fk = b.create_byte_vector(info.first_key.data(), info.has_first_key ? info.first_key.size() : 0);
  b.start_object(6);
  if (fk) { b.prepend_uoffset(fk); b.slot(0); }
  if (info.index_offset) { b.prepend_u64(info.index_offset); b.slot(1); }
  if (info.index_len) { b.prepend_u64(info.index_len); b.slot(2); }
  if (info.filter_offset) { b.prepend_u64(info.filter_offset); b.slot(3); }
  if (info.filter_len) { b.prepend_u64(info.filter_len); b.slot(4); }
  if (int8_t(info.codec) != 0) { b.prepend_i8(int8_t(info.codec)); b.slot(5); }
  uint32_t root = b.end_object();
  b.finish(root);
  return std::vector<uint8_t>(b.data(), b.data() + b.size());
}

std::vector<uint8_t> fb_encode_index(const std::vector<uint64_t>& offsets, const std::vector<uint8_t>& keys,
                                     const std::vector<uint64_t>& key_off) {
  const size_t n = offsets.size();
  FbBuilder b(64 + n * 48 + keys.size());
  std::vector<uint32_t> metas(n);
  for (size_t j = 0; j < n; j++) {
    uint32_t fk = b.create_byte_string(keys.data() + key_off[j], key_off[j + 1] - key_off[j]);
    b.start_object(2);
    if (offsets[j]) { b.prepend_u64(offsets[j]); b.slot(0); }
    if (fk) { b.prepend_uoffset(fk); b.slot(1); }
    metas[j] = b.end_object();
  }
  b.start_vector(4, int(n), 4);
  for (size_t j = n; j-- > 0;) b.prepend_uoffset(metas[j]);
  uint32_t vec = b.end_vector(uint32_t(n));
  b.start_object(1);
  if (vec) { b.prepend_uoffset(vec); b.slot(0); }
  uint32_t root = b.end_object();
  b.finish(root);
  return std::vector<uint8_t>(b.data(), b.data() + b.size());
}

// ------------------------------------------------------------------- reader
static inline uint32_t le32(const uint8_t* p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

// table.go Offset(vtableOffset): 0 when the field is absent.
static bool field(const uint8_t* b, size_t n, uint32_t pos, uint16_t vo, uint32_t* out) {
  if (size_t(pos) + 4 > n) return false;
  int64_t vt = int64_t(pos) - int32_t(le32(b + pos));
  if (vt < 0 || size_t(vt) + 2 > n) return false;
  uint16_t vtlen = uint16_t(b[vt] | b[vt + 1] << 8);
  if (vo < vtlen) {
    if (size_t(vt) + vo + 2 > n) return false;
    *out = uint16_t(b[vt + vo] | b[vt + vo + 1] << 8);
  } else {
    *out = 0;
  }
  return true;
}

static bool field_u64(const uint8_t* b, size_t n, uint32_t pos, uint16_t vo, uint64_t* v) {
  uint32_t o;
  if (!field(b, n, pos, vo, &o)) return false;
  *v = 0;
  if (!o) return true;
  if (size_t(pos) + o + 8 > n) return false;
  *v = uint64_t(le32(b + pos + o)) | uint64_t(le32(b + pos + o + 4)) << 32;
  return true;
}

static bool field_bytes(const uint8_t* b, size_t n, uint32_t pos, uint16_t vo, const uint8_t** p, size_t* len,
                        bool* present) {
  uint32_t o;
  if (!field(b, n, pos, vo, &o)) return false;
  *present = o != 0;
  *p = nullptr;
  *len = 0;
  if (!o) return true;
  size_t at = size_t(pos) + o;
  if (at + 4 > n) return false;
  at += le32(b + at);
  if (at + 4 > n) return false;
  size_t l = le32(b + at);
  if (at + 4 + l > n) return false;
  *p = b + at + 4;
  *len = l;
  return true;
}

bool fb_decode_info(const uint8_t* b, size_t n, InfoFields* out) {
  if (n < 4) return false;
  uint32_t root = le32(b);
  const uint8_t* p;
  size_t l;
  bool present;
  if (!field_bytes(b, n, root, 4, &p, &l, &present)) return false;
  if (!field_u64(b, n, root, 6, &out->index_offset) || !field_u64(b, n, root, 8, &out->index_len) ||
      !field_u64(b, n, root, 10, &out->filter_offset) || !field_u64(b, n, root, 12, &out->filter_len))
    return false;
  uint32_t o;
  if (!field(b, n, root, 14, &o)) return false;
  if (o && size_t(root) + o >= n) return false;
  out->codec = o ? int8_t(b[root + o]) : 0;
  out->has_first_key = present;
  out->first_key.assign(p, p + l);
  return true;
}

bool fb_decode_index(const uint8_t* d, size_t n, std::vector<uint64_t>* offsets, std::vector<uint8_t>* keys,
                     std::vector<uint64_t>* key_off) {
  if (n < 4) return false;
  uint32_t root = le32(d);
  uint32_t o;
  if (!field(d, n, root, 4, &o) || !o) return false;
  size_t vec = size_t(root) + o;
  if (vec + 4 > n) return false;
  vec += le32(d + vec);
  if (vec + 4 > n) return false;
  uint32_t nm = le32(d + vec);
  if (vec + 4 + size_t(nm) * 4 > n) return false;
  offsets->resize(nm);
  key_off->assign(size_t(nm) + 1, 0);
  keys->clear();
  for (uint32_t j = 0; j < nm; j++) {
    size_t ep = vec + 4 + 4 * size_t(j);
    uint32_t tp = uint32_t(ep + le32(d + ep));
    const uint8_t* kp;
    size_t kl;
    bool present;
    if (!field_u64(d, n, tp, 4, &(*offsets)[j]) || !field_bytes(d, n, tp, 6, &kp, &kl, &present)) return false;
    keys->insert(keys->end(), kp, kp + kl);
    (*key_off)[j + 1] = keys->size();
  }
  return true;
}

}  // namespace slate
