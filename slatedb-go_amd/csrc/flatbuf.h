// Host framing: the three flatbuffer tables of the SST footer (schema
// internal/flatbuf/schemas/sst.fbs:11-50) written with the exact byte layout of
// the google/flatbuffers v24.3.25 Go Builder that slatedb-go uses
// (flatbuf.go:62-81 EncodeInfo, :126-139 encodeIndex; manifest_generated.go
// :457-469 BlockMetaT.Pack, :586-606 SsTableIndexT.Pack), and read back the way
// the generated Go accessors do (table.go Offset/Indirect/ByteVector).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace slate {

// Back-to-front buffer with Go Builder semantics: every alignment decision
// depends only on Offset() (bytes written so far), so output bytes equal Go's.
class FbBuilder {
 public:
  explicit FbBuilder(size_t reserve = 256);
  uint32_t offset() const { return uint32_t(buf_.size() - head_); }
  void prep(int size, int additional);
  void prepend_u64(uint64_t v);
  void prepend_i8(int8_t v);
  void prepend_u16(uint16_t v);
  void prepend_uoffset(uint32_t off);
  void prepend_soffset(int32_t off);
  void start_object(int numfields);
  void slot(int i) { vtable_[i] = offset(); }
  uint32_t end_object();
  uint32_t start_vector(int elem, int n, int align);
  uint32_t end_vector(uint32_t n);
  uint32_t create_byte_string(const uint8_t* s, size_t n);  // NUL-terminated
  uint32_t create_byte_vector(const uint8_t* s, size_t n);  // no terminator
  void finish(uint32_t root);
  // finished bytes (valid after finish)
  const uint8_t* data() const { return buf_.data() + head_; }
  size_t size() const { return buf_.size() - head_; }

 private:
  void grow();
  void place_byte(uint8_t b) { buf_[--head_] = b; }
  void place_u32(uint32_t v);
  std::vector<uint8_t> buf_;
  size_t head_;
  int minalign_ = 1;
  std::vector<uint32_t> vtable_;
  uint32_t object_end_ = 0;
  std::vector<uint32_t> vtables_;
};

struct InfoFields {
  uint64_t index_offset = 0, index_len = 0, filter_offset = 0, filter_len = 0;
  int32_t codec = 0;
  bool has_first_key = false;
  std::vector<uint8_t> first_key;
};

// EncodeInfo without the trailing CRC (caller appends BE32 CRC32).
std::vector<uint8_t> fb_encode_info(const InfoFields& info);
// Flatbuffer SsTableIndex bytes (before compression + CRC).
std::vector<uint8_t> fb_encode_index(const std::vector<uint64_t>& offsets, const std::vector<uint8_t>& keys,
                                     const std::vector<uint64_t>& key_off);
// Reader side; return false on a malformed buffer (Go would panic).
bool fb_decode_info(const uint8_t* buf, size_t n, InfoFields* out);
bool fb_decode_index(const uint8_t* buf, size_t n, std::vector<uint64_t>* offsets, std::vector<uint8_t>* keys,
                     std::vector<uint64_t>* key_off);

}  // namespace slate
