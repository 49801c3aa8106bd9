// Temporary: C-ABI entry points not yet backed by kernels (return SLATE_E_INVALID_ARG).
#include "host_ctx.h"
extern "C" {
int slate_block_encode(slate_ctx* ctx, int codec, const uint8_t* data, size_t data_len, const uint16_t* offsets, size_t n_offsets, uint8_t* out, size_t out_cap, size_t* out_len) { return SLATE_E_INVALID_ARG; }
slate_sst_builder* slate_sst_builder_new(slate_ctx* ctx, const slate_sst_config* cfg, int* status) { return nullptr; }
void slate_sst_builder_free(slate_sst_builder* b) {}
int slate_sst_builder_add(slate_sst_builder* b, const uint8_t* key, size_t key_len, const uint8_t* value, size_t value_len, int kind) { return SLATE_E_INVALID_ARG; }
int slate_sst_builder_add_value(slate_sst_builder* b, const uint8_t* key, size_t key_len, const uint8_t* value, size_t value_len) { return SLATE_E_INVALID_ARG; }
int slate_sst_builder_add_batch(slate_sst_builder* b, const uint8_t* keys, const uint64_t* key_off, const uint8_t* values, const uint64_t* value_off, const uint8_t* is_tomb, uint64_t n) { return SLATE_E_INVALID_ARG; }
int slate_sst_builder_next_block(slate_sst_builder* b, uint8_t* out, size_t out_cap, size_t* len, int* present) { return SLATE_E_INVALID_ARG; }
int slate_sst_builder_build(slate_sst_builder* b, slate_sst_table** table) { return SLATE_E_INVALID_ARG; }
void slate_sst_table_free(slate_sst_table* t) {}
int slate_sst_table_info(const slate_sst_table* t, slate_sst_info* info, uint8_t* first_key, size_t first_key_cap) { return SLATE_E_INVALID_ARG; }
size_t slate_sst_table_num_chunks(const slate_sst_table* t) { return 0; }
int slate_sst_table_chunk(const slate_sst_table* t, size_t i, const uint8_t** data, size_t* len) { return SLATE_E_INVALID_ARG; }
size_t slate_sst_table_encoded_len(const slate_sst_table* t) { return 0; }
int slate_sst_table_encode(const slate_sst_table* t, uint8_t* out, size_t out_cap) { return SLATE_E_INVALID_ARG; }
int slate_sst_table_bloom(const slate_sst_table* t, int* present, uint16_t* num_probes, uint8_t* bits, size_t bits_cap, size_t* bits_len) { return SLATE_E_INVALID_ARG; }
int slate_sst_read_info(const uint8_t* sst, size_t sst_len, slate_sst_info* info, uint8_t* first_key, size_t first_key_cap) { return SLATE_E_INVALID_ARG; }
int slate_decode_info(const uint8_t* buf, size_t len, slate_sst_info* info, uint8_t* first_key, size_t first_key_cap) { return SLATE_E_INVALID_ARG; }
int slate_encode_info(const slate_sst_info* info, const uint8_t* first_key, uint8_t* out, size_t out_cap, size_t* out_len) { return SLATE_E_INVALID_ARG; }
int slate_decode_index(slate_ctx* ctx, const uint8_t* buf, size_t len, int codec, slate_index** index) { return SLATE_E_INVALID_ARG; }
void slate_index_free(slate_index* index) {}
size_t slate_index_num_blocks(const slate_index* index) { return 0; }
int slate_index_block_meta(const slate_index* index, size_t i, uint64_t* offset, const uint8_t** first_key, size_t* first_key_len) { return SLATE_E_INVALID_ARG; }
int slate_read_blocks_range(const slate_sst_info* info, const slate_index* index, uint64_t start, uint64_t end, uint64_t* range_start, uint64_t* range_end) { return SLATE_E_INVALID_ARG; }
int slate_read_blocks(slate_ctx* ctx, const slate_sst_info* info, const slate_index* index, uint64_t start, uint64_t end, const uint8_t* data, size_t data_len, uint8_t* out, uint64_t out_cap, uint64_t* out_off, slate_block_meta* meta, slate_row* rows, uint64_t rows_cap, uint64_t* row_base, uint64_t* failed_block) { return SLATE_E_INVALID_ARG; }
int slate_bloom_build(slate_ctx* ctx, const uint8_t* keys, const uint64_t* key_off, uint64_t n, uint32_t bits_per_key, uint8_t* bits, size_t bits_cap, size_t* bits_len, uint16_t* num_probes) { return SLATE_E_INVALID_ARG; }
int slate_bloom_encode(slate_ctx* ctx, uint16_t num_probes, const uint8_t* bits, size_t bits_len, int codec, uint8_t* out, size_t out_cap, size_t* out_len) { return SLATE_E_INVALID_ARG; }
int slate_bloom_decode(slate_ctx* ctx, const uint8_t* buf, size_t len, int codec, uint16_t* num_probes, uint8_t* bits, size_t bits_cap, size_t* bits_len) { return SLATE_E_INVALID_ARG; }
int slate_bloom_has_keys(slate_ctx* ctx, uint16_t num_probes, const uint8_t* bits, size_t bits_len, const uint8_t* keys, const uint64_t* key_off, uint64_t n, uint8_t* out) { return SLATE_E_INVALID_ARG; }
}
