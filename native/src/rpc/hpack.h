// HPACK (RFC 7541) for the native gRPC server: a complete header-block
// decoder (static + dynamic table, Huffman strings, table size updates) and
// the encoder primitives a server needs (literals without indexing, raw
// strings: responses never touch the peer's dynamic table).
#pragma once

#include <cstddef>
#include <cstdint>
#include <deque>
#include <string>
#include <utility>
#include <vector>

namespace mi355x::rpc {

using HeaderList = std::vector<std::pair<std::string, std::string>>;

// Huffman code of RFC 7541 Appendix B (canonical: built from the code lengths).
bool huffman_decode(const uint8_t* p, size_t n, std::string* out);  // false: invalid code or padding
void huffman_encode(const std::string& in, std::string* out);
size_t huffman_encoded_size(const std::string& in);
// sum over symbols of 2^(30 - len): 2^30 for a complete prefix code (tests)
uint64_t huffman_kraft_sum();

class HpackDecoder {
 public:
  explicit HpackDecoder(size_t max_table = 4096) : max_(max_table), limit_(max_table) {}
  // Decodes one complete header block (HEADERS + CONTINUATION fragments).
  // false = COMPRESSION_ERROR (the connection must end).
  bool decode(const uint8_t* p, size_t n, HeaderList* out);
  size_t table_bytes() const { return size_; }
  size_t table_entries() const { return dyn_.size(); }
  size_t max_table() const { return max_; }

 private:
  bool entry(uint64_t index, const std::string** name, const std::string** value) const;
  void insert(std::string name, std::string value);
  void evict(size_t limit);

  std::deque<std::pair<std::string, std::string>> dyn_;  // front = most recent
  size_t size_ = 0;
  size_t max_;    // current maximum (dynamic table size updates)
  size_t limit_;  // our SETTINGS_HEADER_TABLE_SIZE: updates may not exceed it
};

// integer with an N-bit prefix; `first` holds the pattern bits above the prefix
void hpack_put_int(std::string* out, uint64_t v, int prefix_bits, uint8_t first);
// Literal Header Field without Indexing, name from the static table
void hpack_put_literal(std::string* out, uint32_t static_name_index, const std::string& value);
// Literal Header Field without Indexing, literal name
void hpack_put_literal(std::string* out, const std::string& name, const std::string& value);
// Indexed Header Field (static table)
inline void hpack_put_indexed(std::string* out, uint32_t index) { hpack_put_int(out, index, 7, 0x80); }

}  // namespace mi355x::rpc
