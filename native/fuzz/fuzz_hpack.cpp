// HPACK decoder (src/rpc/hpack.cpp): header blocks as kubelet's x/net encoder
// or a hostile peer could send them, several per connection so the dynamic
// table carries state between blocks. Invariants: the table never exceeds its
// maximum; Huffman decode -> encode -> decode is the identity and the encoded
// size prediction is exact.
#include <string>
#include <vector>

#include "../src/rpc/hpack.h"
#include "fuzz_common.h"

using mi355x::fuzz::fail;
using namespace mi355x::rpc;

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  // blocks separated by the two bytes 0xFF 0x00 (rare inside a valid block)
  std::vector<std::pair<const uint8_t*, size_t>> blocks;
  size_t start = 0;
  for (size_t i = 0; i + 1 < size; ++i)
    if (data[i] == 0xFF && data[i + 1] == 0x00) {
      blocks.emplace_back(data + start, i - start);
      start = i + 2;
      ++i;
    }
  blocks.emplace_back(data + start, size - start);

  HpackDecoder dec(4096);
  for (const auto& [p, n] : blocks) {
    HeaderList out;
    if (!dec.decode(p, n, &out)) break;  // COMPRESSION_ERROR ends the connection
    if (dec.table_bytes() > dec.max_table() || dec.max_table() > 4096) fail("dynamic table over its maximum");
    size_t sum = 0;
    for (size_t i = 0; i < dec.table_entries(); ++i) sum += 32;  // every entry costs >= 32 octets
    if (sum > dec.table_bytes()) fail("entry accounting");
  }

  std::string plain;
  if (huffman_decode(data, size, &plain)) {
    std::string enc, back;
    huffman_encode(plain, &enc);
    if (enc.size() != huffman_encoded_size(plain)) fail("huffman size prediction");
    if (!huffman_decode(reinterpret_cast<const uint8_t*>(enc.data()), enc.size(), &back) || back != plain)
      fail("huffman round trip");
  }
  return 0;
}
