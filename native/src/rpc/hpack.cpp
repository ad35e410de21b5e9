// HPACK decoder / encoder primitives (RFC 7541). See hpack.h.
#include "hpack.h"

#include <algorithm>
#include <array>

namespace mi355x::rpc {
namespace {

// Code length in bits of every symbol (0..255, 256 = EOS) of the HPACK Huffman
// code. The code is canonical: codes of one length are consecutive in symbol
// order and follow all shorter codes, so the lengths define it completely.
constexpr uint8_t kHuffLen[257] = {
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28,  //   0.. 15
    28, 28, 28, 28, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 28,  //  16.. 31
    6,  10, 10, 12, 13, 6,  8,  11, 10, 10, 8,  11, 8,  6,  6,  6,   //  ' '..'/'
    5,  5,  5,  6,  6,  6,  6,  6,  6,  6,  7,  8,  15, 6,  12, 10,  //  '0'..'?'
    13, 6,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,   //  '@'..'O'
    7,  7,  7,  7,  7,  7,  7,  7,  8,  7,  8,  13, 19, 13, 14, 6,   //  'P'..'_'
    15, 5,  6,  5,  6,  5,  6,  6,  6,  5,  7,  7,  6,  6,  6,  5,   //  '`'..'o'
    6,  7,  6,  5,  5,  6,  7,  7,  7,  7,  7,  15, 11, 14, 13, 28,  //  'p'..127
    20, 22, 20, 20, 22, 22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23,  // 128..143
    24, 24, 22, 23, 24, 23, 23, 23, 23, 21, 22, 23, 22, 23, 23, 24,  // 144..159
    22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22, 24, 21, 22, 23, 23,  // 160..175
    21, 21, 22, 21, 23, 22, 23, 23, 20, 22, 22, 22, 23, 22, 22, 23,  // 176..191
    26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25,  // 192..207
    19, 21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27,  // 208..223
    20, 24, 20, 21, 22, 21, 21, 23, 22, 22, 25, 25, 24, 24, 26, 23,  // 224..239
    26, 27, 26, 26, 27, 27, 27, 27, 27, 28, 27, 27, 27, 27, 27, 26,  // 240..255
    30};                                                             // EOS

struct HuffTables {
  uint32_t code[257];
  uint32_t first[32];   // first code of each length
  uint32_t count[32];   // number of codes of each length
  uint32_t offset[32];  // index into `order` of the first symbol of each length
  uint16_t order[257];  // symbols sorted by (length, symbol)
};

const HuffTables& huff() {
  static const HuffTables t = [] {
    HuffTables h{};
    for (int s = 0; s < 257; ++s) h.count[kHuffLen[s]]++;
    uint32_t code = 0, idx = 0;
    for (int len = 1; len <= 30; ++len) {
      h.first[len] = code;
      h.offset[len] = idx;
      for (int s = 0; s < 257; ++s)
        if (kHuffLen[s] == len) {
          h.code[s] = code++;
          h.order[idx++] = static_cast<uint16_t>(s);
        }
      code <<= 1;
    }
    return h;
  }();
  return t;
}

struct StaticEntry {
  const char* name;
  const char* value;
};
// RFC 7541 Appendix A
constexpr StaticEntry kStatic[61] = {
    {":authority", ""}, {":method", "GET"}, {":method", "POST"}, {":path", "/"}, {":path", "/index.html"},
    {":scheme", "http"}, {":scheme", "https"}, {":status", "200"}, {":status", "204"}, {":status", "206"},
    {":status", "304"}, {":status", "400"}, {":status", "404"}, {":status", "500"}, {"accept-charset", ""},
    {"accept-encoding", "gzip, deflate"}, {"accept-language", ""}, {"accept-ranges", ""}, {"accept", ""},
    {"access-control-allow-origin", ""}, {"age", ""}, {"allow", ""}, {"authorization", ""},
    {"cache-control", ""}, {"content-disposition", ""}, {"content-encoding", ""}, {"content-language", ""},
    {"content-length", ""}, {"content-location", ""}, {"content-range", ""}, {"content-type", ""},
    {"cookie", ""}, {"date", ""}, {"etag", ""}, {"expect", ""}, {"expires", ""}, {"from", ""}, {"host", ""},
    {"if-match", ""}, {"if-modified-since", ""}, {"if-none-match", ""}, {"if-range", ""},
    {"if-unmodified-since", ""}, {"last-modified", ""}, {"link", ""}, {"location", ""}, {"max-forwards", ""},
    {"proxy-authenticate", ""}, {"proxy-authorization", ""}, {"range", ""}, {"referer", ""}, {"refresh", ""},
    {"retry-after", ""}, {"server", ""}, {"set-cookie", ""}, {"strict-transport-security", ""},
    {"transfer-encoding", ""}, {"user-agent", ""}, {"vary", ""}, {"via", ""}, {"www-authenticate", ""}};

const std::array<std::pair<std::string, std::string>, 61>& static_table() {
  static const auto t = [] {
    std::array<std::pair<std::string, std::string>, 61> a;
    for (size_t i = 0; i < 61; ++i) a[i] = {kStatic[i].name, kStatic[i].value};
    return a;
  }();
  return t;
}

// Integer with an N-bit prefix (RFC 7541 5.1); false on truncation/overflow.
bool get_int(const uint8_t*& p, const uint8_t* end, int prefix_bits, uint64_t* v) {
  if (p >= end) return false;
  const uint8_t mask = static_cast<uint8_t>((1u << prefix_bits) - 1);
  uint64_t x = *p++ & mask;
  if (x < mask) {
    *v = x;
    return true;
  }
  int shift = 0;
  while (true) {
    if (p >= end || shift > 56) return false;
    const uint8_t b = *p++;
    x += static_cast<uint64_t>(b & 0x7F) << shift;
    shift += 7;
    if (!(b & 0x80)) break;
  }
  *v = x;
  return true;
}

bool get_string(const uint8_t*& p, const uint8_t* end, std::string* out) {
  if (p >= end) return false;
  const bool huffman = (*p & 0x80) != 0;
  uint64_t len = 0;
  if (!get_int(p, end, 7, &len)) return false;
  if (len > static_cast<uint64_t>(end - p)) return false;
  bool ok = true;
  if (huffman) {
    out->clear();
    ok = huffman_decode(p, static_cast<size_t>(len), out);
  } else {
    out->assign(reinterpret_cast<const char*>(p), static_cast<size_t>(len));
  }
  p += len;
  return ok;
}

}  // namespace

bool huffman_decode(const uint8_t* p, size_t n, std::string* out) {
  const HuffTables& h = huff();
  uint32_t cur = 0;
  int len = 0;
  for (size_t i = 0; i < n; ++i) {
    for (int b = 7; b >= 0; --b) {
      cur = (cur << 1) | ((p[i] >> b) & 1u);
      ++len;
      if (len > 30) return false;
      if (h.count[len] && cur - h.first[len] < h.count[len]) {
        const uint16_t sym = h.order[h.offset[len] + (cur - h.first[len])];
        if (sym == 256) return false;  // EOS inside a string is an error
        out->push_back(static_cast<char>(sym));
        cur = 0;
        len = 0;
      }
    }
  }
  // padding: at most 7 bits, all ones (a prefix of EOS)
  return len <= 7 && cur == (1u << len) - 1u;
}

size_t huffman_encoded_size(const std::string& in) {
  uint64_t bits = 0;
  for (unsigned char c : in) bits += kHuffLen[c];
  return static_cast<size_t>((bits + 7) / 8);
}

void huffman_encode(const std::string& in, std::string* out) {
  const HuffTables& h = huff();
  uint64_t acc = 0;
  int nbits = 0;
  for (unsigned char c : in) {
    acc = (acc << kHuffLen[c]) | h.code[c];
    nbits += kHuffLen[c];
    while (nbits >= 8) {
      out->push_back(static_cast<char>((acc >> (nbits - 8)) & 0xFF));
      nbits -= 8;
    }
  }
  if (nbits > 0) out->push_back(static_cast<char>(((acc << (8 - nbits)) | ((1u << (8 - nbits)) - 1)) & 0xFF));
}

uint64_t huffman_kraft_sum() {
  uint64_t s = 0;
  for (int i = 0; i < 257; ++i) s += 1ull << (30 - kHuffLen[i]);
  return s;
}

bool HpackDecoder::entry(uint64_t index, const std::string** name, const std::string** value) const {
  if (index == 0) return false;
  if (index <= 61) {
    const auto& e = static_table()[index - 1];
    *name = &e.first;
    *value = &e.second;
    return true;
  }
  const uint64_t d = index - 62;
  if (d >= dyn_.size()) return false;
  *name = &dyn_[d].first;
  *value = &dyn_[d].second;
  return true;
}

void HpackDecoder::evict(size_t limit) {
  while (size_ > limit && !dyn_.empty()) {
    size_ -= dyn_.back().first.size() + dyn_.back().second.size() + 32;
    dyn_.pop_back();
  }
}

void HpackDecoder::insert(std::string name, std::string value) {
  const size_t sz = name.size() + value.size() + 32;
  if (sz > max_) {  // larger than the whole table: empties it (RFC 7541 4.4)
    evict(0);
    return;
  }
  evict(max_ - sz);
  dyn_.emplace_front(std::move(name), std::move(value));
  size_ += sz;
}

bool HpackDecoder::decode(const uint8_t* p, size_t n, HeaderList* out) {
  const uint8_t* end = p + n;
  bool seen_field = false;
  std::string name, value;
  while (p < end) {
    const uint8_t b = *p;
    if (b & 0x80) {  // indexed header field
      uint64_t idx = 0;
      const std::string *nm = nullptr, *val = nullptr;
      if (!get_int(p, end, 7, &idx) || !entry(idx, &nm, &val)) return false;
      out->emplace_back(*nm, *val);
      seen_field = true;
    } else if ((b & 0xE0) == 0x20) {  // dynamic table size update
      if (seen_field) return false;  // only at the start of a block
      uint64_t sz = 0;
      if (!get_int(p, end, 5, &sz) || sz > limit_) return false;
      max_ = static_cast<size_t>(sz);
      evict(max_);
    } else {
      // 01: with incremental indexing (6-bit index); 0000 / 0001: without / never indexed (4-bit)
      const bool indexing = (b & 0xC0) == 0x40;
      uint64_t idx = 0;
      if (!get_int(p, end, indexing ? 6 : 4, &idx)) return false;
      if (idx) {
        const std::string *nm = nullptr, *val = nullptr;
        if (!entry(idx, &nm, &val)) return false;
        name = *nm;
      } else if (!get_string(p, end, &name)) {
        return false;
      }
      if (!get_string(p, end, &value)) return false;
      out->emplace_back(name, value);
      if (indexing) insert(name, value);
      seen_field = true;
    }
  }
  return true;
}

void hpack_put_int(std::string* out, uint64_t v, int prefix_bits, uint8_t first) {
  const uint64_t mask = (1u << prefix_bits) - 1;
  if (v < mask) {
    out->push_back(static_cast<char>(first | v));
    return;
  }
  out->push_back(static_cast<char>(first | mask));
  v -= mask;
  while (v >= 128) {
    out->push_back(static_cast<char>((v & 0x7F) | 0x80));
    v >>= 7;
  }
  out->push_back(static_cast<char>(v));
}

void hpack_put_literal(std::string* out, uint32_t static_name_index, const std::string& value) {
  hpack_put_int(out, static_name_index, 4, 0x00);
  hpack_put_int(out, value.size(), 7, 0x00);
  out->append(value);
}

void hpack_put_literal(std::string* out, const std::string& name, const std::string& value) {
  out->push_back(0x00);
  hpack_put_int(out, name.size(), 7, 0x00);
  out->append(name);
  hpack_put_int(out, value.size(), 7, 0x00);
  out->append(value);
}

}  // namespace mi355x::rpc
