#include "json.h"

#include <cstdio>
#include <cstdlib>
#include <string_view>
#include <unordered_map>
#include <unordered_set>

namespace mi355x::json {
namespace {

// true when a key occurs twice (small objects, the common case, without allocating)
bool repeated_key(const std::vector<std::pair<std::string, Value>>& obj) {
  if (obj.size() <= 16) {
    for (size_t a = 0; a < obj.size(); ++a)
      for (size_t b = a + 1; b < obj.size(); ++b)
        if (obj[a].first == obj[b].first) return true;
    return false;
  }
  std::unordered_set<std::string_view> seen;
  for (const auto& kv : obj)
    if (!seen.insert(kv.first).second) return true;
  return false;
}

}  // namespace

const Value* Value::get(const std::string& key) const {
  if (kind != Object) return nullptr;
  for (const auto& [k, v] : obj)
    if (k == key) return &v;
  return nullptr;
}

Value* Value::get(const std::string& key) {
  if (kind != Object) return nullptr;
  for (auto& [k, v] : obj)
    if (k == key) return &v;
  return nullptr;
}

Value& Value::set(const std::string& key, Value v) {
  if (Value* cur = get(key)) return *cur = std::move(v);
  obj.emplace_back(key, std::move(v));
  return obj.back().second;
}

std::string Value::str(const std::string& key, const std::string& fallback) const {
  const Value* v = get(key);
  if (!v) return fallback;
  if (v->kind == String || v->kind == Number) return v->s;
  return fallback;
}

namespace {

struct Parser {
  explicit Parser(const std::string& text) : t(text) {}
  const std::string& t;
  size_t i = 0;
  std::string err;
  int depth = 0;

  void ws() {
    while (i < t.size() && (t[i] == ' ' || t[i] == '\t' || t[i] == '\n' || t[i] == '\r')) ++i;
  }
  bool fail(const char* what) {
    if (err.empty()) err = std::string(what) + " at byte " + std::to_string(i);
    return false;
  }
  bool lit(const char* w) {
    size_t n = 0;
    while (w[n]) ++n;
    if (t.compare(i, n, w) != 0) return fail("bad literal");
    i += n;
    return true;
  }
  static void utf8(std::string* out, unsigned cp) {
    if (cp < 0x80) {
      out->push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      out->push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out->push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out->push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }
  bool hex4(unsigned* cp) {
    if (i + 4 > t.size()) return fail("short \\u escape");
    unsigned v = 0;
    for (int k = 0; k < 4; ++k) {
      const char c = t[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else return fail("bad \\u escape");
    }
    *cp = v;
    return true;
  }
  bool string(std::string* out) {
    if (i >= t.size() || t[i] != '"') return fail("expected string");
    ++i;
    while (i < t.size()) {
      const char c = t[i++];
      if (c == '"') return true;
      if (static_cast<unsigned char>(c) < 0x20) return fail("control character in string");
      if (c != '\\') {
        out->push_back(c);
        continue;
      }
      if (i >= t.size()) break;
      const char e = t[i++];
      switch (e) {
        case '"': out->push_back('"'); break;
        case '\\': out->push_back('\\'); break;
        case '/': out->push_back('/'); break;
        case 'b': out->push_back('\b'); break;
        case 'f': out->push_back('\f'); break;
        case 'n': out->push_back('\n'); break;
        case 'r': out->push_back('\r'); break;
        case 't': out->push_back('\t'); break;
        case 'u': {
          unsigned cp = 0;
          if (!hex4(&cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00 && i + 1 < t.size() && t[i] == '\\' && t[i + 1] == 'u') {
            const size_t next = i;
            i += 2;
            unsigned lo = 0;
            if (hex4(&lo) && lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else i = next;  // not a low surrogate: that escape is read on its own
          }
          if (cp >= 0xD800 && cp < 0xE000) cp = 0xFFFD;  // a lone surrogate, as Go's encoding/json reads it
          utf8(out, cp);
          break;
        }
        default: return fail("bad escape");
      }
    }
    return fail("unterminated string");
  }
  // RFC 8259: -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)?, kept as its source text
  bool number(Value* v) {
    const size_t s = i;
    auto digit = [&] { return i < t.size() && t[i] >= '0' && t[i] <= '9'; };
    auto digits = [&] {
      if (!digit()) return false;
      while (digit()) ++i;
      return true;
    };
    if (i < t.size() && t[i] == '-') ++i;
    if (i < t.size() && t[i] == '0') {
      ++i;
      if (digit()) return fail("bad number (leading zero)");
    } else if (!digits()) {
      return fail("bad number");
    }
    if (i < t.size() && t[i] == '.') {
      ++i;
      if (!digits()) return fail("bad number (no digits after the point)");
    }
    if (i < t.size() && (t[i] == 'e' || t[i] == 'E')) {
      ++i;
      if (i < t.size() && (t[i] == '+' || t[i] == '-')) ++i;
      if (!digits()) return fail("bad number (no exponent digits)");
    }
    v->kind = Value::Number;
    v->s = t.substr(s, i - s);
    return true;
  }
  bool value(Value* v) {
    if (++depth > 128) return fail("nesting too deep");
    ws();
    if (i >= t.size()) return fail("unexpected end");
    bool ok = true;
    const char c = t[i];
    if (c == '{') {
      ++i;
      v->kind = Value::Object;
      ws();
      if (i < t.size() && t[i] == '}') {
        ++i;
      } else {
        for (;;) {
          ws();
          std::string k;
          if (!string(&k)) return false;
          ws();
          if (i >= t.size() || t[i] != ':') return fail("expected ':'");
          ++i;
          Value m;
          if (!value(&m)) return false;
          v->obj.emplace_back(std::move(k), std::move(m));
          ws();
          if (i < t.size() && t[i] == ',') {
            ++i;
            continue;
          }
          if (i < t.size() && t[i] == '}') {
            ++i;
            break;
          }
          return fail("expected ',' or '}'");
        }
        if (v->obj.size() > 1 && repeated_key(v->obj)) {
          // a repeated key: the last value wins, at the first one's place (Go's encoding/json
          // and Python's json keep the last)
          std::unordered_map<std::string, size_t> at;
          std::vector<std::pair<std::string, Value>> kept;
          kept.reserve(v->obj.size());
          for (auto& kv : v->obj) {
            auto [it, fresh] = at.emplace(kv.first, kept.size());
            if (fresh) kept.push_back(std::move(kv));
            else kept[it->second].second = std::move(kv.second);
          }
          v->obj = std::move(kept);
        }
      }
    } else if (c == '[') {
      ++i;
      v->kind = Value::Array;
      ws();
      if (i < t.size() && t[i] == ']') {
        ++i;
      } else {
        for (;;) {
          Value m;
          if (!value(&m)) return false;
          v->arr.push_back(std::move(m));
          ws();
          if (i < t.size() && t[i] == ',') {
            ++i;
            continue;
          }
          if (i < t.size() && t[i] == ']') {
            ++i;
            break;
          }
          return fail("expected ',' or ']'");
        }
      }
    } else if (c == '"') {
      v->kind = Value::String;
      ok = string(&v->s);
    } else if (c == 't') {
      v->kind = Value::Bool;
      v->b = true;
      ok = lit("true");
    } else if (c == 'f') {
      v->kind = Value::Bool;
      ok = lit("false");
    } else if (c == 'n') {
      ok = lit("null");
    } else {
      ok = number(v);
    }
    --depth;
    return ok;
  }
};

void write(const Value& v, std::string* out) {
  switch (v.kind) {
    case Value::Null: *out += "null"; break;
    case Value::Bool: *out += v.b ? "true" : "false"; break;
    case Value::Number: *out += v.s; break;
    case Value::String: *out += quote(v.s); break;
    case Value::Array:
      out->push_back('[');
      for (size_t k = 0; k < v.arr.size(); ++k) {
        if (k) out->push_back(',');
        write(v.arr[k], out);
      }
      out->push_back(']');
      break;
    case Value::Object:
      out->push_back('{');
      for (size_t k = 0; k < v.obj.size(); ++k) {
        if (k) out->push_back(',');
        *out += quote(v.obj[k].first);
        out->push_back(':');
        write(v.obj[k].second, out);
      }
      out->push_back('}');
      break;
  }
}

}  // namespace

std::optional<Value> parse(const std::string& text, std::string* error) {
  Parser p(text);
  Value v;
  if (!p.value(&v)) {
    if (error) *error = p.err;
    return std::nullopt;
  }
  p.ws();
  if (p.i != text.size()) {
    if (error) *error = "trailing data at byte " + std::to_string(p.i);
    return std::nullopt;
  }
  return v;
}

std::string serialize(const Value& v) {
  std::string out;
  write(v, &out);
  return out;
}

std::string quote(const std::string& s) {
  std::string out = "\"";
  for (const char ch : s) {
    const auto c = static_cast<unsigned char>(ch);
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) {
          char b[8];
          std::snprintf(b, sizeof(b), "\\u%04x", c);
          out += b;
        } else {
          out.push_back(ch);  // UTF-8 passes through (valid JSON)
        }
    }
  }
  out.push_back('"');
  return out;
}

std::map<std::string, std::string> node_labels(const Value& node) {
  std::map<std::string, std::string> out;
  const Value* md = node.get("metadata");
  const Value* labels = md ? md->get("labels") : nullptr;
  if (!labels || labels->kind != Value::Object) return out;
  for (const auto& [k, v] : labels->obj)
    if (v.kind == Value::String) out[k] = v.s;
  return out;
}

}  // namespace mi355x::json
