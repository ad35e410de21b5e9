// The YAML subset configuration files use (see yaml.h).
#include "yaml.h"

#include <cstdint>
#include <vector>

namespace mi355x::yaml {
namespace {

// ---- YAML subset ---------------------------------------------------------------
struct Line {
  int indent;
  std::string text;  // without indentation and trailing comment / whitespace
  int no;
};

// strips a trailing " # comment" outside quotes
std::string strip_comment(const std::string& s) {
  char q = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    if (q) {
      if (c == q && !(q == '"' && i && s[i - 1] == '\\')) q = 0;
    } else if (c == '"' || c == '\'') {
      if (i == 0 || s[i - 1] == ' ' || s[i - 1] == ':' || s[i - 1] == '[' || s[i - 1] == '{' || s[i - 1] == ',')
        q = c;
    } else if (c == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) {
      return s.substr(0, i);
    }
  }
  return s;
}

std::string rtrim(std::string s) {
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.pop_back();
  return s;
}

class Parser {
 public:
  Parser(const std::string& text, std::string* err) : err_(err) {
    int no = 0;
    size_t pos = 0;
    while (pos <= text.size()) {
      size_t nl = text.find('\n', pos);
      if (nl == std::string::npos) nl = text.size();
      raw_.push_back(text.substr(pos, nl - pos));
      pos = nl + 1;
    }
    for (const auto& r : raw_) {
      ++no;
      std::string t = rtrim(r);
      size_t ind = 0;
      while (ind < t.size() && t[ind] == ' ') ++ind;
      std::string body = rtrim(strip_comment(t.substr(ind)));
      if (body.empty() || body == "---" || body == "...") continue;
      lines_.push_back({static_cast<int>(ind), body, no});
    }
  }

  std::optional<json::Value> document() {
    if (lines_.empty()) return json::Value::object();
    const char c0 = lines_[0].text[0];
    if (c0 == '[' || c0 == '{') {  // a flow collection as the document, possibly over several lines
      std::string all;
      for (const auto& l : lines_) all += (all.empty() ? "" : " ") + l.text;
      auto v = scalar_or_flow(all, lines_[0].no);
      if (!err_->empty()) return std::nullopt;
      return v;
    }
    size_t i = 0;
    auto v = block(&i, lines_[0].indent);
    if (v && i < lines_.size()) fail(lines_[i].no, "unexpected content");
    if (!err_->empty()) return std::nullopt;
    return v;
  }

 private:
  void fail(int no, const std::string& why) {
    if (err_->empty()) *err_ = "line " + std::to_string(no) + ": " + why;
  }

  static bool is_seq_item(const std::string& t) { return t == "-" || t.compare(0, 2, "- ") == 0; }

  // position of the ':' that ends a mapping key, or npos
  static size_t key_colon(const std::string& t) {
    char q = 0;
    int depth = 0;
    for (size_t i = 0; i < t.size(); ++i) {
      const char c = t[i];
      if (q) {
        if (c == q) q = 0;
        continue;
      }
      if ((c == '"' || c == '\'') && i == 0) q = c;
      else if (c == '{' || c == '[') ++depth;
      else if (c == '}' || c == ']') --depth;
      else if (c == ':' && depth == 0 && (i + 1 == t.size() || t[i + 1] == ' ')) return i;
    }
    return std::string::npos;
  }

  // nesting bound (block and flow collections): a hostile or broken file
  // must not exhaust the stack (the JSON reader has the same bound)
  static constexpr int kMaxDepth = 128;
  struct Nest {
    explicit Nest(int* d) : d_(d) { ++*d_; }
    ~Nest() { --*d_; }
    int* d_;
  };

  std::optional<json::Value> block(size_t* i, int indent) {
    Nest nest(&depth_);
    if (*i >= lines_.size()) return json::Value{};
    if (depth_ > kMaxDepth) return fail(lines_[*i].no, "nested too deeply"), std::nullopt;
    if (is_seq_item(lines_[*i].text)) return sequence(i, indent);
    return mapping(i, indent);
  }

  std::optional<json::Value> sequence(size_t* i, int indent) {
    json::Value arr;
    arr.kind = json::Value::Array;
    while (*i < lines_.size() && lines_[*i].indent == indent && is_seq_item(lines_[*i].text)) {
      Line& l = lines_[*i];
      std::string rest = l.text.size() > 1 ? l.text.substr(2) : "";
      while (!rest.empty() && rest[0] == ' ') rest.erase(0, 1);
      if (rest.empty()) {  // the item is the nested block below
        ++*i;
        if (*i < lines_.size() && lines_[*i].indent > indent) {
          auto v = block(i, lines_[*i].indent);
          if (!v) return std::nullopt;
          arr.arr.push_back(std::move(*v));
        } else {
          arr.arr.push_back(json::Value{});
        }
        continue;
      }
      const int item_indent = indent + static_cast<int>(l.text.size() - rest.size());
      if (key_colon(rest) != std::string::npos && rest[0] != '{' && rest[0] != '[') {
        // "- key: value": a mapping whose first entry sits on this line
        l.indent = item_indent;
        l.text = rest;
        auto v = mapping(i, item_indent);
        if (!v) return std::nullopt;
        arr.arr.push_back(std::move(*v));
      } else {
        auto v = scalar_or_flow(rest, l.no);
        if (!v) return std::nullopt;
        arr.arr.push_back(std::move(*v));
        ++*i;
      }
    }
    return arr;
  }

  std::optional<json::Value> mapping(size_t* i, int indent) {
    json::Value obj = json::Value::object();
    while (*i < lines_.size() && lines_[*i].indent == indent && !is_seq_item(lines_[*i].text)) {
      const Line l = lines_[*i];
      const size_t c = key_colon(l.text);
      if (c == std::string::npos) {
        fail(l.no, "expected 'key: value'");
        return std::nullopt;
      }
      std::string key = l.text.substr(0, c);
      if (key.size() >= 2 && (key[0] == '"' || key[0] == '\'') && key.back() == key[0])
        key = key.substr(1, key.size() - 2);
      std::string val = c + 1 < l.text.size() ? l.text.substr(c + 1) : "";
      while (!val.empty() && val[0] == ' ') val.erase(0, 1);
      ++*i;
      if (val == "|" || val == "|-" || val == ">" || val == ">-") {  // block scalar
        std::string out;
        int bi = -1;
        size_t r = static_cast<size_t>(l.no);  // raw_ index of the next line
        while (r < raw_.size()) {
          const std::string& rl = raw_[r];
          size_t ind = 0;
          while (ind < rl.size() && rl[ind] == ' ') ++ind;
          if (rtrim(rl).empty()) {
            out += "\n";
            ++r;
            continue;
          }
          if (static_cast<int>(ind) <= indent) break;
          if (bi < 0) bi = static_cast<int>(ind);
          out += rtrim(rl.substr(std::min<size_t>(static_cast<size_t>(bi), ind))) + (val[0] == '>' ? " " : "\n");
          ++r;
        }
        while (*i < lines_.size() && lines_[*i].no <= static_cast<int>(r)) ++*i;
        if (val.size() == 2)
          while (!out.empty() && (out.back() == '\n' || out.back() == ' ')) out.pop_back();
        obj.set(key, json::Value::string(out));
        continue;
      }
      if (val.empty()) {
        if (*i < lines_.size() && lines_[*i].indent > indent) {
          auto v = block(i, lines_[*i].indent);
          if (!v) return std::nullopt;
          obj.set(key, std::move(*v));
        } else if (*i < lines_.size() && lines_[*i].indent == indent && is_seq_item(lines_[*i].text)) {
          auto v = sequence(i, indent);  // "key:\n- item" at the key's indentation
          if (!v) return std::nullopt;
          obj.set(key, std::move(*v));
        } else {
          obj.set(key, json::Value{});
        }
        continue;
      }
      auto v = scalar_or_flow(val, l.no);
      if (!v) return std::nullopt;
      obj.set(key, std::move(*v));
    }
    return obj;
  }

  std::optional<json::Value> scalar_or_flow(const std::string& s, int no) {
    size_t p = 0;
    auto v = flow(s, &p, no, false);
    if (!v) return std::nullopt;
    while (p < s.size() && s[p] == ' ') ++p;
    if (p != s.size()) {
      fail(no, "trailing characters after a value");
      return std::nullopt;
    }
    return v;
  }

  static json::Value plain(const std::string& t) {
    if (t == "true" || t == "True" || t == "TRUE") {
      json::Value v;
      v.kind = json::Value::Bool;
      v.b = true;
      return v;
    }
    if (t == "false" || t == "False" || t == "FALSE") {
      json::Value v;
      v.kind = json::Value::Bool;
      return v;
    }
    if (t == "null" || t == "~" || t.empty()) return json::Value{};
    return json::Value::string(t);
  }

  static void utf8(std::string* out, uint32_t cp) {
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

  // a double-quoted scalar's escape at s[*p] == '\\' (YAML 1.2 5.7); *p ends on its last character
  static bool escape(const std::string& s, size_t* p, std::string* out) {
    const char e = s[++*p];
    switch (e) {
      case '0': out->push_back('\0'); return true;
      case 'a': out->push_back('\a'); return true;
      case 'b': out->push_back('\b'); return true;
      case 't': case '\t': out->push_back('\t'); return true;
      case 'n': out->push_back('\n'); return true;
      case 'v': out->push_back('\v'); return true;
      case 'f': out->push_back('\f'); return true;
      case 'r': out->push_back('\r'); return true;
      case 'e': out->push_back('\x1b'); return true;
      case ' ': case '"': case '/': case '\\': out->push_back(e); return true;
      case 'N': utf8(out, 0x85); return true;
      case '_': utf8(out, 0xA0); return true;
      case 'L': utf8(out, 0x2028); return true;
      case 'P': utf8(out, 0x2029); return true;
      case 'x': case 'u': case 'U': {
        const size_t n = e == 'x' ? 2 : e == 'u' ? 4 : 8;
        if (*p + n >= s.size()) return false;
        uint32_t cp = 0;
        for (size_t k = 1; k <= n; ++k) {
          const char h = s[*p + k];
          const int d = h >= '0' && h <= '9' ? h - '0' : h >= 'a' && h <= 'f' ? h - 'a' + 10
                        : h >= 'A' && h <= 'F' ? h - 'A' + 10 : -1;
          if (d < 0) return false;
          cp = cp * 16 + static_cast<uint32_t>(d);
        }
        if (cp > 0x10FFFF) return false;
        *p += n;
        utf8(out, cp);
        return true;
      }
      default:
        return false;
    }
  }

  // a value starting at s[*p]; in_flow: plain scalars end at , ] }
  std::optional<json::Value> flow(const std::string& s, size_t* p, int no, bool in_flow) {
    Nest nest(&depth_);
    if (depth_ > kMaxDepth) return fail(no, "nested too deeply"), std::nullopt;
    while (*p < s.size() && s[*p] == ' ') ++*p;
    if (*p >= s.size()) return json::Value{};
    const char c = s[*p];
    if (c == '"') {
      std::string out;
      for (++*p; *p < s.size() && s[*p] != '"'; ++*p) {
        if (s[*p] == '\\' && *p + 1 < s.size()) {
          if (!escape(s, p, &out)) return fail(no, "bad escape in a double-quoted scalar"), std::nullopt;
        } else {
          out.push_back(s[*p]);
        }
      }
      if (*p >= s.size()) return fail(no, "unterminated string"), std::nullopt;
      ++*p;
      return json::Value::string(out);
    }
    if (c == '\'') {
      std::string out;
      for (++*p; *p < s.size(); ++*p) {
        if (s[*p] == '\'') {
          if (*p + 1 < s.size() && s[*p + 1] == '\'') {
            out.push_back('\'');
            ++*p;
            continue;
          }
          break;
        }
        out.push_back(s[*p]);
      }
      if (*p >= s.size()) return fail(no, "unterminated string"), std::nullopt;
      ++*p;
      return json::Value::string(out);
    }
    if (c == '[') {
      json::Value arr;
      arr.kind = json::Value::Array;
      ++*p;
      while (true) {
        while (*p < s.size() && s[*p] == ' ') ++*p;
        if (*p < s.size() && s[*p] == ']') {
          ++*p;
          return arr;
        }
        auto v = flow(s, p, no, true);
        if (!v) return std::nullopt;
        arr.arr.push_back(std::move(*v));
        while (*p < s.size() && s[*p] == ' ') ++*p;
        if (*p < s.size() && s[*p] == ',') {
          ++*p;
          continue;
        }
        if (*p < s.size() && s[*p] == ']') {
          ++*p;
          return arr;
        }
        return fail(no, "expected , or ] in a flow sequence"), std::nullopt;
      }
    }
    if (c == '{') {
      json::Value obj = json::Value::object();
      ++*p;
      while (true) {
        while (*p < s.size() && s[*p] == ' ') ++*p;
        if (*p < s.size() && s[*p] == '}') {
          ++*p;
          return obj;
        }
        auto k = flow(s, p, no, true);
        if (!k) return std::nullopt;
        while (*p < s.size() && s[*p] == ' ') ++*p;
        if (*p >= s.size() || s[*p] != ':') return fail(no, "expected : in a flow mapping"), std::nullopt;
        ++*p;
        auto v = flow(s, p, no, true);
        if (!v) return std::nullopt;
        obj.set(k->kind == json::Value::String ? k->s : json::serialize(*k), std::move(*v));
        while (*p < s.size() && s[*p] == ' ') ++*p;
        if (*p < s.size() && s[*p] == ',') {
          ++*p;
          continue;
        }
        if (*p < s.size() && s[*p] == '}') {
          ++*p;
          return obj;
        }
        return fail(no, "expected , or } in a flow mapping"), std::nullopt;
      }
    }
    // plain scalar: to the end (block context) or to , ] } / ": " (flow context)
    size_t e = *p;
    while (e < s.size()) {
      if (in_flow && (s[e] == ',' || s[e] == ']' || s[e] == '}')) break;
      if (in_flow && s[e] == ':' && (e + 1 == s.size() || s[e + 1] == ' ')) break;
      ++e;
    }
    std::string t = rtrim(s.substr(*p, e - *p));
    *p = e;
    return plain(t);
  }

  std::string* err_;
  int depth_ = 0;
  std::vector<std::string> raw_;
  std::vector<Line> lines_;
};

}  // namespace

std::optional<json::Value> parse(const std::string& text, std::string* error) {
  std::string err;
  const size_t first = text.find_first_not_of(" \t\r\n");
  if (first != std::string::npos && (text[first] == '{' || text[first] == '[')) {
    // JSON (a JSON kubeconfig); else a YAML flow collection, whose error is
    // reported only when the text is not JSON either
    if (auto v = json::parse(text, &err)) return v;
    std::string yerr;
    Parser p(text, &yerr);
    if (auto v = p.document()) return v;
    if (error) *error = err;
    return std::nullopt;
  }
  Parser p(text, &err);
  auto v = p.document();
  if (!v && error) *error = err;
  return v;
}

}  // namespace mi355x::yaml
