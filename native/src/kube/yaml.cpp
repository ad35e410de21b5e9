// The YAML subset configuration files use (see yaml.h).
#include "yaml.h"

#include <cctype>
#include <cstdint>
#include <cstring>
#include <map>
#include <optional>
#include <vector>

namespace mi355x::yaml {
namespace {

// ---- YAML subset ---------------------------------------------------------------
struct Line {
  int indent;
  std::string text;  // without indentation and trailing comment / whitespace
  int no;
};

// "# comment" to the end of each line, outside quoted scalars (which may span
// lines). A quote opens a quoted scalar only where a node may start: at the
// start of a line, after a block indicator followed by a blank ("key: ",
// "- ", "? "), after an anchor or tag, and in flow context after '[', '{', ','
// or a value ':'. Anywhere else (a plain scalar such as the key `:'` or
// `a'b`) it is an ordinary character.
std::string strip_comments(const std::string& s) {
  std::string out;
  char q = 0;
  int flow = 0;
  bool at_start = true;  // the next non-blank character begins a node
  auto blank = [](char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; };
  for (size_t k = 0; k < s.size(); ++k) {
    const char ch = s[k];
    const char prev = k ? s[k - 1] : '\n';
    const char next = k + 1 < s.size() ? s[k + 1] : '\n';
    if (q) {
      if (q == '"' && ch == '\\' && k + 1 < s.size()) {
        out += ch;
        out += s[++k];
        continue;
      }
      if (ch == q) {
        if (q == '\'' && k + 1 < s.size() && s[k + 1] == '\'') {
          out += "''";
          ++k;
          continue;
        }
        q = 0;
        at_start = false;
      }
      out += ch;
      continue;
    }
    if (ch == '#' && (prev == ' ' || prev == '\t' || prev == '\n')) {
      while (k < s.size() && s[k] != '\n') ++k;
      if (k < s.size()) out += '\n';
      at_start = true;
      continue;
    }
    out += ch;
    if (ch == '\n') {
      at_start = true;
      continue;
    }
    if (ch == ' ' || ch == '\t' || ch == '\r') continue;
    if (at_start) {
      if (ch == '"' || ch == '\'') {
        q = ch;
        continue;
      }
      if (ch == '[' || ch == '{') {
        flow++;
        continue;
      }
      if ((ch == '-' || ch == '?') && blank(next)) continue;
      if (ch == '&' || ch == '!') {  // an anchor or tag: the node itself follows it
        while (k + 1 < s.size() && !blank(s[k + 1])) out += s[++k];
        continue;
      }
    }
    if (flow > 0) {
      if (ch == ',') {
        at_start = true;
        continue;
      }
      if (ch == ']' || ch == '}') {
        flow--;
        at_start = false;
        continue;
      }
      if (ch == ':' && (blank(next) || prev == '"' || prev == '\'')) {  // after a JSON-like key: adjacent value
        at_start = true;
        continue;
      }
    }
    if (ch == ':' && blank(next)) {
      at_start = true;
      continue;
    }
    at_start = false;
  }
  return out;
}

std::string rtrim(std::string s) {
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.pop_back();
  return s;
}

class Parser {
 public:
  Parser(const std::string& text, std::string* err) : err_(err) {
    int no = 0;
    size_t pos = text.compare(0, 3, "\xEF\xBB\xBF") == 0 ? 3 : 0;  // a UTF-8 byte order mark
    while (pos <= text.size()) {
      size_t nl = text.find('\n', pos);
      if (nl == std::string::npos) nl = text.size();
      raw_.push_back(text.substr(pos, nl - pos));
      pos = nl + 1;
    }
    // One document: directives (%YAML, %TAG) and a `---` may come before it, `...` may end
    // it; a second document is refused. `--- content` starts the document on that line.
    bool started = false, ended = false, directives = false;
    for (auto& r : raw_) {
      ++no;
      const bool marker = r.compare(0, 3, "---") == 0 && (r.size() == 3 || r[3] == ' ' || r[3] == '\t' || r[3] == '\r');
      const bool end = r.compare(0, 3, "...") == 0 && (r.size() == 3 || r[3] == ' ' || r[3] == '\t' || r[3] == '\r');
      if (!started && !marker && r.compare(0, 1, "%") == 0) {
        directives = true;
        r.clear();
        continue;
      }
      if (marker || end) {
        if ((marker && (started || ended)) || (end && ended)) {
          fail(no, "expected a single document in the stream");
          return;
        }
        started = true;
        ended = end;
        r.replace(0, 3, "   ");
      }
      std::string t = rtrim(r);
      size_t ind = 0;
      while (ind < t.size() && t[ind] == ' ') ++ind;
      std::string body = rtrim(strip_comments(t.substr(ind)));
      if (body.empty()) continue;
      if (ended) {
        fail(no, "expected a single document in the stream");
        return;
      }
      if (directives && !started) {
        fail(no, "directives without a document start (---)");
        return;
      }
      started = true;
      lines_.push_back({static_cast<int>(ind), body, no});
    }
    if (directives && !started) fail(1, "directives without a document start (---)");
  }

  std::optional<json::Value> document() {
    if (!err_->empty()) return std::nullopt;
    if (lines_.empty()) return json::Value::object();
    const char c0 = lines_[0].text[0];
    if (c0 == '[' || c0 == '{') {  // a flow collection as the document, possibly over several lines
      std::string all;
      for (const auto& r : raw_) all += rtrim(r) + "\n";  // (markers and directives blanked above)
      auto v = scalar_or_flow(strip_comments(all), lines_[0].no);
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
        if (q == '"' && c == '\\') {
          ++i;  // an escaped character, e.g. \"
        } else if (c == q) {
          if (q == '\'' && i + 1 < t.size() && t[i + 1] == '\'') ++i;  // '' inside a single-quoted key
          else q = 0;
        }
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
  // nodes aliases may copy in one document: a "billion laughs" of nested aliases is refused
  static constexpr size_t kMaxAliasNodes = size_t{1} << 20;
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
    if (key_colon(lines_[*i].text) == std::string::npos) {
      // a scalar or flow collection on the lines below its key (`key:` then `  value`)
      const Line l = lines_[*i];
      ++*i;
      auto v = scalar_or_flow(continued(l.text, l.no, indent - 1, i), l.no);
      if (v && *i < lines_.size() && lines_[*i].indent >= indent) fail(lines_[*i].no, "unexpected content");
      return v;
    }
    return mapping(i, indent);
  }

  std::optional<json::Value> sequence(size_t* i, int indent) {
    json::Value arr;
    arr.kind = json::Value::Array;
    while (*i < lines_.size() && lines_[*i].indent == indent && is_seq_item(lines_[*i].text)) {
      Line& l = lines_[*i];
      std::string rest = l.text.size() > 1 ? l.text.substr(2) : "";
      while (!rest.empty() && rest[0] == ' ') rest.erase(0, 1);
      // `- &a` then a block, `- &a |`, `- &a - x`: the anchor (and tag) name the entry;
      // `- &a k: v` anchors the key (mapping() reads it), inline values keep theirs for flow()
      std::string anchor, tag;
      if (!props(&rest, l.no, true, &anchor, &tag)) return std::nullopt;
      auto keep = [&](json::Value v) {
        if (!tagged(tag, &v, l.no)) return false;
        if (!anchor.empty()) anchors_[anchor] = v;
        arr.arr.push_back(std::move(v));
        return true;
      };
      if (rest.empty()) {  // the item is the nested block below
        ++*i;
        if (*i < lines_.size() && lines_[*i].indent > indent) {
          auto v = block(i, lines_[*i].indent);
          if (!v) return std::nullopt;
          if (!keep(std::move(*v))) return std::nullopt;
        } else {
          if (!keep(json::Value{})) return std::nullopt;
        }
        continue;
      }
      const int item_indent = indent + static_cast<int>(l.text.size() - rest.size());
      if (is_seq_item(rest)) {
        // "- - item": a sequence whose first item sits on this line
        l.indent = item_indent;
        l.text = rest;
        auto v = sequence(i, item_indent);
        if (!v) return std::nullopt;
        if (!keep(std::move(*v))) return std::nullopt;
        continue;
      }
      if (key_colon(rest) != std::string::npos && rest[0] != '{' && rest[0] != '[') {
        // "- key: value": a mapping whose first entry sits on this line
        l.indent = item_indent;
        l.text = rest;
        auto v = mapping(i, item_indent);
        if (!v) return std::nullopt;
        if (!keep(std::move(*v))) return std::nullopt;
      } else if (rest[0] == '|' || rest[0] == '>') {
        ++*i;
        auto v = block_scalar(rest, l.no, indent, i);
        if (!v) return std::nullopt;
        if (!keep(std::move(*v))) return std::nullopt;
      } else {
        ++*i;
        auto v = scalar_or_flow(continued(rest, l.no, indent, i), l.no);
        if (!v) return std::nullopt;
        if (!keep(std::move(*v))) return std::nullopt;
      }
    }
    return arr;
  }

  // Node properties (an anchor, a tag, both in either order) at the start of `*t` when
  // what follows them is a block node: nothing (the block on the next lines), a block
  // scalar or, for a sequence entry, a nested "- item". They are taken off `*t` into
  // *anchor / *tag; properties of an inline value stay for flow().
  bool props(std::string* t, int no, bool entry, std::string* anchor, std::string* tag) {
    std::string r = *t, a, g;
    for (int k = 0; k < 2 && !r.empty() && (r[0] == '&' || r[0] == '!'); ++k) {
      if (r[0] == '&') {
        if (!a.empty()) return true;
        const auto name = take_anchor(&r, no);
        if (!name) return false;
        a = *name;
      } else {
        if (!g.empty()) return true;
        size_t e = 0;
        while (e < r.size() && !space(r[e])) ++e;
        g = r.substr(0, e);
        while (e < r.size() && space(r[e])) ++e;
        r.erase(0, e);
      }
    }
    if (a.empty() && g.empty()) return true;
    if (r.empty() || r[0] == '|' || r[0] == '>' || (entry && is_seq_item(r))) {
      *t = r;
      *anchor = a;
      *tag = g;
    }
    return true;
  }

  // a standard tag on a block node: the node must be of its kind
  bool tagged(const std::string& tag, json::Value* v, int no) {
    if (tag.empty()) return true;
    const auto k = v->kind;
    if (tag == "!!str" && (k == json::Value::String || k == json::Value::Null)) {
      if (k == json::Value::Null) *v = json::Value::string("");  // `key: !!str` is ""
      return true;
    }
    if ((tag == "!!map" && k == json::Value::Object) || (tag == "!!seq" && k == json::Value::Array) ||
        (tag == "!!null" && k == json::Value::Null))
      return true;
    if (tag != "!!str" && tag != "!!map" && tag != "!!seq" && tag != "!!null")
      return fail(no, "unsupported tag " + tag + " on a block node"), false;
    return fail(no, "tag " + tag + " on a block node of another kind"), false;
  }

  std::optional<json::Value> mapping(size_t* i, int indent) {
    json::Value obj = json::Value::object();
    std::vector<json::Value> merges;  // the values of `<<` keys
    const size_t start = *i;
    while (*i < lines_.size() && lines_[*i].indent == indent && !is_seq_item(lines_[*i].text)) {
      const Line l = lines_[*i];
      const size_t c = key_colon(l.text);
      if (c == std::string::npos) {
        fail(l.no, "expected 'key: value'");
        return std::nullopt;
      }
      std::string key = l.text.substr(0, c);
      while (!key.empty() && (key.back() == ' ' || key.back() == '\t')) key.pop_back();
      const auto key_anchor = take_anchor(&key, l.no);  // `&a k: v` anchors the key (as PyYAML reads it)
      if (!key_anchor) return std::nullopt;
      const bool quoted = !key.empty() && (key[0] == '"' || key[0] == '\'');
      if (quoted || (!key.empty() && key[0] == '*')) {  // a quoted key (escapes and '' resolved) or an alias
        auto k = scalar_or_flow(key, l.no);
        if (!k) return std::nullopt;
        if (k->kind != json::Value::String) return fail(l.no, "a key that is not a string"), std::nullopt;
        key = k->s;
      }
      if (!key_anchor->empty()) anchors_[*key_anchor] = json::Value::string(key);
      std::string val = c + 1 < l.text.size() ? l.text.substr(c + 1) : "";
      while (!val.empty() && val[0] == ' ') val.erase(0, 1);
      // an anchor / tag before a block value (`key: &a` then the block, `key: !!str |`);
      // inline values keep theirs for flow()
      std::string anchor, tag;
      if (!props(&val, l.no, false, &anchor, &tag)) return std::nullopt;
      ++*i;
      std::optional<json::Value> v;
      if (!val.empty() && (val[0] == '|' || val[0] == '>')) {  // block scalar
        v = block_scalar(val, l.no, indent, i);
      } else if (val.empty()) {
        if (*i < lines_.size() && lines_[*i].indent > indent)
          v = block(i, lines_[*i].indent);
        else if (*i < lines_.size() && lines_[*i].indent == indent && is_seq_item(lines_[*i].text))
          v = sequence(i, indent);  // "key:\n- item" at the key's indentation
        else
          v = json::Value{};
      } else {
        v = scalar_or_flow(continued(val, l.no, indent, i), l.no);
      }
      if (!v || !tagged(tag, &*v, l.no)) return std::nullopt;
      if (!anchor.empty()) anchors_[anchor] = *v;
      if (key == "<<" && !quoted)
        merges.push_back(std::move(*v));
      else
        obj.set(key, std::move(*v));
    }
    if (!merges.empty() && !merge(&obj, merges, lines_[start].no)) return std::nullopt;
    return obj;
  }

  // `<<: *base` / `<<: [*a, *b]`, the merge key PyYAML's SafeLoader reads: the merged
  // mappings' entries come first (of a list's, the earlier mapping wins), then the
  // mapping's own entries, which override them
  bool merge(json::Value* obj, const std::vector<json::Value>& merges, int no) {
    json::Value out = json::Value::object();
    for (const auto& m : merges) {
      std::vector<const json::Value*> from;
      if (m.kind == json::Value::Object) {
        from.push_back(&m);
      } else if (m.kind == json::Value::Array) {
        for (auto it = m.arr.rbegin(); it != m.arr.rend(); ++it) {
          if (it->kind != json::Value::Object) return fail(no, "expected a mapping for merging"), false;
          from.push_back(&*it);
        }
      } else {
        return fail(no, "expected a mapping or list of mappings for merging"), false;
      }
      for (const json::Value* f : from)
        for (const auto& kv : f->obj) out.set(kv.first, kv.second);
    }
    for (auto& kv : obj->obj) out.set(kv.first, std::move(kv.second));
    *obj = std::move(out);
    return true;
  }

  // A value that goes on over the following lines indented deeper than its
  // parent (`indent`): a folded plain or quoted scalar, or a flow collection.
  // Returns the value's text with the line breaks kept (flow() folds them) and
  // comments removed; consumes those lines. A value alone on its line is returned as is.
  std::string continued(const std::string& first, int no, int indent, size_t* i) {
    // A comment-only line ends a plain scalar, however deep it is indented
    // (`device_count: 2` then `    # two GPUs` is 2, as PyYAML reads it). Inside a
    // quoted scalar or a flow collection the same line is content or a comment
    // the flow reader strips (a comment-like continuation of a quoted scalar,
    // e.g. `  #"`, is not in lines_).
    size_t v = 0;  // past the node's properties (a tag `!x` / `!!str`, an anchor `&a`)
    while (v < first.size() && (first[v] == '!' || first[v] == '&')) {
      while (v < first.size() && first[v] != ' ') ++v;
      while (v < first.size() && first[v] == ' ') ++v;
    }
    const bool plain = v >= first.size() || (first[v] != '"' && first[v] != '\'' && first[v] != '[' && first[v] != '{');
    // the next non-blank raw line decides
    for (size_t r = static_cast<size_t>(no); r < raw_.size(); ++r) {
      const std::string rl = rtrim(raw_[r]);
      size_t ind = 0;
      while (ind < rl.size() && rl[ind] == ' ') ++ind;
      if (ind == rl.size()) continue;
      if (static_cast<int>(ind) <= indent || (plain && rl[ind] == '#')) return first;
      break;
    }
    std::string text = first;
    size_t r = static_cast<size_t>(no);  // raw_ index of the next line
    size_t last = r;
    std::string pending;
    while (r < raw_.size()) {
      const std::string rl = rtrim(raw_[r]);
      size_t ind = 0;
      while (ind < rl.size() && rl[ind] == ' ') ++ind;
      if (ind == rl.size()) {  // blank: a line break inside the value, unless the value ends here
        pending += "\n";
        ++r;
        continue;
      }
      if (static_cast<int>(ind) <= indent || (plain && rl[ind] == '#')) break;
      text += pending + "\n" + rl;
      pending.clear();
      last = ++r;
    }
    while (*i < lines_.size() && lines_[*i].no <= static_cast<int>(last)) ++*i;
    return strip_comments(text);
  }

  // `|` / `>` with an optional chomping (`-` strip, `+` keep, default clip) and
  // indentation indicator, its content on the following lines (YAML 1.2 8.1)
  std::optional<json::Value> block_scalar(const std::string& head, int no, int indent, size_t* i) {
    const bool folded = head[0] == '>';
    char chomp = 0;
    int explicit_indent = 0;
    for (size_t k = 1; k < head.size(); ++k) {
      const char ch = head[k];
      if ((ch == '-' || ch == '+') && !chomp) chomp = ch;
      else if (ch >= '1' && ch <= '9' && !explicit_indent) explicit_indent = ch - '0';
      else if (ch == ' ' || ch == '\t') break;  // a comment may follow (already stripped)
      else return fail(no, "bad block scalar header"), std::nullopt;
    }
    std::vector<std::string> content;  // lines without the block's indentation; "" = blank
    int bi = explicit_indent ? indent + explicit_indent : -1;
    size_t r = static_cast<size_t>(no);
    while (r < raw_.size()) {
      const std::string rl = rtrim(raw_[r]);
      size_t ind = 0;
      while (ind < rl.size() && rl[ind] == ' ') ++ind;
      if (ind == rl.size()) {
        content.emplace_back();
        ++r;
        continue;
      }
      if (static_cast<int>(ind) <= indent) break;
      if (bi < 0) bi = static_cast<int>(ind);
      if (static_cast<int>(ind) < bi) return fail(r + 1, "block scalar line indented less than its first line"), std::nullopt;
      content.push_back(rl.substr(static_cast<size_t>(bi)));
      ++r;
    }
    size_t used = r;
    int trail = 0;
    while (!content.empty() && content.back().empty()) {
      content.pop_back();
      ++trail;
    }
    std::string body;
    if (!folded) {
      for (size_t k = 0; k < content.size(); ++k) body += (k ? "\n" : "") + content[k];
    } else {
      int blanks = 0;
      bool first = true, prev_more = false;
      for (const auto& ln : content) {
        if (ln.empty()) {
          ++blanks;
          continue;
        }
        const bool more = ln[0] == ' ' || ln[0] == '\t';  // more-indented lines keep their breaks
        if (first) body.append(static_cast<size_t>(blanks), '\n');
        else if (!blanks && !more && !prev_more) body += ' ';
        else if (!more && !prev_more) body.append(static_cast<size_t>(blanks), '\n');
        else body.append(static_cast<size_t>(blanks) + 1, '\n');
        body += ln;
        first = false;
        blanks = 0;
        prev_more = more;
      }
    }
    if (!content.empty() && chomp != '-') body += '\n';
    if (chomp == '+') body.append(static_cast<size_t>(trail), '\n');
    while (*i < lines_.size() && lines_[*i].no <= static_cast<int>(used)) ++*i;
    return json::Value::string(body);
  }

  std::optional<json::Value> scalar_or_flow(const std::string& s, int no) {
    size_t p = 0;
    auto v = flow(s, &p, no, false);
    if (!v) return std::nullopt;
    while (p < s.size() && (s[p] == ' ' || s[p] == '\t' || s[p] == '\n')) ++p;
    if (p != s.size()) {
      fail(no, "trailing characters after a value");
      return std::nullopt;
    }
    return v;
  }

  // the name of the anchor `&name` / alias `*name` at s[*p] (*p past it and the blanks after):
  // letters, digits, - and _, as PyYAML scans it; "" when there is none or something other
  // than a blank or ':' (in flow also , ] } ?) follows it
  static std::string anchor_name(const std::string& s, size_t* p, bool in_flow) {
    size_t e = *p + 1;
    while (e < s.size() && (std::isalnum(static_cast<unsigned char>(s[e])) || s[e] == '-' || s[e] == '_')) ++e;
    if (e < s.size() && !space(s[e]) && s[e] != ':' && !(in_flow && std::strchr(",]}?", s[e]) != nullptr))
      return "";
    std::string name = s.substr(*p + 1, e - *p - 1);
    *p = e;
    while (*p < s.size() && (s[*p] == ' ' || s[*p] == '\t')) ++*p;
    return name;
  }

  // the nodes in `v`, counted up to just past the alias budget
  static size_t nodes(const json::Value& v) {
    size_t n = 1;
    for (const auto& e : v.arr) {
      n += nodes(e);
      if (n > kMaxAliasNodes) return n;
    }
    for (const auto& kv : v.obj) {
      n += nodes(kv.second);
      if (n > kMaxAliasNodes) return n;
    }
    return n;
  }

  // a block node's anchor at the start of `t`: its name ("" = none), `t` left with the rest
  std::optional<std::string> take_anchor(std::string* t, int no) {
    if (t->empty() || (*t)[0] != '&') return std::string();
    size_t p = 0;
    std::string name = anchor_name(*t, &p, false);
    if (name.empty()) return fail(no, "expected an anchor name of letters, digits, - or _"), std::nullopt;
    t->erase(0, p);
    return name;
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
    if (t == "null" || t == "Null" || t == "NULL" || t == "~" || t.empty()) return json::Value{};
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
        if (cp >= 0xD800 && cp < 0xDC00 && *p + 6 < s.size() && s[*p + 1] == '\\' && s[*p + 2] == 'u') {
          uint32_t lo = 0;  // a UTF-16 pair written as two escapes
          for (size_t k = 3; k <= 6; ++k) {
            const char h = s[*p + k];
            const int d = h >= '0' && h <= '9' ? h - '0' : h >= 'a' && h <= 'f' ? h - 'a' + 10
                          : h >= 'A' && h <= 'F' ? h - 'A' + 10 : -1;
            lo = d < 0 ? 0 : lo * 16 + static_cast<uint32_t>(d);
            if (d < 0) break;
          }
          if (lo >= 0xDC00 && lo < 0xE000) {
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            *p += 6;
          }
        }
        if (cp >= 0xD800 && cp < 0xE000) cp = 0xFFFD;  // a lone surrogate: no valid UTF-8 for it
        utf8(out, cp);
        return true;
      }
      default:
        return false;
    }
  }

  static bool space(char ch) { return ch == ' ' || ch == '\t' || ch == '\n'; }

  // Line folding inside a flow scalar (YAML 1.2 6.5) at s[*p] == '\n': the
  // trailing white space before the break is dropped from *out (down to
  // `keep`), a single break becomes a space, n empty lines n line feeds; *p
  // ends on the last skipped character.
  static void fold(const std::string& s, size_t* p, std::string* out, size_t keep) {
    out->resize(keep);
    size_t breaks = 1, q = *p + 1;
    while (q < s.size() && (s[q] == ' ' || s[q] == '\t' || s[q] == '\n')) breaks += s[q++] == '\n';
    if (breaks == 1) out->push_back(' ');
    else out->append(breaks - 1, '\n');
    *p = q - 1;
  }

  // a plain scalar's text from s[*p]: to the end (block context) or to , ] } / ": " (flow context), folded.
  // In block context a ": " (or a ':' ending a line) inside it is a mapping where none may start
  // (YAML 1.2 7.3.3): *colon is set and the text so far returned.
  static std::string plain_text(const std::string& s, size_t* p, bool in_flow, bool* colon = nullptr) {
    std::string out;
    size_t keep = 0;
    for (; *p < s.size(); ++*p) {
      const char ch = s[*p];
      if (in_flow && (ch == ',' || ch == ']' || ch == '}')) break;
      if (ch == ':' && (*p + 1 == s.size() || space(s[*p + 1]) ||
                        (in_flow && (s[*p + 1] == ',' || s[*p + 1] == ']' || s[*p + 1] == '}')))) {
        if (in_flow) break;
        if (colon) *colon = true;
        break;
      }
      if (ch == '\n') {
        fold(s, p, &out, keep);
        keep = out.size();
        continue;
      }
      out.push_back(ch);
      if (ch != ' ' && ch != '\t') keep = out.size();
    }
    out.resize(keep);
    return out;
  }

  // a flow mapping key: a plain key is text (as in block mappings), a quoted one its unescaped value
  static std::string flow_key(const json::Value& k, bool quoted) {
    return k.kind == json::Value::String ? k.s
           : k.kind == json::Value::Bool ? (k.b ? "true" : "false")
           : k.kind == json::Value::Null && !quoted ? "null" : json::serialize(k);
  }

  // a value starting at s[*p]; in_flow: plain scalars end at , ] } and ": "; line breaks fold
  std::optional<json::Value> flow(const std::string& s, size_t* p, int no, bool in_flow) {
    Nest nest(&depth_);
    if (depth_ > kMaxDepth) return fail(no, "nested too deeply"), std::nullopt;
    while (*p < s.size() && space(s[*p])) ++*p;
    if (*p >= s.size()) return json::Value{};
    const char c = s[*p];
    if (c == '&') {  // an anchor: the node after it, remembered for its aliases
      const std::string name = anchor_name(s, p, in_flow);
      if (name.empty()) return fail(no, "expected an anchor name of letters, digits, - or _"), std::nullopt;
      auto v = flow(s, p, no, in_flow);
      if (!v) return std::nullopt;
      anchors_[name] = *v;
      return v;
    }
    if (c == '*') {  // an alias: a copy of the anchored node
      const std::string name = anchor_name(s, p, in_flow);
      if (name.empty()) return fail(no, "expected an alias name of letters, digits, - or _"), std::nullopt;
      auto it = anchors_.find(name);
      if (it == anchors_.end()) return fail(no, "found undefined alias '" + name + "'"), std::nullopt;
      aliased_ += nodes(it->second);
      if (aliased_ > kMaxAliasNodes) return fail(no, "aliases expand to too large a document"), std::nullopt;
      return it->second;
    }
    if (c == '!') {  // a standard tag: !!str !!null !!bool !!int !!float !!map !!seq
      size_t e = *p;
      while (e < s.size() && !space(s[e])) ++e;
      const std::string tag = s.substr(*p, e - *p);
      *p = e;
      while (*p < s.size() && (s[*p] == ' ' || s[*p] == '\t')) ++*p;
      std::string anchor;  // `!!str &a x`: the anchor after the tag
      if (*p < s.size() && s[*p] == '&') {
        anchor = anchor_name(s, p, in_flow);
        if (anchor.empty()) return fail(no, "expected an anchor name of letters, digits, - or _"), std::nullopt;
      }
      auto keep = [&](json::Value v) {
        if (!anchor.empty()) anchors_[anchor] = v;
        return v;
      };
      const bool quoted = *p < s.size() && (s[*p] == '"' || s[*p] == '\'');
      if (tag == "!!str" && !quoted) {
        bool colon = false;
        std::string text = plain_text(s, p, in_flow, &colon);
        if (colon) return fail(no, "mapping values are not allowed here"), std::nullopt;
        return keep(json::Value::string(text));
      }
      auto v = flow(s, p, no, in_flow);
      if (!v) return std::nullopt;
      if (tag == "!!null") return keep(json::Value{});
      if (tag == "!!bool" && v->kind == json::Value::String) {
        json::Value b = plain(v->s);
        if (b.kind != json::Value::Bool) return fail(no, "!!bool on a non-boolean"), std::nullopt;
        return keep(b);
      }
      if (tag == "!!str" || tag == "!!bool" || tag == "!!int" || tag == "!!float" || tag == "!!map" ||
          tag == "!!seq")
        return keep(*v);  // numbers stay text, as plain ones do
      return fail(no, "unsupported tag " + tag), std::nullopt;
    }
    if (c == '"') {
      std::string out;
      size_t keep = 0;  // out.size() up to the last character a line break must not trim
      for (++*p; *p < s.size() && s[*p] != '"'; ++*p) {
        if (s[*p] == '\\' && *p + 1 < s.size()) {
          if (s[*p + 1] == '\n') {  // an escaped line break: joined without a space
            ++*p;
            while (*p + 1 < s.size() && (s[*p + 1] == ' ' || s[*p + 1] == '\t')) ++*p;
          } else if (!escape(s, p, &out)) {
            return fail(no, "bad escape in a double-quoted scalar"), std::nullopt;
          }
          keep = out.size();
        } else if (s[*p] == '\n') {
          fold(s, p, &out, keep);
          keep = out.size();
        } else {
          out.push_back(s[*p]);
          if (s[*p] != ' ' && s[*p] != '\t') keep = out.size();
        }
      }
      if (*p >= s.size()) return fail(no, "unterminated string"), std::nullopt;
      ++*p;
      return json::Value::string(out);
    }
    if (c == '\'') {
      std::string out;
      size_t keep = 0;
      for (++*p; *p < s.size(); ++*p) {
        if (s[*p] == '\'') {
          if (*p + 1 < s.size() && s[*p + 1] == '\'') {
            out.push_back('\'');
            keep = out.size();
            ++*p;
            continue;
          }
          break;
        }
        if (s[*p] == '\n') {
          fold(s, p, &out, keep);
          keep = out.size();
          continue;
        }
        out.push_back(s[*p]);
        if (s[*p] != ' ' && s[*p] != '\t') keep = out.size();
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
        while (*p < s.size() && space(s[*p])) ++*p;
        if (*p < s.size() && s[*p] == ']') {
          ++*p;
          return arr;
        }
        const bool quoted_key = s[*p] == '"' || s[*p] == '\'';
        auto v = flow(s, p, no, true);
        if (!v) return std::nullopt;
        while (*p < s.size() && space(s[*p])) ++*p;
        if (*p < s.size() && s[*p] == ':') {  // [k: v]: a single-pair mapping as the entry
          ++*p;
          auto val = flow(s, p, no, true);
          if (!val) return std::nullopt;
          json::Value pair = json::Value::object();
          pair.set(flow_key(*v, quoted_key), std::move(*val));
          v = std::move(pair);
          while (*p < s.size() && space(s[*p])) ++*p;
        }
        arr.arr.push_back(std::move(*v));
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
      std::vector<json::Value> merges;  // the values of `<<` keys
      auto done = [&]() -> std::optional<json::Value> {
        ++*p;
        if (!merges.empty() && !merge(&obj, merges, no)) return std::nullopt;
        return obj;
      };
      ++*p;
      while (true) {
        while (*p < s.size() && space(s[*p])) ++*p;
        if (*p < s.size() && s[*p] == '}') return done();
        const bool quoted_key = s[*p] == '"' || s[*p] == '\'';
        auto k = flow(s, p, no, true);
        if (!k) return std::nullopt;
        while (*p < s.size() && space(s[*p])) ++*p;
        if (*p >= s.size() || s[*p] != ':') return fail(no, "expected : in a flow mapping"), std::nullopt;
        ++*p;
        auto v = flow(s, p, no, true);
        if (!v) return std::nullopt;
        if (!quoted_key && k->kind == json::Value::String && k->s == "<<")
          merges.push_back(std::move(*v));
        else
          obj.set(flow_key(*k, quoted_key), std::move(*v));
        while (*p < s.size() && space(s[*p])) ++*p;
        if (*p < s.size() && s[*p] == ',') {
          ++*p;
          continue;
        }
        if (*p < s.size() && s[*p] == '}') return done();
        return fail(no, "expected , or } in a flow mapping"), std::nullopt;
      }
    }
    if (c == '-' && (*p + 1 == s.size() || space(s[*p + 1])))
      return fail(no, "sequence entries are not allowed here"), std::nullopt;
    if (c == '?' && (*p + 1 == s.size() || space(s[*p + 1])))
      return fail(no, "complex keys (? key) are not supported"), std::nullopt;
    // indicators no plain scalar starts with (in flow , ] } end an empty node instead)
    if (std::strchr("%@`|>", c) != nullptr || (!in_flow && std::strchr(",]}", c) != nullptr))
      return fail(no, std::string("found character '") + c + "' that cannot start any token"), std::nullopt;
    bool colon = false;
    std::string text = plain_text(s, p, in_flow, &colon);
    if (colon) return fail(no, "mapping values are not allowed here"), std::nullopt;
    return plain(text);
  }

  std::string* err_;
  int depth_ = 0;
  std::map<std::string, json::Value> anchors_;  // &name -> the node (aliases copy it)
  size_t aliased_ = 0;                            // nodes copied by aliases so far
  std::vector<std::string> raw_;
  std::vector<Line> lines_;
};

// A JSON document is also YAML 1.1, where a number with an exponent needs a
// '.' and a signed exponent to resolve as a float (PyYAML's float resolver;
// `1e3` and `1.5e3` are text there). Such numbers are kept as their text, as
// a plain YAML scalar would be.
bool yaml11_numeric(const std::string& t) {
  const size_t e = t.find_first_of("eE");
  if (e == std::string::npos) return true;
  return t.find('.') != std::string::npos && e + 1 < t.size() && (t[e + 1] == '+' || t[e + 1] == '-');
}

void retype_json_numbers(json::Value* v) {
  if (v->kind == json::Value::Number && !yaml11_numeric(v->s)) {
    *v = json::Value::string(v->s);
  } else if (v->kind == json::Value::Array) {
    for (auto& x : v->arr) retype_json_numbers(&x);
  } else if (v->kind == json::Value::Object) {
    for (auto& kv : v->obj) retype_json_numbers(&kv.second);
  }
}

}  // namespace

std::optional<json::Value> parse(const std::string& text, std::string* error) {
  std::string err;
  const size_t first = text.find_first_not_of(" \t\r\n");
  if (first != std::string::npos && (text[first] == '{' || text[first] == '[')) {
    // JSON (a JSON kubeconfig); else a YAML flow collection, whose error is
    // reported only when the text is not JSON either
    if (auto v = json::parse(text, &err)) {
      retype_json_numbers(&*v);
      return v;
    }
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
