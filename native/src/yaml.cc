// YAML subset -> Json and viper-style env overlay (see detcore/yaml.h).
#include "detcore/yaml.h"

#include <cctype>
#include <cstdlib>
#include <sstream>

namespace detcore {
namespace {

struct Line {
  int indent;
  std::string text;  // comment-stripped, right-trimmed, without indentation
  std::string raw;   // original line (block scalars)
  int no;
};

std::string RTrim(const std::string& s) {
  size_t e = s.find_last_not_of(" \t\r");
  return e == std::string::npos ? "" : s.substr(0, e + 1);
}
std::string Trim(const std::string& s) {
  size_t b = s.find_first_not_of(" \t\r");
  if (b == std::string::npos) return "";
  return RTrim(s.substr(b));
}

// strip a '#' comment that starts a token (outside quotes)
std::string StripComment(const std::string& s) {
  char q = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (q) {
      if (c == '\\' && q == '"') ++i;
      else if (c == q) q = 0;
    } else if (c == '"' || c == '\'') {
      if (i == 0 || std::isspace(static_cast<unsigned char>(s[i - 1])) || s[i - 1] == ':' || s[i - 1] == '[' ||
          s[i - 1] == '{' || s[i - 1] == ',' || s[i - 1] == '-')
        q = c;
    } else if (c == '#' && (i == 0 || std::isspace(static_cast<unsigned char>(s[i - 1])))) {
      return s.substr(0, i);
    }
  }
  return s;
}

bool IsInt(const std::string& s, int64_t* v) {
  if (s.empty()) return false;
  const char* p = s.c_str();
  char* end = nullptr;
  int base = 10;
  std::string t = s;
  bool neg = false;
  if (t[0] == '+' || t[0] == '-') {
    neg = t[0] == '-';
    t = t.substr(1);
  }
  if (t.size() > 2 && t[0] == '0' && (t[1] == 'x' || t[1] == 'X')) {
    base = 16;
    t = t.substr(2);
  } else if (t.size() > 2 && t[0] == '0' && (t[1] == 'o' || t[1] == 'O')) {
    base = 8;
    t = t.substr(2);
  }
  if (t.empty()) return false;
  for (char c : t)
    if (!(base == 16 ? std::isxdigit(static_cast<unsigned char>(c)) : (c >= '0' && c <= (base == 8 ? '7' : '9')) || c == '_'))
      return false;
  std::string clean;
  for (char c : t)
    if (c != '_') clean.push_back(c);
  p = clean.c_str();
  long long x = std::strtoll(p, &end, base);
  if (*end) return false;
  *v = neg ? -x : x;
  return true;
}

bool IsFloat(const std::string& s, double* v) {
  if (s.empty()) return false;
  std::string l;
  for (char c : s) l.push_back(static_cast<char>(std::tolower(static_cast<unsigned char>(c))));
  if (l == ".inf" || l == "+.inf") { *v = 1e308 * 10; return true; }
  if (l == "-.inf") { *v = -1e308 * 10; return true; }
  bool digit = false, dot_or_exp = false;
  for (char c : l) {
    if (std::isdigit(static_cast<unsigned char>(c))) digit = true;
    else if (c == '.' || c == 'e') dot_or_exp = true;
    else if (c != '+' && c != '-') return false;
  }
  if (!digit || !dot_or_exp) return false;
  char* end = nullptr;
  *v = std::strtod(s.c_str(), &end);
  return *end == 0;
}

std::string Unquote(const std::string& s, int lineno) {
  if (s.size() < 2) throw YamlError("line " + std::to_string(lineno) + ": bad quoted scalar");
  const char q = s[0];
  std::string out;
  for (size_t i = 1; i + 1 < s.size(); ++i) {
    char c = s[i];
    if (q == '\'' && c == '\'' && i + 2 < s.size() && s[i + 1] == '\'') {
      out.push_back('\'');
      ++i;
    } else if (q == '"' && c == '\\' && i + 2 < s.size()) {
      char e = s[++i];
      switch (e) {
        case 'n': out.push_back('\n'); break;
        case 't': out.push_back('\t'); break;
        case 'r': out.push_back('\r'); break;
        case '0': out.push_back('\0'); break;
        case '\\': out.push_back('\\'); break;
        case '"': out.push_back('"'); break;
        case '/': out.push_back('/'); break;
        default: out.push_back('\\'); out.push_back(e);
      }
    } else {
      out.push_back(c);
    }
  }
  return out;
}

// ---------------------------------------------------------------------------------- flow parser
struct Flow {
  const std::string& s;
  size_t i;
  int lineno;
  void ws() {
    while (i < s.size() && std::isspace(static_cast<unsigned char>(s[i]))) ++i;
  }
  [[noreturn]] void fail(const std::string& m) { throw YamlError("line " + std::to_string(lineno) + ": " + m); }
  Json value(const char* stops) {
    ws();
    if (i >= s.size()) fail("unexpected end of flow collection");
    if (s[i] == '[') {
      ++i;
      Json a = Json::array();
      ws();
      if (i < s.size() && s[i] == ']') { ++i; return a; }
      while (true) {
        a.push_back(value(",]"));
        ws();
        if (i < s.size() && s[i] == ',') { ++i; ws(); if (i < s.size() && s[i] == ']') { ++i; return a; } continue; }
        if (i < s.size() && s[i] == ']') { ++i; return a; }
        fail("expected , or ] in flow sequence");
      }
    }
    if (s[i] == '{') {
      ++i;
      Json o = Json::object();
      ws();
      if (i < s.size() && s[i] == '}') { ++i; return o; }
      while (true) {
        Json k = value(":,}");
        ws();
        Json v;
        if (i < s.size() && s[i] == ':') { ++i; v = value(",}"); }
        o[k.is_string() ? k.as_string() : k.dump()] = v;
        ws();
        if (i < s.size() && s[i] == ',') { ++i; ws(); if (i < s.size() && s[i] == '}') { ++i; return o; } continue; }
        if (i < s.size() && s[i] == '}') { ++i; return o; }
        fail("expected , or } in flow mapping");
      }
    }
    if (s[i] == '"' || s[i] == '\'') {
      const char q = s[i];
      size_t j = i + 1;
      while (j < s.size()) {
        if (q == '"' && s[j] == '\\') { j += 2; continue; }
        if (s[j] == q) {
          if (q == '\'' && j + 1 < s.size() && s[j + 1] == '\'') { j += 2; continue; }
          break;
        }
        ++j;
      }
      if (j >= s.size()) fail("unterminated quoted scalar");
      Json out(Unquote(s.substr(i, j - i + 1), lineno));
      i = j + 1;
      return out;
    }
    size_t j = i;
    while (j < s.size()) {
      bool stop = false;
      for (const char* p = stops; *p; ++p)
        if (s[j] == *p && (*p != ':' || j + 1 >= s.size() || std::isspace(static_cast<unsigned char>(s[j + 1])))) stop = true;
      if (stop) break;
      ++j;
    }
    Json out = YamlScalar(Trim(s.substr(i, j - i)));
    i = j;
    return out;
  }
};

// ---------------------------------------------------------------------------------- block parser
class Parser {
 public:
  explicit Parser(const std::string& text) {
    std::stringstream ss(text);
    std::string raw;
    int no = 0;
    while (std::getline(ss, raw)) {
      ++no;
      if (!raw.empty() && raw.back() == '\r') raw.pop_back();
      size_t ind = 0;
      while (ind < raw.size() && raw[ind] == ' ') ++ind;
      if (ind < raw.size() && raw[ind] == '\t') throw YamlError("line " + std::to_string(no) + ": tab indentation");
      std::string t = RTrim(StripComment(raw.substr(ind)));
      all_.push_back(Line{static_cast<int>(ind), t, raw, no});
    }
    for (size_t k = 0; k < all_.size(); ++k)
      if (!all_[k].text.empty() && all_[k].text != "---" && all_[k].text != "...") idx_.push_back(k);
  }

  Json Document() {
    if (idx_.empty()) return Json();
    pos_ = 0;
    Json v = Block(lines(0).indent);
    if (pos_ < idx_.size()) throw YamlError("line " + std::to_string(lines(pos_).no) + ": unexpected indentation");
    return v;
  }

 private:
  Line& lines(size_t p) { return all_[idx_[p]]; }

  static bool IsSeqItem(const std::string& t) { return t == "-" || (t.size() > 1 && t[0] == '-' && t[1] == ' '); }

  // position of the "key: " separator in a block-mapping line, or npos
  static size_t KeySep(const std::string& t) {
    char q = 0;
    int depth = 0;
    for (size_t i = 0; i < t.size(); ++i) {
      char c = t[i];
      if (q) {
        if (c == '\\' && q == '"') ++i;
        else if (c == q) q = 0;
        continue;
      }
      if ((c == '"' || c == '\'') && i == 0) { q = c; continue; }
      if (c == '[' || c == '{') ++depth;
      if (c == ']' || c == '}') --depth;
      if (c == ':' && depth == 0 && (i + 1 == t.size() || t[i + 1] == ' ')) return i;
    }
    return std::string::npos;
  }

  Json Block(int indent) {
    const Line& l = lines(pos_);
    if (IsSeqItem(l.text)) return Sequence(indent);
    if (KeySep(l.text) != std::string::npos) return Mapping(indent);
    // a lone scalar (document is a scalar, or a multi-line flow collection)
    std::string t = l.text;
    ++pos_;
    return Inline(t, l.no, indent);
  }

  // an inline value; joins following deeper lines when a flow collection is still open
  Json Inline(std::string t, int no, int indent) {
    if (!t.empty() && (t[0] == '[' || t[0] == '{')) {
      auto balanced = [](const std::string& s) {
        int d = 0;
        char q = 0;
        for (size_t i = 0; i < s.size(); ++i) {
          char c = s[i];
          if (q) { if (c == '\\' && q == '"') ++i; else if (c == q) q = 0; continue; }
          if (c == '"' || c == '\'') q = c;
          else if (c == '[' || c == '{') ++d;
          else if (c == ']' || c == '}') --d;
        }
        return d <= 0;
      };
      while (!balanced(t) && pos_ < idx_.size() && lines(pos_).indent > indent - 1) {
        t += " " + lines(pos_).text;
        ++pos_;
      }
      Flow f{t, 0, no};
      Json v = f.value("");
      f.ws();
      if (f.i != t.size()) f.fail("trailing characters after flow collection");
      return v;
    }
    if (!t.empty() && (t[0] == '"' || t[0] == '\'')) {
      Flow f{t, 0, no};
      Json v = f.value("");
      f.ws();
      if (f.i != t.size()) f.fail("trailing characters after quoted scalar");
      return v;
    }
    return YamlScalar(t);
  }

  Json BlockScalar(const std::string& head, int parent_indent) {
    const bool folded = head[0] == '>';
    const bool keep = head.find('+') != std::string::npos, strip = head.find('-') != std::string::npos;
    std::vector<std::string> body;
    int ind = -1;
    size_t k = pos_ < idx_.size() ? idx_[pos_] : all_.size();
    // raw lines until a non-blank line at indentation <= parent_indent
    size_t start = (pos_ > 0 ? idx_[pos_ - 1] + 1 : 0);
    (void)k;
    size_t r = start;
    for (; r < all_.size(); ++r) {
      const std::string& raw = all_[r].raw;
      const std::string t = Trim(raw);
      if (t.empty()) { body.push_back(""); continue; }
      if (all_[r].indent <= parent_indent) break;
      if (ind < 0) ind = all_[r].indent;
      body.push_back(raw.size() > static_cast<size_t>(ind) ? raw.substr(ind) : "");
    }
    while (pos_ < idx_.size() && idx_[pos_] < r) ++pos_;
    while (!body.empty() && body.back().empty()) body.pop_back();
    std::string out;
    for (size_t i = 0; i < body.size(); ++i) {
      if (i) out += (folded && !body[i].empty() && !body[i - 1].empty()) ? " " : "\n";
      out += body[i];
    }
    if (!strip && !out.empty()) out += "\n";
    (void)keep;
    return Json(out);
  }

  Json Value(const std::string& rest, int no, int indent) {
    if (rest.empty()) {
      // nested block: deeper indentation, or a sequence at the same indentation as the key
      if (pos_ < idx_.size() && (lines(pos_).indent > indent || (lines(pos_).indent == indent && IsSeqItem(lines(pos_).text))))
        return Block(lines(pos_).indent);
      return Json();
    }
    if (rest[0] == '|' || rest[0] == '>') return BlockScalar(rest, indent);
    return Inline(rest, no, indent + 1);
  }

  Json Mapping(int indent) {
    Json o = Json::object();
    while (pos_ < idx_.size() && lines(pos_).indent == indent && !IsSeqItem(lines(pos_).text)) {
      const Line l = lines(pos_);
      size_t sep = KeySep(l.text);
      if (sep == std::string::npos) throw YamlError("line " + std::to_string(l.no) + ": expected 'key: value'");
      std::string key = Trim(l.text.substr(0, sep));
      if (!key.empty() && (key[0] == '"' || key[0] == '\'')) key = Unquote(key, l.no);
      std::string rest = Trim(l.text.substr(sep + 1));
      ++pos_;
      o[key] = Value(rest, l.no, indent);
    }
    if (pos_ < idx_.size() && lines(pos_).indent > indent)
      throw YamlError("line " + std::to_string(lines(pos_).no) + ": unexpected indentation");
    return o;
  }

  Json Sequence(int indent) {
    Json a = Json::array();
    while (pos_ < idx_.size() && lines(pos_).indent == indent && IsSeqItem(lines(pos_).text)) {
      Line& l = lines(pos_);
      std::string rest = l.text == "-" ? "" : l.text.substr(2);
      size_t lead = 0;
      while (lead < rest.size() && rest[lead] == ' ') ++lead;
      rest = rest.substr(lead);
      if (rest.empty()) {
        ++pos_;
        if (pos_ < idx_.size() && lines(pos_).indent > indent) a.push_back(Block(lines(pos_).indent));
        else a.push_back(Json());
        continue;
      }
      if (IsSeqItem(rest) || (KeySep(rest) != std::string::npos && rest[0] != '[' && rest[0] != '{')) {
        // "- key: v" / "- - x": the item is a block whose first line starts after the dash
        const int inner = indent + 2 + static_cast<int>(lead);
        l.indent = inner;
        l.text = rest;
        a.push_back(Block(inner));
        continue;
      }
      ++pos_;
      if (rest[0] == '|' || rest[0] == '>') a.push_back(BlockScalar(rest, indent));
      else a.push_back(Inline(rest, l.no, indent + 1));
    }
    return a;
  }

  std::vector<Line> all_;
  std::vector<size_t> idx_;
  size_t pos_ = 0;
};

void Leaves(const Json& j, const std::string& prefix, std::vector<std::string>* out) {
  if (j.is_object()) {
    for (auto& kv : j.as_object()) Leaves(kv.second, prefix.empty() ? kv.first : prefix + "." + kv.first, out);
  } else if (!prefix.empty()) {
    out->push_back(prefix);
  }
}

std::string EnvName(const std::string& path) {
  std::string n = "DET_";
  for (char c : path) n.push_back(c == '.' || c == '-' ? '_' : static_cast<char>(std::toupper(static_cast<unsigned char>(c))));
  return n;
}

}  // namespace

Json YamlScalar(const std::string& text) {
  const std::string t = Trim(text);
  if (t.empty() || t == "~" || t == "null" || t == "Null" || t == "NULL") return Json();
  if (t[0] == '"' || t[0] == '\'') return Json(Unquote(t, 0));
  std::string l;
  for (char c : t) l.push_back(static_cast<char>(std::tolower(static_cast<unsigned char>(c))));
  if (l == "true" || l == "yes" || l == "on") return Json(true);
  if (l == "false" || l == "no" || l == "off") return Json(false);
  int64_t iv;
  if (IsInt(t, &iv)) return Json(static_cast<long long>(iv));
  double dv;
  if (IsFloat(t, &dv)) return Json(dv);
  return Json(t);
}

Json ParseYaml(const std::string& text) {
  Parser p(text);
  return p.Document();
}

Json EnvOverlay(const Json& schema, const std::vector<std::string>& extra_paths,
                const std::map<std::string, std::string>& env) {
  std::vector<std::string> paths;
  Leaves(schema, "", &paths);
  paths.insert(paths.end(), extra_paths.begin(), extra_paths.end());
  Json out = Json::object();
  for (const std::string& path : paths) {
    auto it = env.find(EnvName(path));
    if (it == env.end()) continue;
    Json* cur = &out;
    std::stringstream ss(path);
    std::string part;
    std::vector<std::string> parts;
    while (std::getline(ss, part, '.')) parts.push_back(part);
    for (size_t i = 0; i + 1 < parts.size(); ++i) {
      if (!(*cur)[parts[i]].is_object()) (*cur)[parts[i]] = Json::object();
      cur = &(*cur)[parts[i]];
    }
    const std::string& v = it->second;
    // lists/maps may be given in flow syntax (DET_RESOURCE_POOLS='[a, b]')
    (*cur)[parts.back()] = (!v.empty() && (v[0] == '[' || v[0] == '{')) ? ParseYaml(v) : YamlScalar(v);
  }
  return out;
}

}  // namespace detcore
