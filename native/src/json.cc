#include "detcore/json.h"

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>

namespace detcore {

namespace {
const Json kNull;
}

bool Json::as_bool() const {
  if (type_ != Type::Bool) throw JsonError("json: not a bool");
  return b_;
}

int64_t Json::as_int() const {
  if (type_ == Type::Int) return i_;
  if (type_ == Type::Double && std::floor(d_) == d_) return static_cast<int64_t>(d_);
  throw JsonError("json: not an int");
}

double Json::as_double() const {
  if (type_ == Type::Double) return d_;
  if (type_ == Type::Int) return static_cast<double>(i_);
  throw JsonError("json: not a number");
}

const std::string& Json::as_string() const {
  if (type_ != Type::String) throw JsonError("json: not a string");
  return *s_;
}

const Json::Array& Json::as_array() const {
  if (type_ != Type::Array) throw JsonError("json: not an array");
  return *a_;
}

Json::Array& Json::as_array() {
  if (type_ != Type::Array) throw JsonError("json: not an array");
  detach();
  return *a_;
}

const Json::Object& Json::as_object() const {
  if (type_ != Type::Object) throw JsonError("json: not an object");
  return *o_;
}

Json::Object& Json::as_object() {
  if (type_ == Type::Null) {
    type_ = Type::Object;
    o_ = std::make_shared<Object>();
  }
  if (type_ != Type::Object) throw JsonError("json: not an object");
  detach();
  return *o_;
}

void Json::detach() {
  if (a_ && a_.use_count() > 1) a_ = std::make_shared<Array>(*a_);
  if (o_ && o_.use_count() > 1) o_ = std::make_shared<Object>(*o_);
}

bool Json::has(const std::string& k) const {
  return type_ == Type::Object && o_->count(k) > 0;
}

const Json& Json::operator[](const std::string& k) const {
  if (type_ != Type::Object) return kNull;
  auto it = o_->find(k);
  return it == o_->end() ? kNull : it->second;
}

Json& Json::operator[](const std::string& k) { return as_object()[k]; }

const Json& Json::at(const std::string& k) const {
  if (type_ != Type::Object) throw JsonError("json: not an object (key " + k + ")");
  auto it = o_->find(k);
  if (it == o_->end()) throw JsonError("json: missing key " + k);
  return it->second;
}

int64_t Json::get_int(const std::string& k, int64_t dflt) const {
  const Json& v = (*this)[k];
  return v.is_number() ? v.as_int() : dflt;
}
double Json::get_double(const std::string& k, double dflt) const {
  const Json& v = (*this)[k];
  return v.is_number() ? v.as_double() : dflt;
}
bool Json::get_bool(const std::string& k, bool dflt) const {
  const Json& v = (*this)[k];
  return v.is_bool() ? v.as_bool() : dflt;
}
std::string Json::get_string(const std::string& k, const std::string& dflt) const {
  const Json& v = (*this)[k];
  return v.is_string() ? v.as_string() : dflt;
}

size_t Json::size() const {
  if (type_ == Type::Array) return a_->size();
  if (type_ == Type::Object) return o_->size();
  return 0;
}

const Json& Json::operator[](size_t i) const { return as_array().at(i); }
Json& Json::operator[](size_t i) { return as_array().at(i); }

void Json::push_back(Json v) {
  if (type_ == Type::Null) {
    type_ = Type::Array;
    a_ = std::make_shared<Array>();
  }
  as_array().push_back(std::move(v));
}

bool Json::operator==(const Json& o) const {
  if (is_number() && o.is_number()) {
    if (type_ == Type::Int && o.type_ == Type::Int) return i_ == o.i_;
    return as_double() == o.as_double();
  }
  if (type_ != o.type_) return false;
  switch (type_) {
    case Type::Null: return true;
    case Type::Bool: return b_ == o.b_;
    case Type::String: return *s_ == *o.s_;
    case Type::Array: return *a_ == *o.a_;
    case Type::Object: return *o_ == *o.o_;
    default: return false;
  }
}

Json Json::clone() const {
  Json j = *this;
  if (j.a_) {
    Array a;
    for (const auto& v : *j.a_) a.push_back(v.clone());
    j.a_ = std::make_shared<Array>(std::move(a));
  }
  if (j.o_) {
    Object o;
    for (const auto& kv : *j.o_) o.emplace(kv.first, kv.second.clone());
    j.o_ = std::make_shared<Object>(std::move(o));
  }
  return j;
}

std::string format_double(double d) {
  if (!std::isfinite(d)) return "null";
  if (d == 0) return std::signbit(d) ? "-0" : "0";
  char buf[64];
  double a = std::fabs(d);
  // Go encoding/json: 'f' format unless exponent < -6 or >= 21, shortest round-trip digits.
  std::to_chars_result r;
  if (a < 1e-6 || a >= 1e21) {
    r = std::to_chars(buf, buf + sizeof(buf), d, std::chars_format::scientific);
    std::string s(buf, r.ptr);
    // Go prints e-07 as e-07 (two-digit exponent); to_chars prints e-07 too.
    return s;
  }
  r = std::to_chars(buf, buf + sizeof(buf), d, std::chars_format::fixed);
  return std::string(buf, r.ptr);
}

namespace {

void escape_string(std::string& out, const std::string& s) {
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof(buf), "\\u%04x", c);
          out += buf;
        } else {
          out.push_back(static_cast<char>(c));
        }
    }
  }
  out.push_back('"');
}

void newline(std::string& out, int indent, int level) {
  if (indent < 0) return;
  out.push_back('\n');
  out.append(static_cast<size_t>(indent * level), ' ');
}

class Parser {
 public:
  explicit Parser(const std::string& t) : t_(t) {}
  Json parse_document() {
    ws();
    Json v = value();
    ws();
    if (p_ != t_.size()) fail("trailing characters");
    return v;
  }

 private:
  [[noreturn]] void fail(const std::string& m) {
    throw JsonError("json parse error at offset " + std::to_string(p_) + ": " + m);
  }
  void ws() {
    while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\n' || t_[p_] == '\t' || t_[p_] == '\r')) ++p_;
  }
  char peek() { return p_ < t_.size() ? t_[p_] : '\0'; }
  void expect(const char* lit) {
    size_t n = std::strlen(lit);
    if (t_.compare(p_, n, lit) != 0) fail(std::string("expected ") + lit);
    p_ += n;
  }
  Json value() {
    char c = peek();
    if (c == '{') return object();
    if (c == '[') return array();
    if (c == '"') return Json(string());
    if (c == 't') { expect("true"); return Json(true); }
    if (c == 'f') { expect("false"); return Json(false); }
    if (c == 'n') { expect("null"); return Json(); }
    if (c == 'N') { expect("NaN"); return Json(std::nan("")); }
    if (c == 'I') { expect("Infinity"); return Json(HUGE_VAL); }
    return number();
  }
  Json object() {
    Json::Object o;
    ++p_;
    ws();
    if (peek() == '}') { ++p_; return Json(std::move(o)); }
    for (;;) {
      ws();
      if (peek() != '"') fail("expected key");
      std::string k = string();
      ws();
      if (peek() != ':') fail("expected ':'");
      ++p_;
      ws();
      o[k] = value();
      ws();
      if (peek() == ',') { ++p_; continue; }
      if (peek() == '}') { ++p_; break; }
      fail("expected ',' or '}'");
    }
    return Json(std::move(o));
  }
  Json array() {
    Json::Array a;
    ++p_;
    ws();
    if (peek() == ']') { ++p_; return Json(std::move(a)); }
    for (;;) {
      ws();
      a.push_back(value());
      ws();
      if (peek() == ',') { ++p_; continue; }
      if (peek() == ']') { ++p_; break; }
      fail("expected ',' or ']'");
    }
    return Json(std::move(a));
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out.push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }
  uint32_t hex4() {
    if (p_ + 4 > t_.size()) fail("bad \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = t_[p_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string string() {
    std::string s;
    ++p_;
    for (;;) {
      if (p_ >= t_.size()) fail("unterminated string");
      char c = t_[p_++];
      if (c == '"') break;
      if (c != '\\') { s.push_back(c); continue; }
      if (p_ >= t_.size()) fail("bad escape");
      char e = t_[p_++];
      switch (e) {
        case '"': s.push_back('"'); break;
        case '\\': s.push_back('\\'); break;
        case '/': s.push_back('/'); break;
        case 'b': s.push_back('\b'); break;
        case 'f': s.push_back('\f'); break;
        case 'n': s.push_back('\n'); break;
        case 'r': s.push_back('\r'); break;
        case 't': s.push_back('\t'); break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && p_ + 6 <= t_.size() && t_[p_] == '\\' && t_[p_ + 1] == 'u') {
            p_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(s, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return s;
  }
  Json number() {
    size_t start = p_;
    bool is_float = false;
    if (peek() == '-') ++p_;
    if (peek() == 'I') { expect("Infinity"); return Json(-HUGE_VAL); }
    while (p_ < t_.size()) {
      char c = t_[p_];
      if (c >= '0' && c <= '9') { ++p_; continue; }
      if (c == '.' || c == 'e' || c == 'E' || c == '+' || (c == '-' && p_ > start)) { is_float = true; ++p_; continue; }
      break;
    }
    if (p_ == start) fail("unexpected character");
    const char* b = t_.data() + start;
    const char* e = t_.data() + p_;
    if (!is_float) {
      int64_t v = 0;
      auto r = std::from_chars(b, e, v);
      if (r.ec == std::errc() && r.ptr == e) return Json(v);
    }
    double d = 0;
    auto r = std::from_chars(b, e, d);
    if (r.ec != std::errc() || r.ptr != e) fail("bad number");
    return Json(d);
  }
  const std::string& t_;
  size_t p_ = 0;
};

}  // namespace

void Json::dump_to(std::string& out, int indent, int level) const {
  switch (type_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Int: out += std::to_string(i_); break;
    case Type::Double: out += format_double(d_); break;
    case Type::String: escape_string(out, *s_); break;
    case Type::Array: {
      out.push_back('[');
      bool first = true;
      for (const auto& v : *a_) {
        if (!first) out.push_back(',');
        first = false;
        newline(out, indent, level + 1);
        v.dump_to(out, indent, level + 1);
      }
      if (!a_->empty()) newline(out, indent, level);
      out.push_back(']');
      break;
    }
    case Type::Object: {
      out.push_back('{');
      bool first = true;
      for (const auto& kv : *o_) {
        if (!first) out.push_back(',');
        first = false;
        newline(out, indent, level + 1);
        escape_string(out, kv.first);
        out.push_back(':');
        if (indent >= 0) out.push_back(' ');
        kv.second.dump_to(out, indent, level + 1);
      }
      if (!o_->empty()) newline(out, indent, level);
      out.push_back('}');
      break;
    }
  }
}

std::string Json::dump(int indent) const {
  std::string out;
  dump_to(out, indent, 0);
  return out;
}

Json Json::parse(const std::string& text) { return Parser(text).parse_document(); }

}  // namespace detcore
