// Minimal JSON value / parser / serializer for the control plane (configs, protocol messages,
// searcher events, the embedded store).  Objects keep keys sorted (std::map), matching Go's
// encoding/json map marshalling, which the reference relies on for deterministic hparam order.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace detcore {

class Json {
 public:
  enum class Type { Null, Bool, Int, Double, String, Array, Object };
  using Array = std::vector<Json>;
  using Object = std::map<std::string, Json>;

  Json() : type_(Type::Null) {}
  Json(std::nullptr_t) : type_(Type::Null) {}
  Json(bool b) : type_(Type::Bool), b_(b) {}
  Json(int v) : type_(Type::Int), i_(v) {}
  Json(long v) : type_(Type::Int), i_(v) {}
  Json(long long v) : type_(Type::Int), i_(v) {}
  Json(unsigned v) : type_(Type::Int), i_(v) {}
  Json(unsigned long v) : type_(Type::Int), i_(static_cast<int64_t>(v)) {}
  Json(unsigned long long v) : type_(Type::Int), i_(static_cast<int64_t>(v)) {}
  Json(double d) : type_(Type::Double), d_(d) {}
  Json(const char* s) : type_(Type::String), s_(std::make_shared<std::string>(s)) {}
  Json(std::string s) : type_(Type::String), s_(std::make_shared<std::string>(std::move(s))) {}
  Json(Array a) : type_(Type::Array), a_(std::make_shared<Array>(std::move(a))) {}
  Json(Object o) : type_(Type::Object), o_(std::make_shared<Object>(std::move(o))) {}

  static Json array() { return Json(Array{}); }
  static Json object() { return Json(Object{}); }

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_int() const { return type_ == Type::Int; }
  bool is_double() const { return type_ == Type::Double; }
  bool is_number() const { return type_ == Type::Int || type_ == Type::Double; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }

  bool as_bool() const;
  int64_t as_int() const;      // doubles with integral value are accepted
  double as_double() const;    // ints are widened
  const std::string& as_string() const;
  const Array& as_array() const;
  Array& as_array();
  const Object& as_object() const;
  Object& as_object();

  // object access
  bool has(const std::string& k) const;
  const Json& operator[](const std::string& k) const;  // null if missing
  Json& operator[](const std::string& k);              // inserts (converts null to object)
  const Json& at(const std::string& k) const;          // throws if missing
  // typed getters with defaults
  int64_t get_int(const std::string& k, int64_t dflt) const;
  double get_double(const std::string& k, double dflt) const;
  bool get_bool(const std::string& k, bool dflt) const;
  std::string get_string(const std::string& k, const std::string& dflt) const;

  // array access
  size_t size() const;
  const Json& operator[](size_t i) const;
  Json& operator[](size_t i);
  void push_back(Json v);

  std::string dump(int indent = -1) const;
  static Json parse(const std::string& text);

  bool operator==(const Json& o) const;
  bool operator!=(const Json& o) const { return !(*this == o); }

  // deep copy (values share storage copy-on-assign semantics otherwise)
  Json clone() const;

 private:
  void dump_to(std::string& out, int indent, int level) const;
  void detach();
  Type type_;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0;
  std::shared_ptr<std::string> s_;
  std::shared_ptr<Array> a_;
  std::shared_ptr<Object> o_;
};

class JsonError : public std::runtime_error {
 public:
  explicit JsonError(const std::string& m) : std::runtime_error(m) {}
};

// Shortest round-trip formatting of a double as Go's encoding/json does (no NaN/Inf: null).
std::string format_double(double d);

}  // namespace detcore
