// Minimal JSON value / parser / serializer for the executor daemon's control
// plane (request bodies, responses, zygote + worker line protocol).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace bee {

class Json {
 public:
  enum class Type { Null, Bool, Number, String, Array, Object };
  using Array = std::vector<Json>;
  using Object = std::map<std::string, Json>;

  Json() = default;
  Json(std::nullptr_t) {}
  Json(bool b) : type_(Type::Bool), b_(b) {}
  Json(int v) : type_(Type::Number), n_(v) {}
  Json(int64_t v) : type_(Type::Number), n_((double)v) {}
  Json(uint64_t v) : type_(Type::Number), n_((double)v) {}
  Json(double v) : type_(Type::Number), n_(v) {}
  Json(const char* s) : type_(Type::String), s_(std::make_shared<std::string>(s)) {}
  Json(std::string s) : type_(Type::String), s_(std::make_shared<std::string>(std::move(s))) {}
  Json(Array a) : type_(Type::Array), a_(std::make_shared<Array>(std::move(a))) {}
  Json(Object o) : type_(Type::Object), o_(std::make_shared<Object>(std::move(o))) {}

  static Json object() { return Json(Object{}); }
  static Json array() { return Json(Array{}); }
  static Json parse(const std::string& text);  // throws std::runtime_error

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_number() const { return type_ == Type::Number; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }

  bool as_bool(bool dflt = false) const { return is_bool() ? b_ : dflt; }
  double as_number(double dflt = 0) const { return is_number() ? n_ : dflt; }
  int64_t as_int(int64_t dflt = 0) const { return is_number() ? (int64_t)n_ : dflt; }
  const std::string& as_string() const;
  std::string str_or(const std::string& dflt) const { return is_string() ? *s_ : dflt; }
  const Array& as_array() const;
  const Object& as_object() const;
  Array& mut_array();
  Object& mut_object();

  // object access; missing key / non-object -> null
  const Json& operator[](const std::string& key) const;
  Json& set(const std::string& key, Json v);
  bool has(const std::string& key) const;
  void push(Json v) { mut_array().push_back(std::move(v)); }

  std::string dump() const;

 private:
  void dump_to(std::string& out) const;
  Type type_ = Type::Null;
  bool b_ = false;
  double n_ = 0;
  std::shared_ptr<std::string> s_;
  std::shared_ptr<Array> a_;
  std::shared_ptr<Object> o_;
};

void json_escape(const std::string& s, std::string& out);

}  // namespace bee
