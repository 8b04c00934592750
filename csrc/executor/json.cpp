#include "json.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>

namespace bee {

namespace {

const Json kNull;

struct Parser {
  const std::string& s;
  size_t i = 0;

  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json: ") + what + " at offset " + std::to_string(i));
  }
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  bool lit(const char* w) {
    size_t n = strlen(w);
    if (s.compare(i, n, w) == 0) {
      i += n;
      return true;
    }
    return false;
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (i + 4 > s.size()) fail("short \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else fail("bad hex digit");
    }
    return v;
  }
  std::string str() {
    if (s[i] != '"') fail("expected string");
    ++i;
    std::string out;
    while (true) {
      if (i >= s.size()) fail("unterminated string");
      char c = s[i++];
      if (c == '"') break;
      if (c != '\\') {
        out += c;
        continue;
      }
      if (i >= s.size()) fail("bad escape");
      char e = s[i++];
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
            i += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }
  Json value(int depth) {
    if (depth > 200) fail("nesting too deep");
    ws();
    if (i >= s.size()) fail("unexpected end");
    char c = s[i];
    if (c == '{') {
      ++i;
      Json::Object o;
      ws();
      if (i < s.size() && s[i] == '}') { ++i; return Json(std::move(o)); }
      while (true) {
        ws();
        std::string k = str();
        ws();
        if (i >= s.size() || s[i] != ':') fail("expected ':'");
        ++i;
        o[k] = value(depth + 1);
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == '}') { ++i; break; }
        fail("expected ',' or '}'");
      }
      return Json(std::move(o));
    }
    if (c == '[') {
      ++i;
      Json::Array a;
      ws();
      if (i < s.size() && s[i] == ']') { ++i; return Json(std::move(a)); }
      while (true) {
        a.push_back(value(depth + 1));
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == ']') { ++i; break; }
        fail("expected ',' or ']'");
      }
      return Json(std::move(a));
    }
    if (c == '"') return Json(str());
    if (lit("true")) return Json(true);
    if (lit("false")) return Json(false);
    if (lit("null")) return Json(nullptr);
    size_t start = i;
    if (s[i] == '-') ++i;
    while (i < s.size() && (isdigit((unsigned char)s[i]) || s[i] == '.' || s[i] == 'e' || s[i] == 'E' || s[i] == '+' || s[i] == '-')) ++i;
    if (start == i) fail("unexpected character");
    char* end = nullptr;
    std::string num = s.substr(start, i - start);
    double d = strtod(num.c_str(), &end);
    if (!end || *end != '\0') fail("bad number");
    return Json(d);
  }
};

}  // namespace

Json Json::parse(const std::string& text) {
  Parser p{text};
  Json v = p.value(0);
  p.ws();
  if (p.i != text.size()) p.fail("trailing characters");
  return v;
}

const std::string& Json::as_string() const {
  static const std::string empty;
  return is_string() ? *s_ : empty;
}
const Json::Array& Json::as_array() const {
  static const Array empty;
  return is_array() ? *a_ : empty;
}
const Json::Object& Json::as_object() const {
  static const Object empty;
  return is_object() ? *o_ : empty;
}
Json::Array& Json::mut_array() {
  if (!is_array()) { type_ = Type::Array; a_ = std::make_shared<Array>(); }
  return *a_;
}
Json::Object& Json::mut_object() {
  if (!is_object()) { type_ = Type::Object; o_ = std::make_shared<Object>(); }
  return *o_;
}
const Json& Json::operator[](const std::string& key) const {
  if (!is_object()) return kNull;
  auto it = o_->find(key);
  return it == o_->end() ? kNull : it->second;
}
Json& Json::set(const std::string& key, Json v) {
  auto& o = mut_object();
  o[key] = std::move(v);
  return *this;
}
bool Json::has(const std::string& key) const { return is_object() && o_->count(key) > 0; }

void json_escape(const std::string& s, std::string& out) {
  out += '"';
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
          snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += (char)c;
        }
    }
  }
  out += '"';
}

void Json::dump_to(std::string& out) const {
  switch (type_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Number: {
      if (std::isfinite(n_) && n_ == std::floor(n_) && std::fabs(n_) < 9.0e15) {
        out += std::to_string((int64_t)n_);
      } else if (!std::isfinite(n_)) {
        out += "null";
      } else {
        char buf[32];
        snprintf(buf, sizeof buf, "%.17g", n_);
        out += buf;
      }
      break;
    }
    case Type::String: json_escape(*s_, out); break;
    case Type::Array: {
      out += '[';
      bool first = true;
      for (const auto& v : *a_) {
        if (!first) out += ',';
        first = false;
        v.dump_to(out);
      }
      out += ']';
      break;
    }
    case Type::Object: {
      out += '{';
      bool first = true;
      for (const auto& kv : *o_) {
        if (!first) out += ',';
        first = false;
        json_escape(kv.first, out);
        out += ':';
        kv.second.dump_to(out);
      }
      out += '}';
      break;
    }
  }
}

std::string Json::dump() const {
  std::string out;
  dump_to(out);
  return out;
}

}  // namespace bee
