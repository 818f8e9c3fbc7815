// Minimal JSON DOM used as the wire/storage format of the object store.
//
// Kubernetes objects are JSON documents; the reference reaches them through
// client-go's typed structs (vendor/k8s.io/api/core/v1/types.go). We keep the
// document form in the store (so unknown fields, merge patches and the REST
// adapter round-trip losslessly) and parse typed views (api/types.h) out of it
// only where the scheduler needs them.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace xsched {

class Json;
using JsonPtr = std::shared_ptr<const Json>;

class JsonError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Json {
 public:
  enum class Type : uint8_t { Null, Bool, Int, Double, String, Array, Object };
  using Array = std::vector<Json>;
  using Member = std::pair<std::string, Json>;
  using Object = std::vector<Member>;  // insertion ordered; objects are small

  Json() {}
  Json(std::nullptr_t) {}
  Json(bool b) : t_(Type::Bool), i_(b) {}
  Json(int v) : t_(Type::Int), i_(v) {}
  Json(int64_t v) : t_(Type::Int), i_(v) {}
  Json(uint64_t v) : t_(Type::Int), i_(static_cast<int64_t>(v)) {}
  Json(double v) : t_(Type::Double), d_(v) {}
  Json(const char* s) { new (&h_.s) std::string(s); t_ = Type::String; }
  Json(std::string s) { new (&h_.s) std::string(std::move(s)); t_ = Type::String; }
  Json(std::string_view s) { new (&h_.s) std::string(s); t_ = Type::String; }
  Json(const Json& o) { copy_from(o); }
  Json(Json&& o) noexcept { move_from(std::move(o)); }
  // Through a temporary: `j = j["x"]` (a value assigned from inside itself)
  // is built before the old value is destroyed.
  Json& operator=(const Json& o) {
    if (this != &o) {
      Json tmp(o);
      destroy();
      move_from(std::move(tmp));
    }
    return *this;
  }
  Json& operator=(Json&& o) noexcept {
    if (this != &o) {
      Json tmp(std::move(o));
      destroy();
      move_from(std::move(tmp));
    }
    return *this;
  }
  ~Json() { destroy(); }

  static Json array() {
    Json j;
    new (&j.h_.a) Array();
    j.t_ = Type::Array;
    return j;
  }
  static Json object() {
    Json j;
    new (&j.h_.o) Object();
    j.t_ = Type::Object;
    return j;
  }

  Type type() const { return t_; }
  bool is_null() const { return t_ == Type::Null; }
  bool is_bool() const { return t_ == Type::Bool; }
  bool is_int() const { return t_ == Type::Int; }
  bool is_number() const { return t_ == Type::Int || t_ == Type::Double; }
  bool is_string() const { return t_ == Type::String; }
  bool is_array() const { return t_ == Type::Array; }
  bool is_object() const { return t_ == Type::Object; }

  bool as_bool(bool dflt = false) const { return t_ == Type::Bool ? i_ != 0 : dflt; }
  int64_t as_int(int64_t dflt = 0) const {
    if (t_ == Type::Int) return i_;
    if (t_ == Type::Double) return static_cast<int64_t>(d_);
    return dflt;
  }
  double as_double(double dflt = 0.0) const {
    if (t_ == Type::Double) return d_;
    if (t_ == Type::Int) return static_cast<double>(i_);
    return dflt;
  }
  const std::string& as_string() const;  // "" for non-strings
  std::string str_or(std::string_view dflt) const {
    return t_ == Type::String ? h_.s : std::string(dflt);
  }

  const Array& items() const;  // empty for non-arrays
  Array& items_mut();
  const Object& members() const;  // empty for non-objects
  Object& members_mut();

  size_t size() const {
    return t_ == Type::Array ? h_.a.size() : t_ == Type::Object ? h_.o.size() : 0;
  }

  // Object access. get() returns nullptr when missing / not an object.
  const Json* get(std::string_view key) const;
  Json* get_mut(std::string_view key);
  // Path lookup: get_path({"metadata","name"}).
  const Json* path(std::initializer_list<std::string_view> keys) const;
  const Json& operator[](std::string_view key) const;  // null sentinel when missing
  Json& set(std::string_view key, Json v);  // insert or replace
  Json& at_or_create(std::string_view key);  // creates an empty object if missing
  bool erase(std::string_view key);
  void push_back(Json v);

  bool operator==(const Json& o) const;
  bool operator!=(const Json& o) const { return !(*this == o); }

  std::string dump() const;
  void dump_to(std::string& out) const;
  static Json parse(std::string_view text);
  // Calls fn for each element of a top-level JSON array as it is parsed.
  static void parse_array_stream(std::string_view text, const std::function<void(Json&&)>& fn);

  // RFC 7386 JSON merge patch (the "application/merge-patch+json" patch type
  // used by the reference's util.CreateMergePatch callers).
  void merge_patch(const Json& patch);
  // Produce a merge patch that turns `from` into `to`.
  static Json diff_merge_patch(const Json& from, const Json& to);

 private:
  // Scalars live in i_/d_; a string, array or object in h_, whose one live
  // member t_ selects. A value is 48 bytes instead of the 96 that separate
  // string, array and object members took: a pod object's member scan (every
  // field lookup) and deep copy (every store write) touch half the memory.
  Type t_ = Type::Null;
  union {
    int64_t i_ = 0;
    double d_;
  };
  union Heavy {
    std::string s;
    Array a;
    Object o;
    Heavy() {}
    ~Heavy() {}
  } h_;
  void destroy() noexcept {
    switch (t_) {
      case Type::String: h_.s.~basic_string(); break;
      case Type::Array: h_.a.~Array(); break;
      case Type::Object: h_.o.~Object(); break;
      default: break;
    }
    t_ = Type::Null;
  }
  // Into a destroyed (Null) value.
  void copy_from(const Json& o) {
    switch (o.t_) {
      case Type::String: new (&h_.s) std::string(o.h_.s); break;
      case Type::Array: new (&h_.a) Array(o.h_.a); break;
      case Type::Object: new (&h_.o) Object(o.h_.o); break;
      default: i_ = o.i_; break;  // the 8 bytes of either scalar
    }
    t_ = o.t_;
  }
  void move_from(Json&& o) noexcept {
    switch (o.t_) {
      case Type::String: new (&h_.s) std::string(std::move(o.h_.s)); break;
      case Type::Array: new (&h_.a) Array(std::move(o.h_.a)); break;
      case Type::Object: new (&h_.o) Object(std::move(o.h_.o)); break;
      default: i_ = o.i_; break;
    }
    t_ = o.t_;
    o.destroy();
  }
};

inline const Json& json_null() {
  static const Json n;
  return n;
}

// Structural FNV-1a hash of a JSON value (type tags, keys, scalars; object
// members in insertion order). Members named `skip_key` at the top level are
// ignored. Used for the scheduler's pod-template equivalence classes.
uint64_t json_hash(const Json& j, uint64_t h = 1469598103934665603ULL, std::string_view skip_key = {});

}  // namespace xsched
