// Exact Kubernetes resource.Quantity arithmetic.
//
// Semantics follow k8s.io/apimachinery/pkg/api/resource (vendored by the
// reference at vendor/k8s.io/apimachinery/pkg/api/resource/quantity.go):
// decimal (n,u,m,k,M,G,T,P,E), binary (Ki..Ei) and exponent (1e3) suffixes;
// Value()/MilliValue() round UP; canonical string forms preserve the format
// (BinarySI / DecimalSI / DecimalExponent) of the parsed input.
//
// Representation: a signed 128-bit count of nano-units, which is exact for
// every quantity with at most 9 fractional decimal digits up to ~1.7e29.
#pragma once

#include <cstdint>
#include <string>
#include <string_view>

namespace xsched {

using i128 = __int128;

class Quantity {
 public:
  enum class Format : uint8_t { DecimalSI, BinarySI, DecimalExponent };

  Quantity() = default;
  static Quantity from_int(int64_t v, Format f = Format::DecimalSI) {
    Quantity q;
    q.nanos_ = static_cast<i128>(v) * kNano;
    q.fmt_ = f;
    return q;
  }
  static Quantity from_milli(int64_t m, Format f = Format::DecimalSI) {
    Quantity q;
    q.nanos_ = static_cast<i128>(m) * 1000000;
    q.fmt_ = f;
    return q;
  }
  // Throws std::invalid_argument on malformed input (ParseQuantity errors).
  static Quantity parse(std::string_view s);
  static bool try_parse(std::string_view s, Quantity* out);

  int64_t value() const;        // ceil to units (saturating)
  int64_t milli_value() const;  // ceil to milli-units (saturating)
  i128 nanos() const { return nanos_; }
  Format format() const { return fmt_; }
  int sign() const { return nanos_ > 0 ? 1 : nanos_ < 0 ? -1 : 0; }
  bool is_zero() const { return nanos_ == 0; }

  int cmp(const Quantity& o) const { return nanos_ < o.nanos_ ? -1 : nanos_ > o.nanos_ ? 1 : 0; }
  void add(const Quantity& o) { nanos_ += o.nanos_; }
  void sub(const Quantity& o) { nanos_ -= o.nanos_; }
  void neg() { nanos_ = -nanos_; }

  // Canonical string (Quantity.String()).
  std::string str() const;

  bool operator==(const Quantity& o) const { return nanos_ == o.nanos_; }

  static constexpr int64_t kNano = 1000000000;

 private:
  i128 nanos_ = 0;
  Format fmt_ = Format::DecimalSI;
};

}  // namespace xsched
