#include "common/quantity.h"

#include <limits>
#include <stdexcept>

namespace xsched {

namespace {

constexpr i128 kMaxI128 = (static_cast<i128>(1) << 126);  // guard well below overflow

i128 pow10(int e) {
  i128 r = 1;
  for (int i = 0; i < e; ++i) r *= 10;
  return r;
}

int64_t saturate(i128 v) {
  if (v > std::numeric_limits<int64_t>::max()) return std::numeric_limits<int64_t>::max();
  if (v < std::numeric_limits<int64_t>::min()) return std::numeric_limits<int64_t>::min();
  return static_cast<int64_t>(v);
}

// ceil(a / b) for b > 0.
i128 ceil_div(i128 a, i128 b) {
  i128 q = a / b;
  if ((a % b) != 0 && a > 0) q += 1;
  return q;
}

std::string i128_to_string(i128 v) {
  if (v == 0) return "0";
  bool neg = v < 0;
  unsigned __int128 u = neg ? static_cast<unsigned __int128>(-(v + 1)) + 1 : static_cast<unsigned __int128>(v);
  std::string s;
  while (u > 0) {
    s.push_back(static_cast<char>('0' + static_cast<int>(u % 10)));
    u /= 10;
  }
  if (neg) s.push_back('-');
  return std::string(s.rbegin(), s.rend());
}

}  // namespace

bool Quantity::try_parse(std::string_view s, Quantity* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[i] == '+' || s[i] == '-') {
    neg = s[i] == '-';
    ++i;
  }
  // Digits with optional single '.'.
  i128 mant = 0;
  int frac_digits = 0;
  bool seen_dot = false, seen_digit = false;
  int dropped_nonzero = 0;  // fractional digits beyond what we keep (round up)
  for (; i < s.size(); ++i) {
    char c = s[i];
    if (c >= '0' && c <= '9') {
      seen_digit = true;
      if (seen_dot) {
        if (frac_digits >= 18) {  // beyond nano even after largest suffix scale
          if (c != '0') dropped_nonzero = 1;
          continue;
        }
        ++frac_digits;
      }
      if (mant > kMaxI128 / 10) return false;
      mant = mant * 10 + (c - '0');
    } else if (c == '.') {
      if (seen_dot) return false;
      seen_dot = true;
    } else {
      break;
    }
  }
  if (!seen_digit) return false;
  std::string_view suf = s.substr(i);
  Format fmt = Format::DecimalSI;
  int dec_exp = 0;     // power of ten
  int bin_exp = 0;     // power of 1024
  if (suf.empty()) {
  } else if (suf == "n") { dec_exp = -9;
  } else if (suf == "u") { dec_exp = -6;
  } else if (suf == "m") { dec_exp = -3;
  } else if (suf == "k") { dec_exp = 3;
  } else if (suf == "M") { dec_exp = 6;
  } else if (suf == "G") { dec_exp = 9;
  } else if (suf == "T") { dec_exp = 12;
  } else if (suf == "P") { dec_exp = 15;
  } else if (suf == "E") { dec_exp = 18;
  } else if (suf == "Ki") { bin_exp = 1; fmt = Format::BinarySI;
  } else if (suf == "Mi") { bin_exp = 2; fmt = Format::BinarySI;
  } else if (suf == "Gi") { bin_exp = 3; fmt = Format::BinarySI;
  } else if (suf == "Ti") { bin_exp = 4; fmt = Format::BinarySI;
  } else if (suf == "Pi") { bin_exp = 5; fmt = Format::BinarySI;
  } else if (suf == "Ei") { bin_exp = 6; fmt = Format::BinarySI;
  } else if (suf[0] == 'e' || suf[0] == 'E') {
    fmt = Format::DecimalExponent;
    std::string_view ex = suf.substr(1);
    if (ex.empty()) return false;
    bool eneg = false;
    size_t j = 0;
    if (ex[0] == '+' || ex[0] == '-') { eneg = ex[0] == '-'; ++j; }
    if (j >= ex.size()) return false;
    int e = 0;
    for (; j < ex.size(); ++j) {
      if (ex[j] < '0' || ex[j] > '9') return false;
      e = e * 10 + (ex[j] - '0');
      if (e > 40) return false;
    }
    dec_exp = eneg ? -e : e;
  } else {
    return false;
  }
  // value = mant * 10^(dec_exp - frac_digits) * 1024^bin_exp ; nanos = value * 1e9
  int e10 = dec_exp - frac_digits + 9;
  i128 v = mant;
  for (int b = 0; b < bin_exp; ++b) {
    if (v > kMaxI128 / 1024) return false;
    v *= 1024;
  }
  if (e10 >= 0) {
    for (int k = 0; k < e10; ++k) {
      if (v > kMaxI128 / 10) return false;
      v *= 10;
    }
  } else {
    i128 d = pow10(-e10);
    i128 q = v / d;
    if (v % d != 0 || dropped_nonzero) q += 1;  // round up to nano precision
    v = q;
  }
  if (dropped_nonzero && e10 >= 0) v += 1;
  Quantity q;
  q.nanos_ = neg ? -v : v;
  q.fmt_ = fmt;
  *out = q;
  return true;
}

Quantity Quantity::parse(std::string_view s) {
  Quantity q;
  if (!try_parse(s, &q)) throw std::invalid_argument("quantities must match the regular expression: " + std::string(s));
  return q;
}

int64_t Quantity::value() const { return saturate(ceil_div(nanos_, kNano)); }
int64_t Quantity::milli_value() const { return saturate(ceil_div(nanos_, 1000000)); }

std::string Quantity::str() const {
  if (nanos_ == 0) return "0";
  Format fmt = fmt_;
  if (fmt == Format::BinarySI) {
    // Binary only for integral values with |v| >= 1024 (CanonicalizeBytes).
    if (nanos_ % kNano != 0 || (nanos_ > -1024 * static_cast<i128>(kNano) && nanos_ < 1024 * static_cast<i128>(kNano)))
      fmt = Format::DecimalSI;
  }
  if (fmt == Format::BinarySI) {
    i128 v = nanos_ / kNano;
    static const char* suf[] = {"", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
    int e = 0;
    while (e < 6 && v % 1024 == 0) {
      v /= 1024;
      ++e;
    }
    return i128_to_string(v) + suf[e];
  }
  // Decimal: find exponent (multiple of 3, >= -9) such that mantissa integral,
  // choosing the largest such exponent.
  i128 v = nanos_;
  int exp = -9;
  while (v % 1000 == 0 && exp < 18) {
    v /= 1000;
    exp += 3;
  }
  if (fmt == Format::DecimalExponent) {
    if (exp == 0) return i128_to_string(v);
    return i128_to_string(v) + "e" + std::to_string(exp);
  }
  const char* s = "";
  switch (exp) {
    case -9: s = "n"; break;
    case -6: s = "u"; break;
    case -3: s = "m"; break;
    case 0: s = ""; break;
    case 3: s = "k"; break;
    case 6: s = "M"; break;
    case 9: s = "G"; break;
    case 12: s = "T"; break;
    case 15: s = "P"; break;
    case 18: s = "E"; break;
  }
  return i128_to_string(v) + s;
}

}  // namespace xsched
