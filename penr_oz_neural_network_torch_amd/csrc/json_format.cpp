// N9 — native checkpoint array formatter (host C++17).
//
// Renders a float64 tensor exactly as Python's `json.dumps(t.tolist(), indent=4)` would at a
// given nesting level: shortest round-trip digits (std::to_chars), Python `float.__repr__`
// layout (fixed notation for -4 < decpt <= 16, otherwise d.ddde±XX), NaN / Infinity spelled as
// json.dumps does. The reference serialises ~46 bytes per parameter through the pure-Python
// JSON encoder at ~0.9 µs/param (neural_net_model.py:330-336); this path keeps the
// byte-identical file format at native speed.
#include "json_format.h"

#include <charconv>
#include <cmath>
#include <cstring>

namespace pz {
namespace {

void append_repr(std::string& out, double x) {
  if (std::isnan(x)) { out += "NaN"; return; }
  if (std::isinf(x)) { out += x < 0 ? "-Infinity" : "Infinity"; return; }
  if (x == 0.0) { out += std::signbit(x) ? "-0.0" : "0.0"; return; }
  char buf[48];
  auto res = std::to_chars(buf, buf + sizeof(buf), x, std::chars_format::scientific);
  *res.ptr = '\0';
  // buf: [-]d[.ddd]e(+|-)XX
  const char* p = buf;
  bool neg = false;
  if (*p == '-') { neg = true; ++p; }
  char digits[32];
  int nd = 0;
  while (*p && *p != 'e') {
    if (*p != '.') digits[nd++] = *p;
    ++p;
  }
  int exp10 = std::atoi(p + 1);
  const int decpt = exp10 + 1;
  if (neg) out += '-';
  if (decpt <= -4 || decpt > 16) {
    out += digits[0];
    if (nd > 1) { out += '.'; out.append(digits + 1, nd - 1); }
    out += 'e';
    out += exp10 < 0 ? '-' : '+';
    const int ae = exp10 < 0 ? -exp10 : exp10;
    if (ae < 10) out += '0';
    out += std::to_string(ae);
  } else if (decpt <= 0) {
    out += "0.";
    out.append(static_cast<size_t>(-decpt), '0');
    out.append(digits, nd);
  } else if (decpt >= nd) {
    out.append(digits, nd);
    out.append(static_cast<size_t>(decpt - nd), '0');
    out += ".0";
  } else {
    out.append(digits, decpt);
    out += '.';
    out.append(digits + decpt, nd - decpt);
  }
}

void append_indent(std::string& out, int64_t level) { out.append(static_cast<size_t>(4 * level), ' '); }

void render(std::string& out, const double* data, const int64_t* shape, const int64_t* strides, int ndim, int dim,
            int64_t level) {
  if (dim == ndim) { append_repr(out, *data); return; }
  const int64_t n = shape[dim];
  if (n == 0) { out += "[]"; return; }
  out += "[\n";
  for (int64_t i = 0; i < n; ++i) {
    append_indent(out, level + 1);
    render(out, data + i * strides[dim], shape, strides, ndim, dim + 1, level + 1);
    if (i + 1 < n) out += ",\n";
  }
  out += '\n';
  append_indent(out, level);
  out += ']';
}

}  // namespace

std::string format_json_array(const double* data, const int64_t* shape, const int64_t* strides, int ndim,
                              int64_t level) {
  std::string out;
  int64_t numel = 1;
  for (int d = 0; d < ndim; ++d) numel *= shape[d];
  out.reserve(static_cast<size_t>(numel) * (26 + 4 * (level + ndim)) + 16);
  render(out, data, shape, strides, ndim, 0, level);
  return out;
}

std::string repr_double(double x) {
  std::string s;
  append_repr(s, x);
  return s;
}

}  // namespace pz
