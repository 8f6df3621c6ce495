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
#include <stdexcept>
#include <vector>

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

// ------------------------------------------------------------------------------------------
// reader: lift the numeric arrays under one top-level key out of a JSON document
// ------------------------------------------------------------------------------------------
namespace pz {
namespace {

struct Scanner {
  const char* p;
  const char* end;
  std::string& skel;
  std::vector<double>& values;
  std::vector<int64_t>& shapes;
  int64_t next_id = 0;

  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("pz::scan_json_arrays: ") + what);
  }
  // one JSON number (Python's json spelling incl. NaN / Infinity / -Infinity)
  bool number(double& out) {
    ws();
    if (p >= end) return false;
    if (end - p >= 3 && std::memcmp(p, "NaN", 3) == 0) { out = std::nan(""); p += 3; return true; }
    if (end - p >= 8 && std::memcmp(p, "Infinity", 8) == 0) { out = HUGE_VAL; p += 8; return true; }
    if (end - p >= 9 && std::memcmp(p, "-Infinity", 9) == 0) { out = -HUGE_VAL; p += 9; return true; }
    if (!(*p == '-' || (*p >= '0' && *p <= '9'))) return false;
    auto res = std::from_chars(p, end, out);  // correctly rounded, like Python's float()
    if (res.ec != std::errc()) return false;
    p = res.ptr;
    return true;
  }
  // a rectangular nested array of numbers starting at '['; false (position restored) otherwise
  bool numeric_array(std::vector<int64_t>& shape, int depth) {
    const char* start = p;
    const size_t nv = values.size();
    ws();
    if (p >= end || *p != '[') return false;
    ++p;
    ws();
    int64_t count = 0;
    std::vector<int64_t> inner;
    bool nested = false;
    if (p < end && *p == ']') {  // [] is a numeric (empty) row only inside an array
      if (depth == 0) { p = start; return false; }
      ++p;
      shape.assign(1, 0);
      return true;
    }
    while (true) {
      ws();
      if (p < end && *p == '[') {
        std::vector<int64_t> sub;
        if (!numeric_array(sub, depth + 1) || (count > 0 && (!nested || sub != inner))) {
          p = start; values.resize(nv); return false;
        }
        nested = true;
        inner = sub;
      } else {
        double v;
        if (nested || !number(v)) { p = start; values.resize(nv); return false; }
        values.push_back(v);
      }
      ++count;
      ws();
      if (p < end && *p == ',') { ++p; continue; }
      if (p < end && *p == ']') { ++p; break; }
      p = start; values.resize(nv); return false;
    }
    shape.assign(1, count);
    if (nested) shape.insert(shape.end(), inner.begin(), inner.end());
    return true;
  }
  // copy a string literal verbatim
  void string_lit() {
    const char* s = p++;
    while (p < end && *p != '"') p += (*p == '\\') ? 2 : 1;
    if (p >= end) fail("unterminated string");
    ++p;
    skel.append(s, p - s);
  }
  // copy / transform one value. Modes: COPY; IN_KEY (inside the target member: objects' "params"
  // lists switch to PARAMS); PARAMS (a list of parameters: each element is lifted); LIFT (a
  // numeric array becomes one "@@PZ_ARRAY_<k>@@" placeholder)
  enum Mode { COPY, IN_KEY, PARAMS, LIFT };
  void value(Mode mode) {
    ws();
    if (p >= end) fail("unexpected end");
    if (*p == '"') { string_lit(); return; }
    if (*p == '[') {
      if (mode == LIFT) {
        std::vector<int64_t> shape;
        if (numeric_array(shape, 0)) {
          shapes.push_back(static_cast<int64_t>(shape.size()));
          shapes.insert(shapes.end(), shape.begin(), shape.end());
          skel += "\"@@PZ_ARRAY_" + std::to_string(next_id++) + "@@\"";
          return;
        }
      }
      skel += *p++;
      ws();
      if (p < end && *p == ']') { skel += *p++; return; }
      const Mode inner = mode == PARAMS ? LIFT : mode;
      while (true) {
        value(inner);
        ws();
        if (p < end && *p == ',') { skel += *p++; continue; }
        if (p < end && *p == ']') { skel += *p++; return; }
        fail("bad array");
      }
    }
    if (*p == '{') { object(mode == COPY ? COPY : IN_KEY, false); return; }
    const char* s = p;  // number / literal: copy the token
    while (p < end && *p != ',' && *p != ']' && *p != '}' && *p != ' ' && *p != '\n' && *p != '\r' && *p != '\t') ++p;
    skel.append(s, p - s);
  }
  void object(Mode mode, bool top) {
    skel += *p++;  // '{'
    ws();
    if (p < end && *p == '}') { skel += *p++; return; }
    while (true) {
      ws();
      if (p >= end || *p != '"') fail("expected a key");
      const char* k0 = p + 1;
      string_lit();
      const std::string key(k0, p - 1 - k0);
      ws();
      if (p >= end || *p != ':') fail("expected ':'");
      skel += *p++;
      value(top && key == target ? IN_KEY : (mode == IN_KEY && key == "params") ? PARAMS : mode);
      ws();
      if (p < end && *p == ',') { skel += *p++; continue; }
      if (p < end && *p == '}') { skel += *p++; return; }
      fail("bad object");
    }
  }
  std::string target;
};

}  // namespace

void scan_json_arrays(const std::string& text, const std::string& key, std::string& skeleton,
                      std::vector<double>& values, std::vector<int64_t>& shapes) {
  skeleton.clear();
  skeleton.reserve(4096);
  Scanner sc{text.data(), text.data() + text.size(), skeleton, values, shapes};
  sc.target = key;
  sc.ws();
  if (sc.p >= sc.end || *sc.p != '{') throw std::runtime_error("pz::scan_json_arrays: top level must be an object");
  sc.object(Scanner::COPY, true);
}

namespace {

// end of the JSON string starting at p (p points at the opening quote)
const char* skip_string(const char* p, const char* end) {
  ++p;
  while (true) {
    const void* q = std::memchr(p, '"', static_cast<size_t>(end - p));
    if (q == nullptr) throw std::runtime_error("pz::json_null_keys: unterminated string");
    const char* e = static_cast<const char*>(q);
    size_t bs = 0;  // an odd run of backslashes before the quote escapes it
    for (const char* b = e - 1; b >= p && *b == '\\'; --b) ++bs;
    if ((bs & 1) == 0) return e + 1;
    p = e + 1;
  }
}

// end of the JSON value starting at p (after whitespace)
const char* skip_value(const char* p, const char* end) {
  if (p >= end) throw std::runtime_error("pz::json_null_keys: unexpected end");
  if (*p == '"') return skip_string(p, end);
  if (*p != '[' && *p != '{') {
    while (p < end && *p != ',' && *p != ']' && *p != '}' && *p != ' ' && *p != '\n' && *p != '\r' && *p != '\t') ++p;
    return p;
  }
  int depth = 0;
  while (p < end) {
    const char c = *p;
    if (c == '"') { p = skip_string(p, end); continue; }
    if (c == '[' || c == '{') ++depth;
    else if (c == ']' || c == '}') {
      if (--depth == 0) return p + 1;
    }
    ++p;
  }
  throw std::runtime_error("pz::json_null_keys: unterminated container");
}

}  // namespace

std::string json_null_keys(const char* data, size_t n, const std::vector<std::string>& keys) {
  const char* p = data;
  const char* end = data + n;
  auto ws = [&] { while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; };
  ws();
  if (p >= end || *p != '{') throw std::runtime_error("pz::json_null_keys: top level must be an object");
  std::string out;
  out.reserve(4096);
  out += '{';
  ++p;
  bool first = true;
  while (true) {
    ws();
    if (p < end && *p == '}') break;
    if (p >= end || *p != '"') throw std::runtime_error("pz::json_null_keys: expected a key");
    const char* k0 = p;
    p = skip_string(p, end);
    const std::string key(k0 + 1, p - 1 - (k0 + 1));
    ws();
    if (p >= end || *p != ':') throw std::runtime_error("pz::json_null_keys: expected ':'");
    ++p;
    ws();
    const char* v0 = p;
    p = skip_value(p, end);
    if (!first) out += ", ";
    first = false;
    out.append(k0, static_cast<size_t>(v0 - k0) - 0);  // "key": (+ any whitespace)
    bool drop = false;
    for (const auto& k : keys) drop |= k == key;
    if (drop) out += "null";
    else out.append(v0, static_cast<size_t>(p - v0));
    ws();
    if (p < end && *p == ',') { ++p; continue; }
    if (p < end && *p == '}') break;
    throw std::runtime_error("pz::json_null_keys: bad object");
  }
  out += '}';
  return out;
}

}  // namespace pz
