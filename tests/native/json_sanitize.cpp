// Host-only harness for csrc/json_format.cpp, built by tests/test_native_sanitize_cpu.py with
// -fsanitize=address,undefined (the checkpoint reader/writer parses untrusted files).
//
// Modes (argv[1]):
//   repr     read doubles (hex-float text, one per line) from stdin, print repr_double of each
//   roundtrip  format random strided arrays, scan them back, check every value bit-exactly
//   fuzz     feed truncated / mutated checkpoint text to scan_json_arrays and json_null_keys;
//            malformed input must throw std::exception (or parse), never touch memory it does not own
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <random>
#include <string>
#include <vector>

#include "json_format.h"

namespace {

int repr_mode() {
  std::string line;
  while (std::getline(std::cin, line)) {
    if (line.empty()) continue;
    const double x = std::strtod(line.c_str(), nullptr);
    std::cout << pz::repr_double(x) << "\n";
  }
  return 0;
}

double random_double(std::mt19937_64& g) {
  switch (g() % 8) {
    case 0: return std::ldexp(static_cast<double>(g() >> 11), -static_cast<int>(g() % 1100));  // tiny / denormal
    case 1: return -std::ldexp(static_cast<double>(g() >> 11), static_cast<int>(g() % 900));   // huge
    case 2: return static_cast<double>(static_cast<int64_t>(g() % 2000001) - 1000000);         // integers
    case 3: return (g() & 1) ? 0.0 : -0.0;
    default: {
      double d;
      uint64_t bits = g();
      std::memcpy(&d, &bits, 8);
      return std::isfinite(d) ? d : 1.5;
    }
  }
}

int roundtrip_mode() {
  std::mt19937_64 g(20261016);
  int checked = 0;
  for (int it = 0; it < 300; ++it) {
    const int ndim = 1 + static_cast<int>(g() % 3);
    std::vector<int64_t> shape(ndim), strides(ndim);
    int64_t n = 1;
    for (int d = 0; d < ndim; ++d) {
      shape[d] = 1 + static_cast<int64_t>(g() % 6);
      n *= shape[d];
    }
    // row-major strides, sometimes transposed (non-contiguous source)
    int64_t s = 1;
    for (int d = ndim - 1; d >= 0; --d) {
      strides[d] = s;
      s *= shape[d];
    }
    if (ndim == 2 && (g() & 1)) std::swap(strides[0], strides[1]), std::swap(shape[0], shape[1]);
    std::vector<double> data(n);
    for (auto& v : data) v = random_double(g);
    const std::string arr = pz::format_json_array(data.data(), shape.data(), strides.data(), ndim, 1);
    // the checkpoint shape: each layer's "params" list holds its arrays (utils/checkpoint.py)
    const std::string text = "{\n    \"layers\": [\n        {\n            \"algo\": \"linear\",\n"
                             "            \"params\": [\n                " + arr +
                             "\n            ]\n        }\n    ],\n    \"status\": \"Trained\"\n}";
    std::string skeleton;
    std::vector<double> values;
    std::vector<int64_t> shapes;
    pz::scan_json_arrays(text, "layers", skeleton, values, shapes);
    if (static_cast<int64_t>(values.size()) != n || shapes.empty() || shapes[0] != ndim) {
      std::fprintf(stderr, "roundtrip %d: %zu values for %lld, ndim %lld\n", it, values.size(), (long long)n,
                   shapes.empty() ? -1LL : (long long)shapes[0]);
      return 1;
    }
    // values come back in logical (row-major over `shape`) order
    std::vector<int64_t> idx(ndim, 0);
    for (int64_t k = 0; k < n; ++k) {
      int64_t off = 0;
      for (int d = 0; d < ndim; ++d) off += idx[d] * strides[d];
      if (std::memcmp(&values[k], &data[off], 8) != 0) {
        std::fprintf(stderr, "roundtrip %d: value %lld differs (%.17g vs %.17g)\n", it, (long long)k, values[k],
                     data[off]);
        return 1;
      }
      for (int d = ndim - 1; d >= 0; --d) {
        if (++idx[d] < shape[d]) break;
        idx[d] = 0;
      }
      ++checked;
    }
    if (skeleton.find("\"status\"") == std::string::npos || skeleton.find("\"Trained\"") == std::string::npos) {
      std::fprintf(stderr, "roundtrip %d: skeleton lost the status member\n", it);
      return 1;
    }
  }
  std::printf("roundtrip ok %d values\n", checked);
  return 0;
}

int fuzz_mode() {
  std::mt19937_64 g(7);
  const std::string base =
      "{\n    \"model_id\": \"m\\\"q\",\n    \"layers\": [\n        {\n            \"params\": [[[1.5, -2e-300, NaN], "
      "[Infinity, -Infinity, 3]], [0.25, 1e308, -0.0]]\n        }\n    ],\n    \"progress\": "
      "[{\"epoch\": 1, \"cost\": 0.5, \"note\": \"a ] b } c\"}],\n    \"training_buffer\": [[1, 2], [3, 4]],\n    "
      "\"status\": \"Training\"\n}";
  const std::string alphabet = "[]{},:\"\\ 0123456789.eE+-NaInfity\n";
  int parsed = 0, rejected = 0;
  for (int it = 0; it < 20000; ++it) {
    std::string t = base;
    const int kind = static_cast<int>(g() % 3);
    if (kind == 0) {
      t.resize(g() % (t.size() + 1));  // truncation
    } else {
      const int edits = 1 + static_cast<int>(g() % 4);
      for (int e = 0; e < edits && !t.empty(); ++e) {
        const size_t pos = g() % t.size();
        if (kind == 1) t[pos] = alphabet[g() % alphabet.size()];
        else t.erase(pos, 1 + g() % 3);
      }
    }
    try {
      std::string skeleton;
      std::vector<double> values;
      std::vector<int64_t> shapes;
      pz::scan_json_arrays(t, "layers", skeleton, values, shapes);
      ++parsed;
    } catch (const std::exception&) {
      ++rejected;
    }
    try {
      // exact-size heap copy: an overread past the end is an ASan error, not a silent read
      std::vector<char> buf(t.begin(), t.end());
      const std::string meta =
          pz::json_null_keys(buf.data(), buf.size(), {"layers", "training_buffer", "progress"});
      (void)meta;
      ++parsed;
    } catch (const std::exception&) {
      ++rejected;
    }
  }
  std::printf("fuzz ok parsed %d rejected %d\n", parsed, rejected);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "roundtrip";
  if (mode == "repr") return repr_mode();
  if (mode == "roundtrip") return roundtrip_mode();
  if (mode == "fuzz") return fuzz_mode();
  std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
  return 2;
}
