#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace pz {
// json.dumps(nested list, indent=4) text of a strided float64 array at nesting `level`
std::string format_json_array(const double* data, const int64_t* shape, const int64_t* strides, int ndim,
                              int64_t level);
// Python float.__repr__ of x (json.dumps spelling for NaN / Infinity)
std::string repr_double(double x);
// Checkpoint reader: copies the JSON `text` into `skeleton`, except that every rectangular
// numeric array inside the top-level member `key` is replaced by the string "@@PZ_ARRAY_<k>@@"
// and its numbers (correctly rounded, Python json spelling incl. NaN/Infinity) appended to
// `values`; `shapes` receives [ndim, d0, d1, ...] per lifted array. Throws on malformed input.
void scan_json_arrays(const std::string& text, const std::string& key, std::string& skeleton,
                      std::vector<double>& values, std::vector<int64_t>& shapes);
// Metadata reader: the top-level object of [data, data+n) with the VALUES of the top-level
// members named in `keys` replaced by null — skipped structurally (bracket depth, string
// escapes), never parsed, so a multi-GB "layers" member costs one linear byte scan.
std::string json_null_keys(const char* data, size_t n, const std::vector<std::string>& keys);
}  // namespace pz
