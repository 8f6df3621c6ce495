#pragma once

#include <cstdint>
#include <string>

namespace pz {
// json.dumps(nested list, indent=4) text of a strided float64 array at nesting `level`
std::string format_json_array(const double* data, const int64_t* shape, const int64_t* strides, int ndim,
                              int64_t level);
// Python float.__repr__ of x (json.dumps spelling for NaN / Infinity)
std::string repr_double(double x);
}  // namespace pz
