// Host/device-shared plain types of the pz kernels (safe to include from g++ translation units).
#pragma once

#include <stdint.h>

namespace pz {

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_TANH = 3 };

// Stage epilogue spec, passed by value inside kernel argument structs.
// Dropout masks are a pure function of (key, element index): element pair j = idx/2 draws
// bits = mix32(j ^ key); element idx uses the low (even idx) or high (odd idx) 16 bits and is
// kept iff they are >= thresh16. Keys are derived per (seed, layer id) on the host
// (ops/functional.py: layer_key), so each layer's mask is independent and the backward pass
// regenerates it instead of reading a stored mask.
struct EpiSpec {
  int act;            // Act applied between the two dropouts
  int drop_pre;       // != 0: dropout right after the producing op (key_pre)
  int drop_post;      // != 0: dropout after the activation (key_post)
  uint32_t key_pre, key_post;
  uint32_t thresh16;  // drop element iff its 16-bit draw < thresh16  (thresh16 = round(p * 65536))
  float scale;        // 1 / (1 - p)
  float inv_scale;    // (1 - p)
  double scale64;     // the same in double: fp64 kernels (fp64 models) drop out exactly like F.dropout
  double inv_scale64;
  int drop_all;       // p >= 1: every element is dropped
  // Graph-replayed steps: keys above are per (seed, layer) only and the kernel mixes in the
  // epoch read from this device counter (epoch_key). nullptr: the keys are final (eager steps
  // mix the epoch on the host with the same function, so both paths draw identical masks).
  const int* epoch_ptr;
};

}  // namespace pz
