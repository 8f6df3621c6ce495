// Host/device-shared plain types of the pz kernels (safe to include from g++ translation units).
#pragma once

#include <stdint.h>

namespace pz {

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_TANH = 3 };

// stage epilogue spec, passed by value inside kernel argument structs
struct EpiSpec {
  int act;            // Act applied between the two dropouts
  int drop_pre;       // layer id of the dropout right after the producing op, -1 = none
  int drop_post;      // layer id of the dropout after the activation, -1 = none
  uint32_t seed_lo, seed_hi;
  uint32_t thresh16;  // drop element iff its 16-bit draw < thresh16  (thresh16 = round(p * 65536))
  float scale;        // 1 / (1 - p)
  float inv_scale;    // (1 - p)
  int drop_all;       // p >= 1: every element is dropped
};

}  // namespace pz
