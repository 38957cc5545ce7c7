// kernels_consts.h -- layout constants shared by kernels, host planner and the test emulation.
#pragma once
#include "dl_common.h"

namespace mi {
constexpr uint32_t CB_BYTES_STRIDE = KMAX / 8;   // 768 bytes per code-block output row
}  // namespace mi
