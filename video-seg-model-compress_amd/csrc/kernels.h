// Internal (non-ABI) launchers shared between the kernel translation units.
#pragma once
#include "common.h"

namespace drnmi {
// Small-channel LDS-patch conv (patch_conv.hip); returns drnmi_status / hipError_t.
int patch_conv_dispatch(const drnmi_conv_args& p, hipStream_t s);
}  // namespace drnmi
