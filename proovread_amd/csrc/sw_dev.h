// Device-side structures of the SW (seed extension + CIGAR) stage.
#pragma once
#include <stdint.h>

namespace prgpu {
struct SwResident {
    bool loaded = false;
};
inline void sw_release(SwResident &) {}
}  // namespace prgpu
