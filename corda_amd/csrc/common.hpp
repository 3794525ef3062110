// common.hpp — shared device/host definitions for libcordahip (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CHIP_DEV __device__ __forceinline__

#include "../../include/cordahip.h"

// Byte loads from an arbitrary (unaligned) pool offset, assembled into 32-bit words.
CHIP_DEV uint32_t ld_le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
CHIP_DEV uint32_t ld_be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

// Per-key record produced by the key-prep kernels (device-resident, SoA by field).
// scheme: CHIP_SCHEME_* or 0 (unsupported); ok: 1 when the key decodes to a curve point.
struct KeyMeta {
    uint8_t scheme;
    uint8_t ok;
    uint8_t pad[2];
};
