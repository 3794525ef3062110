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

// Wave-level aggregation of per-key counters.  Lanes with `valid` set and equal `key` form a group;
// every member learns its group's leader lane and its rank inside the group, the leader also the
// group size.  One atomic per distinct key per wave instead of one per lane: a batch signed by a
// single notary key would otherwise serialize on one address.  The loop is wave-uniform.  (Capping
// it at a few rounds and letting the rest of the lanes use one atomic each measured no faster on
// the 4,096-key cfg2 batch: the atomics, not the ballot rounds, set the time.)
CHIP_DEV void wave_group(bool valid, uint32_t key, uint32_t& leader, uint32_t& count, uint32_t& rank) {
    const uint32_t lane = __lane_id();
    uint64_t todo = __ballot(valid);
    leader = lane;
    count = 1;
    rank = 0;
    while (todo) {
        const uint32_t l = (uint32_t)__builtin_ctzll(todo);
        const uint32_t kl = __shfl(key, (int)l);
        const bool mine = valid && key == kl;
        const uint64_t m = __ballot(mine);
        if (mine) {
            leader = l;
            rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        }
        if (lane == l) count = (uint32_t)__popcll(m);
        todo &= ~m;
    }
}
