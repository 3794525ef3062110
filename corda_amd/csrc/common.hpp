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
// Exclusive prefix sum of v over the workgroup (every thread must call it; s_wave holds blockDim/64
// words of LDS); `total` = the workgroup's sum.  Lets a workgroup claim its output range with ONE
// atomic on a shared counter: same-address atomics serialize at the memory side (~13 ns each), so
// one per wave on a single counter costs ~0.2 ms per million lanes.
CHIP_DEV uint32_t block_scan_excl(uint32_t v, uint32_t* s_wave, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) s_wave[w] = x;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (uint32_t j = 0; j < nw; j++) {
        const uint32_t c = s_wave[j];
        off += j < w ? c : 0u;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return off + x - v;
}

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
