// atomic_bench.hip — cost of the access patterns the notary commit is built from, 10M lanes, one random
// address per lane (hash of the lane index): a 64-B line read, a returning 32- / 64-bit CAS, a returning
// atomicOr into a bitmap, a 4-B plain store, over footprints from L2-sized to HBM-sized.  Speed only; the
// numbers feed DESIGN.md §3 (why the claim is where it is).
//   hipcc --offload-arch=gfx950 -O3 -o tools/atomic_bench tools/atomic_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ uint32_t mix(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

// mode 0: read the 64-B line; 1: u32 CAS(0 -> i) at line start; 2: u64 CAS at word 14 of the line;
// 3: atomicOr of one bit (footprint = bitmap bytes); 4: plain u32 store; 5: read line + u64 CAS (the lookup)
__global__ void k(int mode, uint64_t n, uint32_t* base, uint64_t lines_mask, uint32_t salt, uint32_t* sink) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t l = (uint64_t)(mix((uint32_t)i ^ salt) ^ ((uint64_t)mix((uint32_t)i + salt) << 7)) & lines_mask;
    uint32_t acc = 0;
    if (mode == 0 || mode == 5) {
        const uint4* p = reinterpret_cast<const uint4*>(base + l * 16);
        const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
        acc = a.x ^ b.y ^ c.z ^ d.w;
        if (mode == 5) {
            unsigned long long* w = reinterpret_cast<unsigned long long*>(base + l * 16 + 14);
            acc ^= (uint32_t)atomicCAS(w, ((unsigned long long)d.w << 32) | d.z, ((unsigned long long)salt << 32) | (i + 1));
        }
    } else if (mode == 1) {
        acc = atomicCAS(base + l * 16, 0u, (uint32_t)i + 1);
    } else if (mode == 2) {
        acc = (uint32_t)atomicCAS(reinterpret_cast<unsigned long long*>(base + l * 16 + 14), 0ull, (unsigned long long)i + 1);
    } else if (mode == 3) {
        acc = atomicOr(base + (l >> 5), 1u << (l & 31));
    } else if (mode == 4) {
        base[l] = (uint32_t)i;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const uint64_t n = 10000000;
    const size_t big = 4ull << 30;   // 4 GiB
    uint32_t* base;
    uint32_t* sink;
    hipMalloc(&base, big);
    hipMalloc(&sink, 64);
    hipMemset(base, 0, big);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[] = {"read64", "cas32", "cas64@w14", "or-bit", "store32", "read64+cas64"};
    const size_t foot[] = {8ull << 20, 32ull << 20, 128ull << 20, 512ull << 20, 2048ull << 20, 4096ull << 20};
    for (int mode = 0; mode < 6; mode++) {
        for (size_t f : foot) {
            // modes 0-2, 5 address 64-B lines; 3 addresses bits (footprint in bytes = bits / 8); 4 addresses words
            uint64_t units = mode == 3 ? f * 8 : (mode == 4 ? f / 4 : f / 64);
            uint64_t mask = units - 1;
            float best = 1e9f;
            for (int rep = 0; rep < 4; rep++) {
                hipMemsetAsync(base, 0, f, 0);
                hipEventRecord(e0, 0);
                hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, mode, n, base, mask, 0x9e3779b9u * (rep + 1), sink);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep && ms < best) best = ms;
            }
            printf("%-14s footprint %5zu MiB  %.3f ms  (%.2f G ops/s)\n", names[mode], f >> 20, best, n / (best * 1e6));
        }
    }
    hipError_t e = hipGetLastError();
    printf("%s\n", hipGetErrorString(e));
    return e != hipSuccess;
}
