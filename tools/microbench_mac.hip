// tools/microbench_mac.hip — the v_mad_u64_u32 (32x32+64 -> 64 MAC) issue rate on gfx950 and whether ordinary
// VALU work issues beside it.  Every kernel runs at full occupancy (2048 blocks x 256 lanes, few VGPRs) with C
// independent MAC chains per lane, so the number is throughput, not latency:
//   mac<C>        C chains of acc = lo(acc) * b + acc                       (1 MAC per step, no other VALU)
//   mac_alu<K>    4 MAC chains + K ordinary VALU ops per MAC, each reading that MAC's result (add / xor / add3 /
//                 lshl_add into accumulators of their own, so none folds)
//   alu<K>        the same K ops per step without the MACs (the chains step by an add instead)
// If the MAC pipe co-issued with ordinary VALU, mac_alu<K> would take max(mac, alu<K>); issuing from one pipe it
// takes their sum.  Prints ms, MAC/s and VALU instr/s (lane-ops) per kernel; the instruction counts of every loop
// body are read from the ISA by tools/microbench_mac_isa.py (the table below uses them).
//   hipcc --offload-arch=gfx950 -O3 -o tools/microbench_mac tools/microbench_mac.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 16384

template <int C>
__global__ void __launch_bounds__(256) k_mac(uint64_t* out, uint32_t seed) {
    const uint32_t b = (seed * 3 + blockIdx.x) | 1u;
    uint64_t acc[C];
#pragma unroll
    for (int c = 0; c < C; c++) acc[c] = seed + c * 977 + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < C; c++) acc[c] = (uint64_t)(uint32_t)acc[c] * b + acc[c];
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < C; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// K ordinary VALU ops per MAC result v (hi / lo halves of the MAC), each into its own accumulator
template <int K>
__device__ __forceinline__ void alu_ops(uint32_t (&x)[4], uint64_t v) {
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    if (K >= 1) x[0] += hi;                       // v_add_u32
    if (K >= 2) x[1] ^= lo;                       // v_xor_b32
    if (K >= 3) x[2] = x[2] + lo + hi;            // v_add3_u32
    if (K >= 4) x[3] = (x[3] << 3) + hi;          // v_lshl_add_u32
}

template <int K>
__global__ void __launch_bounds__(256) k_mac_alu(uint64_t* out, uint32_t seed) {
    const uint32_t b = (seed * 3 + blockIdx.x) | 1u;
    uint64_t acc[4];
    uint32_t x[4][4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        acc[c] = seed + c * 977 + threadIdx.x;
#pragma unroll
        for (int k = 0; k < 4; k++) x[c][k] = c + k;
    }
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            acc[c] = (uint64_t)(uint32_t)acc[c] * b + acc[c];
            alu_ops<K>(x[c], acc[c]);
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) s ^= acc[c] ^ x[c][0] ^ x[c][1] ^ x[c][2] ^ x[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the same ALU ops without MACs: a 64-bit value stepped by two ops per chain (lo += b, hi ^= lo)
template <int K>
__global__ void __launch_bounds__(256) k_alu(uint64_t* out, uint32_t seed) {
    const uint32_t b = (seed * 3 + blockIdx.x) | 1u;
    uint32_t lo[4], hi[4];
    uint32_t x[4][4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        lo[c] = seed + c * 977 + threadIdx.x;
        hi[c] = lo[c] ^ b;
#pragma unroll
        for (int k = 0; k < 4; k++) x[c][k] = c + k;
    }
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            lo[c] += b;
            hi[c] ^= lo[c];
            alu_ops<K>(x[c], ((uint64_t)hi[c] << 32) | lo[c]);
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) s ^= lo[c] ^ x[c][0] ^ x[c][1] ^ x[c][2] ^ x[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint64_t*, uint32_t);

static float run(kfn k, uint64_t* d, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 1u);   // warm
    float best = 1e9f;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(a, 0);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 2u + r);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    hipEventDestroy(a);
    hipEventDestroy(b);
    return best;
}

int main() {
    const int blocks = 2048;
    const double lanes = (double)blocks * 256 * ITERS;
    uint64_t* d;
    if (hipMalloc(&d, (size_t)blocks * 256 * 8) != hipSuccess) return 1;
    struct Row {
        const char* name;
        kfn k;
        int macs, alu;   // per lane per iteration
    } rows[] = {
        {"mac<1>", k_mac<1>, 1, 0},         {"mac<2>", k_mac<2>, 2, 0},         {"mac<4>", k_mac<4>, 4, 0},
        {"mac<8>", k_mac<8>, 8, 0},         {"mac_alu<1>", k_mac_alu<1>, 4, 4}, {"mac_alu<2>", k_mac_alu<2>, 4, 8},
        {"mac_alu<3>", k_mac_alu<3>, 4, 12}, {"mac_alu<4>", k_mac_alu<4>, 4, 16}, {"alu<1>", k_alu<1>, 0, 10},
        {"alu<2>", k_alu<2>, 0, 14},        {"alu<3>", k_alu<3>, 0, 18},        {"alu<4>", k_alu<4>, 0, 23},
    };
    printf("# %d blocks x 256 lanes x %d iterations; per-iteration counts from the ISA (tools/microbench_mac_isa.py; alu<K> includes its step ops, partly fused)\n", blocks, ITERS);
    for (const Row& r : rows) {
        const float ms = run(r.k, d, blocks);
        printf("%-12s %8.3f ms  MAC %7.2f T/s  other VALU %7.2f T/s  (per lane-iter: %d MAC, %d other)\n", r.name, ms,
               r.macs * lanes / (ms * 1e-3) / 1e12, r.alu * lanes / (ms * 1e-3) / 1e12, r.macs, r.alu);
    }
    hipError_t e = hipGetLastError();
    printf("%s\n", hipGetErrorString(e));
    hipFree(d);
    return e != hipSuccess;
}
