// tools/microbench_mul.hip — issue-rate microbenchmark for the multiply instructions a
// 255/256-bit field multiplication can be built from on gfx950 (SURVEY.md §8d asks for a
// measured v_mad_u64_u32 peak).  Each lane runs independent chains (ILP 8) so the number is
// throughput, not latency.  Reports giga-ops/s chip-wide (lane-ops).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CHAINS 8

__global__ void k_mad_u64_u32(uint64_t* out, uint32_t seed) {
    uint32_t a = seed + threadIdx.x, b = seed * 3 + blockIdx.x;
    uint64_t acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = c;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) acc[c] = (uint64_t)((uint32_t)acc[c] ^ a) * (uint64_t)b + acc[c];
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_lo_u32(uint64_t* out, uint32_t seed) {
    uint32_t b = seed * 3 + blockIdx.x;
    uint32_t acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = seed + c + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) acc[c] = (acc[c] ^ (uint32_t)i) * b;   // the xor keeps the loop from folding into b^ITERS
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_hi_u32(uint64_t* out, uint32_t seed) {
    uint32_t b = seed * 3 + blockIdx.x;
    uint32_t acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = seed + c + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) acc[c] = __umulhi(acc[c] | 1u, b) + c;
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad_u24(uint64_t* out, uint32_t seed) {
    uint32_t b = (seed * 3 + blockIdx.x) & 0xffffff;
    uint32_t acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = seed + c + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) acc[c] = __umul24(acc[c], b) + acc[c];
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add_u32(uint64_t* out, uint32_t seed) {
    uint32_t b = seed * 3 + blockIdx.x;
    uint32_t acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = seed + c + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) acc[c] = (acc[c] ^ b) + c;
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma_f64(uint64_t* out, uint32_t seed) {
    double b = 1.0000001 + seed * 1e-9;
    double acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = 1.0 + c + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) acc[c] = __fma_rn(acc[c], b, 0.5);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) s += acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_fma_f32(uint64_t* out, uint32_t seed) {
    float b = 1.0000001f + seed * 1e-9f;
    float acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = 1.0f + c + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) acc[c] = __fmaf_rn(acc[c], b, 0.5f);
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) s += acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

typedef void (*kfn)(uint64_t*, uint32_t);

static double run(kfn k, const char* name, uint64_t* d, int blocks, int threads) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double ops = 5.0 * blocks * threads * (double)ITERS * CHAINS;
    double g = ops / (ms * 1e-3) / 1e9;
    printf("%-14s %10.1f Gop/s (lane-ops)  %8.3f ms\n", name, g, ms / 5);
    return g;
}

int main() {
    int blocks = 256 * 8, threads = 256;
    uint64_t* d;
    hipMalloc(&d, sizeof(uint64_t) * blocks * threads);
    run(k_add_u32, "xor+add_u32", d, blocks, threads);
    run(k_mad_u24, "mad_u32_u24", d, blocks, threads);
    run(k_mul_lo_u32, "mul_lo_u32", d, blocks, threads);
    run(k_mul_hi_u32, "mul_hi_u32", d, blocks, threads);
    run(k_mad_u64_u32, "mad_u64_u32", d, blocks, threads);
    run(k_fma_f32, "fma_f32", d, blocks, threads);
    run(k_fma_f64, "fma_f64", d, blocks, threads);
    hipFree(d);
    return 0;
}
