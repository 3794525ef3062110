// fe_radix_study.hip — the Ed25519 field radix study (SURVEY.md:343-346): GF(2^255 - 19)
// multiplication and squaring in the library's radix 2^25.5 (ten 26/25-bit limbs in 32-bit registers, 64-bit
// column sums, fe25519_dev.hpp) against radix 2^32 (eight saturated 32-bit words: the 8x32 Comba product of
// ec_dev.hpp — one v_mad_u64_u32 + one v_addc per 32x32 product — then the fold 2^256 = 38 mod p).
//
// Each kernel runs a dependent chain of `iters` operations per lane over every CU (8 waves per SIMD) and writes the
// canonical result; the host checks that both radices give the same field elements and prints the time per
// operation.  The per-operation instruction mix comes from the ISA of the same kernels (tools/loopstat.py over
// `hipcc --cuda-device-only -S` of this file: the chain loop holds exactly one operation).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../corda_amd/csrc/fe25519_dev.hpp"
#include "../corda_amd/csrc/ec_dev.hpp"

// ---- radix 2^32: t (512 bits) mod 2^255 - 19, redundant output (< 2^256) ----
CHIP_DEV void reduce_25519(u256& r, const uint32_t t[16]) {
    // u = lo + 38 hi: one v_mad_u64_u32 per word with the running carry as its 64-bit addend
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c = (uint64_t)t[8 + i] * 38u + (uint64_t)t[i] + (c >> 32);
        r.w[i] = (uint32_t)c;
    }
    // fold the top (< 39) once more: r += 38 top; a carry out of that (r within 38 * 39 of 2^256) folds 38 again
    uint32_t top = (uint32_t)(c >> 32) * 38u, cc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = __builtin_addc(r.w[i], i == 0 ? top : 0u, cc, &cc);
    r.w[0] += cc * 38u;
}
CHIP_DEV void fe32_mul(u256& r, const u256& a, const u256& b) {
    uint32_t t[16];
    mul_512(t, a, b);
    reduce_25519(r, t);
}
CHIP_DEV void fe32_sq(u256& r, const u256& a) {
    uint32_t t[16];
    sqr_512(t, a);
    reduce_25519(r, t);
}
// canonical value of a redundant element (< 2^256 < 3p): subtract p while >= p
CHIP_DEV void fe32_canon(uint32_t out[8], const u256& a) {
    static const uint32_t P[8] = {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                                  0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu};
    u256 x = a;
    for (int k = 0; k < 2; k++) {
        u256 y;
        const uint32_t br = u256_sub(y, x, P);
        if (!br) x = y;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = x.w[i];
}

// inputs: 8 words per lane (< p), two operands
__global__ void __launch_bounds__(256) k_mul25(uint32_t n, const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                               uint32_t iters) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n) return;
    fe x, y;
    fe_frombytes(x, in + 16 * l);
    fe_frombytes(y, in + 16 * l + 8);
#pragma unroll 1
    for (uint32_t i = 0; i < iters; i++) fe_mul(x, x, y);
    fe_tobytes(out + 8 * l, x);
}
__global__ void __launch_bounds__(256) k_sq25(uint32_t n, const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                              uint32_t iters) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n) return;
    fe x;
    fe_frombytes(x, in + 16 * l);
#pragma unroll 1
    for (uint32_t i = 0; i < iters; i++) fe_sq(x, x);
    fe_tobytes(out + 8 * l, x);
}
__global__ void __launch_bounds__(256) k_mul32(uint32_t n, const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                               uint32_t iters) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n) return;
    u256 x, y;
    u256_from_c(x, in + 16 * l);
    u256_from_c(y, in + 16 * l + 8);
#pragma unroll 1
    for (uint32_t i = 0; i < iters; i++) fe32_mul(x, x, y);
    fe32_canon(out + 8 * l, x);
}
__global__ void __launch_bounds__(256) k_sq32(uint32_t n, const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                              uint32_t iters) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n) return;
    u256 x;
    u256_from_c(x, in + 16 * l);
#pragma unroll 1
    for (uint32_t i = 0; i < iters; i++) fe32_sq(x, x);
    fe32_canon(out + 8 * l, x);
}

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

int main(int argc, char** argv) {
    const uint32_t n = 256 * 4 * 64 * 8;   // 8 waves per SIMD on 256 CUs
    const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 512;
    std::vector<uint32_t> h(16 * (size_t)n);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (auto& w : h) {
        s ^= s << 13, s ^= s >> 7, s ^= s << 17;
        w = (uint32_t)s;
    }
    for (uint32_t l = 0; l < 2 * n; l++) h[8 * l + 7] &= 0x7fffffffu;   // < 2^255 (and < p with overwhelming odds)
    uint32_t *din, *d25, *d32;
    CK(hipMalloc(&din, h.size() * 4));
    CK(hipMalloc(&d25, (size_t)n * 32));
    CK(hipMalloc(&d32, (size_t)n * 32));
    CK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const uint32_t blocks = n / 256;
    struct K {
        const char* name;
        void (*f)(uint32_t, const uint32_t*, uint32_t*, uint32_t);
        uint32_t* out;
    } ks[] = {{"mul radix 2^25.5", k_mul25, d25}, {"mul radix 2^32  ", k_mul32, d32},
              {"sq  radix 2^25.5", k_sq25, d25}, {"sq  radix 2^32  ", k_sq32, d32}};
    std::vector<uint32_t> r25(8 * (size_t)n), r32(8 * (size_t)n);
    for (int q = 0; q < 4; q++) {
        for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(ks[q].f, dim3(blocks), dim3(256), 0, 0, n, din, ks[q].out, 8u);
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(ks[q].f, dim3(blocks), dim3(256), 0, 0, n, din, ks[q].out, iters);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        // wave-operations per SIMD: n / 64 waves over 1024 SIMDs, `iters` operations each
        const double ns_per_op_per_simd = best * 1e6 / ((double)n / 64 / 1024 * iters);
        printf("%s: %.3f ms for %u lanes x %u = %.2f ns per wave-operation per SIMD (%.0f cycles at 2.4 GHz), %.1f G ops/s\n",
               ks[q].name, best, n, iters, ns_per_op_per_simd, ns_per_op_per_simd * 2.4, (double)n * iters / (best * 1e-3) / 1e9);
        if (q == 1 || q == 3) {
            CK(hipMemcpy(r25.data(), d25, r25.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(r32.data(), d32, r32.size() * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < r25.size(); i++) bad += r25[i] != r32[i];
            printf("  %s: radix 2^32 result %s radix 2^25.5 (%zu differing words)\n", q == 1 ? "mul" : "sq",
                   bad ? "DIFFERS FROM" : "equals", bad);
            if (bad) return 2;
        }
    }
    return 0;
}
