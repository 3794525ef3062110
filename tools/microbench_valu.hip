// tools/microbench_valu.hip — per-opcode VALU issue cost on gfx950 and the clock the chip holds while issuing.
//
// Why: the roofline denominators of the integer kernels (Ed25519 / ECDSA field arithmetic, SHA) are VALU issue
// rates.  The guide (MI355X_MICROARCH.md:54,473) gives 2 cycles per wave64 VALU instruction on a SIMD-32 at
// 2.4 GHz = 78.6 T lane-ops/s; round 3 measured 34 T MAC/s and 40-45 T plain VALU/s without the clock, so the
// two could not be reconciled.  This table settles it: for every opcode the field / hash kernels issue,
// cycles per wave-instruction per SIMD at the in-kernel clock, and that clock.
//
// Each kernel: one loop of UNR x 8 copies of the opcode, in inline asm (no compiler rewriting), over 8
// independent register chains per lane (every instruction reads its chain's previous value), ITERS times.
// Occupancy: 1, 2, 4 and 8 waves per SIMD (256-lane blocks, 256 / 512 / 1024 / 2048 blocks on 256 CUs);
// the kernels use few VGPRs so every level is reachable.  Lane 0 of each block stamps s_memtime (shader clock)
// and s_memrealtime (100 MHz) around the loop into a stamp buffer of its own (vector stores; no output
// value depends on them): clock = median over blocks of d(memtime) / d(memrealtime) x 100 MHz
// (MI355X_MICROARCH.md:503).  Wall time from HIP events (best of 5 after a warm-up of >= 2 s of launches).
//   cycles per wave-instruction per SIMD = wall x clock / (wave-instructions per SIMD)
//   T lane-ops/s = instructions x lanes / wall
// A second table runs dependent chains (one chain per wave, 1 wave per SIMD): latency in cycles.
//   hipcc --offload-arch=gfx950 -O3 -o tools/microbench_valu tools/microbench_valu.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define ITERS 4096
#define UNR 4

// 8 copies of one instruction in ONE asm statement (the compiler's hazard recognizer pads s_nop between separate
// asm statements it cannot see into).  Named operands: 64-bit chains X0..X7, 32-bit chains x0..x7 and h0..h7,
// loop-invariant y, z (32-bit) and Y (64-bit).
#define C8(F) F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7)
#define OPS                                                                                                       \
    [X0] "+v"(X[0]), [X1] "+v"(X[1]), [X2] "+v"(X[2]), [X3] "+v"(X[3]), [X4] "+v"(X[4]), [X5] "+v"(X[5]),         \
        [X6] "+v"(X[6]), [X7] "+v"(X[7]), [x0] "+v"(x[0]), [x1] "+v"(x[1]), [x2] "+v"(x[2]), [x3] "+v"(x[3]),     \
        [x4] "+v"(x[4]), [x5] "+v"(x[5]), [x6] "+v"(x[6]), [x7] "+v"(x[7]), [h0] "+v"(h[0]), [h1] "+v"(h[1]),     \
        [h2] "+v"(h[2]), [h3] "+v"(h[3]), [h4] "+v"(h[4]), [h5] "+v"(h[5]), [h6] "+v"(h[6]), [h7] "+v"(h[7])
#define INS [y] "v"(y), [z] "v"(z), [Y] "v"(Y)
#define SCLOB "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55"
#define RUN(F) asm volatile(C8(F) : OPS : INS : SCLOB)
#define XN(n) "%[x" #n "]"
#define HN(n) "%[h" #n "]"
#define WN(n) "%[X" #n "]"
#define F_ADD(n) "v_add_u32 " XN(n) ", " XN(n) ", %[y]\n\t"
#define F_XOR(n) "v_xor_b32 " XN(n) ", " XN(n) ", %[y]\n\t"
#define F_AND(n) "v_and_b32 " XN(n) ", " XN(n) ", %[y]\n\t"
#define F_SUB(n) "v_sub_u32 " XN(n) ", " XN(n) ", %[y]\n\t"
#define F_ADD3(n) "v_add3_u32 " XN(n) ", " XN(n) ", %[y], %[z]\n\t"
#define F_LSHLADD(n) "v_lshl_add_u32 " XN(n) ", " XN(n) ", 3, %[y]\n\t"
#define F_LSHL(n) "v_lshlrev_b32 " XN(n) ", 3, " XN(n) "\n\t"
#define F_ALIGN(n) "v_alignbit_b32 " XN(n) ", %[y], " XN(n) ", 26\n\t"
#define F_BFE(n) "v_bfe_u32 " XN(n) ", " XN(n) ", 3, 26\n\t"
#define F_MOV(n) "v_mov_b32 " XN(n) ", %[y]\n\t"
#define F_CND(n) "v_cndmask_b32 " XN(n) ", " XN(n) ", %[y], vcc\n\t"
#define F_MULU24(n) "v_mul_u32_u24 " XN(n) ", " XN(n) ", %[y]\n\t"
#define F_MADU24(n) "v_mad_u32_u24 " XN(n) ", " XN(n) ", %[y], %[z]\n\t"
#define F_MULLO(n) "v_mul_lo_u32 " XN(n) ", " XN(n) ", %[y]\n\t"
#define F_MULHI(n) "v_mul_hi_u32 " XN(n) ", " XN(n) ", %[y]\n\t"
#define F_MAC(n) "v_mad_u64_u32 " WN(n) ", s[40:41], %[y], %[z], " WN(n) "\n\t"
#define F_SHR64(n) "v_lshrrev_b64 " WN(n) ", 1, " WN(n) "\n\t"
#define F_SHL64(n) "v_lshlrev_b64 " WN(n) ", 1, " WN(n) "\n\t"
#define F_ADD64(n) "v_lshl_add_u64 " WN(n) ", " WN(n) ", 0, %[Y]\n\t"
#define F_MOV64(n) "v_mov_b64 " WN(n) ", %[Y]\n\t"
#define F_ADDCO(n) "v_add_co_u32 " XN(n) ", s[40:41], " XN(n) ", %[y]\n\t"
#define F_FMA(n) "v_fma_f32 " XN(n) ", %[y], %[z], " XN(n) "\n\t"
#define F_PKFMA(n) "v_pk_fma_f32 " WN(n) ", %[Y], %[Y], " WN(n) "\n\t"
#define F_MAC_ADD(n) F_MAC(n) F_ADD(n)
#define F_MAC_ADD2(n) F_MAC(n) F_ADD(n) "v_xor_b32 " HN(n) ", " HN(n) ", %[z]\n\t"
#define F_MAC_SHR(n) F_MAC(n) "v_lshrrev_b64 " WN(n) ", 1, " WN(n) "\n\t"
#define F_CNDE(n) "v_cndmask_b32_e64 " XN(n) ", " XN(n) ", %[y], s[40:41]\n\t"
#define F_CNDE_VCC(n) "v_cndmask_b32_e64 " XN(n) ", " XN(n) ", %[y], vcc\n\t"
#define F_CND32_MAC(n) "v_cndmask_b32_e32 " XN(n) ", " XN(n) ", %[y], vcc\n\t" F_MAC(n) F_MAC(n) F_MAC(n)
#define F_BFI(n) "v_bfi_b32 " XN(n) ", %[z], " XN(n) ", %[y]\n\t"
#define F_BITOP3(n) "v_bitop3_b32 " XN(n) ", " XN(n) ", %[y], %[z] bitop3:0x96\n\t"
#define F_OR3(n) "v_or3_b32 " XN(n) ", " XN(n) ", %[y], %[z]\n\t"
#define F_PERM(n) "v_perm_b32 " XN(n) ", " XN(n) ", %[y], %[z]\n\t"
#define F_LSHR32(n) "v_lshrrev_b32 " XN(n) ", 3, " XN(n) "\n\t"
#define F_MAX(n) "v_max_u32 " XN(n) ", " XN(n) ", %[y]\n\t"
#define F_ANDOR(n) "v_and_or_b32 " XN(n) ", " XN(n) ", %[y], %[z]\n\t"
#define F_OR(n) "v_or_b32 " XN(n) ", " XN(n) ", %[y]\n\t"
#define F_ADD_SHL(n) F_ADD(n) "v_lshlrev_b32 " HN(n) ", 3, " HN(n) "\n\t"
#define F_ADD_XOR(n) F_ADD(n) "v_xor_b32 " HN(n) ", " HN(n) ", %[z]\n\t"
// a 64-bit add as the 32-bit pair: 8 add_co (lo words x, carries to 8 SGPR pairs), then 8 addc (hi words h)
// reading them 8 instructions later (no hazard padding needed)
#define SP0 "s[40:41]"
#define SP1 "s[42:43]"
#define SP2 "s[44:45]"
#define SP3 "s[46:47]"
#define SP4 "s[48:49]"
#define SP5 "s[50:51]"
#define SP6 "s[52:53]"
#define SP7 "s[54:55]"
#define F_ACO(n) "v_add_co_u32 " XN(n) ", " SP##n ", " XN(n) ", %[y]\n\t"
#define F_ACC(n) "v_addc_co_u32 " HN(n) ", " SP##n ", " HN(n) ", %[z], " SP##n "\n\t"

enum Op {
    OP_ADD_U32, OP_XOR_B32, OP_AND_B32, OP_ADD3_U32, OP_LSHL_ADD_U32, OP_LSHLREV_B32, OP_ALIGNBIT, OP_BFE_U32,
    OP_MOV_B32, OP_CNDMASK, OP_SUB_U32, OP_MUL_U32_U24, OP_MAD_U32_U24, OP_MUL_LO_U32, OP_MUL_HI_U32,
    OP_MAD_U64_U32, OP_LSHRREV_B64, OP_LSHLREV_B64, OP_LSHL_ADD_U64, OP_MOV_B64, OP_ADD_CO_U32, OP_ADD_ADDC_PAIR,
    OP_FMA_F32, OP_PK_FMA_F32, OP_MAC_ADD_11, OP_MAC_ADD_12, OP_MAC_SHIFT64_11, OP_CND_E64, OP_CND_VCCSET, OP_CMP_CND,
    OP_BITOP3, OP_OR3, OP_PERM, OP_LSHRREV_B32, OP_MAX_U32, OP_AND_OR, OP_OR_B32, OP_ADD_SHL_11, OP_ADD_XOR_11, OP_CMP_CND_E32, OP_CND_E64_VCC, OP_CND_E32_MAC, OP_BFI, OP_COUNT
};
struct OpInfo {
    const char* name;
    int per_copy;   // instructions per copy (the pair ops issue 2)
};
static const OpInfo kOps[OP_COUNT] = {
    {"v_add_u32", 1},       {"v_xor_b32", 1},         {"v_and_b32", 1},          {"v_add3_u32", 1},
    {"v_lshl_add_u32", 1},  {"v_lshlrev_b32", 1},     {"v_alignbit_b32", 1},     {"v_bfe_u32", 1},
    {"v_mov_b32", 1},       {"v_cndmask_b32", 1},     {"v_sub_u32", 1},          {"v_mul_u32_u24", 1},
    {"v_mad_u32_u24", 1},   {"v_mul_lo_u32", 1},      {"v_mul_hi_u32", 1},       {"v_mad_u64_u32", 1},
    {"v_lshrrev_b64", 1},   {"v_lshlrev_b64", 1},     {"v_lshl_add_u64", 1},     {"v_mov_b64", 1},
    {"v_add_co_u32", 1},    {"v_add_co+v_addc_co", 2}, {"v_fma_f32", 1},         {"v_pk_fma_f32", 1},
    {"mad_u64 + add_u32 1:1", 2}, {"mad_u64 + 2 add_u32", 3}, {"mad_u64 + lshrrev_b64 1:1", 2},
    {"v_cndmask_b32_e64 s-mask", 1}, {"v_cndmask_b32 vcc (set)", 1}, {"v_cmp + 8 cndmask_e64", 1},
    {"v_bitop3_b32", 1}, {"v_or3_b32", 1}, {"v_perm_b32", 1}, {"v_lshrrev_b32", 1}, {"v_max_u32", 1},
    {"v_and_or_b32", 1}, {"v_or_b32", 1}, {"add_u32 + lshlrev_b32 1:1", 2}, {"add_u32 + xor_b32 1:1", 2},
    {"v_cmp vcc + 8 cndmask_e32", 1}, {"v_cndmask_b32_e64 vcc", 1}, {"cndmask_e32 vcc + 3 mad 1:3", 4},
    {"v_bfi_b32", 1},
};

template <int OP>
__device__ __forceinline__ void step(uint32_t (&x)[8], uint32_t (&h)[8], uint64_t (&X)[8], uint32_t y, uint32_t z,
                                     uint64_t Y) {
    if constexpr (OP == OP_ADD_U32) RUN(F_ADD);
    else if constexpr (OP == OP_XOR_B32) RUN(F_XOR);
    else if constexpr (OP == OP_AND_B32) RUN(F_AND);
    else if constexpr (OP == OP_SUB_U32) RUN(F_SUB);
    else if constexpr (OP == OP_ADD3_U32) RUN(F_ADD3);
    else if constexpr (OP == OP_LSHL_ADD_U32) RUN(F_LSHLADD);
    else if constexpr (OP == OP_LSHLREV_B32) RUN(F_LSHL);
    else if constexpr (OP == OP_ALIGNBIT) RUN(F_ALIGN);
    else if constexpr (OP == OP_BFE_U32) RUN(F_BFE);
    else if constexpr (OP == OP_MOV_B32) RUN(F_MOV);
    else if constexpr (OP == OP_CNDMASK) RUN(F_CND);
    else if constexpr (OP == OP_MUL_U32_U24) RUN(F_MULU24);
    else if constexpr (OP == OP_MAD_U32_U24) RUN(F_MADU24);
    else if constexpr (OP == OP_MUL_LO_U32) RUN(F_MULLO);
    else if constexpr (OP == OP_MUL_HI_U32) RUN(F_MULHI);
    else if constexpr (OP == OP_MAD_U64_U32) RUN(F_MAC);
    else if constexpr (OP == OP_LSHRREV_B64) RUN(F_SHR64);
    else if constexpr (OP == OP_LSHLREV_B64) RUN(F_SHL64);
    else if constexpr (OP == OP_LSHL_ADD_U64) RUN(F_ADD64);
    else if constexpr (OP == OP_MOV_B64) RUN(F_MOV64);
    else if constexpr (OP == OP_ADD_CO_U32) RUN(F_ADDCO);
    else if constexpr (OP == OP_ADD_ADDC_PAIR) asm volatile(C8(F_ACO) C8(F_ACC) : OPS : INS : SCLOB);
    else if constexpr (OP == OP_FMA_F32) RUN(F_FMA);
    else if constexpr (OP == OP_PK_FMA_F32) RUN(F_PKFMA);
    else if constexpr (OP == OP_MAC_ADD_11) RUN(F_MAC_ADD);
    else if constexpr (OP == OP_MAC_ADD_12) RUN(F_MAC_ADD2);
    else if constexpr (OP == OP_MAC_SHIFT64_11) RUN(F_MAC_SHR);
    else if constexpr (OP == OP_CND_E64) asm volatile("s_mov_b64 s[40:41], exec\n\t" C8(F_CNDE) : OPS : INS : SCLOB);
    else if constexpr (OP == OP_CND_VCCSET) asm volatile("s_mov_b64 vcc, exec\n\t" C8(F_CND) : OPS : INS : SCLOB, "vcc");
    else if constexpr (OP == OP_CMP_CND)
        asm volatile("v_cmp_gt_u32 s[40:41], %[y], %[x0]\n\ts_nop 1\n\t" C8(F_CNDE) : OPS : INS : SCLOB);
    else if constexpr (OP == OP_BITOP3) RUN(F_BITOP3);
    else if constexpr (OP == OP_OR3) RUN(F_OR3);
    else if constexpr (OP == OP_PERM) RUN(F_PERM);
    else if constexpr (OP == OP_LSHRREV_B32) RUN(F_LSHR32);
    else if constexpr (OP == OP_MAX_U32) RUN(F_MAX);
    else if constexpr (OP == OP_AND_OR) RUN(F_ANDOR);
    else if constexpr (OP == OP_OR_B32) RUN(F_OR);
    else if constexpr (OP == OP_ADD_SHL_11) RUN(F_ADD_SHL);
    else if constexpr (OP == OP_ADD_XOR_11) RUN(F_ADD_XOR);
    else if constexpr (OP == OP_CMP_CND_E32)
        asm volatile("v_cmp_gt_u32 vcc, %[y], %[x0]\n\ts_nop 1\n\t" C8(F_CND) : OPS : INS : SCLOB, "vcc");
    else if constexpr (OP == OP_CND_E64_VCC)
        asm volatile("v_cmp_gt_u32 vcc, %[y], %[x0]\n\ts_nop 1\n\t" C8(F_CNDE_VCC) : OPS : INS : SCLOB, "vcc");
    else if constexpr (OP == OP_CND_E32_MAC)
        asm volatile("v_cmp_gt_u32 vcc, %[y], %[x0]\n\ts_nop 1\n\t" C8(F_CND32_MAC) : OPS : INS : SCLOB, "vcc");
    else if constexpr (OP == OP_BFI) RUN(F_BFI);
}

template <int OP>
__global__ void __launch_bounds__(256) k_op(uint64_t* out, uint32_t seed, unsigned long long* stamps) {
    uint32_t x[8], h[8];
    uint64_t X[8];
    const uint32_t y = seed * 2654435761u + threadIdx.x, z = y ^ 0x9e3779b9u;
    const uint64_t Y = ((uint64_t)z << 32) | y;
#pragma unroll
    for (int c = 0; c < 8; c++) {
        x[c] = y + c * 977u;
        h[c] = z + c * 131u;
        X[c] = Y + c;
    }
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int u = 0; u < UNR; u++) step<OP>(x, h, X, y, z, Y);
    }
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) s ^= x[c] ^ h[c] ^ X[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// dependent chain: one chain per lane (latency), same opcode
template <int OP>
__global__ void __launch_bounds__(64) k_dep(uint64_t* out, uint32_t seed, unsigned long long* stamps) {
    uint32_t x = seed + threadIdx.x, y = x * 3u + 1u, z = y ^ 0x55u;
    uint64_t X = ((uint64_t)z << 32) | x, Y = X ^ 0x1234567ull;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
#define C4(F) F F F F
#define C32(F) C4(C4(F)) C4(C4(F))
    for (int i = 0; i < ITERS; i++) {
        if constexpr (OP == OP_ADD_U32) asm volatile(C32("v_add_u32 %0, %0, %1\n\t") : "+v"(x) : "v"(y));
        else if constexpr (OP == OP_MUL_LO_U32) asm volatile(C32("v_mul_lo_u32 %0, %0, %1\n\t") : "+v"(x) : "v"(y));
        else if constexpr (OP == OP_MAD_U64_U32)
            asm volatile(C32("v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n\t") : "+v"(X) : "v"(y), "v"(z) : "s40", "s41");
        else if constexpr (OP == OP_LSHRREV_B64) asm volatile(C32("v_lshrrev_b64 %0, 1, %0\n\t") : "+v"(X));
        else if constexpr (OP == OP_LSHL_ADD_U64) asm volatile(C32("v_lshl_add_u64 %0, %0, 0, %1\n\t") : "+v"(X) : "v"(Y));
    }
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x ^ X;
}

typedef void (*kfn)(uint64_t*, uint32_t, unsigned long long*);

struct Meas {
    float ms;
    double ghz;
};

static Meas run(kfn k, int blocks, int threads, uint64_t* d, unsigned long long* st, unsigned long long* hst) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 1u, st);
    float best = 1e9f;
    double ghz = 0;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(a, 0);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 2u + r, st);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) {
            best = ms;
            hipMemcpy(hst, st, (size_t)blocks * 16, hipMemcpyDeviceToHost);
            std::vector<double> f;
            for (int i = 0; i < blocks; i++)
                if (hst[2 * i + 1]) f.push_back((double)hst[2 * i] / (double)hst[2 * i + 1] * 0.1);   // GHz
            std::sort(f.begin(), f.end());
            ghz = f.empty() ? 0 : f[f.size() / 2];
        }
    }
    hipEventDestroy(a);
    hipEventDestroy(b);
    return {best, ghz};
}

template <int OP>
static void row(uint64_t* d, unsigned long long* st, unsigned long long* hst, int cus) {
    printf("%-26s", kOps[OP].name);
    for (int wps : {1, 2, 4, 8}) {
        const int blocks = cus * wps;   // 256-lane blocks: 4 waves per block = one per SIMD
        const Meas m = run(k_op<OP>, blocks, 256, d, st, hst);
        const double winstr = (double)ITERS * UNR * 8 * kOps[OP].per_copy;   // per wave
        const double waves_per_simd = wps;
        const double cyc = m.ms * 1e-3 * m.ghz * 1e9 / (winstr * waves_per_simd);
        const double tops = winstr * 64.0 * blocks * 4 / (m.ms * 1e-3) / 1e12;
        printf(" | %2dw %6.3fms %4.2fGHz %5.2fcyc %6.2fT", wps, m.ms, m.ghz, cyc, tops);
    }
    printf("\n");
}

template <int OP>
static void dep_row(const char* name, uint64_t* d, unsigned long long* st, unsigned long long* hst, int cus) {
    const Meas m = run(k_dep<OP>, cus * 4, 64, d, st, hst);   // one wave per SIMD
    const double instr = (double)ITERS * 32;
    printf("%-26s dependent chain: %6.3f ms at %4.2f GHz = %5.2f cycles per instruction\n", name, m.ms, m.ghz,
           m.ms * 1e-3 * m.ghz * 1e9 / instr);
}

int main(int argc, char** argv) {
    const bool only_new = argc > 1 && (!strcmp(argv[1], "new") || !strcmp(argv[1], "newest"));
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int maxb = cus * 8;
    uint64_t* d;
    unsigned long long *st, *hst;
    if (hipMalloc(&d, (size_t)maxb * 256 * 8) != hipSuccess || hipMalloc(&st, (size_t)maxb * 16) != hipSuccess) return 1;
    hst = (unsigned long long*)malloc((size_t)maxb * 16);
    printf("# %s, %d CUs; %d iterations x %d x 8 copies per wave; columns per occupancy (waves per SIMD): wall, in-kernel "
           "clock (median s_memtime / s_memrealtime), cycles per wave-instruction per SIMD, T lane-ops/s\n",
           p.name, cus, ITERS, UNR);
    // warm the clock up: >= 2 s of back-to-back launches (MI355X_MICROARCH.md:503)
    {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a, 0);
        float ms = 0;
        while (ms < 2000.f) {
            for (int i = 0; i < 50; i++) hipLaunchKernelGGL(k_op<OP_MAD_U64_U32>, dim3(maxb), dim3(256), 0, 0, d, 7u, st);
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
        }
        hipEventDestroy(a);
        hipEventDestroy(b);
    }
    if (!only_new) {
    row<OP_ADD_U32>(d, st, hst, cus);
    row<OP_XOR_B32>(d, st, hst, cus);
    row<OP_AND_B32>(d, st, hst, cus);
    row<OP_SUB_U32>(d, st, hst, cus);
    row<OP_ADD3_U32>(d, st, hst, cus);
    row<OP_LSHL_ADD_U32>(d, st, hst, cus);
    row<OP_LSHLREV_B32>(d, st, hst, cus);
    row<OP_ALIGNBIT>(d, st, hst, cus);
    row<OP_BFE_U32>(d, st, hst, cus);
    row<OP_MOV_B32>(d, st, hst, cus);
    row<OP_CNDMASK>(d, st, hst, cus);
    row<OP_MUL_U32_U24>(d, st, hst, cus);
    row<OP_MAD_U32_U24>(d, st, hst, cus);
    row<OP_MUL_LO_U32>(d, st, hst, cus);
    row<OP_MUL_HI_U32>(d, st, hst, cus);
    row<OP_MAD_U64_U32>(d, st, hst, cus);
    row<OP_LSHRREV_B64>(d, st, hst, cus);
    row<OP_LSHLREV_B64>(d, st, hst, cus);
    row<OP_LSHL_ADD_U64>(d, st, hst, cus);
    row<OP_MOV_B64>(d, st, hst, cus);
    row<OP_ADD_CO_U32>(d, st, hst, cus);
    row<OP_ADD_ADDC_PAIR>(d, st, hst, cus);
    row<OP_FMA_F32>(d, st, hst, cus);
    row<OP_PK_FMA_F32>(d, st, hst, cus);
    row<OP_MAC_ADD_11>(d, st, hst, cus);
    row<OP_MAC_ADD_12>(d, st, hst, cus);
    row<OP_MAC_SHIFT64_11>(d, st, hst, cus);
    }
    const bool only_newest = argc > 1 && !strcmp(argv[1], "newest");
    if (!only_newest) {
    row<OP_CND_E64>(d, st, hst, cus);
    row<OP_CND_VCCSET>(d, st, hst, cus);
    row<OP_CMP_CND>(d, st, hst, cus);
    row<OP_BITOP3>(d, st, hst, cus);
    row<OP_OR3>(d, st, hst, cus);
    row<OP_PERM>(d, st, hst, cus);
    row<OP_LSHRREV_B32>(d, st, hst, cus);
    row<OP_MAX_U32>(d, st, hst, cus);
    row<OP_AND_OR>(d, st, hst, cus);
    row<OP_OR_B32>(d, st, hst, cus);
    row<OP_ADD_SHL_11>(d, st, hst, cus);
    row<OP_ADD_XOR_11>(d, st, hst, cus);
    }
    row<OP_CMP_CND_E32>(d, st, hst, cus);
    row<OP_CND_E64_VCC>(d, st, hst, cus);
    row<OP_CND_E32_MAC>(d, st, hst, cus);
    row<OP_BFI>(d, st, hst, cus);
    if (!only_new) {
    dep_row<OP_ADD_U32>("v_add_u32", d, st, hst, cus);
    dep_row<OP_MUL_LO_U32>("v_mul_lo_u32", d, st, hst, cus);
    dep_row<OP_MAD_U64_U32>("v_mad_u64_u32", d, st, hst, cus);
    dep_row<OP_LSHRREV_B64>("v_lshrrev_b64", d, st, hst, cus);
    dep_row<OP_LSHL_ADD_U64>("v_lshl_add_u64", d, st, hst, cus);
    }
    hipError_t e = hipDeviceSynchronize();
    printf("%s\n", hipGetErrorString(e));
    hipFree(d);
    hipFree(st);
    free(hst);
    return e != hipSuccess;
}
