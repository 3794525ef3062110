// ec_dev.hpp — secp256r1 (P-256) and secp256k1 field, scalar and point arithmetic for gfx950.
//
// Field elements: 8 little-endian u32 words holding any value in [0, 2^256) congruent to the
// element mod p ("redundant" form: both primes exceed 2^255, so one conditional subtraction of p
// gives the canonical value).  Every operation accepts redundant inputs and returns a redundant
// output; fp_canon / fp_is_zero / fp_eq are used where the reference compares values.
//
// Multiplication: product scanning (Comba) over 32-bit limbs.  Each partial product is one
// v_mad_u64_u32 that adds into a 64-bit column accumulator and writes its carry-out to an SGPR
// pair, plus one v_addc_co_u32 that counts the carries in a third word: 2 VALU instructions per
// 32x32 product, no register moves (the compiler's own lowering of `uint64_t p = a*b + t + c`
// needs ~6 instructions per product: it zero-extends every addend through v_mov and adds in 64-bit).
// Reduction: P-256 by the NIST/Solinas word recombination (FIPS 186-4 D.2.3) with 32-bit carry
// chains; secp256k1 by folding with 2^256 = 2^32 + 977 (mod p).  Inversion: Fermat with the
// curve's fixed addition chain (255 squarings + 12 / 15 multiplications).
// Scalars mod n: Montgomery multiplication (R = 2^256): Comba product + Comba REDC.
// Points: Jacobian (X, Y, Z), Z = 0 (exactly) is the point at infinity; tables hold affine points.
#pragma once
#include "common.hpp"
#include "curve_consts.hpp"

enum { CURVE_R1 = 0, CURVE_K1 = 1 };
// Template parameter C of every routine below: the curve in bit 0, plus CURVE_ILP for the
// latency-bound callers (one wave per SIMD: the per-key doubling chains), whose multiplications
// keep all 15 Comba columns in flight instead of one 64-long dependent multiply-add chain.
#define CURVE_ILP 2
#define EC_CURVE(C) ((C) & 1)

struct u256 {
    uint32_t w[8];
};

template <int C> CHIP_DEV const ec_curve_c& curve() { return EC_CURVE(C) == CURVE_R1 ? EC_R1 : EC_K1; }

// ---------------------------------------------------------------------------------------
// multiply-accumulate with carry count: acc (64-bit column) += a * b, top += carry-out.
// gfx950 needs two wait states between a VALU write of an SGPR carry and a VALU read of it as a
// carry-in (the compiler puts s_nop 1 inside its own v_addc chains); the compiler cannot see
// inside this block, so the block carries its own s_nop.
CHIP_DEV void mac(uint64_t& acc, uint32_t& top, uint32_t a, uint32_t b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, %2, %1, 0, %2"
        : "+v"(acc), "+v"(top), "=&s"(cc)
        : "v"(a), "v"(b));
}
// three independent multiply-accumulates in one block: each v_addc reads its carry two VALU
// instructions after the v_mad that wrote it, so no s_nop is needed
CHIP_DEV void mac3(uint64_t& a0, uint32_t& t0, uint32_t x0, uint32_t y0, uint64_t& a1, uint32_t& t1, uint32_t x1,
                   uint32_t y1, uint64_t& a2, uint32_t& t2, uint32_t x2, uint32_t y2) {
    uint64_t c0, c1, c2;
    asm("v_mad_u64_u32 %0, %6, %9, %10, %0\n\t"
        "v_mad_u64_u32 %2, %7, %11, %12, %2\n\t"
        "v_mad_u64_u32 %4, %8, %13, %14, %4\n\t"
        "v_addc_co_u32_e64 %1, %6, %1, 0, %6\n\t"
        "v_addc_co_u32_e64 %3, %7, %3, 0, %7\n\t"
        "v_addc_co_u32_e64 %5, %8, %5, 0, %8"
        : "+v"(a0), "+v"(t0), "+v"(a1), "+v"(t1), "+v"(a2), "+v"(t2), "=&s"(c0), "=&s"(c1), "=&s"(c2)
        : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(x2), "v"(y2));
}
// end of a Comba column: emit the low word, shift the 96-bit accumulator down by 32
CHIP_DEV uint32_t col_next(uint64_t& acc, uint32_t& top) {
    const uint32_t lo = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
    return lo;
}

CHIP_DEV bool u256_is_zero(const u256& a) {
    return (a.w[0] | a.w[1] | a.w[2] | a.w[3] | a.w[4] | a.w[5] | a.w[6] | a.w[7]) == 0;
}
CHIP_DEV bool u256_eq(const u256& a, const u256& b) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d |= a.w[i] ^ b.w[i];
    return d == 0;
}
CHIP_DEV bool u256_eq_c(const u256& a, const uint32_t* b) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d |= a.w[i] ^ b[i];
    return d == 0;
}
// a >= b
CHIP_DEV bool u256_ge(const u256& a, const uint32_t* b) {
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) (void)__builtin_subc(a.w[i], b[i], br, &br);
    return br == 0;
}
// r = a + b, returns carry
CHIP_DEV uint32_t u256_add(u256& r, const u256& a, const uint32_t* b) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = __builtin_addc(a.w[i], b[i], c, &c);
    return c;
}
// r = a - b, returns borrow
CHIP_DEV uint32_t u256_sub(u256& r, const u256& a, const uint32_t* b) {
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = __builtin_subc(a.w[i], b[i], br, &br);
    return br;
}
CHIP_DEV void u256_from_c(u256& r, const uint32_t* c) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = c[i];
}
CHIP_DEV void u256_set_word(u256& r, uint32_t v) {
    r.w[0] = v;
#pragma unroll
    for (int i = 1; i < 8; i++) r.w[i] = 0;
}

// ---------------------------------------------------------------------------------------
// 512-bit product (16 words), Comba
CHIP_DEV void mul_512(uint32_t t[16], const u256& a, const u256& b) {
    uint64_t acc = 0;
    uint32_t top = 0;
#pragma unroll
    for (int k = 0; k < 15; k++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int j = k - i;
            if (j >= 0 && j < 8) mac(acc, top, a.w[i], b.w[j]);
        }
        t[k] = col_next(acc, top);
    }
    t[15] = (uint32_t)acc;
}
// 512-bit product with every column accumulated independently (3 products in flight), then one
// carry pass: the latency variant (CURVE_ILP)
CHIP_DEV void mul_512_ilp(uint32_t t[16], const u256& a, const u256& b) {
    uint64_t acc[15];
    uint32_t top[15];
#pragma unroll
    for (int k = 0; k < 15; k++) {
        acc[k] = 0;
        top[k] = 0;
    }
    // the 64 products in an order that keeps consecutive triples in different columns
    int q[64][2], nq = 0;
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 8; j++) {
            q[nq][0] = i;
            q[nq][1] = j;
            nq++;
        }
#pragma unroll
    for (int s = 0; s + 2 < 64; s += 3) {
        const int i0 = q[s][0], j0 = q[s][1], i1 = q[s + 1][0], j1 = q[s + 1][1], i2 = q[s + 2][0], j2 = q[s + 2][1];
        mac3(acc[i0 + j0], top[i0 + j0], a.w[i0], b.w[j0], acc[i1 + j1], top[i1 + j1], a.w[i1], b.w[j1],
             acc[i2 + j2], top[i2 + j2], a.w[i2], b.w[j2]);
    }
    mac(acc[14], top[14], a.w[7], b.w[7]);   // product 63
    uint64_t c = 0;
    uint32_t ct = 0;
#pragma unroll
    for (int k = 0; k < 15; k++) {
        // column k + carry (96 bits each)
        const uint64_t s0 = acc[k] + c;
        ct += top[k] + (s0 < c ? 1u : 0u);
        t[k] = (uint32_t)s0;
        c = (s0 >> 32) | ((uint64_t)ct << 32);
        ct = 0;
    }
    t[15] = (uint32_t)c;
}
// 512-bit square: off-diagonal products once (Comba), doubled, plus the diagonal
CHIP_DEV void sqr_512(uint32_t t[16], const u256& a) {
    uint64_t acc = 0;
    uint32_t top = 0;
    t[0] = 0;
#pragma unroll
    for (int k = 1; k < 14; k++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int j = k - i;
            if (i < j && j < 8) mac(acc, top, a.w[i], a.w[j]);
        }
        t[k] = col_next(acc, top);
    }
    t[14] = (uint32_t)acc;
    t[15] = (uint32_t)(acc >> 32);
    // double
#pragma unroll
    for (int k = 15; k > 0; k--) t[k] = __builtin_amdgcn_alignbit(t[k], t[k - 1], 31);
    t[0] = 0;
    // + diagonal: a_i^2 into words 2i, 2i+1 with a carry chain
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t sq = (uint64_t)a.w[i] * a.w[i];
        t[2 * i] = __builtin_addc(t[2 * i], (uint32_t)sq, c, &c);
        t[2 * i + 1] = __builtin_addc(t[2 * i + 1], (uint32_t)(sq >> 32), c, &c);
    }
}

// K = 2^256 - p (mod-p value of 2^256), per curve
template <int C> CHIP_DEV uint32_t kword(int i) {
    if (EC_CURVE(C) == CURVE_R1) {   // 2^224 - 2^192 - 2^96 + 1
        const uint32_t K[8] = {1u, 0u, 0u, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xfffffffeu, 0u};
        return K[i];
    } else {               // 2^32 + 977
        const uint32_t K[8] = {977u, 1u, 0u, 0u, 0u, 0u, 0u, 0u};
        return K[i];
    }
}
// r += m K (m in {0, 1} per lane), returns the carry out of 2^256
template <int C> CHIP_DEV uint32_t add_mk(u256& r, uint32_t m) {
    const uint32_t mask = 0u - m;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = __builtin_addc(r.w[i], kword<C>(i) & mask, c, &c);
    return c;
}
template <int C> CHIP_DEV uint32_t sub_mk(u256& r, uint32_t m) {
    const uint32_t mask = 0u - m;
    uint32_t b = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = __builtin_subc(r.w[i], kword<C>(i) & mask, b, &b);
    return b;
}

// secp256k1: t mod p (redundant), p = 2^256 - 2^32 - 977, 2^256 = 2^32 + 977 (mod p)
CHIP_DEV void reduce_k1(u256& r, const uint32_t t[16]) {
    // u = lo + 977 hi + (hi << 32): 9 words, each step one v_mad_u64_u32 of a 64-bit addend
    uint64_t c = 0;
    uint32_t u[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c += (uint64_t)t[i] + (i > 0 ? t[8 + i - 1] : 0u);
        c = (uint64_t)t[8 + i] * 977u + c;
        u[i] = (uint32_t)c;
        c >>= 32;
    }
    c += t[15];   // u[8] (< 2^34)
    // fold u[8] once more: + u8 977 + (u8 << 32)
    const uint32_t h = (uint32_t)c, hh = (uint32_t)(c >> 32);
    uint64_t d = (uint64_t)h * 977u + u[0];
    r.w[0] = (uint32_t)d;
    d >>= 32;
    d += (uint64_t)hh * 977u + (uint64_t)h + u[1];
    r.w[1] = (uint32_t)d;
    d >>= 32;
    uint32_t cc = 0;
    r.w[2] = __builtin_addc(u[2], (uint32_t)d + hh, 0u, &cc);   // d + hh < 2^3: no carry lost
#pragma unroll
    for (int i = 3; i < 8; i++) r.w[i] = __builtin_addc(u[i], 0u, cc, &cc);
    // carry out of 2^256 (rare): add K once more; cannot carry again
    if (cc) (void)add_mk<CURVE_K1>(r, 1u);
}

// P-256: FIPS 186-4 D.2.3 fast reduction, redundant output.
//   T + 2 S1 + 2 S2 + S3 + S4 - D1 - D2 - D3 - D4 with 32-bit carry chains and a signed top word,
//   then top * 2^256 folded as top * (2^224 - 2^192 - 2^96 + 1).
CHIP_DEV void reduce_r1(u256& r, const uint32_t c[16]) {
    uint32_t a[8];
    int32_t top;
    uint32_t cy = 0, bw = 0;
    // U = S1 + S2 = (c15, c14 + c15, c13 + c14, c12 + c13, c11 + c12, 0, 0, 0)  [word 7 .. word 0]
    uint32_t u3, u4, u5, u6, u7, ut;
    u3 = __builtin_addc(c[11], c[12], 0u, &cy);
    u4 = __builtin_addc(c[12], c[13], cy, &cy);
    u5 = __builtin_addc(c[13], c[14], cy, &cy);
    u6 = __builtin_addc(c[14], c[15], cy, &cy);
    u7 = __builtin_addc(c[15], 0u, cy, &cy);
    ut = cy;
    // a = T + 2U
    a[0] = c[0];
    a[1] = c[1];
    a[2] = c[2];
    a[3] = __builtin_addc(c[3], u3 << 1, 0u, &cy);
    a[4] = __builtin_addc(c[4], __builtin_amdgcn_alignbit(u4, u3, 31), cy, &cy);
    a[5] = __builtin_addc(c[5], __builtin_amdgcn_alignbit(u5, u4, 31), cy, &cy);
    a[6] = __builtin_addc(c[6], __builtin_amdgcn_alignbit(u6, u5, 31), cy, &cy);
    a[7] = __builtin_addc(c[7], __builtin_amdgcn_alignbit(u7, u6, 31), cy, &cy);
    top = (int32_t)(cy + ((ut << 1) | (u7 >> 31)));
    // + S3 = (c15, c14, 0, 0, 0, c10, c9, c8)
    a[0] = __builtin_addc(a[0], c[8], 0u, &cy);
    a[1] = __builtin_addc(a[1], c[9], cy, &cy);
    a[2] = __builtin_addc(a[2], c[10], cy, &cy);
    a[3] = __builtin_addc(a[3], 0u, cy, &cy);
    a[4] = __builtin_addc(a[4], 0u, cy, &cy);
    a[5] = __builtin_addc(a[5], 0u, cy, &cy);
    a[6] = __builtin_addc(a[6], c[14], cy, &cy);
    a[7] = __builtin_addc(a[7], c[15], cy, &cy);
    top += (int32_t)cy;
    // + S4 = (c8, c13, c15, c14, c13, c11, c10, c9)
    a[0] = __builtin_addc(a[0], c[9], 0u, &cy);
    a[1] = __builtin_addc(a[1], c[10], cy, &cy);
    a[2] = __builtin_addc(a[2], c[11], cy, &cy);
    a[3] = __builtin_addc(a[3], c[13], cy, &cy);
    a[4] = __builtin_addc(a[4], c[14], cy, &cy);
    a[5] = __builtin_addc(a[5], c[15], cy, &cy);
    a[6] = __builtin_addc(a[6], c[13], cy, &cy);
    a[7] = __builtin_addc(a[7], c[8], cy, &cy);
    top += (int32_t)cy;
    // - D1 = (c10, c8, 0, 0, 0, c13, c12, c11)
    a[0] = __builtin_subc(a[0], c[11], 0u, &bw);
    a[1] = __builtin_subc(a[1], c[12], bw, &bw);
    a[2] = __builtin_subc(a[2], c[13], bw, &bw);
    a[3] = __builtin_subc(a[3], 0u, bw, &bw);
    a[4] = __builtin_subc(a[4], 0u, bw, &bw);
    a[5] = __builtin_subc(a[5], 0u, bw, &bw);
    a[6] = __builtin_subc(a[6], c[8], bw, &bw);
    a[7] = __builtin_subc(a[7], c[10], bw, &bw);
    top -= (int32_t)bw;
    // - D2 = (c11, c9, 0, 0, c15, c14, c13, c12)
    a[0] = __builtin_subc(a[0], c[12], 0u, &bw);
    a[1] = __builtin_subc(a[1], c[13], bw, &bw);
    a[2] = __builtin_subc(a[2], c[14], bw, &bw);
    a[3] = __builtin_subc(a[3], c[15], bw, &bw);
    a[4] = __builtin_subc(a[4], 0u, bw, &bw);
    a[5] = __builtin_subc(a[5], 0u, bw, &bw);
    a[6] = __builtin_subc(a[6], c[9], bw, &bw);
    a[7] = __builtin_subc(a[7], c[11], bw, &bw);
    top -= (int32_t)bw;
    // - D3 = (c12, 0, c10, c9, c8, c15, c14, c13)
    a[0] = __builtin_subc(a[0], c[13], 0u, &bw);
    a[1] = __builtin_subc(a[1], c[14], bw, &bw);
    a[2] = __builtin_subc(a[2], c[15], bw, &bw);
    a[3] = __builtin_subc(a[3], c[8], bw, &bw);
    a[4] = __builtin_subc(a[4], c[9], bw, &bw);
    a[5] = __builtin_subc(a[5], c[10], bw, &bw);
    a[6] = __builtin_subc(a[6], 0u, bw, &bw);
    a[7] = __builtin_subc(a[7], c[12], bw, &bw);
    top -= (int32_t)bw;
    // - D4 = (c13, 0, c11, c10, c9, 0, c15, c14)
    a[0] = __builtin_subc(a[0], c[14], 0u, &bw);
    a[1] = __builtin_subc(a[1], c[15], bw, &bw);
    a[2] = __builtin_subc(a[2], 0u, bw, &bw);
    a[3] = __builtin_subc(a[3], c[9], bw, &bw);
    a[4] = __builtin_subc(a[4], c[10], bw, &bw);
    a[5] = __builtin_subc(a[5], c[11], bw, &bw);
    a[6] = __builtin_subc(a[6], 0u, bw, &bw);
    a[7] = __builtin_subc(a[7], c[13], bw, &bw);
    top -= (int32_t)bw;
    // value = a + top 2^256, top in [-4, 6]: add top (2^224 - 2^192 - 2^96 + 1) with a signed
    // word-by-word carry (the new carry out of 2^256 is then -1, 0 or 1, and non-zero only when a
    // is within |top| 2^224 of 0 or 2^256)
    int64_t s = (int64_t)a[0] + top;
    r.w[0] = (uint32_t)s;
    s >>= 32;
    s += a[1];
    r.w[1] = (uint32_t)s;
    s >>= 32;
    s += a[2];
    r.w[2] = (uint32_t)s;
    s >>= 32;
    s += (int64_t)a[3] - top;
    r.w[3] = (uint32_t)s;
    s >>= 32;
    s += a[4];
    r.w[4] = (uint32_t)s;
    s >>= 32;
    s += a[5];
    r.w[5] = (uint32_t)s;
    s >>= 32;
    s += (int64_t)a[6] - top;
    r.w[6] = (uint32_t)s;
    s >>= 32;
    s += (int64_t)a[7] + top;
    r.w[7] = (uint32_t)s;
    s >>= 32;
    // rare: a carry (+1: add K, may carry again only from values >= p) or a borrow (-1: subtract
    // K, may borrow again only when the value was below K)
    while (s > 0) s -= (int64_t)add_mk<CURVE_R1>(r, 1u) ? 0 : 1;
    while (s < 0) s += (int64_t)sub_mk<CURVE_R1>(r, 1u) ? 0 : 1;
}

// ---------------------------------------------------------------------------------------
// field mod p (redundant form)
template <int C> CHIP_DEV void fp_add(u256& r, const u256& a, const u256& b) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = __builtin_addc(a.w[i], b.w[i], c, &c);
    // a + b = r + c 2^256 = r + c K (mod p); a second carry needs r >= p after the wrap (rare)
    c = add_mk<C>(r, c);
    if (c) (void)add_mk<C>(r, 1u);
}
template <int C> CHIP_DEV void fp_sub(u256& r, const u256& a, const u256& b) {
    uint32_t bw = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = __builtin_subc(a.w[i], b.w[i], bw, &bw);
    // a - b = r - bw 2^256 = r - bw K (mod p); a second borrow needs b - a > p (rare)
    bw = sub_mk<C>(r, bw);
    if (bw) (void)sub_mk<C>(r, 1u);
}
template <int C> CHIP_DEV void fp_neg(u256& r, const u256& a) {
    u256 z;
    u256_set_word(z, 0);
    fp_sub<C>(r, z, a);
}
template <int C> CHIP_DEV void fp_dbl(u256& r, const u256& a) { fp_add<C>(r, a, a); }
// canonical value in [0, p)
template <int C> CHIP_DEV void fp_canon(u256& r, const u256& a) {
    u256 s;
    const uint32_t br = u256_sub(s, a, curve<C>().p);
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = br ? a.w[i] : s.w[i];
}
template <int C> CHIP_DEV bool fp_is_zero(const u256& a) { return u256_is_zero(a) || u256_eq_c(a, curve<C>().p); }
template <int C> CHIP_DEV bool fp_eq(const u256& a, const u256& b) {
    u256 x, y;
    fp_canon<C>(x, a);
    fp_canon<C>(y, b);
    return u256_eq(x, y);
}

template <int C> CHIP_DEV void fp_mul(u256& r, const u256& a, const u256& b) {
    uint32_t t[16];
    if (C & CURVE_ILP) mul_512_ilp(t, a, b);
    else mul_512(t, a, b);
    if (EC_CURVE(C) == CURVE_R1) reduce_r1(r, t);
    else reduce_k1(r, t);
}
template <int C> CHIP_DEV void fp_sqr(u256& r, const u256& a) {
    uint32_t t[16];
    if (C & CURVE_ILP) mul_512_ilp(t, a, a);
    else sqr_512(t, a);
    if (EC_CURVE(C) == CURVE_R1) reduce_r1(r, t);
    else reduce_k1(r, t);
}
template <int C> CHIP_DEV void fp_sqr_n(u256& r, const u256& a, int n) {
    r = a;
#pragma unroll 1
    for (int i = 0; i < n; i++) fp_sqr<C>(r, r);
}
// r = a^e (e little-endian words, a constant exponent: the branch on each bit is wave-uniform)
template <int C> CHIP_DEV void fp_pow(u256& r, const u256& a, const uint32_t* e) {
    u256 acc;
    u256_set_word(acc, 1);
#pragma unroll 1
    for (int k = 255; k >= 0; k--) {
        fp_sqr<C>(acc, acc);
        if ((e[k >> 5] >> (k & 31)) & 1u) fp_mul<C>(acc, acc, a);
    }
    r = acc;
}
// a^(p-2) by the curve's addition chain
template <int C> CHIP_DEV void fp_inv(u256& r, const u256& a) {
    u256 x2, x3, t;
    fp_sqr<C>(x2, a);
    fp_mul<C>(x2, x2, a);       // 2^2 - 1
    fp_sqr<C>(x3, x2);
    fp_mul<C>(x3, x3, a);       // 2^3 - 1
    if (EC_CURVE(C) == CURVE_R1) {
        // p - 2 = ffffffff 00000001 00000000 00000000 00000000 ffffffff ffffffff fffffffd
        u256 x6, x12, x15, x30, x32;
        fp_sqr_n<C>(x6, x3, 3);
        fp_mul<C>(x6, x6, x3);
        fp_sqr_n<C>(x12, x6, 6);
        fp_mul<C>(x12, x12, x6);
        fp_sqr_n<C>(x15, x12, 3);
        fp_mul<C>(x15, x15, x3);
        fp_sqr_n<C>(x30, x15, 15);
        fp_mul<C>(x30, x30, x15);
        fp_sqr_n<C>(x32, x30, 2);
        fp_mul<C>(x32, x32, x2);
        fp_sqr_n<C>(t, x32, 32);
        fp_mul<C>(t, t, a);      // ffffffff 00000001
        fp_sqr_n<C>(t, t, 128);
        fp_mul<C>(t, t, x32);    // ... 00000000 00000000 00000000 ffffffff
        fp_sqr_n<C>(t, t, 32);
        fp_mul<C>(t, t, x32);    // ... ffffffff
        fp_sqr_n<C>(t, t, 30);
        fp_mul<C>(t, t, x30);    // 30 ones
        fp_sqr_n<C>(t, t, 2);
        fp_mul<C>(r, t, a);      // 01
    } else {
        // p - 2 = [223 ones] 0 [22 ones] 0000 1 0 11 0 1
        u256 x6, x9, x11, x22, x44, x88, x176, x220, x223;
        fp_sqr_n<C>(x6, x3, 3);
        fp_mul<C>(x6, x6, x3);
        fp_sqr_n<C>(x9, x6, 3);
        fp_mul<C>(x9, x9, x3);
        fp_sqr_n<C>(x11, x9, 2);
        fp_mul<C>(x11, x11, x2);
        fp_sqr_n<C>(x22, x11, 11);
        fp_mul<C>(x22, x22, x11);
        fp_sqr_n<C>(x44, x22, 22);
        fp_mul<C>(x44, x44, x22);
        fp_sqr_n<C>(x88, x44, 44);
        fp_mul<C>(x88, x88, x44);
        fp_sqr_n<C>(x176, x88, 88);
        fp_mul<C>(x176, x176, x88);
        fp_sqr_n<C>(x220, x176, 44);
        fp_mul<C>(x220, x220, x44);
        fp_sqr_n<C>(x223, x220, 3);
        fp_mul<C>(x223, x223, x3);
        fp_sqr_n<C>(t, x223, 23);
        fp_mul<C>(t, t, x22);
        fp_sqr_n<C>(t, t, 5);
        fp_mul<C>(t, t, a);
        fp_sqr_n<C>(t, t, 3);
        fp_mul<C>(t, t, x2);
        fp_sqr_n<C>(t, t, 2);
        fp_mul<C>(r, t, a);
    }
}

// ---------------------------------------------------------------------------------------
// scalars mod n, Montgomery form (R = 2^256), canonical values in [0, n)
// Comba product, then Comba REDC: column k of t + sum m_i n_j, m_k = (column k) n' for k < 8.
template <int C> CHIP_DEV void mn_mul(u256& r, const u256& a, const u256& b) {
    const ec_curve_c& cv = curve<C>();
    uint32_t t[16];
    if (C & CURVE_ILP) mul_512_ilp(t, a, b);
    else mul_512(t, a, b);
    uint32_t m[8];
    uint64_t acc = 0;
    uint32_t top = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        // acc += t[k]
        const uint64_t prev = acc;
        acc += t[k];
        top += acc < prev;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int j = k - i;
            if (i < k && j >= 0 && j < 8 && i < 8) mac(acc, top, m[i], cv.n[j]);
        }
        if (k < 8) {
            m[k] = (uint32_t)acc * cv.n_minv;
            mac(acc, top, m[k], cv.n[0]);   // zeroes the low word
            (void)col_next(acc, top);
        } else {
            r.w[k - 8] = col_next(acc, top);
        }
    }
    // result = r + acc 2^256 < 2n: one conditional subtraction
    u256 s;
    const uint32_t br = u256_sub(s, r, cv.n);
    if (acc || !br) r = s;
}
template <int C> CHIP_DEV void mn_pow(u256& r, const u256& a_m, const uint32_t* e) {
    const ec_curve_c& cv = curve<C>();
    u256 acc;
    u256_from_c(acc, cv.one_n);
#pragma unroll 1
    for (int k = 255; k >= 0; k--) {
        mn_mul<C>(acc, acc, acc);
        if ((e[k >> 5] >> (k & 31)) & 1u) mn_mul<C>(acc, acc, a_m);
    }
    r = acc;
}

// ---------------------------------------------------------------------------------------
// Variable-time inversion mod n by the binary extended Euclidean algorithm (the inputs are public
// signature values, as in BC's BigInteger.modInverse).  Invariants x1 a = u, x2 a = v (mod n); u, v
// odd; each step replaces the larger of u, v by the difference with its factors of two removed, and
// divides the matching x by the same power of two Montgomery-style (x + m n) / 2^k.  ~180 steps of
// ~150 lane-uniform instructions (selects instead of branches) instead of the ~380 multiplications
// of a Fermat power: the latency of the per-wave inversion kernel.
// x * 2^-k mod m, 1 <= k <= 31, x < m; mminv = -m^-1 mod 2^32
CHIP_DEV void halve_k(u256& x, uint32_t k, const uint32_t* mod, uint32_t mminv) {
    const uint32_t q = (x.w[0] * mminv) & ((1u << k) - 1u);   // x + q m = 0 (mod 2^k)
    uint32_t y[9];
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c = (uint64_t)q * mod[i] + x.w[i] + c;
        y[i] = (uint32_t)c;
        c >>= 32;
    }
    y[8] = (uint32_t)c;
#pragma unroll
    for (int i = 0; i < 8; i++) x.w[i] = __builtin_amdgcn_alignbit(y[i + 1], y[i], k);   // (x + q m) >> k < 2m
    u256 s;
    if (!u256_sub(s, x, mod)) x = s;
}
CHIP_DEV uint32_t u256_ctz_capped(const u256& t) {   // trailing zeros of t (t != 0), capped at 31
    const uint32_t lo = t.w[0];
    return lo ? min((uint32_t)__builtin_ctz(lo), 31u) : 31u;
}
CHIP_DEV void u256_shr_k(u256& t, uint32_t k) {   // 1 <= k <= 31
#pragma unroll
    for (int i = 0; i < 7; i++) t.w[i] = __builtin_amdgcn_alignbit(t.w[i + 1], t.w[i], k);
    t.w[7] >>= k;
}
// plain a^-1 mod m for a in [0, m), m an odd prime (0 -> 0)
CHIP_DEV void modinv_vt(u256& r, const u256& a, const uint32_t* mod, uint32_t mminv) {
    u256 u = a, v, x1, x2;
    u256_from_c(v, mod);
    u256_set_word(x1, 1);
    u256_set_word(x2, 0);
    if (u256_is_zero(u)) {   // no inverse; callers never pass 0, but every loop below must end
        r = u;
        return;
    }
#pragma unroll 1
    while (!(u.w[0] & 1u)) {
        const uint32_t k = u256_ctz_capped(u);
        u256_shr_k(u, k);
        halve_k(x1, k, mod, mminv);
    }
    // each step at least halves u + v: 2 * 256 steps bound the loop for a < m
#pragma unroll 1
    for (int it = 0; it < 520 && !u256_eq(u, v); it++) {
        u256 d, e, t, xt;
        const uint32_t ge = !u256_sub(d, u, v.w);   // u >= v: u - v, else v - u
        (void)u256_sub(e, v, u.w);
        u256 xa, xb;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            t.w[i] = ge ? d.w[i] : e.w[i];
            xa.w[i] = ge ? x1.w[i] : x2.w[i];
            xb.w[i] = ge ? x2.w[i] : x1.w[i];
        }
        // xt = xa - xb (mod m)
        if (u256_sub(xt, xa, xb.w)) (void)u256_add(xt, xt, mod);
#pragma unroll 1
        do {
            const uint32_t k = u256_ctz_capped(t);
            u256_shr_k(t, k);
            halve_k(xt, k, mod, mminv);
        } while (!(t.w[0] & 1u));
#pragma unroll
        for (int i = 0; i < 8; i++) {
            u.w[i] = ge ? t.w[i] : u.w[i];
            v.w[i] = ge ? v.w[i] : t.w[i];
            x1.w[i] = ge ? xt.w[i] : x1.w[i];
            x2.w[i] = ge ? x2.w[i] : xt.w[i];
        }
    }
    r = x1;
}
template <int C> CHIP_DEV void mn_inv_plain(u256& r, const u256& a) { modinv_vt(r, a, curve<C>().n, curve<C>().n_minv); }
// field inversion, variable time (binary extended Euclid; a any redundant value, 0 -> 0): the table
// builders' inversion, ~4x fewer instructions than the addition chain of fp_inv
template <int C> CHIP_DEV void fp_inv_vt(u256& r, const u256& a) {
    u256 c;
    fp_canon<C>(c, a);
    // -p^-1 mod 2^32: P-256 p = -1 (mod 2^32); secp256k1 p = 0xfffffc2f (mod 2^32)
    modinv_vt(r, c, curve<C>().p, EC_CURVE(C) == CURVE_R1 ? 1u : 0xd2253531u);
}
// Montgomery form in, Montgomery form out: (aR)^-1 R^3 R^-1 = a^-1 R
template <int C> CHIP_DEV void mn_inv(u256& r, const u256& a_m) {
    const ec_curve_c& cv = curve<C>();
    u256 inv, r2, r3;
    mn_inv_plain<C>(inv, a_m);
    u256_from_c(r2, cv.r2_n);
    mn_mul<C>(r3, r2, r2);
    mn_mul<C>(r, inv, r3);
}

// ---------------------------------------------------------------------------------------
// points
struct jpt {
    u256 X, Y, Z;
};
struct apt {
    u256 x, y;
};

template <int C> CHIP_DEV void jdbl(jpt& r, const jpt& p) {
    if (EC_CURVE(C) == CURVE_R1) {
        // a = -3: dbl-2001-b
        u256 delta, gamma, beta, alpha, t1, t2, t3;
        fp_sqr<C>(delta, p.Z);
        fp_sqr<C>(gamma, p.Y);
        fp_mul<C>(beta, p.X, gamma);
        fp_sub<C>(t1, p.X, delta);
        fp_add<C>(t2, p.X, delta);
        fp_mul<C>(alpha, t1, t2);
        fp_add<C>(t1, alpha, alpha);
        fp_add<C>(alpha, alpha, t1);            // 3 (X - delta)(X + delta)
        fp_add<C>(t3, p.Y, p.Z);
        fp_sqr<C>(t3, t3);
        fp_sub<C>(t3, t3, gamma);
        fp_sub<C>(r.Z, t3, delta);              // Z3 = (Y+Z)^2 - gamma - delta
        fp_add<C>(t1, beta, beta);
        fp_add<C>(t1, t1, t1);                  // 4 beta
        fp_sqr<C>(t2, alpha);
        fp_sub<C>(t2, t2, t1);
        fp_sub<C>(r.X, t2, t1);                 // X3 = alpha^2 - 8 beta
        fp_sub<C>(t1, t1, r.X);                 // 4 beta - X3
        fp_mul<C>(t1, alpha, t1);
        fp_sqr<C>(gamma, gamma);                // gamma^2
        fp_add<C>(gamma, gamma, gamma);
        fp_add<C>(gamma, gamma, gamma);
        fp_add<C>(gamma, gamma, gamma);         // 8 gamma^2
        fp_sub<C>(r.Y, t1, gamma);
    } else {
        // a = 0: dbl-2009-l
        u256 A, B, Cc, D, E, F, t;
        fp_sqr<C>(A, p.X);
        fp_sqr<C>(B, p.Y);
        fp_sqr<C>(Cc, B);
        fp_add<C>(t, p.X, B);
        fp_sqr<C>(t, t);
        fp_sub<C>(t, t, A);
        fp_sub<C>(t, t, Cc);
        fp_add<C>(D, t, t);
        fp_add<C>(E, A, A);
        fp_add<C>(E, E, A);
        fp_sqr<C>(F, E);
        u256 z3;
        fp_mul<C>(z3, p.Y, p.Z);
        fp_add<C>(r.Z, z3, z3);
        fp_add<C>(t, D, D);
        fp_sub<C>(r.X, F, t);
        fp_sub<C>(t, D, r.X);
        fp_mul<C>(t, E, t);
        fp_add<C>(Cc, Cc, Cc);
        fp_add<C>(Cc, Cc, Cc);
        fp_add<C>(Cc, Cc, Cc);
        fp_sub<C>(r.Y, t, Cc);
    }
}
// Mixed addition r = p + q (q affine) for the comb kernels.  The exceptional case P == Q (H = 0 and r = 0:
// the running sum equals the table point, never for honest signatures, reachable by crafted ones) is not
// computed here: `exc` is set and r is left unspecified; the kernel parks the lane for k_ecdsa_comb_retry.
// Having no doubling call on this path keeps the accumulator in registers (an out-of-line call taking it by
// reference had put it in scratch memory across every addition).
template <int C> CHIP_DEV void jmadd_x(jpt& r, const jpt& p, const apt& q, bool& exc) {
    if (u256_is_zero(p.Z)) {
        r.X = q.x;
        r.Y = q.y;
        u256_set_word(r.Z, 1);
        return;
    }
    u256 Z1Z1, U2, S2, H, HH, I, J, rr, V, t;
    fp_sqr<C>(Z1Z1, p.Z);
    fp_mul<C>(U2, q.x, Z1Z1);
    fp_mul<C>(S2, q.y, p.Z);
    fp_mul<C>(S2, S2, Z1Z1);
    fp_sub<C>(H, U2, p.X);
    fp_sub<C>(rr, S2, p.Y);
    if (fp_is_zero<C>(H)) {
        if (fp_is_zero<C>(rr)) {
            exc = true;
            r = p;
        } else {
            u256_set_word(r.X, 0);
            u256_set_word(r.Y, 0);
            u256_set_word(r.Z, 0);
        }
        return;
    }
    fp_add<C>(rr, rr, rr);
    fp_sqr<C>(HH, H);
    fp_add<C>(I, HH, HH);
    fp_add<C>(I, I, I);
    fp_mul<C>(J, H, I);
    fp_mul<C>(V, p.X, I);
    jpt o;
    fp_sqr<C>(o.X, rr);
    fp_sub<C>(o.X, o.X, J);
    fp_sub<C>(o.X, o.X, V);
    fp_sub<C>(o.X, o.X, V);
    fp_sub<C>(t, V, o.X);
    fp_mul<C>(o.Y, rr, t);
    fp_mul<C>(t, p.Y, J);
    fp_add<C>(t, t, t);
    fp_sub<C>(o.Y, o.Y, t);
    fp_add<C>(t, p.Z, H);
    fp_sqr<C>(t, t);
    fp_sub<C>(t, t, Z1Z1);
    fp_sub<C>(o.Z, t, HH);
    r = o;
}
// the complete mixed addition of the cold kernels (windowed verify, fixed-base table build, retries): the
// P == Q case doubles, out of line so the common path stays small
template <int C> __device__ __attribute__((noinline)) void jdbl_slow(jpt& r, const jpt& p) { jdbl<C>(r, p); }
template <int C> CHIP_DEV void jmadd(jpt& r, const jpt& p, const apt& q) {
    bool exc = false;
    jpt o;
    jmadd_x<C>(o, p, q, exc);
    if (exc) jdbl_slow<C>(r, p);
    else r = o;
}
// complete, with the doubling inline (a kernel that runs only for the rare exceptional lanes)
template <int C> CHIP_DEV void jmadd_full(jpt& r, const jpt& p, const apt& q) {
    bool exc = false;
    jpt o;
    jmadd_x<C>(o, p, q, exc);
    if (exc) jdbl<C>(o, p);
    r = o;
}
