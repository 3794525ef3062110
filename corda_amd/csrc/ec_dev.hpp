// ec_dev.hpp — secp256r1 (P-256) and secp256k1 field, scalar and point arithmetic for gfx950.
//
// Field elements: 8 little-endian u32 words, fully reduced (< p) after every operation.
// Multiplication: 32x32->64 operand-scanning schoolbook (v_mad_u64_u32) into 16 words, then the
// curve's special-form reduction: P-256 by the NIST/Solinas word recombination (FIPS 186-4 D.2.3),
// secp256k1 by folding with 2^256 = 2^32 + 977 (mod p).
// Scalars mod n: Montgomery multiplication (CIOS, R = 2^256).
// Points: Jacobian (X, Y, Z), Z = 0 is the point at infinity; tables hold affine points.
#pragma once
#include "common.hpp"
#include "curve_consts.hpp"

enum { CURVE_R1 = 0, CURVE_K1 = 1 };

struct u256 {
    uint32_t w[8];
};

template <int C> CHIP_DEV const ec_curve_c& curve() { return C == CURVE_R1 ? EC_R1 : EC_K1; }

CHIP_DEV bool u256_is_zero(const u256& a) {
    return (a.w[0] | a.w[1] | a.w[2] | a.w[3] | a.w[4] | a.w[5] | a.w[6] | a.w[7]) == 0;
}
CHIP_DEV bool u256_eq(const u256& a, const u256& b) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d |= a.w[i] ^ b.w[i];
    return d == 0;
}
// a >= b
CHIP_DEV bool u256_ge(const u256& a, const uint32_t* b) {
    uint64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t d = (uint64_t)a.w[i] - b[i] - br;
        br = (d >> 63) & 1;
    }
    return br == 0;
}
// r = a + b, returns carry
CHIP_DEV uint32_t u256_add(u256& r, const u256& a, const uint32_t* b) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c += (uint64_t)a.w[i] + b[i];
        r.w[i] = (uint32_t)c;
        c >>= 32;
    }
    return (uint32_t)c;
}
// r = a - b, returns borrow
CHIP_DEV uint32_t u256_sub(u256& r, const u256& a, const uint32_t* b) {
    uint64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t d = (uint64_t)a.w[i] - b[i] - br;
        r.w[i] = (uint32_t)d;
        br = (d >> 63) & 1;
    }
    return (uint32_t)br;
}
CHIP_DEV void u256_from_c(u256& r, const uint32_t* c) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = c[i];
}

// ---------------------------------------------------------------------------------------
// field mod p
template <int C> CHIP_DEV void fp_add(u256& r, const u256& a, const u256& b) {
    const uint32_t* p = curve<C>().p;
    u256 t, s;
    const uint32_t c = u256_add(t, a, b.w);
    const uint32_t br = u256_sub(s, t, p);
    const bool use_s = c || !br;
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = use_s ? s.w[i] : t.w[i];
}
template <int C> CHIP_DEV void fp_sub(u256& r, const u256& a, const u256& b) {
    const uint32_t* p = curve<C>().p;
    u256 t, s;
    const uint32_t br = u256_sub(t, a, b.w);
    u256_add(s, t, p);
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = br ? s.w[i] : t.w[i];
}
template <int C> CHIP_DEV void fp_neg(u256& r, const u256& a) {
    u256 z;
#pragma unroll
    for (int i = 0; i < 8; i++) z.w[i] = 0;
    fp_sub<C>(r, z, a);
}

// 512-bit product (16 words)
CHIP_DEV void mul_512(uint32_t t[16], const u256& a, const u256& b) {
#pragma unroll
    for (int k = 0; k < 16; k++) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t carry = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            uint64_t p = (uint64_t)a.w[i] * b.w[j] + t[i + j];
            p += carry;
            t[i + j] = (uint32_t)p;
            carry = (uint32_t)(p >> 32);
        }
        t[i + 8] = carry;
    }
}
// 512-bit square: off-diagonal products once, doubled, plus the diagonal
CHIP_DEV void sqr_512(uint32_t t[16], const u256& a) {
#pragma unroll
    for (int k = 0; k < 16; k++) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 7; i++) {
        uint32_t carry = 0;
#pragma unroll
        for (int j = i + 1; j < 8; j++) {
            uint64_t p = (uint64_t)a.w[i] * a.w[j] + t[i + j];
            p += carry;
            t[i + j] = (uint32_t)p;
            carry = (uint32_t)(p >> 32);
        }
        t[i + 8] = carry;
    }
    // double
    uint32_t top = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t v = t[k];
        t[k] = (v << 1) | top;
        top = v >> 31;
    }
    // + diagonal
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t sq = (uint64_t)a.w[i] * a.w[i];
        c += (uint64_t)t[2 * i] + (uint32_t)sq;
        t[2 * i] = (uint32_t)c;
        c >>= 32;
        c += (uint64_t)t[2 * i + 1] + (uint32_t)(sq >> 32);
        t[2 * i + 1] = (uint32_t)c;
        c >>= 32;
    }
}

// secp256k1: t mod p, p = 2^256 - 2^32 - 977
CHIP_DEV void reduce_k1(u256& r, const uint32_t t[16]) {
    // u = lo + hi * 977 + (hi << 32)   (10 words)
    uint32_t u[10];
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c += (uint64_t)t[i] + (uint64_t)t[8 + i] * 977u;
        if (i > 0) c += t[8 + i - 1];
        u[i] = (uint32_t)c;
        c >>= 32;
    }
    c += t[15];
    u[8] = (uint32_t)c;
    u[9] = (uint32_t)(c >> 32);
    // fold u[8..9] (top < 2^34) again: + top * (2^32 + 977)
    const uint64_t top = (uint64_t)u[8] | ((uint64_t)u[9] << 32);
    c = (uint64_t)u[0] + (top & 0xffffffffull) * 977u;
    r.w[0] = (uint32_t)c;
    c >>= 32;
    c += (uint64_t)u[1] + (top >> 32) * 977u + (uint32_t)top;
    r.w[1] = (uint32_t)c;
    c >>= 32;
    c += (uint64_t)u[2] + (top >> 32);
    r.w[2] = (uint32_t)c;
    c >>= 32;
#pragma unroll
    for (int i = 3; i < 8; i++) {
        c += u[i];
        r.w[i] = (uint32_t)c;
        c >>= 32;
    }
    // carry out (value >= 2^256): add 2^32 + 977 once more (cannot overflow again)
    if (c) {
        uint64_t d = (uint64_t)r.w[0] + 977u;
        r.w[0] = (uint32_t)d;
        d >>= 32;
        d += (uint64_t)r.w[1] + 1u;
        r.w[1] = (uint32_t)d;
        d >>= 32;
#pragma unroll
        for (int i = 2; i < 8; i++) {
            d += r.w[i];
            r.w[i] = (uint32_t)d;
            d >>= 32;
        }
    }
    u256 s;
    if (!u256_sub(s, r, EC_K1.p)) r = s;
}

// P-256: FIPS 186-4 D.2.3 fast reduction with 32-bit words
CHIP_DEV void reduce_r1(u256& r, const uint32_t c[16]) {
    int64_t a[8];
    // s1 + 2 s2 + 2 s3 + s4 + s5 - s6 - s7 - s8 - s9, word by word (index 0 = least significant)
    a[0] = (int64_t)c[0] + c[8] + c[9] - c[11] - c[12] - c[13] - c[14];
    a[1] = (int64_t)c[1] + c[9] + c[10] - c[12] - c[13] - c[14] - c[15];
    a[2] = (int64_t)c[2] + c[10] + c[11] - c[13] - c[14] - c[15];
    a[3] = (int64_t)c[3] + 2 * (int64_t)c[11] + 2 * (int64_t)c[12] + c[13] - c[15] - c[8] - c[9];
    a[4] = (int64_t)c[4] + 2 * (int64_t)c[12] + 2 * (int64_t)c[13] + c[14] - c[9] - c[10];
    a[5] = (int64_t)c[5] + 2 * (int64_t)c[13] + 2 * (int64_t)c[14] + c[15] - c[10] - c[11];
    a[6] = (int64_t)c[6] + 2 * (int64_t)c[14] + 2 * (int64_t)c[15] + c[14] + c[13] - c[8] - c[9];
    a[7] = (int64_t)c[7] + 2 * (int64_t)c[15] + c[15] + c[8] - c[10] - c[11] - c[12] - c[13];
    int64_t carry = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        a[i] += carry;
        carry = a[i] >> 32;   // arithmetic shift
        r.w[i] = (uint32_t)a[i];
    }
    // value = r + carry * 2^256, carry in [-4, 6]: bring into [0, p)
    while (carry < 0) {
        carry += u256_add(r, r, EC_R1.p);
    }
    while (carry > 0) {
        carry -= u256_sub(r, r, EC_R1.p);
    }
    u256 s;
    if (!u256_sub(s, r, EC_R1.p)) r = s;
}

template <int C> CHIP_DEV void fp_mul(u256& r, const u256& a, const u256& b) {
    uint32_t t[16];
    mul_512(t, a, b);
    if (C == CURVE_R1) reduce_r1(r, t);
    else reduce_k1(r, t);
}
template <int C> CHIP_DEV void fp_sqr(u256& r, const u256& a) {
    uint32_t t[16];
    sqr_512(t, a);
    if (C == CURVE_R1) reduce_r1(r, t);
    else reduce_k1(r, t);
}
// r = a^e (e little-endian words, a constant exponent: the branch on each bit is wave-uniform),
// left-to-right binary: no per-lane table, so nothing spills to scratch
template <int C> CHIP_DEV void fp_pow(u256& r, const u256& a, const uint32_t* e) {
    u256 acc;
#pragma unroll
    for (int i = 0; i < 8; i++) acc.w[i] = (i == 0);
    for (int k = 255; k >= 0; k--) {
        fp_sqr<C>(acc, acc);
        if ((e[k >> 5] >> (k & 31)) & 1u) fp_mul<C>(acc, acc, a);
    }
    r = acc;
}
template <int C> CHIP_DEV void fp_inv(u256& r, const u256& a) { fp_pow<C>(r, a, curve<C>().p_minus_2); }

// ---------------------------------------------------------------------------------------
// scalars mod n, Montgomery form
template <int C> CHIP_DEV void mn_mul(u256& r, const u256& a, const u256& b) {
    const ec_curve_c& cv = curve<C>();
    uint32_t t[10];
#pragma unroll
    for (int k = 0; k < 10; k++) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            uint64_t p = (uint64_t)a.w[j] * b.w[i] + t[j];
            p += c >> 32;
            t[j] = (uint32_t)p;
            c = p;
        }
        uint64_t s = (uint64_t)t[8] + (c >> 32);
        t[8] = (uint32_t)s;
        t[9] = (uint32_t)(s >> 32);
        const uint32_t m = t[0] * cv.n_minv;
        uint64_t p = (uint64_t)m * cv.n[0] + t[0];
        c = p;
#pragma unroll
        for (int j = 1; j < 8; j++) {
            p = (uint64_t)m * cv.n[j] + t[j];
            p += c >> 32;
            t[j - 1] = (uint32_t)p;
            c = p;
        }
        s = (uint64_t)t[8] + (c >> 32);
        t[7] = (uint32_t)s;
        t[8] = t[9] + (uint32_t)(s >> 32);
    }
    u256 res, sub;
#pragma unroll
    for (int i = 0; i < 8; i++) res.w[i] = t[i];
    const uint32_t br = u256_sub(sub, res, cv.n);
    if (t[8] || !br) res = sub;
    r = res;
}
template <int C> CHIP_DEV void mn_pow(u256& r, const u256& a_m, const uint32_t* e) {
    const ec_curve_c& cv = curve<C>();
    u256 acc;
    u256_from_c(acc, cv.one_n);
    for (int k = 255; k >= 0; k--) {
        mn_mul<C>(acc, acc, acc);
        if ((e[k >> 5] >> (k & 31)) & 1u) mn_mul<C>(acc, acc, a_m);
    }
    r = acc;
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
    if (C == CURVE_R1) {
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

// r = p + q (q affine, not infinity).  Exact for every input: infinity, p == q, p == -q.
template <int C> CHIP_DEV void jmadd(jpt& r, const jpt& p, const apt& q) {
    if (u256_is_zero(p.Z)) {
        r.X = q.x;
        r.Y = q.y;
#pragma unroll
        for (int i = 0; i < 8; i++) r.Z.w[i] = (i == 0);
        return;
    }
    u256 Z1Z1, U2, S2, H, HH, I, J, rr, V, t;
    fp_sqr<C>(Z1Z1, p.Z);
    fp_mul<C>(U2, q.x, Z1Z1);
    fp_mul<C>(S2, q.y, p.Z);
    fp_mul<C>(S2, S2, Z1Z1);
    fp_sub<C>(H, U2, p.X);
    fp_sub<C>(rr, S2, p.Y);
    if (u256_is_zero(H)) {
        if (u256_is_zero(rr)) {
            jdbl<C>(r, p);
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) r.X.w[i] = r.Y.w[i] = r.Z.w[i] = 0;
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
