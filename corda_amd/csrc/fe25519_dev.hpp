// fe25519_dev.hpp — GF(2^255-19) arithmetic and Ed25519 group operations for gfx950.
//
// Representation: ten unsigned 32-bit limbs, radix 2^25.5 (even limbs 26 bits, odd 25 bits).
// Products are 32x32->64 multiply-accumulates (v_mad_u64_u32: one per ~4.2 cycles per SIMD, 36.5e12 MAC/s at
// 2.38 GHz measured by tools/microbench_valu.hip, profiles/r04/microbench_valu_a.txt; it does not co-issue
// with the dual-issue 32-bit ops), column sums stay below 2^63 under these bounds:
//   "carried" limb : even < 2^26, odd < 2^25 (+2^17 on limb 1)   — every mul/sq output
//   "loose"   limb : even < 3*2^26, odd < 3*2^25                 — carried + carried or
//                                                                   carried + 2p - carried
// fe_mul / fe_sq accept loose inputs (19*g < 2^32 and every column < 2^62.2).  fe_sub requires a
// carried subtrahend.  The point formulas below are arranged so no other inputs occur.
#pragma once
#include "common.hpp"
#include "curve_consts.hpp"

struct fe {
    uint32_t v[10];
};

#define M26 0x3ffffffu
#define M25 0x1ffffffu

// 2p limbs
#define P2_0 0x7ffffdau
#define P2_E 0x7fffffeu
#define P2_O 0x3fffffeu
// 4p limbs
#define P4_0 0xfffffb4u
#define P4_E 0xffffffcu
#define P4_O 0x7fffffcu

CHIP_DEV void fe_0(fe& h) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = 0;
}
CHIP_DEV void fe_1(fe& h) {
    fe_0(h);
    h.v[0] = 1;
}
CHIP_DEV void fe_from_c(fe& h, const fe_c& c) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = c.v[i];
}
CHIP_DEV void fe_add(fe& h, const fe& f, const fe& g) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + g.v[i];
}
// h = f + 2p - g   (g carried)
CHIP_DEV void fe_sub(fe& h, const fe& f, const fe& g) {
    h.v[0] = f.v[0] + P2_0 - g.v[0];
#pragma unroll
    for (int i = 1; i < 10; i++) h.v[i] = f.v[i] + ((i & 1) ? P2_O : P2_E) - g.v[i];
}
// h = f + 4p - g   (g < 2^27 even / 2^26 odd, e.g. a sum of two carried values)
CHIP_DEV void fe_sub4(fe& h, const fe& f, const fe& g) {
    h.v[0] = f.v[0] + P4_0 - g.v[0];
#pragma unroll
    for (int i = 1; i < 10; i++) h.v[i] = f.v[i] + ((i & 1) ? P4_O : P4_E) - g.v[i];
}
CHIP_DEV void fe_neg(fe& h, const fe& f) {
    fe z;
    fe_0(z);
    fe_sub(h, z, f);
}
CHIP_DEV void fe_cmov(fe& h, const fe& f, bool c) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = c ? f.v[i] : h.v[i];
}

// carry-propagate ten 64-bit column sums into a carried element
CHIP_DEV void fe_carry64(fe& h, uint64_t t[10]) {
    uint64_t c;
    c = t[0] >> 26; t[1] += c; t[0] &= M26;
    c = t[4] >> 26; t[5] += c; t[4] &= M26;
    c = t[1] >> 25; t[2] += c; t[1] &= M25;
    c = t[5] >> 25; t[6] += c; t[5] &= M25;
    c = t[2] >> 26; t[3] += c; t[2] &= M26;
    c = t[6] >> 26; t[7] += c; t[6] &= M26;
    c = t[3] >> 25; t[4] += c; t[3] &= M25;
    c = t[7] >> 25; t[8] += c; t[7] &= M25;
    c = t[4] >> 26; t[5] += c; t[4] &= M26;
    c = t[8] >> 26; t[9] += c; t[8] &= M26;
    c = t[9] >> 25; t[9] &= M25; t[0] += c * 19;
    c = t[0] >> 26; t[1] += c; t[0] &= M26;
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = (uint32_t)t[i];
}
// normalise a loose element (limbs < 2^31) into carried form
CHIP_DEV void fe_carry(fe& h) {
    uint32_t c;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        if (k & 1) { c = h.v[k] >> 25; h.v[k] &= M25; }
        else { c = h.v[k] >> 26; h.v[k] &= M26; }
        h.v[k + 1] += c;
    }
    c = h.v[9] >> 25;
    h.v[9] &= M25;
    h.v[0] += c * 19;
    c = h.v[0] >> 26;
    h.v[0] &= M26;
    h.v[1] += c;
}

CHIP_DEV uint64_t mul32(uint32_t a, uint32_t b) { return (uint64_t)a * (uint64_t)b; }

// t = f * g column sums (f, g loose).  coefficient(i,j) = (2 if i,j odd) * (19 if i+j >= 10)
CHIP_DEV void fe_mul_cols(uint64_t t[10], const fe& f, const fe& g) {
    uint32_t g19[10], f2[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        g19[i] = g.v[i] * 19u;
        f2[i] = (i & 1) ? (f.v[i] << 1) : f.v[i];
    }
#pragma unroll
    for (int k = 0; k < 10; k++) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
        for (int j = 0; j < 10; j++) {
            const int k = (i + j) % 10;
            const bool both_odd = (i & 1) && (j & 1);
            const uint32_t fa = both_odd ? f2[i] : f.v[i];
            const uint32_t gb = (i + j >= 10) ? g19[j] : g.v[j];
            t[k] += mul32(fa, gb);
        }
    }
}
CHIP_DEV void fe_mul(fe& h, const fe& f, const fe& g) {
    uint64_t t[10];
    fe_mul_cols(t, f, g);
    fe_carry64(h, t);
}
// h = 2 f g
CHIP_DEV void fe_mul2(fe& h, const fe& f, const fe& g) {
    uint64_t t[10];
    fe_mul_cols(t, f, g);
#pragma unroll
    for (int k = 0; k < 10; k++) t[k] <<= 1;
    fe_carry64(h, t);
}
// squaring column sums: pairs i<=j, coefficient (i==j ? 1 : 2) * (2 if both odd) * (19 if wrap)
CHIP_DEV void fe_sq_cols(uint64_t t[10], const fe& f) {
    uint32_t f2[10], f19[10], f38[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        f2[i] = f.v[i] << 1;
        f19[i] = f.v[i] * 19u;
        f38[i] = f.v[i] * 38u;
    }
#pragma unroll
    for (int k = 0; k < 10; k++) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
        for (int j = i; j < 10; j++) {
            const int k = (i + j) % 10;
            const bool wrap = (i + j) >= 10;
            const bool io = i & 1, jo = j & 1;
            uint32_t a, b;
            if (i == j) {
                // coefficient: (2 if odd) * (19 if wrap)
                if (io && wrap) { a = f.v[i]; b = f38[j]; }
                else if (io) { a = f.v[i]; b = f2[j]; }
                else if (wrap) { a = f.v[i]; b = f19[j]; }
                else { a = f.v[i]; b = f.v[j]; }
            } else {
                // coefficient: 2 * (2 if both odd) * (19 if wrap); 38 only ever multiplies an odd
                // limb (< 3*2^25), 19 any limb (< 3*2^26): every factor stays below 2^32
                if (io && jo) {
                    if (wrap) { a = f2[i]; b = f38[j]; }
                    else { a = f2[i]; b = f2[j]; }
                } else if (wrap) {
                    a = f2[i]; b = f19[j];
                } else {
                    a = f2[i]; b = f.v[j];
                }
            }
            t[k] += mul32(a, b);
        }
    }
}
CHIP_DEV void fe_sq(fe& h, const fe& f) {
    uint64_t t[10];
    fe_sq_cols(t, f);
    fe_carry64(h, t);
}
CHIP_DEV void fe_sq2(fe& h, const fe& f) {
    uint64_t t[10];
    fe_sq_cols(t, f);
#pragma unroll
    for (int k = 0; k < 10; k++) t[k] <<= 1;
    fe_carry64(h, t);
}
// (a local accumulator: with h aliasing f — fe_sqn(x, x, 2) in fe_pow22523 — the compiler kept ~380 registers
// live through the square-root chain, so every kernel decoding a key ran at 1 wave per SIMD)
CHIP_DEV void fe_sqn(fe& h, const fe& f, int n) {
    fe t;
    fe_sq(t, f);
    for (int i = 1; i < n; i++) fe_sq(t, t);
    h = t;
}

// z^(2^250 - 1) and helpers for inversion / square roots
CHIP_DEV void fe_pow_common(fe& z250, fe& z11, const fe& z) {
    fe z2, z9, t, z5, z10, z20, z50, z100;
    fe_sq(z2, z);            // 2
    fe_sq(t, z2);
    fe_sq(t, t);             // 8
    fe_mul(z9, t, z);        // 9
    fe_mul(z11, z9, z2);     // 11
    fe_sq(t, z11);           // 22
    fe_mul(z5, t, z9);       // 2^5 - 1
    fe_sqn(t, z5, 5);
    fe_mul(z10, t, z5);      // 2^10 - 1
    fe_sqn(t, z10, 10);
    fe_mul(z20, t, z10);     // 2^20 - 1
    fe_sqn(t, z20, 20);
    fe_mul(t, t, z20);       // 2^40 - 1
    fe_sqn(t, t, 10);
    fe_mul(z50, t, z10);     // 2^50 - 1
    fe_sqn(t, z50, 50);
    fe_mul(z100, t, z50);    // 2^100 - 1
    fe_sqn(t, z100, 100);
    fe_mul(t, t, z100);      // 2^200 - 1
    fe_sqn(t, t, 50);
    fe_mul(z250, t, z50);    // 2^250 - 1
}
// (both write a local and copy it out: callers pass h aliasing z, e.g. ge_frombytes' fe_pow22523(X, X))
CHIP_DEV void fe_invert(fe& h, const fe& z) {
    fe z250, z11, r;
    fe_pow_common(z250, z11, z);
    fe_sqn(z250, z250, 5);   // 2^255 - 32
    fe_mul(r, z250, z11);    // 2^255 - 21 = p - 2
    h = r;
}
// (the two squarings written out: as fe_sqn(x, x, 2) the whole square root compiled to ~380 live registers)
CHIP_DEV void fe_pow22523(fe& h, const fe& z) {
    fe z250, z11, r, t;
    fe_pow_common(z250, z11, z);
    fe_sq(t, z250);
    fe_sq(t, t);             // 2^252 - 4
    fe_mul(r, t, z);         // 2^252 - 3
    h = r;
}

// canonical encoding into 8 little-endian words (input carried or loose < 2^31 limbs)
CHIP_DEV void fe_tobytes(uint32_t w[8], const fe& f) {
    fe h = f;
    fe_carry(h);
    uint32_t q = (h.v[0] + 19u) >> 26;
#pragma unroll
    for (int i = 1; i < 10; i++) q = (h.v[i] + q) >> ((i & 1) ? 25 : 26);
    h.v[0] += 19u * q;
    uint32_t c;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        if (k & 1) { c = h.v[k] >> 25; h.v[k] &= M25; }
        else { c = h.v[k] >> 26; h.v[k] &= M26; }
        h.v[k + 1] += c;
    }
    h.v[9] &= M25;
    w[0] = h.v[0] | (h.v[1] << 26);
    w[1] = (h.v[1] >> 6) | (h.v[2] << 19);
    w[2] = (h.v[2] >> 13) | (h.v[3] << 13);
    w[3] = (h.v[3] >> 19) | (h.v[4] << 6);
    w[4] = h.v[5] | (h.v[6] << 25);
    w[5] = (h.v[6] >> 7) | (h.v[7] << 19);
    w[6] = (h.v[7] >> 13) | (h.v[8] << 12);
    w[7] = (h.v[8] >> 20) | (h.v[9] << 6);
}
// low 255 bits of 8 little-endian words (value may be >= p: i2p decode tolerates it)
CHIP_DEV void fe_frombytes(fe& h, const uint32_t w[8]) {
    h.v[0] = w[0] & M26;
    h.v[1] = ((w[0] >> 26) | (w[1] << 6)) & M25;
    h.v[2] = ((w[1] >> 19) | (w[2] << 13)) & M26;
    h.v[3] = ((w[2] >> 13) | (w[3] << 19)) & M25;
    h.v[4] = (w[3] >> 6) & M26;
    h.v[5] = w[4] & M25;
    h.v[6] = ((w[4] >> 25) | (w[5] << 7)) & M26;
    h.v[7] = ((w[5] >> 19) | (w[6] << 13)) & M25;
    h.v[8] = ((w[6] >> 12) | (w[7] << 20)) & M26;
    h.v[9] = (w[7] >> 6) & M25;
}
CHIP_DEV bool fe_isnonzero(const fe& f) {
    uint32_t w[8];
    fe_tobytes(w, f);
    return (w[0] | w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7]) != 0;
}
CHIP_DEV uint32_t fe_isnegative(const fe& f) {
    uint32_t w[8];
    fe_tobytes(w, f);
    return w[0] & 1;
}

// ---------------------------------------------------------------------------------------
// Group elements (twisted Edwards a = -1, extended coordinates; ref10 naming)
struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };       // completed: x = X/Z, y = Y/T
struct ge_cached { fe YpX, YmX, Z, T2d; };
struct ge_niels { fe ypx, ymx, xy2d; };

CHIP_DEV void ge_p2_0(ge_p2& r) { fe_0(r.X); fe_1(r.Y); fe_1(r.Z); }
CHIP_DEV void ge_p3_0(ge_p3& r) { fe_0(r.X); fe_1(r.Y); fe_1(r.Z); fe_0(r.T); }

CHIP_DEV void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
    fe_mul(r.X, p.X, p.T);
    fe_mul(r.Y, p.Z, p.Y);
    fe_mul(r.Z, p.Z, p.T);
}
CHIP_DEV void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
    fe_mul(r.X, p.X, p.T);
    fe_mul(r.Y, p.Z, p.Y);
    fe_mul(r.Z, p.Z, p.T);
    fe_mul(r.T, p.X, p.Y);
}
// r = 2p (p2 -> p1p1); output limbs: X, T carried; Y < 2^27; Z loose
CHIP_DEV void ge_p2_dbl(ge_p1p1& r, const ge_p2& p) {
    fe XX, YY, B, A, s;
    fe_sq(XX, p.X);
    fe_sq(YY, p.Y);
    fe_sq2(B, p.Z);
    fe_add(s, p.X, p.Y);
    fe_sq(A, s);
    fe_add(r.Y, YY, XX);          // < 2^27
    fe_sub(r.Z, YY, XX);          // loose
    fe_sub4(r.X, A, r.Y);         // A - (YY + XX)
    fe_carry(r.X);
    fe_add(s, B, XX);             // 2Z^2 + XX
    fe_sub(r.T, s, YY);           // B - (YY - XX)
    fe_carry(r.T);
}
CHIP_DEV void ge_p3_to_p2(ge_p2& r, const ge_p3& p) { r.X = p.X; r.Y = p.Y; r.Z = p.Z; }

// r = p + q (neg: p - q); q cached with carried coordinates
CHIP_DEV void ge_add_cached(ge_p1p1& r, const ge_p3& p, const ge_cached& q, bool neg) {
    fe ypx, ymx, A, B, C, D2, qp, qm, z1, z2;
    fe_add(ypx, p.Y, p.X);
    fe_sub(ymx, p.Y, p.X);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        qp.v[i] = neg ? q.YmX.v[i] : q.YpX.v[i];
        qm.v[i] = neg ? q.YpX.v[i] : q.YmX.v[i];
    }
    fe_mul(A, ypx, qp);
    fe_mul(B, ymx, qm);
    fe_mul(C, q.T2d, p.T);
    fe_mul2(D2, p.Z, q.Z);
    fe_sub(r.X, A, B);
    fe_add(r.Y, A, B);
    fe_add(z1, D2, C);
    fe_sub(z2, D2, C);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        r.Z.v[i] = neg ? z2.v[i] : z1.v[i];
        r.T.v[i] = neg ? z1.v[i] : z2.v[i];
    }
}
// r = p + q (neg: p - q); q affine Niels; pZ2 = 2 * p.Z carried
CHIP_DEV void ge_madd(ge_p1p1& r, const ge_p3& p, const fe& pZ2, const ge_niels& q, bool neg) {
    fe ypx, ymx, A, B, C, qp, qm, z1, z2;
    fe_add(ypx, p.Y, p.X);
    fe_sub(ymx, p.Y, p.X);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        qp.v[i] = neg ? q.ymx.v[i] : q.ypx.v[i];
        qm.v[i] = neg ? q.ypx.v[i] : q.ymx.v[i];
    }
    fe_mul(A, ypx, qp);
    fe_mul(B, ymx, qm);
    fe_mul(C, q.xy2d, p.T);
    fe_sub(r.X, A, B);
    fe_add(r.Y, A, B);
    fe_add(z1, pZ2, C);
    fe_sub(z2, pZ2, C);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        r.Z.v[i] = neg ? z2.v[i] : z1.v[i];
        r.T.v[i] = neg ? z1.v[i] : z2.v[i];
    }
}
CHIP_DEV void ge_p3_to_cached(ge_cached& r, const ge_p3& p) {
    fe_add(r.YpX, p.Y, p.X);
    fe_carry(r.YpX);
    fe_sub(r.YmX, p.Y, p.X);
    fe_carry(r.YmX);
    r.Z = p.Z;
    fe c;
    fe_from_c(c, ED_D2);
    fe_mul(r.T2d, p.T, c);
}
CHIP_DEV void ge_p3_dbl(ge_p1p1& r, const ge_p3& p) {
    ge_p2 q;
    ge_p3_to_p2(q, p);
    ge_p2_dbl(r, q);
}

// canonical encoding of a projective point: y with bit 255 = sign(x)
CHIP_DEV void ge_tobytes(uint32_t w[8], const fe& X, const fe& Y, const fe& Z) {
    fe zi, x, y;
    fe_invert(zi, Z);
    fe_mul(x, X, zi);
    fe_mul(y, Y, zi);
    fe_tobytes(w, y);
    w[7] |= fe_isnegative(x) << 31;
}

// GroupElement(curve, bytes) decompression (i2p 0.2.0 semantics). Returns false if
// "not a valid point".  w: 8 LE words of the encoded point.
CHIP_DEV bool ge_frombytes(ge_p3& h, const uint32_t w[8]) {
    fe u, v, v3, vxx, chk, one, d;
    fe_1(one);
    fe_frombytes(h.Y, w);
    fe_sq(u, h.Y);
    fe_from_c(d, ED_D);
    fe_mul(v, u, d);
    fe_add(v, v, one);           // v = d y^2 + 1
    fe_sub(u, u, one);           // u = y^2 - 1
    fe_carry(u);
    fe_carry(v);
    fe_sq(v3, v);
    fe_mul(v3, v3, v);           // v^3
    fe_sq(h.X, v3);
    fe_mul(h.X, h.X, v);
    fe_mul(h.X, h.X, u);         // u v^7
    fe_pow22523(h.X, h.X);       // (u v^7)^((p-5)/8)
    fe_mul(h.X, h.X, v3);
    fe_mul(h.X, h.X, u);         // u v^3 (u v^7)^((p-5)/8)
    fe_sq(vxx, h.X);
    fe_mul(vxx, vxx, v);
    fe_sub(chk, vxx, u);
    if (fe_isnonzero(chk)) {
        fe_add(chk, vxx, u);
        if (fe_isnonzero(chk)) return false;
        fe s;
        fe_from_c(s, ED_SQRTM1);
        fe_mul(h.X, h.X, s);
    }
    if (fe_isnegative(h.X) != (w[7] >> 31)) {
        fe_neg(h.X, h.X);
        fe_carry(h.X);
    }
    fe_1(h.Z);
    fe_mul(h.T, h.X, h.Y);
    return true;
}
