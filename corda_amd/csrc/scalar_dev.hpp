// scalar_dev.hpp — arithmetic modulo the Ed25519 group order L = 2^252 + c (c < 2^125) and the
// scalar recodings used by the verify kernel.  Scalars are 8 little-endian u32 words.
#pragma once
#include "common.hpp"
#include "curve_consts.hpp"

// c = L - 2^252 = 0x14def9dea2f79cd65812631a5cf5d3ed
#define SC_C0 0x5cf5d3edu
#define SC_C1 0x5812631au
#define SC_C2 0xa2f79cd6u
#define SC_C3 0x14def9deu

// r = (r * 2^32 + w) mod L, r < L on input and output.
// t = q 2^252 + u0 (u0 < 2^252, q < 2^33); 2^252 = -c (mod L) so t = u0 - q c, in (-2^158, 2^252).
CHIP_DEV void sc_horner_step(uint32_t r[8], uint32_t w) {
    uint32_t t[9];
    t[0] = w;
#pragma unroll
    for (int i = 0; i < 8; i++) t[i + 1] = r[i];
    const uint64_t q = ((uint64_t)t[8] << 4) | (t[7] >> 28);
    t[7] &= 0x0fffffffu;
    const uint32_t ql = (uint32_t)q, qh = (uint32_t)(q >> 32);
    // qc = q * c, 6 words
    uint32_t qc[6];
    uint64_t acc = (uint64_t)ql * SC_C0;
    qc[0] = (uint32_t)acc;
    acc = (acc >> 32) + (uint64_t)ql * SC_C1;
    qc[1] = (uint32_t)acc;
    acc = (acc >> 32) + (uint64_t)ql * SC_C2;
    qc[2] = (uint32_t)acc;
    acc = (acc >> 32) + (uint64_t)ql * SC_C3;
    qc[3] = (uint32_t)acc;
    qc[4] = (uint32_t)(acc >> 32);
    qc[5] = 0;
    if (qh) {   // + c << 32
        uint64_t s = (uint64_t)qc[1] + SC_C0;
        qc[1] = (uint32_t)s;
        s = (s >> 32) + qc[2] + SC_C1;
        qc[2] = (uint32_t)s;
        s = (s >> 32) + qc[3] + SC_C2;
        qc[3] = (uint32_t)s;
        s = (s >> 32) + qc[4] + SC_C3;
        qc[4] = (uint32_t)s;
        qc[5] = (uint32_t)(s >> 32);
    }
    // u = t[0..7] - qc
    uint64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t sub = (i < 6 ? (uint64_t)qc[i] : 0ull) + br;
        const uint64_t d = (uint64_t)t[i] - sub;
        r[i] = (uint32_t)d;
        br = (d >> 63) & 1;   // borrow (t[i] < sub)
    }
    if (br) {   // negative: + L
        uint64_t s = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            s += (uint64_t)r[i] + ED_L[i];
            r[i] = (uint32_t)s;
            s >>= 32;
        }
    }
}
// 512-bit little-endian (16 words) mod L
CHIP_DEV void sc_reduce512(uint32_t r[8], const uint32_t x[16]) {
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = 0;
#pragma unroll
    for (int i = 15; i >= 0; i--) sc_horner_step(r, x[i]);
}
CHIP_DEV void sc_reduce256(uint32_t r[8], const uint32_t x[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = 0;
#pragma unroll
    for (int i = 7; i >= 0; i--) sc_horner_step(r, x[i]);
}
// r = (a - b) mod L for a, b < L
CHIP_DEV void sc_sub(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
    uint64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t d = (uint64_t)a[i] - (uint64_t)b[i] - br;
        r[i] = (uint32_t)d;
        br = (d >> 63) & 1;
    }
    if (br) {
        uint64_t s = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            s += (uint64_t)r[i] + ED_L[i];
            r[i] = (uint32_t)s;
            s >>= 32;
        }
    }
}

CHIP_DEV uint32_t sel8(const uint32_t v[8], uint32_t i) {
    uint32_t r = v[0];
#pragma unroll
    for (int k = 1; k < 8; k++) r = (i == (uint32_t)k) ? v[k] : r;
    return r;
}

// Number of carries i2p/ref10 GroupElement.slide() drops off digit 255 for scalar s.
// Only reachable for s >= 2^255 (carries below that never overflow: SURVEY/DESIGN note);
// exact literal simulation of the recoding over a 256-bit register.
CHIP_DEV uint32_t slide_drops(const uint32_t s[8]) {
    // ref10 slide() over the bits of s, word by word: word k (static after unrolling) and its successor hold
    // every bit a window anchored in word k looks at (<= 6 ahead), so no register is indexed dynamically
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = s[k];
    uint32_t drops = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        for (uint32_t j = 0; j < 32; j++) {
            const uint32_t i = 32u * k + j;
            if (!((v[k] >> j) & 1u)) continue;
            int acc = 1;
            for (uint32_t b = 1; b <= 6 && i + b < 256; b++) {
                const uint32_t pos = j + b;   // bit of the 64-bit window (v[k+1] : v[k])
                const uint64_t win = ((uint64_t)(k < 7 ? v[k < 7 ? k + 1 : 7] : 0u) << 32) | v[k];
                if (!((win >> pos) & 1u)) continue;
                if (acc + (1 << b) <= 15) {
                    acc += 1 << b;
                    if (pos < 32) v[k] &= ~(1u << pos);
                    else if (k < 7) v[k < 7 ? k + 1 : 7] &= ~(1u << (pos - 32));
                } else if (acc - (1 << b) >= -15) {
                    acc -= 1 << b;
                    // v += 2^(32k + pos) (binary increment), overflow past bit 255 = the dropped carry
                    uint64_t c = 0;
#pragma unroll
                    for (int q = k; q < 8; q++) {
                        const uint32_t add = (q == k && pos < 32) ? (1u << pos)
                                             : ((q == k + 1 && pos >= 32) ? (1u << (pos - 32)) : 0u);
                        c += (uint64_t)v[q] + add;
                        v[q] = (uint32_t)c;
                        c >>= 32;
                    }
                    drops += (uint32_t)c;
                } else {
                    break;
                }
            }
        }
    }
    return drops;
}

// signed radix-16 recoding of a < 2^253: 64 digits in [-8, 7] (top digit <= 2), returned as
// 64 biased nibbles (digit + 8) packed little-endian into 8 words.
CHIP_DEV void sc_recode16(uint32_t out[8], const uint32_t a[8]) {
    int carry = 0;
#pragma unroll
    for (int w = 0; w < 8; w++) {
        uint32_t o = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            int v = (int)((a[w] >> (4 * k)) & 15u) + carry;
            carry = (v + 8) >> 4;
            v -= carry << 4;
            o |= (uint32_t)(v + 8) << (4 * k);
        }
        out[w] = o;
    }
}
// signed radix-256 recoding of a < 2^253: 32 digits in [-128, 127] (top <= 17), biased by 128
CHIP_DEV void sc_recode256(uint32_t out[8], const uint32_t a[8]) {
    int carry = 0;
#pragma unroll
    for (int w = 0; w < 8; w++) {
        uint32_t o = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            int v = (int)((a[w] >> (8 * k)) & 255u) + carry;
            carry = (v + 128) >> 8;
            v -= carry << 8;
            o |= (uint32_t)(v + 128) << (8 * k);
        }
        out[w] = o;
    }
}
// shift a 256-bit little-endian register left by n (n < 32)
CHIP_DEV void shl256(uint32_t v[8], int n) {
#pragma unroll
    for (int k = 7; k > 0; k--) v[k] = (v[k] << n) | (v[k - 1] >> (32 - n));
    v[0] <<= n;
}
