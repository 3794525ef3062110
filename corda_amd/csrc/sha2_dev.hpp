// sha2_dev.hpp — FIPS 180-4 SHA-256 / SHA-512 compression functions for gfx950 device code.
// One lane = one message; block words are supplied by the caller (big-endian already packed).
#pragma once
#include "common.hpp"

__device__ __constant__ const uint32_t SHA256_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

__device__ __constant__ const uint64_t SHA512_K[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

// LUT index = S0 << 2 | S1 << 1 | S2
#define BITOP3_XOR3 0x96
#define BITOP3_CH 0xCA    // S0 ? S1 : S2
#define BITOP3_MAJ 0xE8
// 16 rounds (SHA-256 and SHA-512) with the round function's variables rotated by name (8 rounds = one full rotation: no moves), the
// message schedule in place in w[16] (static indices: the 16 rounds of a group are unrolled, the 5 groups are not)
#define SHA2_16(BODY)                                                                                          \
    BODY(0, a, b, c, d, e, f, g, hh) BODY(1, hh, a, b, c, d, e, f, g) BODY(2, g, hh, a, b, c, d, e, f)          \
    BODY(3, f, g, hh, a, b, c, d, e) BODY(4, e, f, g, hh, a, b, c, d) BODY(5, d, e, f, g, hh, a, b, c)          \
    BODY(6, c, d, e, f, g, hh, a, b) BODY(7, b, c, d, e, f, g, hh, a) BODY(8, a, b, c, d, e, f, g, hh)          \
    BODY(9, hh, a, b, c, d, e, f, g) BODY(10, g, hh, a, b, c, d, e, f) BODY(11, f, g, hh, a, b, c, d, e)        \
    BODY(12, e, f, g, hh, a, b, c, d) BODY(13, d, e, f, g, hh, a, b, c) BODY(14, c, d, e, f, g, hh, a, b)       \
    BODY(15, b, c, d, e, f, g, hh, a)
CHIP_DEV uint32_t rotr32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
CHIP_DEV uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

CHIP_DEV void sha256_init(uint32_t h[8]) {
    h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
    h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
}
// w: 16 big-endian message words (clobbered as the schedule ring).  Three-input logic as v_bitop3_b32 (xor3 / ch /
// maj: dual-issue class on gfx950), rotates as v_alignbit_b32; rounds in unrolled groups of 16 with the state
// rotated by name (8 rounds = one rotation) and the schedule ring at static indices.
#define SHA256_ROUND(a, b, c, d, e, f, g, hh, kw)                                                                \
    do {                                                                                                         \
        const uint32_t S1_ = __builtin_amdgcn_bitop3_b32(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25), BITOP3_XOR3); \
        const uint32_t t1_ = hh + S1_ + __builtin_amdgcn_bitop3_b32(e, f, g, BITOP3_CH) + (kw);                   \
        const uint32_t S0_ = __builtin_amdgcn_bitop3_b32(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22), BITOP3_XOR3); \
        d += t1_;                                                                                                \
        hh = t1_ + S0_ + __builtin_amdgcn_bitop3_b32(a, b, c, BITOP3_MAJ);                                      \
    } while (0)
CHIP_DEV void sha256_compress(uint32_t h[8], uint32_t w[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#define SHA256_R0(j, A, B, C, D, E, F, G, H) SHA256_ROUND(A, B, C, D, E, F, G, H, SHA256_K[j] + w[j]);
    SHA2_16(SHA256_R0)
#undef SHA256_R0
#pragma unroll 1
    for (int r = 16; r < 64; r += 16) {
#define SHA256_RS(j, A, B, C, D, E, F, G, H)                                                                   \
        {                                                                                                      \
            const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];                                       \
            w[j] += __builtin_amdgcn_bitop3_b32(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3, BITOP3_XOR3) +       \
                    w[(j + 9) & 15] + __builtin_amdgcn_bitop3_b32(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10, BITOP3_XOR3); \
            SHA256_ROUND(A, B, C, D, E, F, G, H, SHA256_K[r + j] + w[j]);                                      \
        }
        SHA2_16(SHA256_RS)
#undef SHA256_RS
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

CHIP_DEV void sha512_init(uint64_t h[8]) {
    h[0] = 0x6a09e667f3bcc908ull; h[1] = 0xbb67ae8584caa73bull; h[2] = 0x3c6ef372fe94f82bull;
    h[3] = 0xa54ff53a5f1d36f1ull; h[4] = 0x510e527fade682d1ull; h[5] = 0x9b05688c2b3e6c1full;
    h[6] = 0x1f83d9abfb41bd6bull; h[7] = 0x5be0cd19137e2179ull;
}
// 64-bit rotates / shifts / three-input logic on the 32-bit halves: one v_alignbit_b32 per half for a rotate (the
// compiler otherwise builds them from two 64-bit shifts and two ORs), one v_bitop3_b32 per half for xor3 / ch / maj
// (a dual-issue class instruction on gfx950: tools/microbench_valu.hip)
CHIP_DEV uint64_t u64_of(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
template <int N>
CHIP_DEV uint64_t rotr64h(uint64_t x) {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if (N < 32) return u64_of(__builtin_amdgcn_alignbit(hi, lo, N), __builtin_amdgcn_alignbit(lo, hi, N));
    return u64_of(__builtin_amdgcn_alignbit(lo, hi, N - 32), __builtin_amdgcn_alignbit(hi, lo, N - 32));
}
template <int N>
CHIP_DEV uint64_t shr64h(uint64_t x) {   // N < 32
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    return u64_of(__builtin_amdgcn_alignbit(hi, lo, N), hi >> N);
}
template <uint32_t LUT>
CHIP_DEV uint64_t bitop3_64(uint64_t a, uint64_t b, uint64_t c) {
    return u64_of(__builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, LUT),
                  __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), LUT));
}

// one round of SHA-512 on the rotating state (a..hh renamed by the caller's unrolled sequence)
#define SHA512_ROUND(a, b, c, d, e, f, g, hh, kw)                                                                \
    do {                                                                                                         \
        const uint64_t S1_ = bitop3_64<BITOP3_XOR3>(rotr64h<14>(e), rotr64h<18>(e), rotr64h<41>(e));            \
        const uint64_t t1_ = hh + S1_ + bitop3_64<BITOP3_CH>(e, f, g) + (kw);                                   \
        const uint64_t S0_ = bitop3_64<BITOP3_XOR3>(rotr64h<28>(a), rotr64h<34>(a), rotr64h<39>(a));            \
        d += t1_;                                                                                                \
        hh = t1_ + S0_ + bitop3_64<BITOP3_MAJ>(a, b, c);                                                        \
    } while (0)
CHIP_DEV void sha512_compress(uint64_t h[8], uint64_t w[16]) {
    uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#define SHA512_R0(j, A, B, C, D, E, F, G, H) SHA512_ROUND(A, B, C, D, E, F, G, H, SHA512_K[j] + w[j]);
    SHA2_16(SHA512_R0)
#undef SHA512_R0
#pragma unroll 1
    for (int r = 16; r < 80; r += 16) {
#define SHA512_RS(j, A, B, C, D, E, F, G, H)                                                                   \
        {                                                                                                      \
            const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];                                       \
            w[j] += bitop3_64<BITOP3_XOR3>(rotr64h<1>(w15), rotr64h<8>(w15), shr64h<7>(w15)) + w[(j + 9) & 15] + \
                    bitop3_64<BITOP3_XOR3>(rotr64h<19>(w2), rotr64h<61>(w2), shr64h<6>(w2));                   \
            SHA512_ROUND(A, B, C, D, E, F, G, H, SHA512_K[r + j] + w[j]);                                      \
        }
        SHA2_16(SHA512_RS)
#undef SHA512_RS
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// big-endian word at byte offset q of a pool byte string p[0..len) followed by the SHA-2 padding
// byte 0x80 and zeros (q may be negative: those bytes read as 0).  Aligned dword loads when the
// word lies inside the string.
CHIP_DEV uint32_t comp_word(const uint8_t* p, uint32_t len, int64_t q) {
    if (q >= 0 && q + 4 <= (int64_t)len) {
        const uint32_t sh = (uint32_t)((uintptr_t)(p + q) & 3u);
        const uint32_t* ap = reinterpret_cast<const uint32_t*>(p + q - sh);   // pointer arithmetic: stays global
        uint32_t lo = ap[0];
        uint32_t v = lo;
        if (sh) {
            const uint32_t hi = ap[1];   // in bounds: q + 4 <= len and the word straddles
            v = __builtin_amdgcn_alignbyte(hi, lo, sh);
        }
        return __builtin_bswap32(v);
    }
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int64_t j = q + k;
        uint32_t by = 0;
        if (j >= 0 && j < (int64_t)len) by = p[j];
        else if (j == (int64_t)len) by = 0x80u;
        v = (v << 8) | by;
    }
    return v;
}

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));   // dwordx4 at dword alignment

// the 64-byte block at p (inside the string) as 16 big-endian words: four 4-byte-aligned dwordx4 loads and one
// dword (the bytes are realigned with v_alignbyte), all independent; every load overlaps the block, so none can
// touch a page the string does not
CHIP_DEV void block_words(uint32_t w[16], const uint8_t* p) {
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t* ap = reinterpret_cast<const uint32_t*>(p - sh);
    uint32_t d[17];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const u32x4_a4 v = *reinterpret_cast<const u32x4_a4*>(ap + 4 * k);
        d[4 * k] = v.x;
        d[4 * k + 1] = v.y;
        d[4 * k + 2] = v.z;
        d[4 * k + 3] = v.w;
    }
    d[16] = sh ? ap[16] : 0u;
#pragma unroll
    for (int j = 0; j < 16; j++) w[j] = __builtin_bswap32(__builtin_amdgcn_alignbyte(d[j + 1], d[j], sh));
}

// SHA-256 of pool bytes p[0..len): state words in H (big-endian digest words).  Whole blocks are fetched one
// block ahead of the compression (block_words), so a block's loads are in flight while the previous one is
// compressed; the tail block(s) with the padding go through comp_word
CHIP_DEV void sha256_bytes(uint32_t H[8], const uint8_t* p, uint32_t len) {
    uint32_t w[16], nx[16];
    sha256_init(H);
    const uint64_t total = len;
    const uint32_t nblocks = (uint32_t)((total + 9 + 63) / 64);
    const uint32_t nfull = len / 64;   // blocks wholly inside the string
    if (nfull) block_words(nx, p);
    for (uint32_t b = 0; b < nblocks; b++) {
        if (b < nfull) {
#pragma unroll
            for (int j = 0; j < 16; j++) w[j] = nx[j];
            if (b + 1 < nfull) block_words(nx, p + (uint64_t)(b + 1) * 64);
        } else {
#pragma unroll
            for (int j = 0; j < 16; j++) w[j] = comp_word(p, len, (int64_t)b * 64 + 4 * j);
        }
        if (b == nblocks - 1) {
            w[14] = (uint32_t)((total * 8) >> 32);
            w[15] = (uint32_t)(total * 8);
        }
        sha256_compress(H, w);
    }
}
