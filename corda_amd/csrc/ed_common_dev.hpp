// ed_common_dev.hpp — pieces shared by the two Ed25519 verify schedules (ed25519.hip: windowed
// Straus with doublings; ed25519_comb.hip: per-key comb tables): the i2p challenge hash, the
// effective S of i2p's slide() recoding, and table row load/store helpers.
#pragma once
#include "fe25519_dev.hpp"
#include "scalar_dev.hpp"
#include "sha2_dev.hpp"

// SHA-512(R || Abyte || M) as a little-endian 512-bit integer (16 words)
//   i2p EdDSAEngine.engineVerify: digest.update(Rbyte); digest.update(key.getAbyte()); digest.update(M)
CHIP_DEV void ed_challenge(uint32_t hx[16], const uint32_t R[8], const uint32_t Ab[8], const uint8_t* m, uint32_t ml) {
    uint64_t H[8];
    sha512_init(H);
    const uint64_t total = 64ull + ml;
    const uint32_t nblocks = (uint32_t)((total + 17 + 127) / 128);
    for (uint32_t b = 0; b < nblocks; b++) {
        uint64_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            uint64_t v;
            if (b == 0 && j < 8) {
                const uint32_t lo = (j < 4) ? R[2 * j] : Ab[2 * (j - 4)];
                const uint32_t hi = (j < 4) ? R[2 * j + 1] : Ab[2 * (j - 4) + 1];
                v = ((uint64_t)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
            } else {
                // message bytes at offset (block byte - 64), SHA padding byte 0x80 after the end
                const int64_t q = (int64_t)b * 128 + 8 * j - 64;
                v = ((uint64_t)comp_word(m, ml, q) << 32) | comp_word(m, ml, q + 4);
            }
            w[j] = v;
        }
        if (b == nblocks - 1) {
            w[14] = 0;
            w[15] = total * 8;
        }
        sha512_compress(H, w);
    }
    // digest bytes are big-endian state words; as a little-endian integer word 2j = bswap(hi32(H_j))
#pragma unroll
    for (int j = 0; j < 8; j++) {
        hx[2 * j] = __builtin_bswap32((uint32_t)(H[j] >> 32));
        hx[2 * j + 1] = __builtin_bswap32((uint32_t)H[j]);
    }
}

// The scalar i2p actually multiplies B by: S (not range checked) recoded by ref10 slide(), which
// drops a carry past digit 255 (only reachable for S >= 2^255), reduced mod L.
CHIP_DEV void ed_effective_s(uint32_t s[8], const uint32_t S[8]) {
    sc_reduce256(s, S);
    if (S[7] >> 31) {
        const uint32_t d = slide_drops(S);
        uint32_t k2[8];
#pragma unroll
        for (int q = 0; q < 8; q++) k2[q] = ED_2_256_MOD_L[q];
        for (uint32_t t = 0; t < d; t++) sc_sub(s, s, k2);
    }
}

// cached point row: YpX, YmX, Z, T2d (40 words)
CHIP_DEV void ed_store_cached(uint32_t* dst, const ge_cached& c) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        dst[i] = c.YpX.v[i];
        dst[10 + i] = c.YmX.v[i];
        dst[20 + i] = c.Z.v[i];
        dst[30 + i] = c.T2d.v[i];
    }
}
CHIP_DEV void ed_load_cached(ge_cached& c, const uint32_t* __restrict__ src) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
#pragma unroll
    for (int q = 0; q < 10; q++) {
        const uint4 x = s4[q];
        const uint32_t vals[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int idx = 4 * q + e;
            const int f = idx / 10, l = idx % 10;
            if (f == 0) c.YpX.v[l] = vals[e];
            else if (f == 1) c.YmX.v[l] = vals[e];
            else if (f == 2) c.Z.v[l] = vals[e];
            else c.T2d.v[l] = vals[e];
        }
    }
}
// extended point row: X, Y, Z, T (40 words)
CHIP_DEV void ed_store_p3(uint32_t* dst, const ge_p3& p) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        dst[i] = p.X.v[i];
        dst[10 + i] = p.Y.v[i];
        dst[20 + i] = p.Z.v[i];
        dst[30 + i] = p.T.v[i];
    }
}
CHIP_DEV void ed_load_p3(ge_p3& p, const uint32_t* __restrict__ src) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        p.X.v[i] = src[i];
        p.Y.v[i] = src[10 + i];
        p.Z.v[i] = src[20 + i];
        p.T.v[i] = src[30 + i];
    }
}
