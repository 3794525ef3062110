// ed_common_dev.hpp — pieces shared by the two Ed25519 verify schedules (ed25519.hip: windowed
// Straus with doublings; ed25519_comb.hip: per-key comb tables): the i2p challenge hash, the
// effective S of i2p's slide() recoding, and table row load/store helpers.
#pragma once
#include "fe25519_dev.hpp"
#include "scalar_dev.hpp"
#include "sha2_dev.hpp"

// big-endian word of message bytes m[q .. q+4) followed by the SHA-2 padding byte 0x80 and zeros, from the message's
// aligned dwords D (d1 = index of the last dword holding a message byte: every load stays inside dwords that hold
// message bytes, so it never leaves the message's pages); sh = the message's address mod 4.  Branch-free.
CHIP_DEV uint32_t msg_be_word(const uint32_t* __restrict__ D, int32_t d1, uint32_t sh, uint32_t ml, int32_t q) {
    const int32_t k = q >> 2;
    const uint32_t lo = D[min(k, d1)], hi = D[min(k + 1, d1)];
    const uint32_t be = __builtin_bswap32(__builtin_amdgcn_alignbyte(hi, lo, sh));
    const int32_t valid = (int32_t)ml - q;                     // message bytes in this word (may be <= 0)
    const uint32_t vs = (uint32_t)min(max(valid, 0), 4);
    const uint32_t keep = (uint32_t)~(0xffffffffull >> (8 * vs));
    const uint32_t pad = (uint32_t)(0x80000000ull >> (8 * vs)) & (uint32_t)((int32_t)~valid >> 31);
    return (be & keep) | pad;
}

// SHA-512(R || Abyte || M) as a little-endian 512-bit integer (16 words)
//   i2p EdDSAEngine.engineVerify: digest.update(Rbyte); digest.update(key.getAbyte()); digest.update(M)
// `safe`: any valid byte address (an empty message reads nothing of its own)
CHIP_DEV void ed_challenge(uint32_t hx[16], const uint32_t R[8], const uint32_t Ab[8], const uint8_t* m, uint32_t ml,
                           const uint8_t* safe) {
    uint64_t H[8];
    sha512_init(H);
    const uint64_t total = 64ull + ml;
    const uint32_t nblocks = (uint32_t)((total + 17 + 127) / 128);
    const uint8_t* base = ml ? m : safe;
    const uint32_t sh = (uint32_t)((uintptr_t)base & 3u);
    const uint32_t* D = reinterpret_cast<const uint32_t*>(base - sh);
    const int32_t d1 = ml ? (int32_t)((sh + ml + 3) >> 2) - 1 : 0;
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
                const int32_t q = (int32_t)b * 128 + 8 * j - 64;
                v = ((uint64_t)msg_be_word(D, d1, sh, ml, q) << 32) | msg_be_word(D, d1, sh, ml, q + 4);
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

// ---- signed table rows: the sign of a digit applied by addressing (Y+X / Y-X swapped) and one bit select ----
// (m & a) | (~m & b) as one v_bfi_b32 (the compiler otherwise emits v_cndmask_b32_e32 on VCC, which issues at
// about a quarter of the rate when several follow each other: tools/microbench_valu.hip)
CHIP_DEV uint32_t bit_select(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}
// affine Niels entry with the sign applied by addressing: q+ = [ypx, ymx], q- = [ymx, ypx] (-Q negates x),
// xy2d as stored; neg reported for the caller's C term
CHIP_DEV void ed_load_niels_signed(fe& qp, fe& qm, fe& xy2d, const uint32_t* __restrict__ e, bool neg) {
    const uint2* p = reinterpret_cast<const uint2*>(e + (neg ? 10 : 0));
    const uint2* m = reinterpret_cast<const uint2*>(e + (neg ? 0 : 10));
    const uint4* x = reinterpret_cast<const uint4*>(e + 20);
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const uint2 a = p[k], b = m[k];
        qp.v[2 * k] = a.x;
        qp.v[2 * k + 1] = a.y;
        qm.v[2 * k] = b.x;
        qm.v[2 * k + 1] = b.y;
    }
    const uint4 x0 = x[0], x1 = x[1];
    const uint2 x2 = reinterpret_cast<const uint2*>(e + 28)[0];
    xy2d.v[0] = x0.x; xy2d.v[1] = x0.y; xy2d.v[2] = x0.z; xy2d.v[3] = x0.w;
    xy2d.v[4] = x1.x; xy2d.v[5] = x1.y; xy2d.v[6] = x1.z; xy2d.v[7] = x1.w;
    xy2d.v[8] = x2.x; xy2d.v[9] = x2.y;
}
// r = p + (+-q), q affine Niels loaded signed (qp, qm swapped for -q); pZ2 = 2 p.Z; the sign of the xy2d term
// is the one select left (z1 / z2 swap, negm = all-ones for -q)
CHIP_DEV void ge_madd_signed(ge_p1p1& r, const ge_p3& p, const fe& pZ2, const fe& qp, const fe& qm, const fe& xy2d,
                             uint32_t negm) {
    fe ypx, ymx, A, B, C, z1, z2;
    fe_add(ypx, p.Y, p.X);
    fe_sub(ymx, p.Y, p.X);
    fe_mul(A, ypx, qp);
    fe_mul(B, ymx, qm);
    fe_mul(C, xy2d, p.T);
    fe_sub(r.X, A, B);
    fe_add(r.Y, A, B);
    fe_add(z1, pZ2, C);
    fe_sub(z2, pZ2, C);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        r.Z.v[i] = bit_select(negm, z2.v[i], z1.v[i]);
        r.T.v[i] = bit_select(negm, z1.v[i], z2.v[i]);
    }
}
// k_ed_comb_hash: h = SHA-512(R || A || M) mod L and the effective S, recoded (h: signed radix-2^W bytes for
// the table half; S: signed radix-2^16 digits for [S]B) into the hand-off rows of bmid.  Its SHA-512 state
// sets the register budget, so the [S]B additions run in a kernel of their own at twice the occupancy.
// row j of a window as the signed multiple +-j: Y+X / Y-X swapped by address for -j
CHIP_DEV void ed_load_row_signed(ge_cached& q, const uint32_t* __restrict__ row, bool neg) {
    const uint2* p = reinterpret_cast<const uint2*>(row + (neg ? 10 : 0));
    const uint2* m = reinterpret_cast<const uint2*>(row + (neg ? 0 : 10));
    const uint4* zt = reinterpret_cast<const uint4*>(row + 20);
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const uint2 a = p[k], b = m[k];
        q.YpX.v[2 * k] = a.x;
        q.YpX.v[2 * k + 1] = a.y;
        q.YmX.v[2 * k] = b.x;
        q.YmX.v[2 * k + 1] = b.y;
    }
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const uint4 x = zt[k];
        const uint32_t v[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int i = 4 * k + e;
            if (i < 10) q.Z.v[i] = v[e];
            else q.T2d.v[i - 10] = v[e];
        }
    }
}
// r = p + (+-q): q = [Y+X, Y-X, 2Z, 2dT] loaded signed (QZ2 = false: the row holds Z, as the Straus tables);
// negm = all-ones for -q (its 2dT term negated: Z and T of the completed point trade places), as a per-lane
// bit mask (v_bfi, no lane-mask register)
template <bool QZ2 = true>
CHIP_DEV void ge_add_row(ge_p1p1& r, const ge_p3& p, const ge_cached& q, uint32_t negm) {
    fe ypx, ymx, A, B, C, D2, z1, z2;
    fe_add(ypx, p.Y, p.X);
    fe_sub(ymx, p.Y, p.X);
    fe_mul(A, ypx, q.YpX);
    fe_mul(B, ymx, q.YmX);
    fe_mul(C, q.T2d, p.T);
    if (QZ2) fe_mul(D2, p.Z, q.Z);
    else fe_mul2(D2, p.Z, q.Z);
    fe_sub(r.X, A, B);
    fe_add(r.Y, A, B);
    fe_add(z1, D2, C);
    fe_sub(z2, D2, C);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        r.Z.v[i] = bit_select(negm, z2.v[i], z1.v[i]);
        r.T.v[i] = bit_select(negm, z1.v[i], z2.v[i]);
    }
}

