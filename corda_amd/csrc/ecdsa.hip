// ecdsa.hip — K2: SHA256withECDSA verification for ECDSA_SECP256R1_SHA256 (scheme 3) and
// ECDSA_SECP256K1_SHA256 (scheme 2) with BouncyCastle 1.57 semantics as selected by
// Crypto.isValid (core/.../crypto/Crypto.kt:615-625):
//   - StdDSAEncoder.decode: exactly one DER SEQUENCE of exactly two INTEGERs, minimal definite
//     lengths, no trailing bytes (DER re-encoding must equal the input); an empty INTEGER or one
//     ASN1Integer calls malformed (redundant leading 00 / FF byte) -> exception.  Failure ->
//     CHIP_SIG_DECODE.
//   - e = SHA-256(M) (256-bit n: no truncation); r, s outside [1, n-1] -> INVALID (negative / zero
//     DER integers land here); w = s^-1, u1 = e w, u2 = r w mod n; R = u1 G + u2 Q;
//     R = infinity -> INVALID; accept iff x(R) mod n == r (checked projectively as BC does:
//     X == r Z^2 or, when r + n < p, X == (r + n) Z^2).  High-s is valid.
// Schedule (lane-uniform, no divergence except the rare exceptional additions): 4-bit signed
// windows for u2 from a per-key affine table {1..8}Q built by K2b, 8-bit signed windows for u1
// from a 129-entry affine G table staged in LDS.
#include "ec_dev.hpp"
#include "sha2_dev.hpp"
#include "runtime.hpp"

#define EC_TAB_STRIDE EC_KEY_TABLE_WORDS

__device__ __constant__ const uint8_t SPKI_R1_PFX[26] = {0x30, 0x59, 0x30, 0x13, 0x06, 0x07, 0x2a, 0x86, 0x48,
                                                        0xce, 0x3d, 0x02, 0x01, 0x06, 0x08, 0x2a, 0x86, 0x48,
                                                        0xce, 0x3d, 0x03, 0x01, 0x07, 0x03, 0x42, 0x00};
__device__ __constant__ const uint8_t SPKI_K1_PFX[23] = {0x30, 0x56, 0x30, 0x10, 0x06, 0x07, 0x2a, 0x86,
                                                        0x48, 0xce, 0x3d, 0x02, 0x01, 0x06, 0x05, 0x2b,
                                                        0x81, 0x04, 0x00, 0x0a, 0x03, 0x42, 0x00};

CHIP_DEV bool match_prefix(const uint8_t* p, const uint8_t* pfx, int n, uint8_t second_len_byte, uint8_t bitstr_len) {
    bool ok = true;
    for (int i = 0; i < n; i++) {
        uint8_t want = pfx[i];
        if (i == 1) want = second_len_byte;
        if (i == n - 2) want = bitstr_len;
        ok = ok && (p[i] == want);
    }
    return ok;
}

CHIP_DEV void load_be256(u256& r, const uint8_t* p) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[7 - i] = ld_be32(p + 4 * i);
}

template <int C>
CHIP_DEV bool ec_decode_point(apt& q, const uint8_t* pt, uint32_t len) {
    const ec_curve_c& cv = curve<C>();
    if (len == 65 && pt[0] == 0x04) {
        load_be256(q.x, pt + 1);
        load_be256(q.y, pt + 33);
        if (u256_ge(q.x, cv.p) || u256_ge(q.y, cv.p)) return false;
    } else if (len == 33 && (pt[0] == 0x02 || pt[0] == 0x03)) {
        load_be256(q.x, pt + 1);
        if (u256_ge(q.x, cv.p)) return false;
        u256 rhs, t;
        fp_sqr<C>(rhs, q.x);
        fp_mul<C>(rhs, rhs, q.x);
        if (C == CURVE_R1) {   // - 3x
            fp_add<C>(t, q.x, q.x);
            fp_add<C>(t, t, q.x);
            fp_sub<C>(rhs, rhs, t);
        }
        u256 b;
        u256_from_c(b, cv.b);
        fp_add<C>(rhs, rhs, b);
        fp_pow<C>(q.y, rhs, cv.p_plus_1_div_4);
        if ((q.y.w[0] & 1u) != (uint32_t)(pt[0] & 1)) fp_neg<C>(q.y, q.y);
    } else {
        return false;
    }
    // on-curve: y^2 == x^3 + a x + b
    u256 lhs, rhs, t, b;
    fp_sqr<C>(lhs, q.y);
    fp_sqr<C>(rhs, q.x);
    fp_mul<C>(rhs, rhs, q.x);
    if (C == CURVE_R1) {
        fp_add<C>(t, q.x, q.x);
        fp_add<C>(t, t, q.x);
        fp_sub<C>(rhs, rhs, t);
    }
    u256_from_c(b, cv.b);
    fp_add<C>(rhs, rhs, b);
    return u256_eq(lhs, rhs);
}

CHIP_DEV void store_apt(uint32_t* dst, const apt& a) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        dst[i] = a.x.w[i];
        dst[8 + i] = a.y.w[i];
    }
}
CHIP_DEV void load_apt(apt& a, const uint32_t* src) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    const uint4 v0 = s4[0], v1 = s4[1], v2 = s4[2], v3 = s4[3];
    a.x.w[0] = v0.x; a.x.w[1] = v0.y; a.x.w[2] = v0.z; a.x.w[3] = v0.w;
    a.x.w[4] = v1.x; a.x.w[5] = v1.y; a.x.w[6] = v1.z; a.x.w[7] = v1.w;
    a.y.w[0] = v2.x; a.y.w[1] = v2.y; a.y.w[2] = v2.z; a.y.w[3] = v2.w;
    a.y.w[4] = v3.x; a.y.w[5] = v3.y; a.y.w[6] = v3.z; a.y.w[7] = v3.w;
}

// {1..8} Q in affine form: Jacobian multiples, one shared inversion (Montgomery's trick)
template <int C>
CHIP_DEV void ec_build_table(uint32_t* tab, const apt& q) {
    jpt P[8];
    P[0].X = q.x;
    P[0].Y = q.y;
#pragma unroll
    for (int i = 0; i < 8; i++) P[0].Z.w[i] = (i == 0);
    jdbl<C>(P[1], P[0]);
    for (int k = 2; k < 8; k++) jmadd<C>(P[k], P[k - 1], q);
    u256 acc[8];
    acc[0] = P[0].Z;
    for (int k = 1; k < 8; k++) fp_mul<C>(acc[k], acc[k - 1], P[k].Z);
    u256 inv;
    fp_inv<C>(inv, acc[7]);
    for (int k = 7; k >= 0; k--) {
        u256 zi, zi2, zi3;
        if (k > 0) fp_mul<C>(zi, inv, acc[k - 1]);
        else zi = inv;
        if (k > 0) fp_mul<C>(inv, inv, P[k].Z);
        fp_sqr<C>(zi2, zi);
        fp_mul<C>(zi3, zi2, zi);
        apt a;
        fp_mul<C>(a.x, P[k].X, zi2);
        fp_mul<C>(a.y, P[k].Y, zi3);
        store_apt(tab + 16 * (k + 1), a);
    }
}

// ---- K2b: per unique key ----
__global__ void __launch_bounds__(256) k_ecdsa_key_prep(uint64_t n_keys, const uint8_t* __restrict__ key_data,
                                                        const uint64_t* __restrict__ key_off,
                                                        const uint32_t* __restrict__ key_len, KeyMeta* meta,
                                                        uint32_t* __restrict__ table) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_keys) return;
    const uint8_t* p = key_data + key_off[k];
    const uint32_t len = key_len[k];
    int scheme = 0;
    const uint8_t* pt = nullptr;
    uint32_t ptlen = 0;
    if (len == 91 && match_prefix(p, SPKI_R1_PFX, 26, 0x59, 0x42)) { scheme = CHIP_SCHEME_R1; pt = p + 26; ptlen = 65; }
    else if (len == 59 && match_prefix(p, SPKI_R1_PFX, 26, 0x39, 0x22)) { scheme = CHIP_SCHEME_R1; pt = p + 26; ptlen = 33; }
    else if (len == 88 && match_prefix(p, SPKI_K1_PFX, 23, 0x56, 0x42)) { scheme = CHIP_SCHEME_K1; pt = p + 23; ptlen = 65; }
    else if (len == 56 && match_prefix(p, SPKI_K1_PFX, 23, 0x36, 0x22)) { scheme = CHIP_SCHEME_K1; pt = p + 23; ptlen = 33; }
    if (!scheme) return;   // not ECDSA r1/k1 (Ed25519 keys are prepared by ed25519.hip)
    KeyMeta m;
    m.scheme = (uint8_t)scheme;
    m.pad[0] = m.pad[1] = 0;
    apt q;
    bool ok;
    uint32_t* tab = table + k * EC_TAB_STRIDE;
    if (scheme == CHIP_SCHEME_R1) {
        ok = ec_decode_point<CURVE_R1>(q, pt, ptlen);
        if (ok) ec_build_table<CURVE_R1>(tab, q);
    } else {
        ok = ec_decode_point<CURVE_K1>(q, pt, ptlen);
        if (ok) ec_build_table<CURVE_K1>(tab, q);
    }
    m.ok = ok ? 1 : 0;
    meta[k] = m;
}

// ---- DER (BC 1.57 StdDSAEncoder + re-encode equality) ----
CHIP_DEV bool der_len(const uint8_t* p, uint32_t avail, uint32_t& hdr, uint32_t& L) {
    if (avail < 1) return false;
    const uint32_t b = p[0];
    if (b < 0x80) { hdr = 1; L = b; return true; }
    if (b == 0x80) return false;
    const uint32_t nb = b & 0x7f;
    if (nb > 4 || nb + 1 > avail) return false;
    if (p[1] == 0) return false;
    uint32_t v = 0;
    for (uint32_t i = 0; i < nb; i++) v = (v << 8) | p[1 + i];
    if (v < 0x80) return false;
    hdr = 1 + nb;
    L = v;
    return true;
}
// INTEGER content -> value; oor when value <= 0 or >= 2^256
CHIP_DEV void der_int(u256& v, bool& oor, const uint8_t* c, uint32_t n) {
#pragma unroll
    for (int i = 0; i < 8; i++) v.w[i] = 0;
    oor = false;
    if (c[0] & 0x80) { oor = true; return; }
    uint32_t i = 0;
    while (i < n && c[i] == 0) i++;
    if (i == n || n - i > 32) { oor = true; return; }
    for (uint32_t k = i; k < n; k++) {
        const uint32_t pos = n - 1 - k;   // byte position from the least significant end
        v.w[pos >> 2] |= (uint32_t)c[k] << (8 * (pos & 3));
    }
}
CHIP_DEV bool der_decode(const uint8_t* sig, uint32_t len, u256& r, bool& roor, u256& s, bool& soor) {
    uint32_t hdr, L;
    if (len < 2 || sig[0] != 0x30) return false;
    if (!der_len(sig + 1, len - 1, hdr, L)) return false;
    if (1 + hdr + L != len) return false;
    const uint8_t* p = sig + 1 + hdr;
    uint32_t rem = L;
    const uint8_t* val[2];
    uint32_t vl[2];
    for (int k = 0; k < 2; k++) {
        if (rem < 2 || p[0] != 0x02) return false;
        uint32_t h2, l2;
        if (!der_len(p + 1, rem - 1, h2, l2)) return false;
        if (1 + h2 + l2 > rem) return false;
        if (l2 == 0) return false;
        const uint8_t* c = p + 1 + h2;   // ASN1Integer malformed-integer rule
        if (l2 > 1 && ((c[0] == 0x00 && !(c[1] & 0x80)) || (c[0] == 0xff && (c[1] & 0x80)))) return false;
        val[k] = c;
        vl[k] = l2;
        p += 1 + h2 + l2;
        rem -= 1 + h2 + l2;
    }
    if (rem != 0) return false;
    der_int(r, roor, val[0], vl[0]);
    der_int(s, soor, val[1], vl[1]);
    return true;
}

// signed radix-2^w recoding of a 256-bit scalar: ndig digits biased by 2^(w-1), plus final carry
template <int W>
CHIP_DEV uint32_t recode(uint32_t out[8], const u256& a) {
    int carry = 0;
    const int per = 32 / W;
#pragma unroll
    for (int wd = 0; wd < 8; wd++) {
        uint32_t o = 0;
#pragma unroll
        for (int k = 0; k < per; k++) {
            int v = (int)((a.w[wd] >> (W * k)) & ((1u << W) - 1)) + carry;
            carry = (v + (1 << (W - 1))) >> W;
            v -= carry << W;
            o |= (uint32_t)(v + (1 << (W - 1))) << (W * k);
        }
        out[wd] = o;
    }
    return (uint32_t)carry;
}
CHIP_DEV void shl256_(uint32_t v[8], int n) {
#pragma unroll
    for (int k = 7; k > 0; k--) v[k] = (v[k] << n) | (v[k - 1] >> (32 - n));
    v[0] <<= n;
}

template <int C>
CHIP_DEV void add_digit(jpt& acc, const apt& e, int d) {
    if (d == 0) return;
    apt a = e;
    if (d < 0) fp_neg<C>(a.y, a.y);
    jmadd<C>(acc, acc, a);
}

template <int C>
__global__ void __launch_bounds__(256) k_ecdsa_verify(const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                                                      const uint32_t* __restrict__ key_idx,
                                                      const uint32_t* __restrict__ msg_idx,
                                                      const uint8_t* __restrict__ sig_data,
                                                      const uint64_t* __restrict__ sig_off,
                                                      const uint32_t* __restrict__ sig_len,
                                                      const uint8_t* __restrict__ msg_data,
                                                      const uint64_t* __restrict__ msg_off,
                                                      const uint32_t* __restrict__ msg_len,
                                                      const uint32_t* __restrict__ table, uint8_t* __restrict__ status) {
    __shared__ uint32_t gtab[EC_G_ENTRIES * 16];
    const ec_aff_c* G = (C == CURVE_R1) ? EC_R1_G_TABLE : EC_K1_G_TABLE;
    for (int i = threadIdx.x; i < EC_G_ENTRIES * 16; i += blockDim.x) {
        const ec_aff_c& e = G[i >> 4];
        gtab[i] = (i & 15) < 8 ? e.x[i & 7] : e.y[i & 7];
    }
    __syncthreads();
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= *count) return;
    const uint32_t i = list[gid];
    const ec_curve_c& cv = curve<C>();
    u256 r, s;
    bool roor, soor;
    if (!der_decode(sig_data + sig_off[i], sig_len[i], r, roor, s, soor)) {
        status[i] = CHIP_SIG_DECODE;
        return;
    }
    // r, s in [1, n-1]
    if (roor || soor || u256_is_zero(r) || u256_is_zero(s) || u256_ge(r, cv.n) || u256_ge(s, cv.n)) {
        status[i] = CHIP_INVALID;
        return;
    }
    // e = SHA-256(M), big-endian integer; reduce once mod n (e < 2^256 < 2n)
    const uint32_t mi = msg_idx[i];
    uint32_t H[8];
    sha256_bytes(H, msg_data + msg_off[mi], msg_len[mi]);
    u256 e;
#pragma unroll
    for (int k = 0; k < 8; k++) e.w[k] = H[7 - k];
    {
        u256 t;
        if (!u256_sub(t, e, cv.n)) e = t;
    }
    // w = s^-1 mod n (Fermat, Montgomery domain); u1 = e w, u2 = r w
    u256 r2n, sm, wm, u1, u2;
    u256_from_c(r2n, cv.r2_n);
    mn_mul<C>(sm, s, r2n);
    mn_pow<C>(wm, sm, cv.n_minus_2);
    mn_mul<C>(u1, e, wm);
    mn_mul<C>(u2, r, wm);
    // R = u1 G + u2 Q
    uint32_t dq[8], dg[8];
    const uint32_t cq = recode<4>(dq, u2);
    const uint32_t cg = recode<8>(dg, u1);
    const uint32_t* qt = table + (uint64_t)key_idx[i] * EC_TAB_STRIDE;
    jpt acc;
#pragma unroll
    for (int k = 0; k < 8; k++) acc.X.w[k] = acc.Y.w[k] = acc.Z.w[k] = 0;
    apt ent;
    // top window (position 64): the recodings' final carries
    if (cq) {
        load_apt(ent, qt + 16);
        add_digit<C>(acc, ent, 1);
    }
    if (cg) {
        load_apt(ent, gtab + 16);
        add_digit<C>(acc, ent, 1);
    }
    for (int w = 63; w >= 0; w--) {
        jdbl<C>(acc, acc);
        jdbl<C>(acc, acc);
        jdbl<C>(acc, acc);
        jdbl<C>(acc, acc);
        const int d = (int)(dq[7] >> 28) - 8;
        shl256_(dq, 4);
        const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
        load_apt(ent, qt + 16 * ad);
        add_digit<C>(acc, ent, d);
        if ((w & 1) == 0) {
            const int g = (int)(dg[7] >> 24) - 128;
            shl256_(dg, 8);
            const uint32_t ag = (uint32_t)(g < 0 ? -g : g);
            const uint32_t* ge = gtab + 16 * ag;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                ent.x.w[k] = ge[k];
                ent.y.w[k] = ge[8 + k];
            }
            add_digit<C>(acc, ent, g);
        }
    }
    if (u256_is_zero(acc.Z)) {
        status[i] = CHIP_INVALID;
        return;
    }
    // x(R) mod n == r  <=>  X == r Z^2  or  (r + n < p and X == (r + n) Z^2)
    u256 z2, t;
    fp_sqr<C>(z2, acc.Z);
    fp_mul<C>(t, r, z2);
    bool ok = u256_eq(t, acc.X);
    if (!ok) {
        u256 rn;
        const uint32_t c = u256_add(rn, r, cv.n);
        if (!c && !u256_ge(rn, cv.p)) {
            fp_mul<C>(t, rn, z2);
            ok = u256_eq(t, acc.X);
        }
    }
    status[i] = ok ? CHIP_VALID : CHIP_INVALID;
}

void launch_ecdsa_key_prep(hipStream_t st, uint64_t n_keys, const uint8_t* key_data, const uint64_t* key_off,
                           const uint32_t* key_len, KeyMeta* meta, uint32_t* ectab) {
    if (!n_keys) return;
    const uint32_t blocks = (uint32_t)((n_keys + 255) / 256);
    hipLaunchKernelGGL(k_ecdsa_key_prep, dim3(blocks), dim3(256), 0, st, n_keys, key_data, key_off, key_len, meta,
                       ectab);
}

void launch_ecdsa_verify(hipStream_t st, int scheme, uint64_t n, const uint32_t* list, const uint32_t* count,
                         const chip_sig_batch* b, const uint32_t* ectab, uint8_t* status) {
    if (!n) return;
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    if (scheme == CHIP_SCHEME_R1)
        hipLaunchKernelGGL(k_ecdsa_verify<CURVE_R1>, dim3(blocks), dim3(256), 0, st, list, count, b->key_idx,
                           b->msg_idx, b->sig_data, b->sig_off, b->sig_len, b->msg_data, b->msg_off, b->msg_len,
                           ectab, status);
    else
        hipLaunchKernelGGL(k_ecdsa_verify<CURVE_K1>, dim3(blocks), dim3(256), 0, st, list, count, b->key_idx,
                           b->msg_idx, b->sig_data, b->sig_off, b->sig_len, b->msg_data, b->msg_off, b->msg_len,
                           ectab, status);
}

// ---------------------------------------------------------------------------------------
// K2c: per-key comb path (keys that sign many signatures of a batch).  R = u1 G + u2 Q with no
// doublings: u2 in signed radix-16 digits over 65 windows from a per-key table of 2^(4w) {1..8} Q
// (built for the batch by k_ecdsa_comb_chain / k_ecdsa_comb_fill on the second stream, normalised to
// affine so every addition is a mixed one), u1 in signed radix-256 digits over 33 windows from the
// fixed tables EC_<C>_G_COMB.  s^-1 is one Fermat inversion per EC_INV_BATCH signatures (Montgomery's
// trick, k_ecdsa_comb_inv).  96 mixed additions instead of 256 doublings + 96 mixed additions; the same
// BC 1.57 semantics as k_ecdsa_verify (identical DER / range / x(R) mod n checks).
#include "comb_tables.hpp"

#define EC_COMB_QWIN 65
#define EC_COMB_QENT 8
#define EC_COMB_JW 24
// affine table per key, then (after all keys) the Jacobian scratch it is normalised from
#define EC_COMB_KEY_WORDS (EC_COMB_QWIN * EC_COMB_QENT * 16)
#define EC_COMB_JAC_WORDS (EC_COMB_QWIN * EC_COMB_QENT * EC_COMB_JW)
#define EC_INV_BATCH 16

CHIP_DEV void store_jpt(uint32_t* d, const jpt& p) {
    uint4* d4 = reinterpret_cast<uint4*>(d);
    d4[0] = make_uint4(p.X.w[0], p.X.w[1], p.X.w[2], p.X.w[3]);
    d4[1] = make_uint4(p.X.w[4], p.X.w[5], p.X.w[6], p.X.w[7]);
    d4[2] = make_uint4(p.Y.w[0], p.Y.w[1], p.Y.w[2], p.Y.w[3]);
    d4[3] = make_uint4(p.Y.w[4], p.Y.w[5], p.Y.w[6], p.Y.w[7]);
    d4[4] = make_uint4(p.Z.w[0], p.Z.w[1], p.Z.w[2], p.Z.w[3]);
    d4[5] = make_uint4(p.Z.w[4], p.Z.w[5], p.Z.w[6], p.Z.w[7]);
}
CHIP_DEV void store_u256(uint32_t* d, const u256& v) {
    uint4* d4 = reinterpret_cast<uint4*>(d);
    d4[0] = make_uint4(v.w[0], v.w[1], v.w[2], v.w[3]);
    d4[1] = make_uint4(v.w[4], v.w[5], v.w[6], v.w[7]);
}
CHIP_DEV void load_u256(u256& v, const uint32_t* s) {
    const uint4* s4 = reinterpret_cast<const uint4*>(s);
    const uint4 a = s4[0], b = s4[1];
    v.w[0] = a.x; v.w[1] = a.y; v.w[2] = a.z; v.w[3] = a.w;
    v.w[4] = b.x; v.w[5] = b.y; v.w[6] = b.z; v.w[7] = b.w;
}
CHIP_DEV void load_jpt(jpt& p, const uint32_t* s) {
    const uint4* s4 = reinterpret_cast<const uint4*>(s);
    uint4 v;
    v = s4[0]; p.X.w[0] = v.x; p.X.w[1] = v.y; p.X.w[2] = v.z; p.X.w[3] = v.w;
    v = s4[1]; p.X.w[4] = v.x; p.X.w[5] = v.y; p.X.w[6] = v.z; p.X.w[7] = v.w;
    v = s4[2]; p.Y.w[0] = v.x; p.Y.w[1] = v.y; p.Y.w[2] = v.z; p.Y.w[3] = v.w;
    v = s4[3]; p.Y.w[4] = v.x; p.Y.w[5] = v.y; p.Y.w[6] = v.z; p.Y.w[7] = v.w;
    v = s4[4]; p.Z.w[0] = v.x; p.Z.w[1] = v.y; p.Z.w[2] = v.z; p.Z.w[3] = v.w;
    v = s4[5]; p.Z.w[4] = v.x; p.Z.w[5] = v.y; p.Z.w[6] = v.z; p.Z.w[7] = v.w;
}

// r = p + q, both Jacobian (add-2007-bl); exact for infinity, p == q and p == -q.  r may alias p.
template <int C> CHIP_DEV void jadd(jpt& r, const jpt& p, const jpt& q) {
    if (u256_is_zero(p.Z)) { r = q; return; }
    if (u256_is_zero(q.Z)) { r = p; return; }
    u256 Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, rr, V, t;
    fp_sqr<C>(Z1Z1, p.Z);
    fp_sqr<C>(Z2Z2, q.Z);
    fp_mul<C>(U1, p.X, Z2Z2);
    fp_mul<C>(U2, q.X, Z1Z1);
    fp_mul<C>(S1, p.Y, q.Z);
    fp_mul<C>(S1, S1, Z2Z2);
    fp_mul<C>(S2, q.Y, p.Z);
    fp_mul<C>(S2, S2, Z1Z1);
    fp_sub<C>(H, U2, U1);
    fp_sub<C>(rr, S2, S1);
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
    fp_add<C>(I, H, H);
    fp_sqr<C>(I, I);
    fp_mul<C>(J, H, I);
    fp_mul<C>(V, U1, I);
    jpt o;
    fp_sqr<C>(o.X, rr);
    fp_sub<C>(o.X, o.X, J);
    fp_sub<C>(o.X, o.X, V);
    fp_sub<C>(o.X, o.X, V);
    fp_sub<C>(t, V, o.X);
    fp_mul<C>(o.Y, rr, t);
    fp_mul<C>(t, S1, J);
    fp_add<C>(t, t, t);
    fp_sub<C>(o.Y, o.Y, t);
    fp_add<C>(t, p.Z, q.Z);
    fp_sqr<C>(t, t);
    fp_sub<C>(t, t, Z1Z1);
    fp_sub<C>(t, t, Z2Z2);
    fp_mul<C>(o.Z, t, H);
    r = o;
}

CHIP_DEV bool ec_key_ok(const KeyMeta* meta, uint64_t k, int scheme) {
    const KeyMeta m = meta[k];
    return m.scheme == scheme && m.ok;
}

// chain: P_w = 2^(4w) Q for w = 0..64 into entry 1 of every window of the Jacobian scratch
// (256 serial doublings per key)
template <int C>
CHIP_DEV void ec_comb_chain(const uint32_t* __restrict__ ectab, uint32_t* __restrict__ jac, uint64_t k) {
    apt q;
    load_apt(q, ectab + k * EC_TAB_STRIDE + 16);
    jpt P;
    P.X = q.x;
    P.Y = q.y;
#pragma unroll
    for (int i = 0; i < 8; i++) P.Z.w[i] = (i == 0);
    uint32_t* tab = jac + k * EC_COMB_JAC_WORDS;
    for (int w = 0; w < EC_COMB_QWIN; w++) {
        store_jpt(tab + (uint32_t)w * EC_COMB_QENT * EC_COMB_JW, P);
        if (w + 1 == EC_COMB_QWIN) break;
#pragma unroll 1
        for (int b = 0; b < 4; b++) jdbl<C>(P, P);
    }
}
// fill: entries j = 2..8 of window w = j P_w (Jacobian scratch), then to affine.  A lane takes
// EC_FILL_GROUP windows so that one Fermat inversion serves 8 EC_FILL_GROUP entries (Montgomery's
// trick; the prefix products are parked in the x slots of the affine entries)
#define EC_FILL_GROUP 8
#define EC_FILL_LANES ((EC_COMB_QWIN - 1) / EC_FILL_GROUP)
template <int C>
CHIP_DEV void ec_comb_fill(uint32_t* __restrict__ jac, uint32_t* __restrict__ out, uint32_t w0, uint32_t w1) {
    u256 acc, z, t;
#pragma unroll
    for (int i = 0; i < 8; i++) acc.w[i] = (i == 0);
    for (uint32_t w = w0; w < w1; w++) {
        uint32_t* e = jac + w * EC_COMB_QENT * EC_COMB_JW;
        uint32_t* o = out + w * EC_COMB_QENT * 16;
        jpt P, A;
        load_jpt(P, e);
        store_u256(o, acc);
        fp_mul<C>(acc, acc, P.Z);
        jdbl<C>(A, P);
        store_jpt(e + EC_COMB_JW, A);
        store_u256(o + 16, acc);
        fp_mul<C>(acc, acc, A.Z);
#pragma unroll 1
        for (int j = 3; j <= EC_COMB_QENT; j++) {
            jadd<C>(A, A, P);
            store_jpt(e + (uint32_t)(j - 1) * EC_COMB_JW, A);
            store_u256(o + (uint32_t)(j - 1) * 16, acc);
            fp_mul<C>(acc, acc, A.Z);
        }
    }
    fp_inv<C>(acc, acc);   // entries are j 2^(4w) Q, never infinity for a valid key
    for (uint32_t w = w1; w-- > w0;) {
        const uint32_t* e = jac + w * EC_COMB_QENT * EC_COMB_JW;
        uint32_t* o = out + w * EC_COMB_QENT * 16;
#pragma unroll 1
        for (int j = EC_COMB_QENT - 1; j >= 0; j--) {
            u256 zi, zi2, pre, x, y;
            load_u256(pre, o + (uint32_t)j * 16);
            load_u256(z, e + (uint32_t)j * EC_COMB_JW + 16);
            fp_mul<C>(zi, acc, pre);
            fp_mul<C>(acc, acc, z);
            fp_sqr<C>(zi2, zi);
            load_u256(x, e + (uint32_t)j * EC_COMB_JW);
            load_u256(y, e + (uint32_t)j * EC_COMB_JW + 8);
            fp_mul<C>(x, x, zi2);
            fp_mul<C>(t, zi2, zi);
            fp_mul<C>(y, y, t);
            store_u256(o + (uint32_t)j * 16, x);
            store_u256(o + (uint32_t)j * 16 + 8, y);
        }
    }
}
// one launch for both curves: r1 and k1 keys build concurrently (lane per key)
__global__ void __launch_bounds__(64) k_ecdsa_comb_chain(uint64_t n_keys, const KeyMeta* __restrict__ meta,
                                                         const uint32_t* __restrict__ ectab, uint32_t* __restrict__ jac) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_keys) return;
    if (ec_key_ok(meta, k, CHIP_SCHEME_R1)) ec_comb_chain<CURVE_R1>(ectab, jac, k);
    else if (ec_key_ok(meta, k, CHIP_SCHEME_K1)) ec_comb_chain<CURVE_K1>(ectab, jac, k);
}
// lane per key x group of windows (the last group also takes window 64)
__global__ void __launch_bounds__(256) k_ecdsa_comb_fill(uint64_t n_keys, const KeyMeta* __restrict__ meta,
                                                         uint32_t* __restrict__ ctab, uint32_t* __restrict__ jac) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t k = g / EC_FILL_LANES;
    const uint32_t grp = (uint32_t)(g % EC_FILL_LANES);
    if (k >= n_keys) return;
    const uint32_t w0 = grp * EC_FILL_GROUP;
    const uint32_t w1 = (grp + 1 == EC_FILL_LANES) ? EC_COMB_QWIN : w0 + EC_FILL_GROUP;
    uint32_t* e = jac + k * EC_COMB_JAC_WORDS;
    uint32_t* out = ctab + k * EC_COMB_KEY_WORDS;
    if (ec_key_ok(meta, k, CHIP_SCHEME_R1)) ec_comb_fill<CURVE_R1>(e, out, w0, w1);
    else if (ec_key_ok(meta, k, CHIP_SCHEME_K1)) ec_comb_fill<CURVE_K1>(e, out, w0, w1);
}

// hand-off between the kernels, SoA by list position: acc X/Y/Z (24 words), u2 (8), r (8), state (1).
// Before k_ecdsa_comb_g the X slots hold e, the Y slots s R and the Z slots s^-1 R.
#define EC_MID_WORDS 41

CHIP_DEV void mid_store(uint32_t* mid, uint64_t cap, uint32_t gid, int slot, const u256& v) {
#pragma unroll
    for (int k = 0; k < 8; k++) mid[(uint64_t)(slot + k) * cap + gid] = v.w[k];
}
CHIP_DEV void mid_load(u256& v, const uint32_t* mid, uint64_t cap, uint32_t gid, int slot) {
#pragma unroll
    for (int k = 0; k < 8; k++) v.w[k] = mid[(uint64_t)(slot + k) * cap + gid];
}

// DER, range checks, e = SHA-256(M), s R (Montgomery form mod n)
template <int C>
__global__ void __launch_bounds__(256) k_ecdsa_comb_pre(const uint32_t* __restrict__ list,
                                                        const uint32_t* __restrict__ count,
                                                        const uint32_t* __restrict__ msg_idx,
                                                        const uint8_t* __restrict__ sig_data,
                                                        const uint64_t* __restrict__ sig_off,
                                                        const uint32_t* __restrict__ sig_len,
                                                        const uint8_t* __restrict__ msg_data,
                                                        const uint64_t* __restrict__ msg_off,
                                                        const uint32_t* __restrict__ msg_len, uint32_t* __restrict__ mid,
                                                        uint64_t cap, uint8_t* __restrict__ status) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= *count) return;
    const uint32_t i = list[gid];
    const ec_curve_c& cv = curve<C>();
    uint32_t* st_word = mid + (uint64_t)40 * cap + gid;
    u256 r, s;
    bool roor, soor;
    if (!der_decode(sig_data + sig_off[i], sig_len[i], r, roor, s, soor)) {
        status[i] = CHIP_SIG_DECODE;
        *st_word = 0;
        return;
    }
    if (roor || soor || u256_is_zero(r) || u256_is_zero(s) || u256_ge(r, cv.n) || u256_ge(s, cv.n)) {
        status[i] = CHIP_INVALID;
        *st_word = 0;
        return;
    }
    const uint32_t mi = msg_idx[i];
    uint32_t H[8];
    sha256_bytes(H, msg_data + msg_off[mi], msg_len[mi]);
    u256 e;
#pragma unroll
    for (int k = 0; k < 8; k++) e.w[k] = H[7 - k];
    {
        u256 t;
        if (!u256_sub(t, e, cv.n)) e = t;
    }
    u256 r2n, sm;
    u256_from_c(r2n, cv.r2_n);
    mn_mul<C>(sm, s, r2n);
    mid_store(mid, cap, gid, 0, e);
    mid_store(mid, cap, gid, 8, sm);
    mid_store(mid, cap, gid, 32, r);
    *st_word = 1;
}

// s^-1 R for EC_INV_BATCH signatures per lane: prefix products of s R (parked in the Z slots), one
// Fermat inversion of the product, then back to front.  Rejected signatures count as 1.  Lane l of a
// wave takes positions base + j 64 + l, so every step is a coalesced row.
template <int C>
__global__ void __launch_bounds__(64) k_ecdsa_comb_inv(const uint32_t* __restrict__ count, uint32_t* __restrict__ mid,
                                                       uint64_t cap) {
    const uint32_t n = *count;
    const uint32_t base = blockIdx.x * 64u * EC_INV_BATCH + threadIdx.x;
    if (base >= n) return;
    const ec_curve_c& cv = curve<C>();
    u256 acc, sm;
    u256_from_c(acc, cv.one_n);
    for (int j = 0; j < EC_INV_BATCH; j++) {
        const uint32_t gid = base + 64u * j;
        if (gid >= n) break;
        if (!mid[(uint64_t)40 * cap + gid]) continue;
        mid_store(mid, cap, gid, 16, acc);
        mid_load(sm, mid, cap, gid, 8);
        mn_mul<C>(acc, acc, sm);
    }
    mn_pow<C>(acc, acc, cv.n_minus_2);
    for (int j = EC_INV_BATCH - 1; j >= 0; j--) {
        const uint32_t gid = base + 64u * j;
        if (gid >= n || !mid[(uint64_t)40 * cap + gid]) continue;
        u256 pre, w;
        mid_load(pre, mid, cap, gid, 16);
        mid_load(sm, mid, cap, gid, 8);
        mn_mul<C>(w, acc, pre);
        mn_mul<C>(acc, acc, sm);
        mid_store(mid, cap, gid, 16, w);
    }
}

// u1 = e s^-1, u2 = r s^-1 and u1 G from the fixed comb
template <int C>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k_ecdsa_comb_g(const uint32_t* __restrict__ count, uint32_t* __restrict__ mid,
                                                      uint64_t cap) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= *count || !mid[(uint64_t)40 * cap + gid]) return;
    u256 e, r, wm, u1, u2;
    mid_load(e, mid, cap, gid, 0);
    mid_load(wm, mid, cap, gid, 16);
    mid_load(r, mid, cap, gid, 32);
    mn_mul<C>(u1, e, wm);
    mn_mul<C>(u2, r, wm);
    uint32_t dg[8];
    const uint32_t cg = recode<8>(dg, u1);
    jpt acc;
#pragma unroll
    for (int k = 0; k < 8; k++) acc.X.w[k] = acc.Y.w[k] = acc.Z.w[k] = 0;
    const uint32_t* G = (C == CURVE_R1) ? EC_R1_G_COMB : EC_K1_G_COMB;
    apt ga;
#pragma unroll 1
    for (int wd = 0; wd < 8; wd++) {
        const uint32_t cur = dg[wd];
#pragma unroll 1
        for (int q = 0; q < 4; q++) {
            const int d = (int)((cur >> (8 * q)) & 255u) - 128;
            if (!d) continue;
            const uint32_t w = (uint32_t)(wd * 4 + q);
            load_apt(ga, G + (w * EC_COMB_GENT + (uint32_t)(d < 0 ? -d : d)) * 16);
            add_digit<C>(acc, ga, d);
        }
    }
    if (cg) {
        load_apt(ga, G + (32u * EC_COMB_GENT + 1u) * 16);
        add_digit<C>(acc, ga, 1);
    }
    mid_store(mid, cap, gid, 0, acc.X);
    mid_store(mid, cap, gid, 8, acc.Y);
    mid_store(mid, cap, gid, 16, acc.Z);
    mid_store(mid, cap, gid, 24, u2);
}

// u2 Q half: one mixed addition per non-zero radix-16 digit from the key's affine table, then
// x(R) mod n == r exactly as k_ecdsa_verify checks it
template <int C>
__global__ void __launch_bounds__(256) k_ecdsa_comb_q(const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                                                      const uint32_t* __restrict__ key_idx,
                                                      const uint32_t* __restrict__ ctab, const uint32_t* __restrict__ mid,
                                                      uint64_t cap, uint8_t* __restrict__ status) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= *count || !mid[(uint64_t)40 * cap + gid]) return;
    const uint32_t i = list[gid];
    const ec_curve_c& cv = curve<C>();
    jpt acc;
    apt ent;
    u256 u2, r;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        acc.X.w[k] = mid[(uint64_t)k * cap + gid];
        acc.Y.w[k] = mid[(uint64_t)(8 + k) * cap + gid];
        acc.Z.w[k] = mid[(uint64_t)(16 + k) * cap + gid];
        u2.w[k] = mid[(uint64_t)(24 + k) * cap + gid];
        r.w[k] = mid[(uint64_t)(32 + k) * cap + gid];
    }
    uint32_t dq[8];
    const uint32_t cq = recode<4>(dq, u2);
    const uint32_t* qt = ctab + (uint64_t)key_idx[i] * EC_COMB_KEY_WORDS;
#pragma unroll 1
    for (int wd = 0; wd < 8; wd++) {
        const uint32_t cur = dq[wd];
#pragma unroll 1
        for (int q = 0; q < 8; q++) {
            const int d = (int)((cur >> (4 * q)) & 15u) - 8;
            if (!d) continue;
            const uint32_t w = (uint32_t)(wd * 8 + q);
            load_apt(ent, qt + (w * EC_COMB_QENT + (uint32_t)(d < 0 ? -d : d) - 1) * 16);
            add_digit<C>(acc, ent, d);
        }
    }
    if (cq) {
        load_apt(ent, qt + (64u * EC_COMB_QENT) * 16);
        add_digit<C>(acc, ent, 1);
    }
    if (u256_is_zero(acc.Z)) {
        status[i] = CHIP_INVALID;
        return;
    }
    u256 z2, t;
    fp_sqr<C>(z2, acc.Z);
    fp_mul<C>(t, r, z2);
    bool ok = u256_eq(t, acc.X);
    if (!ok) {
        u256 rn;
        const uint32_t c = u256_add(rn, r, cv.n);
        if (!c && !u256_ge(rn, cv.p)) {
            fp_mul<C>(t, rn, z2);
            ok = u256_eq(t, acc.X);
        }
    }
    status[i] = ok ? CHIP_VALID : CHIP_INVALID;
}

uint64_t ecdsa_comb_key_words() { return EC_COMB_KEY_WORDS + EC_COMB_JAC_WORDS; }

void launch_ecdsa_comb_build(hipStream_t st, uint64_t n_keys, const KeyMeta* meta, const uint32_t* ectab,
                             uint32_t* ctab) {
    if (!n_keys) return;
    uint32_t* jac = ctab + n_keys * EC_COMB_KEY_WORDS;
    hipLaunchKernelGGL(k_ecdsa_comb_chain, dim3((uint32_t)((n_keys + 63) / 64)), dim3(64), 0, st, n_keys, meta, ectab,
                       jac);
    hipLaunchKernelGGL(k_ecdsa_comb_fill, dim3((uint32_t)((n_keys * EC_FILL_LANES + 255) / 256)), dim3(256), 0, st, n_keys,
                       meta, ctab, jac);
}

uint64_t ecdsa_comb_mid_words() { return EC_MID_WORDS; }

template <int C>
static void comb_pre(hipStream_t st, uint64_t n, const uint32_t* list, const uint32_t* count, const chip_sig_batch* b,
                     uint32_t* mid, uint8_t* status) {
    hipLaunchKernelGGL(k_ecdsa_comb_pre<C>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, list, count,
                       b->msg_idx, b->sig_data, b->sig_off, b->sig_len, b->msg_data, b->msg_off, b->msg_len, mid,
                       (uint64_t)n, status);
    hipLaunchKernelGGL(k_ecdsa_comb_inv<C>, dim3((uint32_t)((n + 64 * EC_INV_BATCH - 1) / (64 * EC_INV_BATCH))), dim3(64),
                       0, st, count, mid, (uint64_t)n);
    hipLaunchKernelGGL(k_ecdsa_comb_g<C>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, count, mid, (uint64_t)n);
}

void launch_ecdsa_comb_pre(hipStream_t st, int scheme, uint64_t n, const uint32_t* list, const uint32_t* count,
                           const chip_sig_batch* b, uint32_t* mid, uint8_t* status) {
    if (!n) return;
    if (scheme == CHIP_SCHEME_R1) comb_pre<CURVE_R1>(st, n, list, count, b, mid, status);
    else comb_pre<CURVE_K1>(st, n, list, count, b, mid, status);
}
void launch_ecdsa_comb_q(hipStream_t st, int scheme, uint64_t n, const uint32_t* list, const uint32_t* count,
                         const chip_sig_batch* b, const uint32_t* ctab, const uint32_t* mid, uint8_t* status) {
    if (!n) return;
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    if (scheme == CHIP_SCHEME_R1)
        hipLaunchKernelGGL(k_ecdsa_comb_q<CURVE_R1>, dim3(blocks), dim3(256), 0, st, list, count, b->key_idx, ctab, mid,
                           (uint64_t)n, status);
    else
        hipLaunchKernelGGL(k_ecdsa_comb_q<CURVE_K1>, dim3(blocks), dim3(256), 0, st, list, count, b->key_idx, ctab, mid,
                           (uint64_t)n, status);
}
