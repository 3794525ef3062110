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
//
// Two schedules, identical results:
//   * windowed (k_ecdsa_verify, keys with few signatures): 4-bit signed windows for u2 from a
//     per-key affine table {1..8}Q (k_ecdsa_key_table), 8-bit signed windows for u1 from a 129-entry
//     affine G table staged in LDS; 256 doublings per signature.
//   * comb (keys that sign many signatures of the batch): no doublings per signature.  Work lists
//     grouped by key (k_ec_group_*), then
//       k_ecdsa_comb_pre<C> DER, range checks, e = SHA-256(M), s R and the wavefront-level part of the
//                           batched s^-1: prefix / suffix products across the 64 lanes (shuffles)
//       k_ecdsa_comb_inv    one inversion per wave product (binary extended Euclid), both curves
//       k_ecdsa_comb_g<C>   s^-1 = (wave product)^-1 * prefix * suffix, u1, u2, and u1 G from the
//                           fixed radix-2^EC_GW comb (built on the device at context start)
//       k_ecdsa_comb_q<C>   u2 Q from the per-key radix-16 table (65 windows x {1..8}) + the x(R) check
//     the per-key tables (k_ecdsa_comb_chain / _fill) are built on the context's second stream while
//     the main stream runs classify, pre, inv and g.
#include "ec_dev.hpp"
#include "sha2_dev.hpp"
#include "runtime.hpp"
#ifndef EC_G_PF
#define EC_G_PF 1   // software-pipelined G-comb gathers in k_ecdsa_comb_g (A/B: +0.9-1.0 %, profiles/r03/ab_ecdsa_g_prefetch.txt)
#endif
#include <cstdlib>

#define EC_TAB_STRIDE EC_KEY_TABLE_WORDS

// the signature-batch pointers a retry lane reads (kernel argument)
struct chip_sig_batch_dev {
    const uint32_t *key_idx, *msg_idx;
    const uint8_t* sig_data;
    const uint64_t* sig_off;
    const uint32_t* sig_len;
    const uint8_t* msg_data;
    const uint64_t* msg_off;
    const uint32_t* msg_len;
};

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

// x^3 + a x + b
template <int C>
CHIP_DEV void curve_rhs(u256& rhs, const u256& x) {
    u256 t, b;
    fp_sqr<C>(rhs, x);
    fp_mul<C>(rhs, rhs, x);
    if (EC_CURVE(C) == CURVE_R1) {   // - 3x
        fp_add<C>(t, x, x);
        fp_add<C>(t, t, x);
        fp_sub<C>(rhs, rhs, t);
    }
    u256_from_c(b, curve<C>().b);
    fp_add<C>(rhs, rhs, b);
}

// BC ECCurve.decodePoint: uncompressed 04||X||Y or compressed 02/03||X, coordinates < p, on the curve
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
        u256 rhs;
        curve_rhs<C>(rhs, q.x);
        fp_pow<C>(q.y, rhs, cv.p_plus_1_div_4);
        fp_canon<C>(q.y, q.y);
        if ((q.y.w[0] & 1u) != (uint32_t)(pt[0] & 1)) {
            fp_neg<C>(q.y, q.y);
            fp_canon<C>(q.y, q.y);
        }
    } else {
        return false;
    }
    // on-curve: y^2 == x^3 + a x + b
    u256 lhs, rhs;
    fp_sqr<C>(lhs, q.y);
    curve_rhs<C>(rhs, q.x);
    return fp_eq<C>(lhs, rhs);
}

CHIP_DEV void store_apt(uint32_t* dst, const apt& a) {
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    d4[0] = make_uint4(a.x.w[0], a.x.w[1], a.x.w[2], a.x.w[3]);
    d4[1] = make_uint4(a.x.w[4], a.x.w[5], a.x.w[6], a.x.w[7]);
    d4[2] = make_uint4(a.y.w[0], a.y.w[1], a.y.w[2], a.y.w[3]);
    d4[3] = make_uint4(a.y.w[4], a.y.w[5], a.y.w[6], a.y.w[7]);
}
CHIP_DEV void load_apt(apt& a, const uint32_t* src) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    const uint4 v0 = s4[0], v1 = s4[1], v2 = s4[2], v3 = s4[3];
    a.x.w[0] = v0.x; a.x.w[1] = v0.y; a.x.w[2] = v0.z; a.x.w[3] = v0.w;
    a.x.w[4] = v1.x; a.x.w[5] = v1.y; a.x.w[6] = v1.z; a.x.w[7] = v1.w;
    a.y.w[0] = v2.x; a.y.w[1] = v2.y; a.y.w[2] = v2.z; a.y.w[3] = v2.w;
    a.y.w[4] = v3.x; a.y.w[5] = v3.y; a.y.w[6] = v3.z; a.y.w[7] = v3.w;
}
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
    load_u256(p.X, s);
    load_u256(p.Y, s + 8);
    load_u256(p.Z, s + 16);
}
CHIP_DEV void jpt_inf(jpt& p) {
    u256_set_word(p.X, 0);
    u256_set_word(p.Y, 0);
    u256_set_word(p.Z, 0);
}
CHIP_DEV void jpt_from_aff(jpt& p, const apt& a) {
    p.X = a.x;
    p.Y = a.y;
    u256_set_word(p.Z, 1);
}
// affine (x, y) = (X / Z^2, Y / Z^3) given zi = 1 / Z
template <int C>
CHIP_DEV void jpt_to_aff(apt& a, const jpt& p, const u256& zi) {
    u256 zi2, zi3;
    fp_sqr<C>(zi2, zi);
    fp_mul<C>(zi3, zi2, zi);
    fp_mul<C>(a.x, p.X, zi2);
    fp_mul<C>(a.y, p.Y, zi3);
}

// {1..8} Q in affine form: Jacobian multiples, one shared inversion (Montgomery's trick).  The
// windowed schedule's per-key table; entry 1 (= Q) was stored by the key prep.
template <int C>
CHIP_DEV void ec_build_table(uint32_t* tab) {
    apt q;
    load_apt(q, tab + 16);
    jpt A, P[7];
    jpt_from_aff(A, q);
    jdbl<C>(P[0], A);                               // 2Q
#pragma unroll 1
    for (int k = 1; k < 7; k++) jmadd<C>(P[k], P[k - 1], q);
    u256 acc[7];
    acc[0] = P[0].Z;
#pragma unroll 1
    for (int k = 1; k < 7; k++) fp_mul<C>(acc[k], acc[k - 1], P[k].Z);
    u256 inv;
    fp_inv_vt<C>(inv, acc[6]);
#pragma unroll 1
    for (int k = 6; k >= 0; k--) {
        u256 zi;
        if (k > 0) {
            fp_mul<C>(zi, inv, acc[k - 1]);
            fp_mul<C>(inv, inv, P[k].Z);
        } else {
            zi = inv;
        }
        apt a;
        jpt_to_aff<C>(a, P[k], zi);
        store_apt(tab + 16 * (k + 2), a);
    }
}

// ---- K2b: per unique key: SPKI scheme lookup + decode (Crypto.findSignatureScheme, decodePoint) ----
__global__ void __launch_bounds__(256) k_ecdsa_key_prep(uint64_t n_keys, const uint8_t* __restrict__ key_data,
                                                        const uint64_t* __restrict__ key_off,
                                                        const uint32_t* __restrict__ key_len, KeyMeta* meta,
                                                        uint32_t* __restrict__ table, const uint32_t* __restrict__ skip) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_keys || (skip && *skip)) return;
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
    const bool ok = scheme == CHIP_SCHEME_R1 ? ec_decode_point<CURVE_R1>(q, pt, ptlen)
                                             : ec_decode_point<CURVE_K1>(q, pt, ptlen);
    if (ok) store_apt(table + k * EC_TAB_STRIDE + 16, q);
    m.ok = ok ? 1 : 0;
    meta[k] = m;
}

__global__ void __launch_bounds__(64) k_ecdsa_key_table(uint64_t n_keys, const KeyMeta* __restrict__ meta,
                                                        uint32_t* __restrict__ table, const uint32_t* __restrict__ skip) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_keys || (skip && *skip)) return;
    const KeyMeta m = meta[k];
    if (!m.ok) return;
    if (m.scheme == CHIP_SCHEME_R1) ec_build_table<CURVE_R1>(table + k * EC_TAB_STRIDE);
    else if (m.scheme == CHIP_SCHEME_K1) ec_build_table<CURVE_K1>(table + k * EC_TAB_STRIDE);
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
    // by destination byte (unrolled: every word index static, so v stays in registers), the loads independent
#pragma unroll
    for (uint32_t pos = 0; pos < 32; pos++) {   // byte position from the least significant end
        const uint32_t b = pos < n - i ? (uint32_t)c[n - 1 - pos] : 0u;
        v.w[pos >> 2] |= b << (8 * (pos & 3));
    }
}
CHIP_DEV bool der_decode(const uint8_t* sig, uint32_t len, u256& r, bool& roor, u256& s, bool& soor) {
    uint32_t hdr, L;
    if (len < 2 || sig[0] != 0x30) return false;
    if (!der_len(sig + 1, len - 1, hdr, L)) return false;
    if (1 + hdr + L != len) return false;
    // the two INTEGERs as byte offsets into sig (no array of pointers: with the LDS-staged source the walk reads
    // through generic pointers, and an array of them went to scratch)
    uint32_t at = 1 + hdr, rem = L;
    uint32_t v0 = 0, l0 = 0, v1 = 0, l1 = 0;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        if (rem < 2 || sig[at] != 0x02) return false;
        uint32_t h2, l2;
        if (!der_len(sig + at + 1, rem - 1, h2, l2)) return false;
        if (1 + h2 + l2 > rem) return false;
        if (l2 == 0) return false;
        const uint32_t c = at + 1 + h2;   // ASN1Integer malformed-integer rule
        if (l2 > 1 && ((sig[c] == 0x00 && !(sig[c + 1] & 0x80)) || (sig[c] == 0xff && (sig[c + 1] & 0x80)))) return false;
        if (k == 0) { v0 = c; l0 = l2; } else { v1 = c; l1 = l2; }
        at += 1 + h2 + l2;
        rem -= 1 + h2 + l2;
    }
    if (rem != 0) return false;
    der_int(r, roor, sig + v0, l0);
    der_int(s, soor, sig + v1, l1);
    return true;
}

// DER, range checks and e = SHA-256(M) reduced mod n.  Returns the status to report when the
// signature stops here (0xff: go on with the arithmetic).
template <int C>
CHIP_DEV uint32_t ecdsa_front(u256& r, u256& s, u256& e, const uint8_t* sig, uint32_t siglen, const uint8_t* msg,
                              uint32_t msglen) {
    const ec_curve_c& cv = curve<C>();
    bool roor, soor;
    if (!der_decode(sig, siglen, r, roor, s, soor)) return CHIP_SIG_DECODE;
    if (roor || soor || u256_is_zero(r) || u256_is_zero(s) || u256_ge(r, cv.n) || u256_ge(s, cv.n)) return CHIP_INVALID;
    uint32_t H[8];
    sha256_bytes(H, msg, msglen);
#pragma unroll
    for (int k = 0; k < 8; k++) e.w[k] = H[7 - k];
    u256 t;
    if (!u256_sub(t, e, cv.n)) e = t;   // e < 2^256 < 2n
    return 0xffu;
}

// ecdsa_front with the signature staged in this lane's LDS slot first: up to EC_SIG_STAGE_DW independent dword
// loads, issued together, instead of the DER walk's chain of dependent byte loads from global memory (each
// waiting for the one before).  DER signatures of both curves are at most 72 bytes; longer ones take the plain path.
#define EC_SIG_STAGE_DW 21   // 84 bytes: 72 + up to 3 bytes of misalignment (odd stride: no LDS bank conflicts)
template <int C>
CHIP_DEV uint32_t ecdsa_front_staged(u256& r, u256& s, u256& e, const uint8_t* sig, uint32_t siglen, const uint8_t* msg,
                                     uint32_t msglen, uint32_t* lslot) {
    const uint32_t sh = (uint32_t)((uintptr_t)sig & 3u);
    const bool staged = sh + siglen <= 4u * EC_SIG_STAGE_DW;
    if (staged) {
        const uint32_t* ap = reinterpret_cast<const uint32_t*>(sig - sh);   // aligned dwords overlapping the signature
        const uint32_t ndw = (sh + siglen + 3u) >> 2;
#pragma unroll
        for (int k = 0; k < EC_SIG_STAGE_DW; k++)
            if ((uint32_t)k < ndw) lslot[k] = ap[k];
    }
    // one inlined walk over either source (generic loads)
    return ecdsa_front<C>(r, s, e, staged ? reinterpret_cast<const uint8_t*>(lslot) + sh : sig, siglen, msg, msglen);
}

// x(R) mod n == r  <=>  X == r Z^2  or  (r + n < p and X == (r + n) Z^2); R = infinity -> false
template <int C>
CHIP_DEV bool ecdsa_check(const jpt& acc, const u256& r) {
    if (fp_is_zero<C>(acc.Z)) return false;
    u256 z2, t;
    fp_sqr<C>(z2, acc.Z);
    fp_mul<C>(t, r, z2);
    if (fp_eq<C>(t, acc.X)) return true;
    u256 rn;
    const uint32_t c = u256_add(rn, r, curve<C>().n);
    if (c || u256_ge(rn, curve<C>().p)) return false;
    fp_mul<C>(t, rn, z2);
    return fp_eq<C>(t, acc.X);
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
// the comb kernels' digit addition: the exceptional case sets `exc` (jmadd_x)
template <int C>
CHIP_DEV void add_digit_x(jpt& acc, const apt& e, int d, bool& exc) {
    if (d == 0) return;
    apt a = e;
    if (d < 0) fp_neg<C>(a.y, a.y);
    jmadd_x<C>(acc, acc, a, exc);
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
    if (blockIdx.x * blockDim.x >= *count) return;   // whole block past the list: skip the table load
    const ec_aff_c* G = (EC_CURVE(C) == CURVE_R1) ? EC_R1_G_TABLE : EC_K1_G_TABLE;
    for (int i = threadIdx.x; i < EC_G_ENTRIES * 16; i += blockDim.x) {
        const ec_aff_c& e = G[i >> 4];
        gtab[i] = (i & 15) < 8 ? e.x[i & 7] : e.y[i & 7];
    }
    __syncthreads();
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= *count) return;
    const uint32_t i = list[gid];
    const ec_curve_c& cv = curve<C>();
    u256 r, s, e;
    const uint32_t mi = msg_idx[i];
    const uint32_t st0 = ecdsa_front<C>(r, s, e, sig_data + sig_off[i], sig_len[i], msg_data + msg_off[mi], msg_len[mi]);
    if (st0 != 0xffu) {
        status[i] = (uint8_t)st0;
        return;
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
    jpt_inf(acc);
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
#pragma unroll 1
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
    status[i] = ecdsa_check<C>(acc, r) ? CHIP_VALID : CHIP_INVALID;
}

// ---- Crypto.decodePublicKey of an ECDSA r1 / k1 SPKI (BC decodePoint) for the Kryo front end: ok = the point
// decodes; kind 1 also requires the uncompressed encoding BCECPublicKey re-encodes
__global__ void __launch_bounds__(256) k_ecdsa_key_check(uint64_t n, const uint8_t* __restrict__ pool,
                                                         const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ len,
                                                         const uint8_t* __restrict__ kind, uint8_t* __restrict__ ok) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = pool + off[i];
    const uint32_t l = len[i];
    int scheme = 0;
    const uint8_t* pt = nullptr;
    uint32_t ptlen = 0;
    if (l == 91 && match_prefix(p, SPKI_R1_PFX, 26, 0x59, 0x42)) { scheme = CHIP_SCHEME_R1; pt = p + 26; ptlen = 65; }
    else if (l == 59 && match_prefix(p, SPKI_R1_PFX, 26, 0x39, 0x22)) { scheme = CHIP_SCHEME_R1; pt = p + 26; ptlen = 33; }
    else if (l == 88 && match_prefix(p, SPKI_K1_PFX, 23, 0x56, 0x42)) { scheme = CHIP_SCHEME_K1; pt = p + 23; ptlen = 65; }
    else if (l == 56 && match_prefix(p, SPKI_K1_PFX, 23, 0x36, 0x22)) { scheme = CHIP_SCHEME_K1; pt = p + 23; ptlen = 33; }
    if (!scheme) return;
    apt q;
    bool good = scheme == CHIP_SCHEME_R1 ? ec_decode_point<CURVE_R1>(q, pt, ptlen) : ec_decode_point<CURVE_K1>(q, pt, ptlen);
    if (kind[i]) good = good && ptlen == 65;
    ok[i] = good ? 1 : 0;
}

void launch_ecdsa_key_check(hipStream_t st, uint64_t n, const uint8_t* pool, const uint64_t* off, const uint32_t* len,
                            const uint8_t* kind, uint8_t* ok) {
    if (!n) return;
    hipLaunchKernelGGL(k_ecdsa_key_check, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, n, pool, off, len, kind, ok);
}

void launch_ecdsa_key_prep(hipStream_t st, uint64_t n_keys, const uint8_t* key_data, const uint64_t* key_off,
                           const uint32_t* key_len, KeyMeta* meta, uint32_t* ectab, const uint32_t* skip) {
    if (!n_keys) return;
    const uint32_t blocks = (uint32_t)((n_keys + 255) / 256);
    hipLaunchKernelGGL(k_ecdsa_key_prep, dim3(blocks), dim3(256), 0, st, n_keys, key_data, key_off, key_len, meta,
                       ectab, skip);
}
void launch_ecdsa_key_table(hipStream_t st, uint64_t n_keys, const KeyMeta* meta, uint32_t* ectab,
                            const uint32_t* skip) {
    if (!n_keys) return;
    hipLaunchKernelGGL(k_ecdsa_key_table, dim3((uint32_t)((n_keys + 63) / 64)), dim3(64), 0, st, n_keys, meta, ectab,
                       skip);
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
// Fixed-base G comb: entry (w, j) = j 2^(EC_GW w) G for windows w < EC_GWIN, j = 1..2^(EC_GW-1),
// affine, 16 words each.  u1 < n < 2^256 in signed radix-2^EC_GW digits: EC_GWIN digits cover
// EC_GW * EC_GWIN >= 257 bits, so the recoding never leaves a final carry.  Built once per context
// (k_ecdsa_gcomb_build: one lane per entry, 2^(EC_GW w) G by doublings, the multiple by
// double-and-add, one inversion to affine).
#ifndef EC_GW
#define EC_GW 16   // measured: 12 -> 76.0M, 14 -> 77.3M, 16 -> 78.4M cfg3 sigs/s (P-256 only 71.6 -> 74.2M)
#endif
#define EC_GWIN ((256 + EC_GW) / EC_GW)
#define EC_GENT (1u << (EC_GW - 1))
#define EC_GCOMB_WORDS ((uint64_t)EC_GWIN * EC_GENT * 16)

template <int C>
__global__ void __launch_bounds__(64) k_ecdsa_gcomb_build(uint32_t* __restrict__ out) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= EC_GWIN * EC_GENT) return;
    const uint32_t w = g / EC_GENT, j = g % EC_GENT + 1;
    const ec_aff_c& G = (EC_CURVE(C) == CURVE_R1) ? EC_R1_G_TABLE[1] : EC_K1_G_TABLE[1];
    jpt P;
    u256_from_c(P.X, G.x);
    u256_from_c(P.Y, G.y);
    u256_set_word(P.Z, 1);
#pragma unroll 1
    for (uint32_t b = 0; b < EC_GW * w; b++) jdbl<C>(P, P);
    u256 zi;
    apt base;
    fp_inv_vt<C>(zi, P.Z);
    jpt_to_aff<C>(base, P, zi);
    jpt acc;
    jpt_inf(acc);
#pragma unroll 1
    for (int bit = EC_GW - 1; bit >= 0; bit--) {
        jdbl<C>(acc, acc);
        if ((j >> bit) & 1u) jmadd<C>(acc, acc, base);
    }
    fp_inv_vt<C>(zi, acc.Z);
    apt a;
    jpt_to_aff<C>(a, acc, zi);
    fp_canon<C>(a.x, a.x);
    fp_canon<C>(a.y, a.y);
    store_apt(out + ((uint64_t)w * EC_GENT + (j - 1)) * 16, a);
}

uint64_t ecdsa_gcomb_words() { return 2 * EC_GCOMB_WORDS; }
void launch_ecdsa_gcomb_build(hipStream_t st, uint32_t* gcomb) {
    const uint32_t lanes = EC_GWIN * EC_GENT;
    hipLaunchKernelGGL(k_ecdsa_gcomb_build<CURVE_R1>, dim3((lanes + 63) / 64), dim3(64), 0, st, gcomb);
    hipLaunchKernelGGL(k_ecdsa_gcomb_build<CURVE_K1>, dim3((lanes + 63) / 64), dim3(64), 0, st, gcomb + EC_GCOMB_WORDS);
}

// ---------------------------------------------------------------------------------------
// Per-key comb tables: window w (0..64) holds j 2^(4w) Q for j = 1..8, affine (16 words each).
#define EC_COMB_QWIN 65
#define EC_COMB_QENT 8
#define EC_COMB_JW 24
// affine table per key, then (after all keys) the Jacobian scratch it is normalised from
// (a secp256k1 key's GLV table, 26 x 16 entries + beta x, 9,984 words, is the larger: see EC_GLV_*)
#define EC_COMB_KEY_WORDS 9984
#define EC_COMB_JAC_WORDS (EC_COMB_QWIN * EC_COMB_QENT * EC_COMB_JW)

// ---- GLV for secp256k1 (BC 1.57's GLVTypeBEndomorphism on the k1 path; CHIP_EC_GLV, default on) ----
// lambda Q = (beta x, y) with beta^3 = 1 (mod p), lambda^3 = 1 (mod n).  u2 = a1 + lambda a2 (mod n) with
// |a1|, |a2| < 2^128 (the rounded-lattice split: c_i = round(u2 g_i / 2^384), a2 = c1 (-b1) + c2 (-b2),
// a1 = u2 - lambda a2), so u2 Q = a1 Q + a2 (lambda Q) needs only the table's windows 0..32: a secp256k1 key's
// table is 26 windows of {1..16} 2^(5w) Q plus beta x of each entry (EC_GLV_BETA_AT): 52 additions per signature
// instead of 65, and a chain of 125 doublings instead of 256 (the 129-bit halves take radix 32 for the table memory
// the 256-bit scalar took at radix 16).
// Constants checked in tools/glv_constants.py (lambda G = (beta Gx, Gy), the split's identity and bound).
#define EC_GLV_W 5                                             // window bits of the GLV table
#define EC_GLV_ENT 16                                          // entries per window: signed digits |d| <= 16
#define EC_GLV_WIN 26                                          // windows of a 129-bit signed radix-32 recoding
#ifndef EC_GLV_LO
#define EC_GLV_LO 13                                           // windows [0, 13) built and added with the low half
#endif
#ifndef EC_GLV_FILL_GROUP
#define EC_GLV_FILL_GROUP 2                                    // windows per fill lane (7 of a launch's 8-9 groups)
#endif
#define EC_GLV_BETA_AT (EC_GLV_WIN * EC_GLV_ENT * 16)            // beta x of entry (w, j): + (w * 16 + j - 1) * 8
static_assert(EC_GLV_BETA_AT + EC_GLV_WIN * EC_GLV_ENT * 8 <= EC_COMB_KEY_WORDS, "GLV table");
static_assert(EC_GLV_WIN * EC_GLV_W >= 130, "GLV windows cover a 129-bit recoding");
static_assert(EC_GLV_WIN * EC_GLV_ENT * EC_COMB_JW <= EC_COMB_QWIN * EC_COMB_QENT * EC_COMB_JW, "GLV scratch");
static_assert(EC_COMB_QWIN * EC_COMB_QENT * 16 <= EC_COMB_KEY_WORDS, "P-256 table");
__device__ __constant__ const uint32_t K1_BETA[8] = {0x719501eeu, 0xc1396c28u, 0x12f58995u, 0x9cf04975u,
                                                     0xac3434e9u, 0x6e64479eu, 0x657c0710u, 0x7ae96a2bu};
__device__ __constant__ const uint32_t K1_GLV_G1[8] = {0x45dbb031u, 0xe893209au, 0x71e8ca7fu, 0x3daa8a14u,
                                                       0x9284eb15u, 0xe86c90e4u, 0xa7d46bcdu, 0x3086d221u};
__device__ __constant__ const uint32_t K1_GLV_G2[8] = {0x8ac47f71u, 0x1571b4aeu, 0x9df506c6u, 0x221208acu,
                                                       0x0abfe4c4u, 0x6f547fa9u, 0x010e8828u, 0xe4437ed6u};
// -b1 R, -b2 R, -lambda R (mod n): Montgomery multipliers, so mn_mul gives the plain product mod n
__device__ __constant__ const uint32_t K1_GLV_MB1R[8] = {0x0ad9263cu, 0xc50468d0u, 0xfaa6ed42u, 0x1b1c8205u,
                                                         0x8ac47f71u, 0x1571b4aeu, 0x9df506c6u, 0x221208acu};
__device__ __constant__ const uint32_t K1_GLV_MB2R[8] = {0x6a144696u, 0x0cac5e50u, 0xf3ba5939u, 0x1e8a8dc5u,
                                                         0xba244fceu, 0x176cdf65u, 0x8e173580u, 0xc25575ebu};
__device__ __constant__ const uint32_t K1_GLV_MLR[8] = {0x06a3d4a3u, 0xcf54734fu, 0x2b820beeu, 0x8e1af539u,
                                                        0xad96826du, 0x8c5699f9u, 0x7aa729c6u, 0xacd7bfe8u};
__device__ __constant__ const uint32_t K1_N_HALF[8] = {0x681b20a0u, 0xdfe92f46u, 0x57a4501du, 0x5d576e73u,
                                                       0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu};
// round(k g / 2^384) for k, g < 2^256 (< 2^128 + 1)
CHIP_DEV void glv_round_shift(u256& c, const u256& k, const uint32_t* g) {
    u256 gg;
    u256_from_c(gg, g);
    uint32_t t[16];
    mul_512(t, k, gg);
    uint32_t cy = 0;
    const uint32_t rb = t[11] >> 31;
    c.w[0] = __builtin_addc(t[12], rb, 0u, &cy);
    c.w[1] = __builtin_addc(t[13], 0u, cy, &cy);
    c.w[2] = __builtin_addc(t[14], 0u, cy, &cy);
    c.w[3] = __builtin_addc(t[15], 0u, cy, &cy);
    c.w[4] = cy;
    c.w[5] = c.w[6] = c.w[7] = 0;
}
// (a + b) mod n for a, b < n
CHIP_DEV void mn_add_k1(u256& r, const u256& a, const u256& b) {
    const uint32_t c = u256_add(r, a, b.w);
    u256 s;
    const uint32_t br = u256_sub(s, r, EC_K1.n);
    if (c || !br) r = s;
}
// u2 (< n) -> |a1|, |a2| < 2^128 with their signs: u2 = s1 |a1| + lambda s2 |a2| (mod n)
CHIP_DEV void glv_split(const u256& u2, u256& a1, bool& neg1, u256& a2, bool& neg2) {
    u256 c1, c2, x1, x2, r1, r2, m;
    glv_round_shift(c1, u2, K1_GLV_G1);
    glv_round_shift(c2, u2, K1_GLV_G2);
    u256_from_c(m, K1_GLV_MB1R);
    mn_mul<CURVE_K1>(x1, c1, m);
    u256_from_c(m, K1_GLV_MB2R);
    mn_mul<CURVE_K1>(x2, c2, m);
    mn_add_k1(r2, x1, x2);
    u256_from_c(m, K1_GLV_MLR);
    mn_mul<CURVE_K1>(x1, r2, m);
    mn_add_k1(r1, x1, u2);
    // the signed representative: r > n / 2 -> -(n - r)
    neg1 = u256_ge(r1, K1_N_HALF) && !u256_eq_c(r1, K1_N_HALF);
    neg2 = u256_ge(r2, K1_N_HALF) && !u256_eq_c(r2, K1_N_HALF);
    u256 nn, nr;
    u256_from_c(nn, EC_K1.n);
    (void)u256_sub(nr, nn, r1.w);
    a1 = neg1 ? nr : r1;
    (void)u256_sub(nr, nn, r2.w);
    a2 = neg2 ? nr : r2;
}

CHIP_DEV bool ec_key_ok(const KeyMeta* meta, uint64_t k, int scheme) {
    const KeyMeta m = meta[k];
    return m.scheme == scheme && m.ok;
}

// chain: P_w = 2^(4w) Q (Jacobian) for windows [wa, wb) into entry 0 of each window of the scratch
// (4 serial doublings per window, 256 per key: the latency of this kernel is the per-key table's
// critical path).  Run in two launches (windows 0..31, then 32..64 continuing from P_31) so the low
// half of the table is filled — and the signatures' low-window additions run — while the chain
// still doubles towards the high half.
template <int C>
CHIP_DEV void ec_comb_chain(const uint32_t* __restrict__ ectab, uint32_t* __restrict__ jac, uint64_t k, uint32_t wa,
                            uint32_t wb, uint32_t ent = EC_COMB_QENT, uint32_t wbits = 4) {
    uint32_t* tab = jac + k * EC_COMB_JAC_WORDS;
    jpt P;
    uint32_t w = wa;
    if (wa == 0) {
        apt q;
        load_apt(q, ectab + k * EC_TAB_STRIDE + 16);
        jpt_from_aff(P, q);
        store_jpt(tab, P);
        w = 1;
    } else {
        load_jpt(P, tab + (wa - 1) * ent * EC_COMB_JW);
    }
#pragma unroll 1
    for (; w < wb; w++) {
#pragma unroll 1
        for (uint32_t b = 0; b < wbits; b++) jdbl<C>(P, P);
        store_jpt(tab + w * ent * EC_COMB_JW, P);
    }
}
// The same chain on a lane pair per key (adjacent lanes of a wave; both hold the point): each doubling's field
// operations are split between the two lanes — P-256's 3M + 5S as four steps of one operation per lane, secp256k1's
// 2M + 5S likewise — and the halves exchanged by DPP quad permutes (one v_mov_dpp per word), so the serial chain
// per key, the critical path of the ECDSA table build, carries about half the dependent operations per doubling.
CHIP_DEV uint32_t ec_pair_swap(uint32_t v) {   // the partner lane's v (lanes 2i <-> 2i+1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
}
CHIP_DEV void u256_swap_in(u256& out, const u256& mine) {
#pragma unroll
    for (int i = 0; i < 8; i++) out.w[i] = ec_pair_swap(mine.w[i]);
}
CHIP_DEV void u256_sel(u256& r, uint32_t m, const u256& a, const u256& b) {   // m all-ones: a, else b
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = (a.w[i] & m) | (b.w[i] & ~m);
}
// r = 2p on a lane pair (odd: all-ones on the odd lane); p, r the same on both lanes
template <int C>
CHIP_DEV void jdbl_pair(jpt& r, const jpt& p, uint32_t odd) {
    u256 mine, other, a, b;
    if (EC_CURVE(C) == CURVE_R1) {
        // dbl-2001-b.  1: delta = Z^2 (even), gamma = Y^2 (odd)
        u256 delta, gamma, alpha, beta, a2, g2, yz2, y3m, t1, t2;
        u256_sel(a, odd, p.Y, p.Z);
        fp_sqr<C>(mine, a);
        u256_swap_in(other, mine);
        u256_sel(delta, odd, other, mine);
        u256_sel(gamma, odd, mine, other);
        // 2: (X - delta)(X + delta) (even), beta = X gamma (odd)
        fp_sub<C>(t1, p.X, delta);
        fp_add<C>(t2, p.X, delta);
        u256_sel(a, odd, p.X, t1);
        u256_sel(b, odd, gamma, t2);
        fp_mul<C>(mine, a, b);
        u256_swap_in(other, mine);
        u256_sel(alpha, odd, other, mine);
        u256_sel(beta, odd, mine, other);
        fp_add<C>(t1, alpha, alpha);
        fp_add<C>(alpha, alpha, t1);            // 3 (X - delta)(X + delta)
        // 3: alpha^2 (even), gamma^2 (odd)
        u256_sel(a, odd, gamma, alpha);
        fp_sqr<C>(mine, a);
        u256_swap_in(other, mine);
        u256_sel(a2, odd, other, mine);
        u256_sel(g2, odd, mine, other);
        fp_add<C>(t1, beta, beta);
        fp_add<C>(t1, t1, t1);                  // 4 beta
        fp_sub<C>(t2, a2, t1);
        fp_sub<C>(r.X, t2, t1);                 // X3 = alpha^2 - 8 beta
        // 4: (Y + Z)^2 (even), alpha (4 beta - X3) (odd)
        fp_sub<C>(t1, t1, r.X);
        fp_add<C>(t2, p.Y, p.Z);
        u256_sel(a, odd, alpha, t2);
        u256_sel(b, odd, t1, t2);
        fp_mul<C>(mine, a, b);
        u256_swap_in(other, mine);
        u256_sel(yz2, odd, other, mine);
        u256_sel(y3m, odd, mine, other);
        fp_sub<C>(t1, yz2, gamma);
        fp_sub<C>(r.Z, t1, delta);              // Z3 = (Y+Z)^2 - gamma - delta
        fp_add<C>(g2, g2, g2);
        fp_add<C>(g2, g2, g2);
        fp_add<C>(g2, g2, g2);                  // 8 gamma^2
        fp_sub<C>(r.Y, y3m, g2);
    } else {
        // dbl-2009-l.  1: A = X^2 (even), B = Y^2 (odd)
        u256 A, B, Cc, D, E, F, T, yz, y3m, t;
        u256_sel(a, odd, p.Y, p.X);
        fp_sqr<C>(mine, a);
        u256_swap_in(other, mine);
        u256_sel(A, odd, other, mine);
        u256_sel(B, odd, mine, other);
        fp_add<C>(E, A, A);
        fp_add<C>(E, E, A);                     // E = 3A
        // 2: F = E^2 (even), C = B^2 (odd)
        u256_sel(a, odd, B, E);
        fp_sqr<C>(mine, a);
        u256_swap_in(other, mine);
        u256_sel(F, odd, other, mine);
        u256_sel(Cc, odd, mine, other);
        // 3: (X + B)^2 (even), Y Z (odd)
        fp_add<C>(t, p.X, B);
        u256_sel(a, odd, p.Y, t);
        u256_sel(b, odd, p.Z, t);
        fp_mul<C>(mine, a, b);
        u256_swap_in(other, mine);
        u256_sel(T, odd, other, mine);
        u256_sel(yz, odd, mine, other);
        fp_sub<C>(t, T, A);
        fp_sub<C>(t, t, Cc);
        fp_add<C>(D, t, t);
        fp_add<C>(r.Z, yz, yz);
        fp_add<C>(t, D, D);
        fp_sub<C>(r.X, F, t);
        // 4: E (D - X3) (both lanes compute it: one operation, no exchange)
        fp_sub<C>(t, D, r.X);
        fp_mul<C>(y3m, E, t);
        fp_add<C>(Cc, Cc, Cc);
        fp_add<C>(Cc, Cc, Cc);
        fp_add<C>(Cc, Cc, Cc);
        fp_sub<C>(r.Y, y3m, Cc);
    }
}
template <int C>
CHIP_DEV void ec_comb_chain2(const uint32_t* __restrict__ ectab, uint32_t* __restrict__ jac, uint64_t k, uint32_t wa,
                             uint32_t wb, uint32_t odd, uint32_t ent = EC_COMB_QENT, uint32_t wbits = 4) {
    uint32_t* tab = jac + k * EC_COMB_JAC_WORDS;
    jpt P;
    uint32_t w = wa;
    if (wa == 0) {
        apt q;
        load_apt(q, ectab + k * EC_TAB_STRIDE + 16);
        jpt_from_aff(P, q);
        if (!odd) store_jpt(tab, P);
        w = 1;
    } else {
        load_jpt(P, tab + (wa - 1) * ent * EC_COMB_JW);
    }
#pragma unroll 1
    for (; w < wb; w++) {
#pragma unroll 1
        for (uint32_t b = 0; b < wbits; b++) jdbl_pair<C>(P, P, odd);
        if (!odd) store_jpt(tab + w * ent * EC_COMB_JW, P);
    }
}

// fill, for windows [w0, w1) of one key:
//   1. P_w to affine with one inversion for the group (Montgomery's trick; prefix products parked in
//      the x slots of the output entries)
//   2. j P_w for j = 2..8: one doubling and six mixed additions, Jacobian into the scratch
//   3. those 7 (w1 - w0) entries to affine with one more shared inversion
#define EC_FILL_GROUP 4   // measured: 1 -> 68.9M, 2 -> 73.4M, 4 -> 75.3M, 8 -> 74.6M, 16 -> 59.7M cfg3 sigs/s
template <int C>
CHIP_DEV void ec_comb_fill(uint32_t* __restrict__ jac, uint32_t* __restrict__ out, uint32_t w0, uint32_t w1,
                           uint32_t* __restrict__ bx, uint32_t ent = EC_COMB_QENT) {
    // bx (GLV, secp256k1): beta x of every entry written beside the table
    auto beta_x = [&](uint32_t w, uint32_t j, const apt& a) {
        if (!bx) return;
        u256 b, t;
        u256_from_c(b, K1_BETA);
        fp_mul<C>(t, a.x, b);
        store_u256(bx + (w * ent + j) * 8, t);
    };
    u256 acc, z, inv;
    // 1.
    u256_set_word(acc, 1);
#pragma unroll 1
    for (uint32_t w = w0; w < w1; w++) {
        store_u256(out + w * ent * 16, acc);
        load_u256(z, jac + w * ent * EC_COMB_JW + 16);
        fp_mul<C>(acc, acc, z);
    }
    fp_inv_vt<C>(inv, acc);   // entries are 2^(4w) Q, never infinity for a valid key
#pragma unroll 1
    for (uint32_t w = w1; w-- > w0;) {
        uint32_t* o = out + w * ent * 16;
        jpt P;
        u256 pre, zi;
        load_jpt(P, jac + w * ent * EC_COMB_JW);
        load_u256(pre, o);
        fp_mul<C>(zi, inv, pre);
        fp_mul<C>(inv, inv, P.Z);
        apt a;
        jpt_to_aff<C>(a, P, zi);
        store_apt(o, a);
        beta_x(w, 0, a);
    }
    // 2.
    u256_set_word(acc, 1);
#pragma unroll 1
    for (uint32_t w = w0; w < w1; w++) {
        uint32_t* e = jac + w * ent * EC_COMB_JW;
        uint32_t* o = out + w * ent * 16;
        apt a;
        load_apt(a, o);
        jpt A;
        jpt_from_aff(A, a);
        jdbl<C>(A, A);
        bool exc = false;   // j a + a with 2 <= j <= 7 is never P == Q (prime order n > 8)
#pragma unroll 1
        for (int j = 2; j <= (int)ent; j++) {
            if (j > 2) jmadd_x<C>(A, A, a, exc);
            store_jpt(e + (uint32_t)(j - 1) * EC_COMB_JW, A);
            store_u256(o + (uint32_t)(j - 1) * 16, acc);
            fp_mul<C>(acc, acc, A.Z);
        }
    }
    // 3.
    fp_inv_vt<C>(inv, acc);
#pragma unroll 1
    for (uint32_t w = w1; w-- > w0;) {
        const uint32_t* e = jac + w * ent * EC_COMB_JW;
        uint32_t* o = out + w * ent * 16;
#pragma unroll 1
        for (int j = (int)ent - 1; j >= 1; j--) {
            jpt A;
            u256 pre, zi;
            load_jpt(A, e + (uint32_t)j * EC_COMB_JW);
            load_u256(pre, o + (uint32_t)j * 16);
            fp_mul<C>(zi, inv, pre);
            fp_mul<C>(inv, inv, A.Z);
            apt a;
            jpt_to_aff<C>(a, A, zi);
            store_apt(o + (uint32_t)j * 16, a);
            beta_x(w, (uint32_t)j, a);
        }
    }
}
// one launch for both curves: r1 and k1 keys build concurrently (lane per key)
__global__ void __launch_bounds__(64) k_ecdsa_comb_chain(uint64_t n_keys, const KeyMeta* __restrict__ meta,
                                                         const uint32_t* __restrict__ ectab, uint32_t* __restrict__ jac,
                                                         uint32_t prio, uint32_t wa, uint32_t wb,
                                                         const uint32_t* __restrict__ skip, uint32_t glv) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_keys || (skip && *skip)) return;
    // the chain is the latency-bound critical path of the step: win VALU arbitration against the
    // throughput kernels of the main stream that share its SIMDs
    if (prio) __builtin_amdgcn_s_setprio(3);
    // GLV: a secp256k1 table's windows [0, 13) with the low half, [13, 26) with the high one
    const uint32_t wak = glv ? (wa ? EC_GLV_LO : 0u) : wa, wbk = glv ? (wa ? EC_GLV_WIN : EC_GLV_LO) : wb;
    if (ec_key_ok(meta, k, CHIP_SCHEME_R1)) ec_comb_chain<CURVE_R1 | CURVE_ILP>(ectab, jac, k, wa, wb);
    else if (ec_key_ok(meta, k, CHIP_SCHEME_K1))
        ec_comb_chain<CURVE_K1 | CURVE_ILP>(ectab, jac, k, wak, wbk, glv ? EC_GLV_ENT : EC_COMB_QENT, glv ? EC_GLV_W : 4);
}
#ifndef EC_CHAIN_PAIR
#define EC_CHAIN_PAIR 1   // the chain on lane pairs (k_ecdsa_comb_chain2); CHIP_EC_CHAIN_PAIR=0: one lane per key
#endif
// two lanes per key (both lanes of a pair take the same exits: the same key)
__global__ void __launch_bounds__(64) k_ecdsa_comb_chain2(uint64_t n_keys, const KeyMeta* __restrict__ meta,
                                                          const uint32_t* __restrict__ ectab, uint32_t* __restrict__ jac,
                                                          uint32_t prio, uint32_t wa, uint32_t wb,
                                                          const uint32_t* __restrict__ skip, uint32_t glv) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t k = g >> 1;
    const uint32_t odd = (g & 1u) ? ~0u : 0u;
    if (k >= n_keys || (skip && *skip)) return;
    if (prio) __builtin_amdgcn_s_setprio(3);
    const uint32_t wak = glv ? (wa ? EC_GLV_LO : 0u) : wa, wbk = glv ? (wa ? EC_GLV_WIN : EC_GLV_LO) : wb;
    if (ec_key_ok(meta, k, CHIP_SCHEME_R1)) ec_comb_chain2<CURVE_R1 | CURVE_ILP>(ectab, jac, k, wa, wb, odd);
    else if (ec_key_ok(meta, k, CHIP_SCHEME_K1))
        ec_comb_chain2<CURVE_K1 | CURVE_ILP>(ectab, jac, k, wak, wbk, odd, glv ? EC_GLV_ENT : EC_COMB_QENT,
                                             glv ? EC_GLV_W : 4);
}
// lane per key x group of `gw` windows of [wa, wb) (the fill is latency-bound: fewer windows per
// lane = more lanes, at one shared inversion pair per lane)
#ifndef EC_FILL_WAVES
#define EC_FILL_WAVES 1   // waves per SIMD the table fill's registers must leave room for (170 VGPRs = 2 waves; 3: 2 spilled)
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(EC_FILL_WAVES))) k_ecdsa_comb_fill(uint64_t n_keys, const KeyMeta* __restrict__ meta,
                                                         uint32_t* __restrict__ ctab, uint32_t* __restrict__ jac,
                                                         uint32_t wa, uint32_t wb, uint32_t gw, uint32_t ng,
                                                         const uint32_t* __restrict__ skip, uint32_t glv) {
    // ng lanes per key: P-256's (wb - wa) / gw groups, or more when the GLV half needs them (the rest return)
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t k = g / ng;
    const uint32_t grp = (uint32_t)(g % ng);
    if (k >= n_keys || (skip && *skip)) return;
    const uint32_t w0 = wa + grp * gw;
    const uint32_t w1 = w0 + gw < wb ? w0 + gw : wb;
    uint32_t* e = jac + k * EC_COMB_JAC_WORDS;
    uint32_t* out = ctab + k * EC_COMB_KEY_WORDS;
    if (ec_key_ok(meta, k, CHIP_SCHEME_R1)) {
        if (w0 < w1) ec_comb_fill<CURVE_R1>(e, out, w0, w1, nullptr);
    } else if (ec_key_ok(meta, k, CHIP_SCHEME_K1)) {
        if (!glv) {
            if (w0 < w1) ec_comb_fill<CURVE_K1>(e, out, w0, w1, nullptr);
            return;
        }
        // the launch's group grp over the curve's own half, [0, 13) or [13, 26), EC_GLV_FILL_GROUP windows a lane: a
        // window's 15 additions are twice P-256's 7, so half the windows keep the lanes' serial chains even
        const uint32_t lo = wa ? EC_GLV_LO : 0u, hi = wa ? EC_GLV_WIN : EC_GLV_LO;
        const uint32_t v0 = lo + grp * EC_GLV_FILL_GROUP, v1 = min(v0 + EC_GLV_FILL_GROUP, hi);
        if (v0 < v1) ec_comb_fill<CURVE_K1>(e, out, v0, v1, out + EC_GLV_BETA_AT, EC_GLV_ENT);
    }
}

// ---- work lists grouped by key (counting sort), so the lanes of a wave read one key's table ----
// key_count[k] = signatures of key k in its curve's list (k_classify's histogram); a key's
// signatures occupy [key_base[k], key_base[k] + key_count[k]) of the grouped list of its curve.
__global__ void __launch_bounds__(256) k_ec_group_base(uint64_t n_keys, const KeyMeta* __restrict__ meta,
                                                       const uint32_t* __restrict__ key_count,
                                                       uint32_t* __restrict__ key_base, uint32_t* __restrict__ ctr) {
    // one atomic per workgroup per curve (block prefix sums)
    __shared__ uint32_t s_wave[4], s_base[2];
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t c = 0;
    int curve = -1;
    if (k < n_keys) {
        const KeyMeta m = meta[k];
        c = key_count[k];
        if (m.ok && c && (m.scheme == CHIP_SCHEME_R1 || m.scheme == CHIP_SCHEME_K1)) curve = m.scheme == CHIP_SCHEME_R1 ? 0 : 1;
    }
    uint32_t tot0, tot1;
    const uint32_t ex0 = block_scan_excl(curve == 0 ? c : 0u, s_wave, tot0);
    const uint32_t ex1 = block_scan_excl(curve == 1 ? c : 0u, s_wave, tot1);
    if (threadIdx.x == 0) {
        s_base[0] = tot0 ? atomicAdd(&ctr[0], tot0) : 0u;
        s_base[1] = tot1 ? atomicAdd(&ctr[1], tot1) : 0u;
    }
    __syncthreads();
    if (curve >= 0) key_base[k] = s_base[curve] + (curve == 0 ? ex0 : ex1);
}
// one lane per (curve list, position): grid covers 2 n lanes, [0, n) r1 and [n, 2n) k1; the slot
// inside the key's range is the signature's key rank from k_classify (no atomics)
__global__ void __launch_bounds__(256) k_ec_group_scatter(uint64_t n, const uint32_t* __restrict__ lists,
                                                          const uint32_t* __restrict__ counts,
                                                          const uint32_t* __restrict__ key_idx,
                                                          const uint32_t* __restrict__ key_base,
                                                          const uint32_t* __restrict__ key_rank, uint32_t* __restrict__ out) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int L = g < n ? 0 : 1;
    const uint64_t pos = g - (uint64_t)L * n;
    const uint32_t cnt = counts[L == 0 ? LIST_R1 : LIST_K1];
    if (pos >= cnt) return;
    const uint32_t i = lists[(uint64_t)(L == 0 ? LIST_R1 : LIST_K1) * n + pos];
    out[(uint64_t)L * n + key_base[key_idx[i]] + key_rank[i]] = i;
}

// ---- signature kernels, SoA hand-off by list position (`cap` = list capacity) ----
//   pre (A): DER, range, e = SHA-256(M), s R; wave prefix / suffix products of s R
//            slots 0-7 e, 8-15 exclusive prefix, 16-23 exclusive suffix, 32-39 r, 40 state;
//            wave product -> wp[wave]
//   inv (B): wp[wave] -> wp[wave]^-1 (one Fermat inversion per wave of signatures)
//   g   (C): s^-1 = wp^-1 * prefix * suffix, u1 = e s^-1, u2 = r s^-1, u1 G;
//            slots 0-23 u1 G (X, Y, Z), 24-31 u2
//   q   (D): + u2 Q from the key's table, x(R) mod n == r
#define EC_MID_WORDS 42   // + word 41: the GLV signs and carries HALF 0 hands to HALF 1 (secp256k1)

CHIP_DEV void mid_store(uint32_t* mid, uint64_t cap, uint32_t gid, int slot, const u256& v) {
#pragma unroll
    for (int k = 0; k < 8; k++) mid[(uint64_t)(slot + k) * cap + gid] = v.w[k];
}
CHIP_DEV void mid_load(u256& v, const uint32_t* mid, uint64_t cap, uint32_t gid, int slot) {
#pragma unroll
    for (int k = 0; k < 8; k++) v.w[k] = mid[(uint64_t)(slot + k) * cap + gid];
}

CHIP_DEV void wave_shfl_up(u256& o, const u256& v, int d) {
#pragma unroll
    for (int k = 0; k < 8; k++) o.w[k] = (uint32_t)__shfl_up((int)v.w[k], d, 64);
}
CHIP_DEV void wave_shfl_down(u256& o, const u256& v, int d) {
#pragma unroll
    for (int k = 0; k < 8; k++) o.w[k] = (uint32_t)__shfl_down((int)v.w[k], d, 64);
}

// A.  The wave-level part of the batched inversion: inclusive prefix and suffix products of s R
// across the 64 lanes (Hillis-Steele scans over shuffles); the exclusive products stay with the
// lane, the wave's total goes to k_ecdsa_comb_inv.  Lanes without an arithmetic signature pass the
// Montgomery one.  Every lane of a live wave takes part.
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
                                                        uint32_t* __restrict__ wp, uint64_t cap,
                                                        uint8_t* __restrict__ status) {
    const uint32_t n = *count;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if ((gid & ~63u) >= n) return;   // whole wave past the list: wave-uniform exit
    const ec_curve_c& cv = curve<C>();
    const int lane = (int)__lane_id();
    const bool live = gid < n;
    u256 r, s, e, sm;
    bool go = false;
    __shared__ uint32_t s_sig[256 * EC_SIG_STAGE_DW];
    if (live) {
        const uint32_t i = list[gid];
        const uint32_t mi = msg_idx[i];
        const uint32_t st0 = ecdsa_front_staged<C>(r, s, e, sig_data + sig_off[i], sig_len[i], msg_data + msg_off[mi],
                                                   msg_len[mi], s_sig + threadIdx.x * EC_SIG_STAGE_DW);
        if (st0 != 0xffu) status[i] = (uint8_t)st0;
        go = st0 == 0xffu;
    }
    if (go) {
        u256 r2n;
        u256_from_c(r2n, cv.r2_n);
        mn_mul<C>(sm, s, r2n);
    } else {
        u256_from_c(sm, cv.one_n);
    }
    u256 pre = sm, suf = sm, o, t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        wave_shfl_up(o, pre, d);
        mn_mul<C>(t, pre, o);
        if (lane >= d) pre = t;
        wave_shfl_down(o, suf, d);
        mn_mul<C>(t, suf, o);
        if (lane + d < 64) suf = t;
    }
    if (lane == 63) store_u256(wp + (uint64_t)(gid >> 6) * 8, pre);
    u256 ep, es;
    wave_shfl_up(ep, pre, 1);
    wave_shfl_down(es, suf, 1);
    if (lane == 0) u256_from_c(ep, cv.one_n);
    if (lane == 63) u256_from_c(es, cv.one_n);
    if (!live) return;
    mid[(uint64_t)40 * cap + gid] = go ? 1u : 0u;
    if (!go) return;
    mid_store(mid, cap, gid, 0, e);
    mid_store(mid, cap, gid, 8, ep);
    mid_store(mid, cap, gid, 16, es);
    mid_store(mid, cap, gid, 32, r);
}

// B.  One inversion per wave product (binary extended Euclid, mn_inv), both curves in one launch: lanes [0, nw) r1 waves,
// [nw, 2 nw) k1 waves (nw = the wave capacity of one list).
__global__ void __launch_bounds__(64) k_ecdsa_comb_inv(const uint32_t* __restrict__ counts, uint32_t* __restrict__ wp_r1,
                                                       uint32_t* __restrict__ wp_k1, uint32_t nw) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const bool k1 = g >= nw;
    const uint32_t w = k1 ? g - nw : g;
    const uint32_t n = counts[k1 ? LIST_K1 : LIST_R1];
    if (w >= (n + 63) / 64) return;
    uint32_t* p = (k1 ? wp_k1 : wp_r1) + (uint64_t)w * 8;
    u256 v, inv;
    load_u256(v, p);
    if (k1) mn_inv<CURVE_K1 | CURVE_ILP>(inv, v);
    else mn_inv<CURVE_R1 | CURVE_ILP>(inv, v);
    store_u256(p, inv);
}

// C.  s^-1, u1, u2 and u1 G from the fixed comb.
template <int C>
CHIP_DEV void comb_g_body(uint32_t blk, const uint32_t* __restrict__ count, const uint32_t* __restrict__ gcomb,
                          uint32_t* __restrict__ mid, const uint32_t* __restrict__ wp, uint64_t cap, uint32_t park_all) {
    const uint32_t gid = blk * blockDim.x + threadIdx.x;
    if (gid >= *count || mid[(uint64_t)40 * cap + gid] != 1u) return;
    u256 e, r, ep, es, winv, wm, u1, u2;
    mid_load(ep, mid, cap, gid, 8);
    mid_load(es, mid, cap, gid, 16);
    load_u256(winv, wp + (uint64_t)(gid >> 6) * 8);
    mn_mul<C>(wm, winv, ep);
    mn_mul<C>(wm, wm, es);
    mid_load(e, mid, cap, gid, 0);
    mid_load(r, mid, cap, gid, 32);
    mn_mul<C>(u1, e, wm);
    mn_mul<C>(u2, r, wm);
    jpt acc;
    jpt_inf(acc);
    const uint32_t* G = gcomb + (EC_CURVE(C) == CURVE_R1 ? 0 : EC_GCOMB_WORDS);
    int carry = 0;
    apt ga;
    bool exc = false;
    // the signed radix-2^EC_GW digit of window w (windows in order: the carry runs low to high)
    auto digit = [&](int w) -> int {
        const int b = w * EC_GW;   // bits [b, b + EC_GW) of u1
        uint32_t bits;
        if (b >= 256) bits = 0;
        else if ((b & 31) + EC_GW <= 32 || (b >> 5) == 7) bits = u1.w[b >> 5] >> (b & 31);
        else bits = __builtin_amdgcn_alignbit(u1.w[(b >> 5) + 1], u1.w[b >> 5], b & 31);
        int v = (int)(bits & ((1u << EC_GW) - 1)) + carry;
        carry = (v + (1 << (EC_GW - 1)) - 1) >> EC_GW;   // digits in [-2^(W-1) + 1, 2^(W-1)]
        return v - (carry << EC_GW);
    };
#if EC_G_PF
    // software-pipelined gathers: window w + 1's G entry is loaded while window w's addition runs (a zero
    // digit loads entry 1 and skips the addition)
    int vn = digit(0);
    apt gn;
    load_apt(gn, G + ((uint32_t)(vn < 0 ? -vn : vn) - (vn != 0)) * 16);
#pragma unroll
    for (int w = 0; w < EC_GWIN; w++) {
        const int v = vn;
        ga = gn;
        if (w + 1 < EC_GWIN) {
            vn = digit(w + 1);
            load_apt(gn, G + ((uint64_t)(w + 1) * EC_GENT + (uint32_t)(vn < 0 ? -vn : vn) - (vn != 0)) * 16);
        }
        if (v != 0) {
            if (v < 0) fp_neg<C>(ga.y, ga.y);
            jmadd_x<C>(acc, acc, ga, exc);
        }
    }
#else
#pragma unroll
    for (int w = 0; w < EC_GWIN; w++) {
        const int v = digit(w);
        if (v != 0) {
            const uint32_t av = (uint32_t)(v < 0 ? -v : v);
            load_apt(ga, G + ((uint64_t)w * EC_GENT + av - 1) * 16);
            if (v < 0) fp_neg<C>(ga.y, ga.y);
            jmadd_x<C>(acc, acc, ga, exc);
        }
    }
#endif
    if (exc || park_all) {   // finished by k_ecdsa_comb_retry (park_all: CHIP_FLAG_EC_RETRY_ALL, tests)
        mid[(uint64_t)40 * cap + gid] = 2u;
        return;
    }
    mid_store(mid, cap, gid, 0, acc.X);
    mid_store(mid, cap, gid, 8, acc.Y);
    mid_store(mid, cap, gid, 16, acc.Z);
    mid_store(mid, cap, gid, 24, u2);
}
// both curves in one grid (blocks [0, half) P-256, the rest secp256k1): the secp256k1 blocks fill
// the chip while the last P-256 waves drain instead of waiting for a second launch
#ifndef EC_G_WAVES
#define EC_G_WAVES 3   // as EC_Q0_WAVES, for k_ecdsa_comb_g: 210 VGPRs = 2 waves; at 3 waves (70 spilled) the front end
                       // runs 2.71-2.76 -> 2.28 ms, cfg3 88.5-89.5 -> 90.5-91.2M (profiles/r05/ab_r05k.txt)
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(EC_G_WAVES))) k_ecdsa_comb_g(const uint32_t* __restrict__ counts,
                                                      const uint32_t* __restrict__ gcomb, uint32_t* __restrict__ mid_r1,
                                                      uint32_t* __restrict__ mid_k1, const uint32_t* __restrict__ wp_r1,
                                                      const uint32_t* __restrict__ wp_k1, uint64_t cap, uint32_t half,
                                                      uint32_t park_all) {
    if (blockIdx.x < half) comb_g_body<CURVE_R1>(blockIdx.x, counts + LIST_R1, gcomb, mid_r1, wp_r1, cap, park_all);
    else comb_g_body<CURVE_K1>(blockIdx.x - half, counts + LIST_K1, gcomb, mid_k1, wp_k1, cap, park_all);
}

// D.  u2 Q half: one mixed addition per non-zero radix-16 digit from the key's affine table, then
// x(R) mod n == r exactly as k_ecdsa_verify checks it.  The list is grouped by key and consecutive
// blocks run on one XCD, so a key's 33 KB table is read from one L2.
// Two launches: HALF 0 adds the digits of windows 0..31 (the low half of the table, filled first)
// and parks the Jacobian sum in the hand-off area; HALF 1 adds windows 32..64 and checks x(R).
template <int C, int HALF>
CHIP_DEV void comb_q_body(uint32_t blk, const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                          const uint32_t* __restrict__ key_idx, const uint32_t* __restrict__ ctab,
                          uint32_t* __restrict__ mid, uint64_t cap, uint8_t* __restrict__ status, uint32_t glv) {
    const uint32_t n = *count;
    const uint32_t gid = blk * blockDim.x + threadIdx.x;
    if (gid >= n || mid[(uint64_t)40 * cap + gid] != 1u) return;
    const uint32_t i = list[gid];
    bool exc = false;
    jpt acc;
    apt ent;
    u256 u2, r;
    mid_load(acc.X, mid, cap, gid, 0);
    mid_load(acc.Y, mid, cap, gid, 8);
    mid_load(acc.Z, mid, cap, gid, 16);
    mid_load(u2, mid, cap, gid, 24);
    mid_load(r, mid, cap, gid, 32);
    const uint32_t* qt = ctab + (uint64_t)key_idx[i] * EC_COMB_KEY_WORDS;
    if (EC_CURVE(C) == CURVE_K1 && glv) {
        // u2 Q = s1 |a1| Q + s2 |a2| (lambda Q): per radix-32 window one entry of Q's table and one of lambda Q's
        // (beta x, y).  HALF 0 splits u2 and adds windows [0, 13) (the low half of the table), then hands |a1|, |a2|
        // (in u2's slot), the signs and the digit carries (word 41) to HALF 1, which adds [13, 26) and checks.
        u256 a1, a2;
        bool n1, n2;
        int cy1 = 0, cy2 = 0;
        if (HALF == 0) {
            glv_split(u2, a1, n1, a2, n2);
        } else {
            const uint32_t f = mid[(uint64_t)41 * cap + gid];
            n1 = f & 1u;
            n2 = (f >> 1) & 1u;
            cy1 = (int)((f >> 2) & 1u);
            cy2 = (int)((f >> 3) & 1u);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                a1.w[q] = u2.w[q];
                a2.w[q] = u2.w[4 + q];
                a1.w[4 + q] = 0;
                a2.w[4 + q] = 0;
            }
        }
        const uint32_t* bxt = qt + EC_GLV_BETA_AT;
        // |a| < 2^128 in four words, shifted down one window at a time (no dynamically indexed register array); the
        // signed digit of the window (its 5 low bits + carry, in [-15, 16]); the last window ends with no carry
        uint32_t s1[4], s2[4];
        constexpr int SK = HALF ? EC_GLV_LO * EC_GLV_W : 0, SW = SK / 32, SB = SK % 32;   // HALF 1 resumes at window 13
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t l1 = q + SW < 4 ? a1.w[q + SW] : 0u, h1 = q + SW + 1 < 4 ? a1.w[q + SW + 1] : 0u;
            const uint32_t l2 = q + SW < 4 ? a2.w[q + SW] : 0u, h2 = q + SW + 1 < 4 ? a2.w[q + SW + 1] : 0u;
            s1[q] = SB ? __builtin_amdgcn_alignbit(h1, l1, SB) : l1;
            s2[q] = SB ? __builtin_amdgcn_alignbit(h2, l2, SB) : l2;
        }
        auto digit = [](uint32_t (&a)[4], int& cy) -> int {
            const int v = (int)(a[0] & 31u) + cy;
#pragma unroll
            for (int q = 0; q < 3; q++) a[q] = __builtin_amdgcn_alignbit(a[q + 1], a[q], EC_GLV_W);
            a[3] >>= EC_GLV_W;
            cy = (v + 15) >> 5;
            return v - (cy << 5);
        };
#pragma unroll 1
        for (uint32_t w = HALF ? EC_GLV_LO : 0u; w < (HALF ? EC_GLV_WIN : EC_GLV_LO); w++) {
            int d = digit(s1, cy1);
            if (n1) d = -d;
            if (d) {
                load_apt(ent, qt + (w * EC_GLV_ENT + (uint32_t)(d < 0 ? -d : d) - 1) * 16);
                add_digit_x<C>(acc, ent, d, exc);
            }
            d = digit(s2, cy2);
            if (n2) d = -d;
            if (d) {
                const uint32_t e = w * EC_GLV_ENT + (uint32_t)(d < 0 ? -d : d) - 1;
                load_u256(ent.x, bxt + e * 8);
                load_u256(ent.y, qt + e * 16 + 8);
                add_digit_x<C>(acc, ent, d, exc);
            }
        }
        if (exc) {
            mid[(uint64_t)40 * cap + gid] = 2u;
            return;
        }
        if (HALF == 0) {
            mid_store(mid, cap, gid, 0, acc.X);
            mid_store(mid, cap, gid, 8, acc.Y);
            mid_store(mid, cap, gid, 16, acc.Z);
            u256 h;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                h.w[q] = a1.w[q];
                h.w[4 + q] = a2.w[q];
            }
            mid_store(mid, cap, gid, 24, h);
            mid[(uint64_t)41 * cap + gid] = (n1 ? 1u : 0u) | (n2 ? 2u : 0u) | ((uint32_t)cy1 << 2) | ((uint32_t)cy2 << 3);
            return;
        }
        status[i] = ecdsa_check<C>(acc, r) ? CHIP_VALID : CHIP_INVALID;
        return;
    }
    uint32_t dq[8];
    const uint32_t cq = recode<4>(dq, u2);
#pragma unroll 1
    for (int wd = HALF * 4; wd < HALF * 4 + 4; wd++) {
        const uint32_t cur = dq[wd];
#pragma unroll 1
        for (int q = 0; q < 8; q++) {
            const int d = (int)((cur >> (4 * q)) & 15u) - 8;
            if (!d) continue;
            const uint32_t w = (uint32_t)(wd * 8 + q);
            load_apt(ent, qt + (w * EC_COMB_QENT + (uint32_t)(d < 0 ? -d : d) - 1) * 16);
            add_digit_x<C>(acc, ent, d, exc);
        }
    }
    if (HALF == 0) {
        if (exc) {
            mid[(uint64_t)40 * cap + gid] = 2u;
            return;
        }
        mid_store(mid, cap, gid, 0, acc.X);
        mid_store(mid, cap, gid, 8, acc.Y);
        mid_store(mid, cap, gid, 16, acc.Z);
        return;
    }
    if (cq) {
        load_apt(ent, qt + (64u * EC_COMB_QENT) * 16);
        add_digit_x<C>(acc, ent, 1, exc);
    }
    if (exc) {
        mid[(uint64_t)40 * cap + gid] = 2u;
        return;
    }
    status[i] = ecdsa_check<C>(acc, r) ? CHIP_VALID : CHIP_INVALID;
}
// both curves in one grid, as k_ecdsa_comb_g.  EC_Q0_WAVES: waves per SIMD HALF 0's registers must leave room for.
// Left to itself the compiler gives HALF 0 194 VGPRs (2 waves) against HALF 1's 156 (3 waves), and HALF 0 issued at
// 5.05 cycles per VALU instruction against 4.04 (profiles/r05/cfg3_pmc_sq.csv); capped at 3 waves (168 VGPRs, 36
// spilled) it runs 1.72-1.79 -> 1.44 ms, cfg3 83.8-84.2 -> 88.1-88.7M (profiles/r05/ab_r05j.txt)
#ifndef EC_Q0_WAVES
#define EC_Q0_WAVES 3
#endif
#ifndef EC_Q1_WAVES
#define EC_Q1_WAVES 3   // HALF 1 with the GLV windows of secp256k1 compiles to 170 VGPRs: held to 3 waves per SIMD
#endif
template <int HALF>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HALF == 0 ? EC_Q0_WAVES : EC_Q1_WAVES)))
k_ecdsa_comb_q(const uint32_t* __restrict__ list_r1,
                                                      const uint32_t* __restrict__ list_k1,
                                                      const uint32_t* __restrict__ counts,
                                                      const uint32_t* __restrict__ key_idx,
                                                      const uint32_t* __restrict__ ctab,
                                                      uint32_t* __restrict__ mid_r1,
                                                      uint32_t* __restrict__ mid_k1, uint64_t cap,
                                                      uint8_t* __restrict__ status, uint32_t half, uint32_t glv) {
    if (blockIdx.x < half)
        comb_q_body<CURVE_R1, HALF>(blockIdx.x, list_r1, counts + LIST_R1, key_idx, ctab, mid_r1, cap, status, glv);
    else
        comb_q_body<CURVE_K1, HALF>(blockIdx.x - half, list_k1, counts + LIST_K1, key_idx, ctab, mid_k1, cap, status,
                                    glv);
}

// E.  Lanes parked by an exceptional addition (mid state 2) verified again from their bytes with complete
// additions: e, s^-1, u1, u2, then u1 G + u2 Q by one double-and-add over both scalars (Shamir).  Runs for
// every batch; for honest inputs no lane is parked and every wave exits at its first load.
template <int C>
CHIP_DEV void comb_retry_body(uint32_t blk, const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                              const chip_sig_batch_dev& b, const uint32_t* __restrict__ ectab,
                              const uint32_t* __restrict__ mid, uint64_t cap, uint8_t* __restrict__ status) {
    const uint32_t gid = blk * blockDim.x + threadIdx.x;
    if (gid >= *count || mid[(uint64_t)40 * cap + gid] != 2u) return;
    const ec_curve_c& cv = curve<C>();
    const uint32_t i = list[gid];
    const uint32_t mi = b.msg_idx[i];
    u256 r, s, e;
    const uint32_t st0 = ecdsa_front<C>(r, s, e, b.sig_data + b.sig_off[i], b.sig_len[i], b.msg_data + b.msg_off[mi],
                                        b.msg_len[mi]);
    if (st0 != 0xffu) {
        status[i] = (uint8_t)st0;
        return;
    }
    u256 r2n, sm, inv, u1, u2;
    u256_from_c(r2n, cv.r2_n);
    mn_mul<C>(sm, s, r2n);
    mn_inv<C>(inv, sm);   // s^-1 R
    mn_mul<C>(u1, e, inv);
    mn_mul<C>(u2, r, inv);
    const ec_aff_c& g = (EC_CURVE(C) == CURVE_R1) ? EC_R1_G_TABLE[1] : EC_K1_G_TABLE[1];
    apt G, Q;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        G.x.w[k] = g.x[k];
        G.y.w[k] = g.y[k];
    }
    load_apt(Q, ectab + (uint64_t)b.key_idx[i] * EC_TAB_STRIDE + 16);
    jpt acc;
    jpt_inf(acc);
#pragma unroll 1
    for (int bit = 255; bit >= 0; bit--) {
        if (!u256_is_zero(acc.Z)) jdbl<C>(acc, acc);
        if ((u1.w[bit >> 5] >> (bit & 31)) & 1u) jmadd_full<C>(acc, acc, G);
        if ((u2.w[bit >> 5] >> (bit & 31)) & 1u) jmadd_full<C>(acc, acc, Q);
    }
    status[i] = ecdsa_check<C>(acc, r) ? CHIP_VALID : CHIP_INVALID;
}
__global__ void __launch_bounds__(256) k_ecdsa_comb_retry(const uint32_t* __restrict__ list_r1,
                                                          const uint32_t* __restrict__ list_k1,
                                                          const uint32_t* __restrict__ counts, chip_sig_batch_dev b,
                                                          const uint32_t* __restrict__ ectab,
                                                          const uint32_t* __restrict__ mid_r1,
                                                          const uint32_t* __restrict__ mid_k1, uint64_t cap,
                                                          uint8_t* __restrict__ status, uint32_t half) {
    if (blockIdx.x < half) comb_retry_body<CURVE_R1>(blockIdx.x, list_r1, counts + LIST_R1, b, ectab, mid_r1, cap, status);
    else comb_retry_body<CURVE_K1>(blockIdx.x - half, list_k1, counts + LIST_K1, b, ectab, mid_k1, cap, status);
}

uint64_t ecdsa_comb_key_words() { return EC_COMB_KEY_WORDS + EC_COMB_JAC_WORDS; }

// CHIP_EC_GLV=0: secp256k1 through the full 65-window table like P-256 (round 5)
static uint32_t ec_glv() {
    static const uint32_t on = [] {
        const char* e = getenv("CHIP_EC_GLV");
        return e ? (uint32_t)(e[0] != '0') : 1u;
    }();
    return on;
}
// table halves: windows [0, EC_LO_WIN) and [EC_LO_WIN, 65); fill groups cover EC_FILL_GROUP windows each
#define EC_LO_WIN 32
void launch_ecdsa_comb_chain(hipStream_t st, uint64_t n_keys, const KeyMeta* meta, const uint32_t* ectab,
                             uint32_t* ctab, int half, const uint32_t* skip) {
    if (!n_keys) return;
    uint32_t* jac = ctab + n_keys * EC_COMB_KEY_WORDS;
    static const uint32_t prio = [] {
        const char* e = getenv("CHIP_CHAIN_PRIO");
        return e ? (uint32_t)(e[0] != '0') : 1u;
    }();
    const uint32_t wa = half ? EC_LO_WIN : 0, wb = half ? EC_COMB_QWIN : EC_LO_WIN;
    static const bool pair = [] {
        const char* e = getenv("CHIP_EC_CHAIN_PAIR");
        return e ? e[0] != '0' : EC_CHAIN_PAIR != 0;
    }();
    if (pair)
        hipLaunchKernelGGL(k_ecdsa_comb_chain2, dim3((uint32_t)((2 * n_keys + 63) / 64)), dim3(64), 0, st, n_keys, meta,
                           ectab, jac, prio, wa, wb, skip, ec_glv());
    else
        hipLaunchKernelGGL(k_ecdsa_comb_chain, dim3((uint32_t)((n_keys + 63) / 64)), dim3(64), 0, st, n_keys, meta,
                           ectab, jac, prio, wa, wb, skip, ec_glv());
}
void launch_ecdsa_comb_fill(hipStream_t st, uint64_t n_keys, const KeyMeta* meta, uint32_t* ctab, int half,
                            const uint32_t* skip) {
    if (!n_keys) return;
    uint32_t* jac = ctab + n_keys * EC_COMB_KEY_WORDS;
    static const uint32_t gw = [] {
        const char* e = getenv("CHIP_EC_FILL_GROUP");
        const uint32_t v = e ? (uint32_t)strtoul(e, nullptr, 10) : EC_FILL_GROUP;
        return v ? v : 1u;
    }();
    const uint32_t wa = half ? EC_LO_WIN : 0, wb = half ? EC_COMB_QWIN : EC_LO_WIN;
    const uint32_t kw = half ? EC_GLV_WIN - EC_GLV_LO : EC_GLV_LO;   // a secp256k1 GLV table's windows in this half
    const uint32_t ng = std::max((wb - wa + gw - 1) / gw, ec_glv() ? (kw + EC_GLV_FILL_GROUP - 1) / EC_GLV_FILL_GROUP : 0u);
    hipLaunchKernelGGL(k_ecdsa_comb_fill, dim3((uint32_t)((n_keys * ng + 255) / 256)), dim3(256), 0, st, n_keys, meta,
                       ctab, jac, wa, wb, gw, ng, skip, ec_glv());
}

// words of the hand-off area per list position, and of the wave products per list
uint64_t ecdsa_comb_mid_words() { return EC_MID_WORDS; }
uint64_t ecdsa_comb_wp_words(uint64_t n) { return ((n + 63) / 64) * 8; }

void launch_ecdsa_group(hipStream_t st, uint64_t n, uint64_t n_keys, const KeyMeta* meta, const uint32_t* key_count,
                        uint32_t* key_base, const uint32_t* key_rank, uint32_t* ctr, const uint32_t* lists,
                        const uint32_t* counts, const uint32_t* key_idx, uint32_t* grouped) {
    if (!n || !n_keys) return;
    hipLaunchKernelGGL(k_ec_group_base, dim3((uint32_t)((n_keys + 255) / 256)), dim3(256), 0, st, n_keys, meta, key_count,
                       key_base, ctr);
    hipLaunchKernelGGL(k_ec_group_scatter, dim3((uint32_t)((2 * n + 255) / 256)), dim3(256), 0, st, n, lists, counts,
                       key_idx, key_base, key_rank, grouped);
}

template <int C>
static void comb_sig(hipStream_t st, uint64_t n, const uint32_t* list, const uint32_t* count, const chip_sig_batch* b,
                     uint32_t* mid, uint32_t* wp, uint8_t* status) {
    hipLaunchKernelGGL(k_ecdsa_comb_pre<C>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, list, count, b->msg_idx,
                       b->sig_data, b->sig_off, b->sig_len, b->msg_data, b->msg_off, b->msg_len, mid, wp, (uint64_t)n,
                       status);
}
void launch_ecdsa_comb_pre(hipStream_t st, int scheme, uint64_t n, const uint32_t* list, const uint32_t* count,
                           const chip_sig_batch* b, uint32_t* mid, uint32_t* wp, uint8_t* status) {
    if (!n) return;
    if (scheme == CHIP_SCHEME_R1) comb_sig<CURVE_R1>(st, n, list, count, b, mid, wp, status);
    else comb_sig<CURVE_K1>(st, n, list, count, b, mid, wp, status);
}
void launch_ecdsa_comb_inv(hipStream_t st, uint64_t n, const uint32_t* counts, uint32_t* wp_r1, uint32_t* wp_k1) {
    if (!n) return;
    const uint32_t nw = (uint32_t)((n + 63) / 64);
    hipLaunchKernelGGL(k_ecdsa_comb_inv, dim3((2 * nw + 63) / 64), dim3(64), 0, st, counts, wp_r1, wp_k1, nw);
}
void launch_ecdsa_comb_g(hipStream_t st, uint64_t n, const uint32_t* counts, const uint32_t* gcomb, uint32_t* mid_r1,
                         uint32_t* mid_k1, const uint32_t* wp_r1, const uint32_t* wp_k1, bool park_all) {
    if (!n) return;
    const uint32_t half = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(k_ecdsa_comb_g, dim3(2 * half), dim3(256), 0, st, counts, gcomb, mid_r1, mid_k1, wp_r1, wp_k1,
                       (uint64_t)n, half, park_all ? 1u : 0u);
}
void launch_ecdsa_comb_retry(hipStream_t st, uint64_t n, const uint32_t* list_r1, const uint32_t* list_k1,
                             const uint32_t* counts, const chip_sig_batch* b, const uint32_t* ectab,
                             const uint32_t* mid_r1, const uint32_t* mid_k1, uint8_t* status) {
    if (!n) return;
    const uint32_t half = (uint32_t)((n + 255) / 256);
    chip_sig_batch_dev d{b->key_idx, b->msg_idx, b->sig_data, b->sig_off, b->sig_len, b->msg_data, b->msg_off, b->msg_len};
    hipLaunchKernelGGL(k_ecdsa_comb_retry, dim3(2 * half), dim3(256), 0, st, list_r1, list_k1, counts, d, ectab, mid_r1,
                       mid_k1, (uint64_t)n, status, half);
}
void launch_ecdsa_comb_q(hipStream_t st, uint64_t n, const uint32_t* list_r1, const uint32_t* list_k1,
                         const uint32_t* counts, const chip_sig_batch* b, const uint32_t* ctab, uint32_t* mid_r1,
                         uint32_t* mid_k1, uint8_t* status, int table_half) {
    if (!n) return;
    const uint32_t half = (uint32_t)((n + 255) / 256);
    if (table_half)
        hipLaunchKernelGGL(k_ecdsa_comb_q<1>, dim3(2 * half), dim3(256), 0, st, list_r1, list_k1, counts, b->key_idx, ctab,
                           mid_r1, mid_k1, (uint64_t)n, status, half, ec_glv());
    else
        hipLaunchKernelGGL(k_ecdsa_comb_q<0>, dim3(2 * half), dim3(256), 0, st, list_r1, list_k1, counts, b->key_idx, ctab,
                           mid_r1, mid_k1, (uint64_t)n, status, half, ec_glv());
}
