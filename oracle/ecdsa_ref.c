/* oracle/ecdsa_ref.c — CPU restatement of SHA256withECDSA verification with the semantics of
 * org.bouncycastle:bcprov-jdk15on:1.57 as selected by Crypto.isValid (Crypto.kt:615-625) for
 * ECDSA_SECP256K1_SHA256 (id 2, Crypto.kt:84-96) and ECDSA_SECP256R1_SHA256 (id 3, :99-111).
 * TEST INFRASTRUCTURE (see oracle.h).  The jar is not vendored; restated from BC 1.57's
 * published DSABase.engineVerify / StdDSAEncoder.decode / ECDSASigner.verifySignature
 * (SURVEY.md §8a "ECDSA contract"):
 *   - DER: exactly one SEQUENCE of exactly two INTEGERs, definite minimal lengths, DER
 *     re-encoding must equal the input (so no trailing bytes, no long-form short lengths);
 *     an INTEGER whose content is malformed in ASN1Integer's sense (a redundant leading 00 or FF
 *     byte) or empty -> exception.  Any failure -> SignatureException (SIG_DECODE).
 *     (The malformed-INTEGER rule is restated from BC's ASN1Integer.isMalformed; no reference test
 *     pins it — parity unpinned for that one case.)
 *   - e = SHA-256(M) as a big-endian integer (n is 256 bits: no truncation).
 *   - r or s outside [1, n-1] -> false.  w = s^-1, u1 = e w, u2 = r w (mod n),
 *     R = u1 G + u2 Q; R = infinity -> false; accept iff x(R) mod n == r.  High-s is valid.
 * Arithmetic: 4 x 64-bit limbs, Montgomery multiplication with 128-bit products. */
#include "oracle_int.h"
#include <string.h>

typedef struct { uint64_t w[4]; } u256;

typedef struct {
    u256 m;        /* modulus            */
    uint64_t minv; /* -m^-1 mod 2^64     */
    u256 r2;       /* R^2 mod m          */
    u256 one;      /* R mod m            */
} mont;

typedef struct {
    mont fp, fn;
    u256 a_m, b_m;   /* curve a, b in Montgomery form (fp) */
    int a_is_m3;     /* unused by the generic formulas; documentation */
    u256 gx, gy;     /* affine generator, plain */
} curve;

static curve C_R1, C_K1;
static int ec_ready = 0;

static int hexval(char c) { return c <= '9' ? c - '0' : (c | 32) - 'a' + 10; }
static void u256_from_hex(u256* r, const char* h) {
    memset(r, 0, sizeof *r);
    int n = 0;
    for (const char* p = h; *p; p++) {
        if (*p == ' ') continue;
        n++;
    }
    int bit = 0;
    for (int i = (int)strlen(h) - 1; i >= 0; i--) {
        if (h[i] == ' ') continue;
        uint64_t v = (uint64_t)hexval(h[i]);
        r->w[bit / 64] |= v << (bit % 64);
        bit += 4;
    }
    (void)n;
}
static void u256_from_be(u256* r, const uint8_t b[32]) {
    for (int i = 0; i < 4; i++) {
        uint64_t x = 0;
        for (int j = 0; j < 8; j++) x = (x << 8) | b[(3 - i) * 8 + j];
        r->w[i] = x;
    }
}
static void u256_to_be(uint8_t b[32], const u256* r) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) b[(3 - i) * 8 + j] = (uint8_t)(r->w[i] >> (56 - 8 * j));
}
static int u256_cmp(const u256* a, const u256* b) {
    for (int i = 3; i >= 0; i--) {
        if (a->w[i] != b->w[i]) return a->w[i] > b->w[i] ? 1 : -1;
    }
    return 0;
}
static int u256_iszero(const u256* a) { return !(a->w[0] | a->w[1] | a->w[2] | a->w[3]); }
static uint64_t u256_add(u256* r, const u256* a, const u256* b) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
        c += (u128)a->w[i] + b->w[i];
        r->w[i] = (uint64_t)c;
        c >>= 64;
    }
    return (uint64_t)c;
}
static uint64_t u256_sub(u256* r, const u256* a, const u256* b) {
    uint64_t bw = 0;
    for (int i = 0; i < 4; i++) {
        u128 d = (u128)a->w[i] - b->w[i] - bw;
        r->w[i] = (uint64_t)d;
        bw = (uint64_t)(d >> 64) & 1;
    }
    return bw;
}
/* modular add/sub for values < m */
static void mod_add(const mont* M, u256* r, const u256* a, const u256* b) {
    u256 t;
    uint64_t c = u256_add(&t, a, b);
    u256 s;
    uint64_t bw = u256_sub(&s, &t, &M->m);
    if (c || !bw) *r = s; else *r = t;
}
static void mod_sub(const mont* M, u256* r, const u256* a, const u256* b) {
    u256 t;
    uint64_t bw = u256_sub(&t, a, b);
    if (bw) u256_add(&t, &t, &M->m);
    *r = t;
}
/* Montgomery product a*b*R^-1 mod m (CIOS) */
static void mont_mul(const mont* M, u256* r, const u256* a, const u256* b) {
    uint64_t t[6] = {0};
    for (int i = 0; i < 4; i++) {
        u128 c = 0;
        for (int j = 0; j < 4; j++) {
            c += (u128)a->w[j] * b->w[i] + t[j];
            t[j] = (uint64_t)c;
            c >>= 64;
        }
        u128 s = (u128)t[4] + (uint64_t)c;
        t[4] = (uint64_t)s;
        t[5] = (uint64_t)(s >> 64);
        uint64_t q = t[0] * M->minv;
        c = (u128)q * M->m.w[0] + t[0];
        c >>= 64;
        for (int j = 1; j < 4; j++) {
            c += (u128)q * M->m.w[j] + t[j];
            t[j - 1] = (uint64_t)c;
            c >>= 64;
        }
        s = (u128)t[4] + (uint64_t)c;
        t[3] = (uint64_t)s;
        t[4] = t[5] + (uint64_t)(s >> 64);
    }
    u256 res = {{t[0], t[1], t[2], t[3]}}, s2;
    uint64_t bw = u256_sub(&s2, &res, &M->m);
    if (t[4] || !bw) res = s2;
    *r = res;
}
static void mont_init(mont* M, const char* hex) {
    u256_from_hex(&M->m, hex);
    /* minv = -m^-1 mod 2^64 by Newton iteration */
    uint64_t x = 1;
    for (int i = 0; i < 7; i++) x *= 2 - M->m.w[0] * x;
    M->minv = (uint64_t)0 - x;
    /* one = 2^256 mod m, computed as (2^256 - m) mod m since m > 2^255 */
    u256 z = {{0, 0, 0, 0}};
    u256_sub(&M->one, &z, &M->m);
    /* r2 = one * 2^256 mod m by 256 doublings */
    u256 t = M->one;
    for (int i = 0; i < 256; i++) mod_add(M, &t, &t, &t);
    M->r2 = t;
}
static void to_mont(const mont* M, u256* r, const u256* a) { mont_mul(M, r, a, &M->r2); }
static void from_mont(const mont* M, u256* r, const u256* a) {
    u256 one = {{1, 0, 0, 0}};
    mont_mul(M, r, a, &one);
}
/* a^e for e = m - 2 (Fermat inverse), a in Montgomery form */
static void mont_inv(const mont* M, u256* r, const u256* a) {
    u256 e, two = {{2, 0, 0, 0}};
    u256_sub(&e, &M->m, &two);
    u256 acc = M->one;
    for (int i = 255; i >= 0; i--) {
        mont_mul(M, &acc, &acc, &acc);
        if ((e.w[i / 64] >> (i % 64)) & 1) mont_mul(M, &acc, &acc, a);
    }
    *r = acc;
}

static void curve_init(curve* c, const char* p, const char* n, const char* a, const char* b,
                       const char* gx, const char* gy) {
    mont_init(&c->fp, p);
    mont_init(&c->fn, n);
    u256 t;
    u256_from_hex(&t, a); to_mont(&c->fp, &c->a_m, &t);
    u256_from_hex(&t, b); to_mont(&c->fp, &c->b_m, &t);
    u256_from_hex(&c->gx, gx);
    u256_from_hex(&c->gy, gy);
}
static void ec_init(void) {
    if (ec_ready) return;
    curve_init(&C_R1, "FFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF",
               "FFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551",
               "FFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFC",
               "5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B",
               "6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296",
               "4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5");
    curve_init(&C_K1, "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F",
               "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141",
               "0", "7",
               "79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798",
               "483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8");
    ec_ready = 1;
}
void orc_ec_init(void) { ec_init(); }
static const curve* curve_of(int scheme) { return scheme == ORC_SCHEME_R1 ? &C_R1 : &C_K1; }

/* Jacobian point, coordinates in Montgomery form; Z == 0 <=> infinity */
typedef struct { u256 X, Y, Z; } jpt;

static void jdbl(const curve* c, jpt* r, const jpt* p) {
    const mont* F = &c->fp;
    if (u256_iszero(&p->Z)) { *r = *p; return; }
    u256 XX, YY, YYYY, ZZ, S, M, T, t, u;
    mont_mul(F, &XX, &p->X, &p->X);
    mont_mul(F, &YY, &p->Y, &p->Y);
    mont_mul(F, &YYYY, &YY, &YY);
    mont_mul(F, &ZZ, &p->Z, &p->Z);
    mod_add(F, &t, &p->X, &YY); mont_mul(F, &t, &t, &t); mod_sub(F, &t, &t, &XX); mod_sub(F, &t, &t, &YYYY);
    mod_add(F, &S, &t, &t);
    mod_add(F, &M, &XX, &XX); mod_add(F, &M, &M, &XX);
    mont_mul(F, &u, &ZZ, &ZZ); mont_mul(F, &u, &u, &c->a_m); mod_add(F, &M, &M, &u);
    mont_mul(F, &T, &M, &M); mod_sub(F, &T, &T, &S); mod_sub(F, &T, &T, &S);
    jpt q;
    q.X = T;
    mod_add(F, &t, &p->Y, &p->Z); mont_mul(F, &t, &t, &t); mod_sub(F, &t, &t, &YY); mod_sub(F, &q.Z, &t, &ZZ);
    mod_sub(F, &t, &S, &T); mont_mul(F, &t, &M, &t);
    u = YYYY; mod_add(F, &u, &u, &u); mod_add(F, &u, &u, &u); mod_add(F, &u, &u, &u);
    mod_sub(F, &q.Y, &t, &u);
    *r = q;
}
static void jadd(const curve* c, jpt* r, const jpt* p, const jpt* q) {
    const mont* F = &c->fp;
    if (u256_iszero(&p->Z)) { *r = *q; return; }
    if (u256_iszero(&q->Z)) { *r = *p; return; }
    u256 Z1Z1, Z2Z2, U1, U2, S1, S2, H, R, I, J, V, t;
    mont_mul(F, &Z1Z1, &p->Z, &p->Z);
    mont_mul(F, &Z2Z2, &q->Z, &q->Z);
    mont_mul(F, &U1, &p->X, &Z2Z2);
    mont_mul(F, &U2, &q->X, &Z1Z1);
    mont_mul(F, &S1, &p->Y, &q->Z); mont_mul(F, &S1, &S1, &Z2Z2);
    mont_mul(F, &S2, &q->Y, &p->Z); mont_mul(F, &S2, &S2, &Z1Z1);
    mod_sub(F, &H, &U2, &U1);
    mod_sub(F, &R, &S2, &S1);
    if (u256_iszero(&H)) {
        if (u256_iszero(&R)) { jdbl(c, r, p); return; }
        memset(r, 0, sizeof *r);   /* P + (-P) = infinity */
        return;
    }
    mod_add(F, &R, &R, &R);
    mod_add(F, &I, &H, &H); mont_mul(F, &I, &I, &I);
    mont_mul(F, &J, &H, &I);
    mont_mul(F, &V, &U1, &I);
    jpt o;
    mont_mul(F, &o.X, &R, &R); mod_sub(F, &o.X, &o.X, &J); mod_sub(F, &o.X, &o.X, &V); mod_sub(F, &o.X, &o.X, &V);
    mod_sub(F, &t, &V, &o.X); mont_mul(F, &o.Y, &R, &t);
    mont_mul(F, &t, &S1, &J); mod_add(F, &t, &t, &t); mod_sub(F, &o.Y, &o.Y, &t);
    mod_add(F, &t, &p->Z, &q->Z); mont_mul(F, &t, &t, &t); mod_sub(F, &t, &t, &Z1Z1); mod_sub(F, &t, &t, &Z2Z2);
    mont_mul(F, &o.Z, &t, &H);
    *r = o;
}

/* BC decodePoint: 04||X||Y or 02/03||X; coordinates must be < p; point must satisfy the curve
 * equation (ECPoint.isValid).  Writes plain big-endian X||Y. */
int orc_ecdsa_decode_key(int scheme, const uint8_t* pt, size_t len, uint8_t xy[64]) {
    ec_init();
    const curve* c = curve_of(scheme);
    const mont* F = &c->fp;
    u256 x, y, xm, ym, lhs, rhs, t;
    if (len == 65 && pt[0] == 0x04) {
        u256_from_be(&x, pt + 1);
        u256_from_be(&y, pt + 33);
        if (u256_cmp(&x, &F->m) >= 0 || u256_cmp(&y, &F->m) >= 0) return -1;
        to_mont(F, &xm, &x); to_mont(F, &ym, &y);
    } else if (len == 33 && (pt[0] == 0x02 || pt[0] == 0x03)) {
        u256_from_be(&x, pt + 1);
        if (u256_cmp(&x, &F->m) >= 0) return -1;
        to_mont(F, &xm, &x);
        /* y = sqrt(x^3 + a x + b) = rhs^((p+1)/4) (p = 3 mod 4 for both curves) */
        mont_mul(F, &rhs, &xm, &xm); mont_mul(F, &rhs, &rhs, &xm);
        mont_mul(F, &t, &c->a_m, &xm); mod_add(F, &rhs, &rhs, &t); mod_add(F, &rhs, &rhs, &c->b_m);
        u256 e, one = {{1, 0, 0, 0}};
        u256_add(&e, &F->m, &one);
        for (int i = 0; i < 2; i++) { /* e >>= 1 twice */
            e.w[0] = (e.w[0] >> 1) | (e.w[1] << 63); e.w[1] = (e.w[1] >> 1) | (e.w[2] << 63);
            e.w[2] = (e.w[2] >> 1) | (e.w[3] << 63); e.w[3] >>= 1;
        }
        u256 acc = F->one;
        for (int i = 255; i >= 0; i--) {
            mont_mul(F, &acc, &acc, &acc);
            if ((e.w[i / 64] >> (i % 64)) & 1) mont_mul(F, &acc, &acc, &rhs);
        }
        ym = acc;
        from_mont(F, &y, &ym);
        if ((int)(y.w[0] & 1) != (pt[0] & 1)) {
            u256 z = {{0, 0, 0, 0}};
            mod_sub(F, &ym, &z, &ym);
            from_mont(F, &y, &ym);
        }
    } else {
        return -1;
    }
    /* on-curve: y^2 == x^3 + a x + b */
    mont_mul(F, &lhs, &ym, &ym);
    mont_mul(F, &rhs, &xm, &xm); mont_mul(F, &rhs, &rhs, &xm);
    mont_mul(F, &t, &c->a_m, &xm); mod_add(F, &rhs, &rhs, &t); mod_add(F, &rhs, &rhs, &c->b_m);
    if (u256_cmp(&lhs, &rhs) != 0) return -1;
    u256_to_be(xy, &x);
    u256_to_be(xy + 32, &y);
    return 0;
}

/* StdDSAEncoder.decode + DER re-encode equality (BC 1.57). */
static int der_len(const uint8_t* p, size_t avail, size_t* hdr, size_t* len) {
    if (avail < 1) return -1;
    uint8_t b = p[0];
    if (b < 0x80) { *hdr = 1; *len = b; return 0; }
    if (b == 0x80) return -1;                      /* indefinite: BER, re-encode differs */
    size_t nb = b & 0x7f;
    if (nb > 4 || nb + 1 > avail) return -1;
    if (p[1] == 0) return -1;                      /* non-minimal long form              */
    size_t L = 0;
    for (size_t i = 0; i < nb; i++) L = (L << 8) | p[1 + i];
    if (L < 0x80) return -1;                       /* long form for a short length       */
    *hdr = 1 + nb; *len = L;
    return 0;
}
/* two's-complement INTEGER content -> 32-byte magnitude; oor=1 if value <= 0 or >= 2^256 */
static void der_int_value(const uint8_t* c, size_t n, uint8_t out[32], int* oor) {
    memset(out, 0, 32);
    *oor = 0;
    if (c[0] & 0x80) { *oor = 1; return; }         /* negative                           */
    size_t i = 0;
    while (i < n && c[i] == 0) i++;
    if (i == n) { *oor = 1; return; }              /* zero                               */
    if (n - i > 32) { *oor = 1; return; }          /* >= 2^256                           */
    memcpy(out + 32 - (n - i), c + i, n - i);
}
int orc_der_decode(const uint8_t* sig, size_t len, uint8_t r[32], uint8_t s[32], int* r_oor, int* s_oor) {
    size_t hdr, L;
    if (len < 2 || sig[0] != 0x30) return -1;
    if (der_len(sig + 1, len - 1, &hdr, &L)) return -1;
    if (1 + hdr + L != len) return -1;             /* trailing or truncated              */
    const uint8_t* p = sig + 1 + hdr;
    size_t rem = L;
    const uint8_t* val[2];
    size_t vlen[2];
    for (int k = 0; k < 2; k++) {
        if (rem < 2 || p[0] != 0x02) return -1;
        size_t h2, l2;
        if (der_len(p + 1, rem - 1, &h2, &l2)) return -1;
        if (1 + h2 + l2 > rem) return -1;
        if (l2 == 0) return -1;                    /* BigInteger of zero length          */
        const uint8_t* c = p + 1 + h2;             /* ASN1Integer: malformed integer     */
        if (l2 > 1 && ((c[0] == 0x00 && !(c[1] & 0x80)) || (c[0] == 0xff && (c[1] & 0x80)))) return -1;
        val[k] = p + 1 + h2;
        vlen[k] = l2;
        p += 1 + h2 + l2;
        rem -= 1 + h2 + l2;
    }
    if (rem != 0) return -1;                       /* s.size() != 2                      */
    der_int_value(val[0], vlen[0], r, r_oor);
    der_int_value(val[1], vlen[1], s, s_oor);
    return 0;
}

int orc_ecdsa_verify(int scheme, const uint8_t xy[64], const uint8_t* sig, size_t siglen,
                     const uint8_t* msg, size_t msglen) {
    ec_init();
    const curve* c = curve_of(scheme);
    const mont* F = &c->fp;
    const mont* N = &c->fn;
    uint8_t rb[32], sb[32], eb[32];
    int roor, soor;
    if (orc_der_decode(sig, siglen, rb, sb, &roor, &soor)) return ORC_SIG_DECODE;
    orc_sha256(msg, msglen, eb);
    if (roor || soor) return ORC_INVALID;
    u256 r, s, e;
    u256_from_be(&r, rb);
    u256_from_be(&s, sb);
    u256_from_be(&e, eb);
    if (u256_cmp(&r, &N->m) >= 0 || u256_cmp(&s, &N->m) >= 0) return ORC_INVALID;
    if (u256_cmp(&e, &N->m) >= 0) u256_sub(&e, &e, &N->m);
    u256 sm, wm, em, rm, u1m, u2m, u1, u2;
    to_mont(N, &sm, &s);
    mont_inv(N, &wm, &sm);
    to_mont(N, &em, &e);
    to_mont(N, &rm, &r);
    mont_mul(N, &u1m, &em, &wm);
    mont_mul(N, &u2m, &rm, &wm);
    from_mont(N, &u1, &u1m);
    from_mont(N, &u2, &u2m);
    /* R = u1 G + u2 Q, Shamir double-and-add (exact group arithmetic) */
    jpt G, Q, GQ, R;
    to_mont(F, &G.X, &c->gx); to_mont(F, &G.Y, &c->gy); G.Z = F->one;
    u256 qx, qy;
    u256_from_be(&qx, xy); u256_from_be(&qy, xy + 32);
    to_mont(F, &Q.X, &qx); to_mont(F, &Q.Y, &qy); Q.Z = F->one;
    jadd(c, &GQ, &G, &Q);
    memset(&R, 0, sizeof R);
    for (int i = 255; i >= 0; i--) {
        jdbl(c, &R, &R);
        int b1 = (u1.w[i / 64] >> (i % 64)) & 1, b2 = (u2.w[i / 64] >> (i % 64)) & 1;
        if (b1 && b2) jadd(c, &R, &R, &GQ);
        else if (b1) jadd(c, &R, &R, &G);
        else if (b2) jadd(c, &R, &R, &Q);
    }
    if (u256_iszero(&R.Z)) return ORC_INVALID;
    u256 zi, zi2, xm, x;
    mont_inv(F, &zi, &R.Z);
    mont_mul(F, &zi2, &zi, &zi);
    mont_mul(F, &xm, &R.X, &zi2);
    from_mont(F, &x, &xm);
    if (u256_cmp(&x, &N->m) >= 0) u256_sub(&x, &x, &N->m);
    return u256_cmp(&x, &r) == 0 ? ORC_VALID : ORC_INVALID;
}

/* test helper: affine x||y (BE) of k*G */
int orc_ecdsa_scalarmult_base(int scheme, const uint8_t k[32], uint8_t xy[64]) {
    ec_init();
    const curve* c = curve_of(scheme);
    const mont* F = &c->fp;
    jpt G, R;
    to_mont(F, &G.X, &c->gx); to_mont(F, &G.Y, &c->gy); G.Z = F->one;
    memset(&R, 0, sizeof R);
    for (int i = 255; i >= 0; i--) {
        jdbl(c, &R, &R);
        if ((k[31 - i / 8] >> (i % 8)) & 1) jadd(c, &R, &R, &G);
    }
    if (u256_iszero(&R.Z)) return -1;
    u256 zi, zi2, zi3, t, x, y;
    mont_inv(F, &zi, &R.Z);
    mont_mul(F, &zi2, &zi, &zi);
    mont_mul(F, &zi3, &zi2, &zi);
    mont_mul(F, &t, &R.X, &zi2); from_mont(F, &x, &t);
    mont_mul(F, &t, &R.Y, &zi3); from_mont(F, &y, &t);
    u256_to_be(xy, &x);
    u256_to_be(xy + 32, &y);
    return 0;
}
