/* oracle/ed25519_ref.c — CPU restatement of Ed25519 verification with the semantics of
 * net.i2p.crypto:eddsa:0.2.0 EdDSAEngine as reached through Corda's X509EdDSAEngine
 * (core/.../internal/X509EdDSAEngine.kt:40) from Crypto.isValid (Crypto.kt:615-625).
 * TEST INFRASTRUCTURE (see oracle.h).  The jar is not vendored in /root/reference; this
 * follows its published algorithm (SURVEY.md §8a "Ed25519 contract"):
 *   - siglen != 64                -> SignatureException("signature length is wrong")
 *   - h = SHA-512(sig[0:32] || Abyte || M) reduced mod L   (Abyte = canonical re-encoding of A)
 *   - S = sig[32:64] as a little-endian integer, NOT range checked (S >= L accepted)
 *   - R' = h*(-A) + S*B computed by GroupElement.doubleScalarMultiplyVariableTime with the
 *     ref10 slide() signed-window recoding (carry out of digit 255 dropped)
 *   - accept iff canonical encode(R') == sig[0:32] bytewise
 *   - key decode GroupElement(curve, bytes): y read from 255 bits (y >= p tolerated),
 *     x = sqrt((y^2-1)/(d y^2+1)) else "not a valid point", sign fixed by bit 255 (x = 0 with
 *     the sign bit set tolerated). No small-order / subgroup check.
 * Field: radix 2^51, five 64-bit limbs with 128-bit products (a plain scalar restatement). */
#include "oracle_int.h"
#include <string.h>

typedef struct { uint64_t v[5]; } fe;
#define MASK51 ((1ull << 51) - 1)

static void fe_0(fe* h) { memset(h, 0, sizeof *h); }
static void fe_1(fe* h) { fe_0(h); h->v[0] = 1; }
static void fe_copy(fe* h, const fe* f) { *h = *f; }

static void fe_carry(fe* h) {
    uint64_t c;
    for (int k = 0; k < 2; k++) {
        c = h->v[0] >> 51; h->v[0] &= MASK51; h->v[1] += c;
        c = h->v[1] >> 51; h->v[1] &= MASK51; h->v[2] += c;
        c = h->v[2] >> 51; h->v[2] &= MASK51; h->v[3] += c;
        c = h->v[3] >> 51; h->v[3] &= MASK51; h->v[4] += c;
        c = h->v[4] >> 51; h->v[4] &= MASK51; h->v[0] += 19 * c;
    }
}
static void fe_add(fe* h, const fe* f, const fe* g) {
    for (int i = 0; i < 5; i++) h->v[i] = f->v[i] + g->v[i];
    fe_carry(h);
}
/* h = f - g + 4p (keeps limbs positive for reduced-ish inputs) */
static void fe_sub(fe* h, const fe* f, const fe* g) {
    static const uint64_t P4[5] = {0x1fffffffffffb4ull, 0x1ffffffffffffcull, 0x1ffffffffffffcull,
                                   0x1ffffffffffffcull, 0x1ffffffffffffcull};
    for (int i = 0; i < 5; i++) h->v[i] = f->v[i] + P4[i] - g->v[i];
    fe_carry(h);
}
static void fe_neg(fe* h, const fe* f) { fe z; fe_0(&z); fe_sub(h, &z, f); }
static void fe_mul(fe* h, const fe* f, const fe* g) {
    const uint64_t *a = f->v, *b = g->v;
    u128 t[5];
    uint64_t b19[5];
    for (int i = 0; i < 5; i++) b19[i] = 19 * b[i];
    t[0] = (u128)a[0] * b[0] + (u128)a[1] * b19[4] + (u128)a[2] * b19[3] + (u128)a[3] * b19[2] + (u128)a[4] * b19[1];
    t[1] = (u128)a[0] * b[1] + (u128)a[1] * b[0] + (u128)a[2] * b19[4] + (u128)a[3] * b19[3] + (u128)a[4] * b19[2];
    t[2] = (u128)a[0] * b[2] + (u128)a[1] * b[1] + (u128)a[2] * b[0] + (u128)a[3] * b19[4] + (u128)a[4] * b19[3];
    t[3] = (u128)a[0] * b[3] + (u128)a[1] * b[2] + (u128)a[2] * b[1] + (u128)a[3] * b[0] + (u128)a[4] * b19[4];
    t[4] = (u128)a[0] * b[4] + (u128)a[1] * b[3] + (u128)a[2] * b[2] + (u128)a[3] * b[1] + (u128)a[4] * b[0];
    uint64_t r[5];
    u128 c = 0;
    for (int i = 0; i < 5; i++) {
        t[i] += c;
        r[i] = (uint64_t)t[i] & MASK51;
        c = t[i] >> 51;
    }
    u128 x = (u128)c * 19 + r[0];
    r[0] = (uint64_t)x & MASK51;
    r[1] += (uint64_t)(x >> 51);
    for (int i = 0; i < 5; i++) h->v[i] = r[i];
    fe_carry(h);
}
static void fe_sq(fe* h, const fe* f) { fe_mul(h, f, f); }

/* ref10-style fe_frombytes: low 255 bits, value may be >= p (i2p Ed25519LittleEndianEncoding.decode) */
static void fe_frombytes(fe* h, const uint8_t s[32]) {
    uint64_t w[4];
    for (int i = 0; i < 4; i++) {
        uint64_t x = 0;
        for (int j = 7; j >= 0; j--) x = (x << 8) | s[8 * i + j];
        w[i] = x;
    }
    w[3] &= 0x7fffffffffffffffull;
    h->v[0] = w[0] & MASK51;
    h->v[1] = ((w[0] >> 51) | (w[1] << 13)) & MASK51;
    h->v[2] = ((w[1] >> 38) | (w[2] << 26)) & MASK51;
    h->v[3] = ((w[2] >> 25) | (w[3] << 39)) & MASK51;
    h->v[4] = (w[3] >> 12) & MASK51;
}
/* canonical little-endian encoding (fully reduced mod p) */
static void fe_tobytes(uint8_t s[32], const fe* f) {
    fe t = *f;
    fe_carry(&t);
    /* now t < 2^255 + small; subtract p if t >= p */
    uint64_t q = (t.v[0] + 19) >> 51;
    q = (t.v[1] + q) >> 51;
    q = (t.v[2] + q) >> 51;
    q = (t.v[3] + q) >> 51;
    q = (t.v[4] + q) >> 51;
    t.v[0] += 19 * q;
    uint64_t c;
    c = t.v[0] >> 51; t.v[0] &= MASK51; t.v[1] += c;
    c = t.v[1] >> 51; t.v[1] &= MASK51; t.v[2] += c;
    c = t.v[2] >> 51; t.v[2] &= MASK51; t.v[3] += c;
    c = t.v[3] >> 51; t.v[3] &= MASK51; t.v[4] += c;
    t.v[4] &= MASK51;
    uint64_t w[4];
    w[0] = t.v[0] | (t.v[1] << 51);
    w[1] = (t.v[1] >> 13) | (t.v[2] << 38);
    w[2] = (t.v[2] >> 26) | (t.v[3] << 25);
    w[3] = (t.v[3] >> 39) | (t.v[4] << 12);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}
static int fe_isnonzero(const fe* f) {
    uint8_t s[32];
    fe_tobytes(s, f);
    uint8_t r = 0;
    for (int i = 0; i < 32; i++) r |= s[i];
    return r != 0;
}
static int fe_isnegative(const fe* f) {
    uint8_t s[32];
    fe_tobytes(s, f);
    return s[0] & 1;
}
/* h = f^e for a 256-bit little-endian exponent (square-and-multiply, oracle only) */
static void fe_pow(fe* h, const fe* f, const uint8_t e[32]) {
    fe r, b = *f;
    fe_1(&r);
    for (int i = 255; i >= 0; i--) {
        fe_sq(&r, &r);
        if ((e[i >> 3] >> (i & 7)) & 1) fe_mul(&r, &r, &b);
    }
    *h = r;
}
/* exponents: p-2 and (p-5)/8 little-endian */
static uint8_t EXP_PM2[32], EXP_P58[32];
static fe FE_D, FE_D2, FE_SQRTM1;
static fe BX, BY;
static int g_init = 0;
typedef struct { fe X, Y, Z, T; } ge_;
static ge_ Bi_tab[8];   /* odd multiples {1,3,..,15}B, filled by ed_init */

static void fe_invert(fe* h, const fe* f) { fe_pow(h, f, EXP_PM2); }
static void fe_from_u32(fe* h, uint32_t x) { fe_0(h); h->v[0] = x; }

/* ---- group: extended twisted Edwards coordinates (a = -1) ---- */
typedef struct { fe X, Y, Z, T; } ge;

static void ge_identity(ge* p) { fe_0(&p->X); fe_1(&p->Y); fe_1(&p->Z); fe_0(&p->T); }
static void ge_add(ge* r, const ge* p, const ge* q) {
    fe a, b, c, d, e, f, g, h, t;
    fe_sub(&a, &p->Y, &p->X); fe_sub(&t, &q->Y, &q->X); fe_mul(&a, &a, &t);
    fe_add(&b, &p->Y, &p->X); fe_add(&t, &q->Y, &q->X); fe_mul(&b, &b, &t);
    fe_mul(&c, &p->T, &q->T); fe_mul(&c, &c, &FE_D2);
    fe_mul(&d, &p->Z, &q->Z); fe_add(&d, &d, &d);
    fe_sub(&e, &b, &a); fe_sub(&f, &d, &c); fe_add(&g, &d, &c); fe_add(&h, &b, &a);
    fe_mul(&r->X, &e, &f); fe_mul(&r->Y, &g, &h); fe_mul(&r->T, &e, &h); fe_mul(&r->Z, &f, &g);
}
static void ge_neg(ge* r, const ge* p) { fe_neg(&r->X, &p->X); r->Y = p->Y; r->Z = p->Z; fe_neg(&r->T, &p->T); }
static void ge_sub(ge* r, const ge* p, const ge* q) { ge n; ge_neg(&n, q); ge_add(r, p, &n); }
static void ge_dbl(ge* r, const ge* p) {
    fe a, b, c, e, g, f, h, t;
    fe_sq(&a, &p->X); fe_sq(&b, &p->Y); fe_sq(&c, &p->Z); fe_add(&c, &c, &c);
    fe_add(&t, &p->X, &p->Y); fe_sq(&e, &t); fe_sub(&e, &e, &a); fe_sub(&e, &e, &b);
    /* D = -A ; G = D + B = B - A ; F = G - C ; H = D - B = -A - B */
    fe_sub(&g, &b, &a); fe_sub(&f, &g, &c); fe_add(&h, &a, &b); fe_neg(&h, &h);
    fe_mul(&r->X, &e, &f); fe_mul(&r->Y, &g, &h); fe_mul(&r->T, &e, &h); fe_mul(&r->Z, &f, &g);
}
static void ge_tobytes(uint8_t s[32], const ge* p) {
    fe zi, x, y;
    fe_invert(&zi, &p->Z);
    fe_mul(&x, &p->X, &zi);
    fe_mul(&y, &p->Y, &zi);
    fe_tobytes(s, &y);
    s[31] |= (uint8_t)(fe_isnegative(&x) << 7);
}
/* GroupElement(curve, byte[] s) — i2p 0.2.0 decompression; returns -1 on "not a valid point" */
static int ge_frombytes(ge* p, const uint8_t s[32]) {
    fe y, yy, u, v, v3, x, vxx, chk, one;
    fe_1(&one);
    fe_frombytes(&y, s);
    fe_sq(&yy, &y);
    fe_sub(&u, &yy, &one);
    fe_mul(&v, &yy, &FE_D); fe_add(&v, &v, &one);
    fe_sq(&v3, &v); fe_mul(&v3, &v3, &v);
    fe_sq(&x, &v3); fe_mul(&x, &x, &v); fe_mul(&x, &x, &u);
    fe_pow(&x, &x, EXP_P58);
    fe_mul(&x, &x, &v3); fe_mul(&x, &x, &u);
    fe_sq(&vxx, &x); fe_mul(&vxx, &vxx, &v);
    fe_sub(&chk, &vxx, &u);
    if (fe_isnonzero(&chk)) {
        fe_add(&chk, &vxx, &u);
        if (fe_isnonzero(&chk)) return -1;
        fe_mul(&x, &x, &FE_SQRTM1);
    }
    if (fe_isnegative(&x) != ((s[31] >> 7) & 1)) fe_neg(&x, &x);
    p->X = x; p->Y = y; fe_1(&p->Z); fe_mul(&p->T, &x, &y);
    return 0;
}

static void ed_init(void) {
    if (g_init) return;
    /* p = 2^255 - 19 little-endian */
    uint8_t p[32];
    memset(p, 0xff, 32); p[0] = 0xed; p[31] = 0x7f;
    /* p - 2 */
    memcpy(EXP_PM2, p, 32); EXP_PM2[0] = 0xeb;
    /* (p - 5) / 8 = 2^252 - 3 */
    memset(EXP_P58, 0xff, 32); EXP_P58[0] = 0xfd; EXP_P58[31] = 0x0f;
    fe a, b, one;
    fe_1(&one);
    /* d = -121665 / 121666 */
    fe_from_u32(&a, 121665); fe_from_u32(&b, 121666);
    fe_invert(&b, &b); fe_mul(&FE_D, &a, &b); fe_neg(&FE_D, &FE_D);
    fe_add(&FE_D2, &FE_D, &FE_D);
    /* sqrt(-1) = 2^((p-1)/4) */
    uint8_t e[32];
    memset(e, 0xff, 32); e[0] = 0xfb; e[31] = 0x1f;   /* (p-1)/4 = 2^253 - 5 */
    fe two; fe_from_u32(&two, 2);
    fe_pow(&FE_SQRTM1, &two, e);
    /* B: y = 4/5, x even */
    fe_from_u32(&a, 4); fe_from_u32(&b, 5); fe_invert(&b, &b); fe_mul(&BY, &a, &b);
    uint8_t yb[32]; fe_tobytes(yb, &BY);
    g_init = 1;
    ge B; ge_frombytes(&B, yb);
    BX = B.X;
    ge B2; ge_dbl(&B2, &B);
    ge* Bi = (ge*)Bi_tab;
    Bi[0] = B;
    for (int i = 1; i < 8; i++) ge_add(&Bi[i], &Bi[i - 1], &B2);
}

/* ---- scalars mod L = 2^252 + 27742317777372353535851937790883648493 ---- */
static const uint8_t L_LE[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                                 0xa2, 0xde, 0xf9, 0xde, 0x14, 0, 0, 0, 0, 0, 0, 0, 0,
                                 0, 0, 0, 0, 0, 0, 0, 0x10};
/* generic restatement of Ed25519ScalarOps.reduce (ref10 sc_reduce): 512-bit LE -> mod L */
void orc_ed_init(void) { ed_init(); }
void orc_ed25519_sc_reduce64(const uint8_t in[64], uint8_t out[32]) {
    uint64_t Lw[4], r[5] = {0};
    for (int i = 0; i < 4; i++) {
        uint64_t x = 0;
        for (int j = 7; j >= 0; j--) x = (x << 8) | L_LE[8 * i + j];
        Lw[i] = x;
    }
    for (int bit = 511; bit >= 0; bit--) {
        /* r = 2r + bit */
        for (int i = 4; i > 0; i--) r[i] = (r[i] << 1) | (r[i - 1] >> 63);
        r[0] = (r[0] << 1) | ((in[bit >> 3] >> (bit & 7)) & 1);
        /* if r >= L: r -= L  (r < 2L < 2^254 fits) */
        int ge_ = 1;
        if (r[4]) ge_ = 1;
        else {
            for (int i = 3; i >= 0; i--) {
                if (r[i] != Lw[i]) { ge_ = r[i] > Lw[i]; break; }
            }
        }
        if (ge_) {
            u128 bw = 0;
            for (int i = 0; i < 4; i++) {
                u128 d = (u128)r[i] - Lw[i] - bw;
                r[i] = (uint64_t)d;
                bw = (d >> 64) ? 1 : 0;
            }
            r[4] -= (uint64_t)bw;
        }
    }
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t)(r[i] >> (8 * j));
}

/* GroupElement.slide(byte[] a) — i2p 0.2.0 / ref10.  Returns how many carries fell off
 * digit 255 (the effective scalar is then a - drops*2^256). */
int orc_ed25519_slide(const uint8_t a[32], int8_t r[256]) {
    int drops = 0;
    for (int i = 0; i < 256; i++) r[i] = (int8_t)(1 & (a[i >> 3] >> (i & 7)));
    for (int i = 0; i < 256; i++) {
        if (!r[i]) continue;
        for (int b = 1; b <= 6 && i + b < 256; b++) {
            if (!r[i + b]) continue;
            if (r[i] + (r[i + b] << b) <= 15) {
                r[i] = (int8_t)(r[i] + (r[i + b] << b));
                r[i + b] = 0;
            } else if (r[i] - (r[i + b] << b) >= -15) {
                r[i] = (int8_t)(r[i] - (r[i + b] << b));
                int k;
                for (k = i + b; k < 256; k++) {
                    if (!r[k]) { r[k] = 1; break; }
                    r[k] = 0;
                }
                if (k == 256) drops++;
            } else
                break;
        }
    }
    return drops;
}

/* GroupElement.doubleScalarMultiplyVariableTime(A, a, b) = a*A + b*B, i2p 0.2.0 structure:
 * odd-multiple tables {1,3,...,15}·P, slide() digits, scan from the top nonzero digit. */
static void double_scalarmult(ge* r, const ge* A, const uint8_t a[32], const uint8_t b[32]) {
    ge Ai[8], A2;
    ge_dbl(&A2, A);
    Ai[0] = *A;
    for (int i = 1; i < 8; i++) ge_add(&Ai[i], &Ai[i - 1], &A2);
    int8_t as[256], bs[256];
    orc_ed25519_slide(a, as);
    orc_ed25519_slide(b, bs);
    ge_identity(r);
    int i;
    for (i = 255; i >= 0; i--)
        if (as[i] || bs[i]) break;
    for (; i >= 0; i--) {
        ge_dbl(r, r);
        if (as[i] > 0) ge_add(r, r, &Ai[as[i] / 2]);
        else if (as[i] < 0) ge_sub(r, r, &Ai[(-as[i]) / 2]);
        const ge* Bi = (const ge*)Bi_tab;
        if (bs[i] > 0) ge_add(r, r, &Bi[bs[i] / 2]);
        else if (bs[i] < 0) ge_sub(r, r, &Bi[(-bs[i]) / 2]);
    }
}

int orc_ed25519_decode_key(const uint8_t a[32], uint8_t abyte[32]) {
    ed_init();
    ge A;
    if (ge_frombytes(&A, a) != 0) return -1;
    ge_tobytes(abyte, &A);   /* EdDSAPublicKey.Abyte = A.toByteArray() */
    return 0;
}

int orc_ed25519_verify(const uint8_t a[32], const uint8_t* sig, size_t siglen, const uint8_t* msg,
                       size_t msglen) {
    ed_init();
    ge A, Aneg, R;
    if (ge_frombytes(&A, a) != 0) return ORC_KEY_INVALID;
    if (siglen != 64) return ORC_SIG_DECODE;
    uint8_t abyte[32];
    ge_tobytes(abyte, &A);
    orc_sha512_ctx c;
    uint8_t h64[64], h[32];
    orc_sha512_init(&c);
    orc_sha512_update(&c, sig, 32);
    orc_sha512_update(&c, abyte, 32);
    orc_sha512_update(&c, msg, msglen);
    orc_sha512_final(&c, h64);
    orc_ed25519_sc_reduce64(h64, h);
    ge_neg(&Aneg, &A);
    double_scalarmult(&R, &Aneg, h, sig + 32);
    uint8_t rc[32];
    ge_tobytes(rc, &R);
    return memcmp(rc, sig, 32) == 0 ? ORC_VALID : ORC_INVALID;
}

/* test helper: encode [s]B (s little-endian, any 256-bit value, plain double-and-add) */
void orc_ed25519_scalarmult_base(const uint8_t s[32], uint8_t out[32]) {
    ed_init();
    ge B, r;
    B.X = BX; B.Y = BY; fe_1(&B.Z); fe_mul(&B.T, &BX, &BY);
    ge_identity(&r);
    for (int i = 255; i >= 0; i--) {
        ge_dbl(&r, &r);
        if ((s[i >> 3] >> (i & 7)) & 1) ge_add(&r, &r, &B);
    }
    ge_tobytes(out, &r);
}
/* test helper: encode a*P + b*B for an encoded point P (exact, double-and-add) */
int orc_ed25519_double_scalarmult_plain(const uint8_t p[32], const uint8_t a[32], const uint8_t b[32],
                                        uint8_t out[32]) {
    ed_init();
    ge P, B, r;
    if (ge_frombytes(&P, p) != 0) return -1;
    B.X = BX; B.Y = BY; fe_1(&B.Z); fe_mul(&B.T, &BX, &BY);
    ge_identity(&r);
    for (int i = 255; i >= 0; i--) {
        ge_dbl(&r, &r);
        if ((a[i >> 3] >> (i & 7)) & 1) ge_add(&r, &r, &P);
        if ((b[i >> 3] >> (i & 7)) & 1) ge_add(&r, &r, &B);
    }
    ge_tobytes(out, &r);
    return 0;
}
