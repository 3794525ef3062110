// ed25519.hip — K1b (key prep) and K1 (batch verify) for EDDSA_ED25519_SHA512 on gfx950.
//
// Semantics: i2p eddsa 0.2.0 EdDSAEngine.engineVerify as reached from Crypto.isValid
// (core/.../crypto/Crypto.kt:615-625) through X509EdDSAEngine (core/.../internal/X509EdDSAEngine.kt:40):
//   h  = SHA-512(R || Abyte || M) mod L,  Abyte = canonical re-encoding of the decoded key
//   S  = sig[32:64] little-endian, not range checked; i2p's slide() drops a carry past digit 255
//        (only possible for S >= 2^255), so the effective scalar is S - drops*2^256
//   R' = [h](-A) + [S]B ; accept iff canonical encode(R') == sig[0:32]
// Since R' is a group element the scalar-multiplication schedule is free: here a lane-uniform
// fixed-window schedule (no divergence) — signed radix-16 digits for A from a per-key table
// of 0..8 x (-A) in global memory, signed radix-256 digits for B from a 129-entry affine table
// staged in LDS; 252 doublings + 64 A-adds + 32 B-adds per signature.
#include "ed_common_dev.hpp"
#include "runtime.hpp"

#include <cstdlib>
#ifndef ED_STRAUS_OCC
#define ED_STRAUS_OCC 1
#endif
#define ED_TAB_ENTRIES 9
#define ED_TAB_WORDS (ED_TAB_ENTRIES * 40)

// SPKI prefix of an Ed25519 key (X509 SubjectPublicKeyInfo, OID 1.3.101.112)
__device__ __constant__ const uint8_t SPKI_ED[12] = {0x30, 0x2a, 0x30, 0x05, 0x06, 0x03, 0x2b, 0x65, 0x70, 0x03, 0x21, 0x00};

// ---- K1b: per unique key.  Ed25519 keys only; other schemes are handled by ecdsa.hip ----
// TABLE = false (eager comb batches): no Straus table, so the kernel needs a third of the registers and its
// workgroups find room beside the batch-wide kernels it runs next to
// OCC: waves per SIMD the registers must leave room for (CHIP_ED_KEYPREP_OCC; 1 = the compiler's choice)
template <bool TABLE, int OCC = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) k_ed25519_key_prep(uint64_t n_keys, const uint8_t* __restrict__ key_data,
                                                          const uint64_t* __restrict__ key_off,
                                                          const uint32_t* __restrict__ key_len, KeyMeta* meta,
                                                          uint32_t* __restrict__ abytes, uint32_t* __restrict__ table,
                                                          uint32_t* __restrict__ nega, const uint32_t* __restrict__ skip) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_keys || (skip && *skip)) return;
#if !ED_NO_PRIO
    __builtin_amdgcn_s_setprio(3);   // a latency chain per key (the square root) ahead of the comb tables
#endif
    const uint8_t* p = key_data + key_off[k];
    const uint32_t len = key_len[k];
    bool is_ed = (len == 44);
    if (is_ed) {
#pragma unroll
        for (int i = 0; i < 12; i++) is_ed = is_ed && (p[i] == SPKI_ED[i]);
    }
    if (!is_ed) return;   // left for the ECDSA key prep (meta zero-initialised = unsupported)
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = ld_le32(p + 12 + 4 * i);
    ge_p3 A;
    KeyMeta m;
    m.scheme = CHIP_SCHEME_ED25519;
    m.pad[0] = m.pad[1] = 0;
    if (!ge_frombytes(A, w)) {
        m.ok = 0;
        meta[k] = m;
        return;
    }
    m.ok = 1;
    // Abyte = A.toByteArray(): canonical y, sign of x (Z = 1)
    uint32_t ab[8];
    fe_tobytes(ab, A.Y);
    ab[7] |= fe_isnegative(A.X) << 31;
#pragma unroll
    for (int i = 0; i < 8; i++) abytes[k * 8 + i] = ab[i];
    // table[j] = j * (-A), j = 0..8, cached form
    ge_p3 nA = A;
    fe_neg(nA.X, A.X);
    fe_carry(nA.X);
    fe_neg(nA.T, A.T);
    fe_carry(nA.T);
    if (nega) ed_store_p3(nega + k * 40, nA);   // -A in extended form: base of the per-key comb (ed25519_comb.hip)
    if (!TABLE) {   // every signature takes the comb (eager tables): no Straus table
        meta[k] = m;
        return;
    }
    uint32_t* tab = table + k * ED_TAB_WORDS;
    ge_cached c, c1;
    fe_1(c.YpX); fe_1(c.YmX); fe_1(c.Z); fe_0(c.T2d);
    ed_store_cached(tab, c);
    ge_p3_to_cached(c1, nA);
    ed_store_cached(tab + 40, c1);
    ge_p1p1 t;
    ge_p3 P;
    ge_p3_dbl(t, nA);
    ge_p1p1_to_p3(P, t);
    ge_p3_to_cached(c, P);
    ed_store_cached(tab + 80, c);
    for (int j = 3; j <= 8; j++) {
        ge_add_cached(t, P, c1, false);
        ge_p1p1_to_p3(P, t);
        ge_p3_to_cached(c, P);
        ed_store_cached(tab + 40 * j, c);
    }
    meta[k] = m;
}

// ---- K1: batch verify over the compacted list of Ed25519 signatures needing arithmetic ----
// OCC: waves per SIMD the register allocation must leave room for (1: the compiler's choice, 248 VGPRs = 2 waves;
// 3: <= 168 VGPRs, a few spilled long-lived words), CHIP_ED_STRAUS_OCC
template <int OCC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) k_ed25519_verify(const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                                                        const uint32_t* __restrict__ key_idx,
                                                        const uint32_t* __restrict__ msg_idx,
                                                        const uint8_t* __restrict__ sig_data,
                                                        const uint64_t* __restrict__ sig_off,
                                                        const uint8_t* __restrict__ msg_data,
                                                        const uint64_t* __restrict__ msg_off,
                                                        const uint32_t* __restrict__ msg_len,
                                                        const uint32_t* __restrict__ abytes,
                                                        const uint32_t* __restrict__ table, uint8_t* __restrict__ status) {
    __shared__ uint32_t btab[ED_B_ENTRIES * 30];
    if (blockIdx.x * blockDim.x >= *count) return;   // whole block past the list: skip the table load
    for (int i = threadIdx.x; i < ED_B_ENTRIES * 30; i += blockDim.x) {
        const niels_c& e = ED_B_TABLE[i / 30];
        const int f = (i % 30) / 10, l = i % 10;
        btab[i] = f == 0 ? e.ypx[l] : (f == 1 ? e.ymx[l] : e.xy2d[l]);
    }
    __syncthreads();
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= *count) return;
    const uint32_t i = list[gid];
    const uint32_t k = key_idx[i];
    const uint32_t mi = msg_idx[i];
    const uint8_t* sig = sig_data + sig_off[i];
    uint32_t R[8], S[8], Ab[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        R[q] = ld_le32(sig + 4 * q);
        S[q] = ld_le32(sig + 32 + 4 * q);
        Ab[q] = abytes[(uint64_t)k * 8 + q];
    }
    // h = SHA-512(R || Abyte || M) mod L
    uint32_t hx[16], h[8], s[8];
    ed_challenge(hx, R, Ab, msg_data + msg_off[mi], msg_len[mi], sig);
    sc_reduce512(h, hx);
    // effective S (slide() carry drop) reduced mod L
    ed_effective_s(s, S);
    uint32_t ea[8], eb[8];
    sc_recode16(ea, h);
    sc_recode256(eb, s);
    const uint32_t* tab = table + (uint64_t)k * ED_TAB_WORDS;

    // windows w = 63..0 of 4 bits: 4 doublings, + the A digit's row of the key table (signed radix 16), and at
    // every even w + the B digit's entry of the LDS table (signed radix 256).  Window 63 starts from the
    // identity (no doubling, no multiplication: identity + q = (q+ - q-, q+ + q-, 2Z, 2Z)); the loop runs the
    // windows in (even, odd) pairs, so nothing in it is conditional and it carries only the projective r.
    ge_p2 r;
    ge_p1p1 t;
    ge_p3 u;
    ge_cached ca;
    fe qp, qm, xy2d, z2;
    auto a_digit = [&]() -> int {
        const int d = (int)(ea[7] >> 28) - 8;
        shl256(ea, 4);
        return d;
    };
    auto doublings = [&]() {   // r -> u = 16 r
#pragma unroll 1
        for (int q = 0; q < 3; q++) {
            ge_p2_dbl(t, r);
            ge_p1p1_to_p2(r, t);
        }
        ge_p2_dbl(t, r);
        ge_p1p1_to_p3(u, t);
    };
    auto a_add = [&]() {       // t = u + d (-A)
        const int d = a_digit();
        ed_load_row_signed(ca, tab + 40 * (uint32_t)(d < 0 ? -d : d), d < 0);
        ge_add_row<false>(t, u, ca, (uint32_t)(d >> 31));
    };
    auto b_add = [&]() {       // t = t + e B (affine Niels entry |e| of the LDS table, signed)
        const int e = (int)(eb[7] >> 24) - 128;
        shl256(eb, 8);
        const uint32_t ie = (uint32_t)(e < 0 ? -e : e);
        const uint32_t* ent = btab + 30 * ie;
        const uint32_t* pp = ent + (e < 0 ? 10 : 0);
        const uint32_t* pm = ent + (e < 0 ? 0 : 10);
#pragma unroll
        for (int l = 0; l < 10; l++) {
            qp.v[l] = pp[l];
            qm.v[l] = pm[l];
            xy2d.v[l] = ent[20 + l];
        }
        fe_mul(u.X, t.X, t.T);
        fe_mul(u.Y, t.Z, t.Y);
        fe_mul2(z2, t.Z, t.T);
        fe_mul(u.T, t.X, t.Y);
        ge_madd_signed(t, u, z2, qp, qm, xy2d, (uint32_t)(e >> 31));
    };
    {   // window 63 (odd: no B digit)
        const int d = a_digit();
        ed_load_row_signed(ca, tab + 40 * (uint32_t)(d < 0 ? -d : d), d < 0);
        fe_sub(t.X, ca.YpX, ca.YmX);
        fe_add(t.Y, ca.YpX, ca.YmX);
        fe_add(t.Z, ca.Z, ca.Z);
        t.T = t.Z;
        ge_p1p1_to_p2(r, t);
    }
#pragma unroll 1
    for (int w = 62; w > 0; w -= 2) {
        doublings();           // window w (even)
        a_add();
        b_add();
        ge_p1p1_to_p2(r, t);
        doublings();           // window w - 1 (odd)
        a_add();
        ge_p1p1_to_p2(r, t);
    }
    doublings();               // window 0
    a_add();
    b_add();
    ge_p1p1_to_p2(r, t);
    uint32_t enc[8];
    ge_tobytes(enc, r.X, r.Y, r.Z);
    bool eq = true;
#pragma unroll
    for (int q = 0; q < 8; q++) eq = eq && (enc[q] == R[q]);
    status[i] = eq ? CHIP_VALID : CHIP_INVALID;
}

// ---- the split Straus path's table half (launch_ed_straus_split) ----
// The same lane-uniform schedule as k_ed25519_verify without its B additions, SHA-512 and inversion: h's signed
// radix-16 digits come from the row (k_ed_comb_hash<false, true>), [S]B (completed) from k_ed_comb_bhalf, and R'
// leaves projective for the batched-inversion finish.
// early: the row of position p is the signature's (launch_ed_straus_front), else the position's
template <int OCC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) k_ed25519_verify_a(const uint32_t* __restrict__ list,
                                                          const uint32_t* __restrict__ count,
                                                          const uint32_t* __restrict__ key_idx,
                                                          const uint32_t* __restrict__ table,
                                                          const uint32_t* __restrict__ bmid, uint32_t row_words,
                                                          uint32_t hd_word, uint32_t* __restrict__ xyz, uint64_t cap,
                                                          uint32_t early) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= *count) return;
    const uint32_t i = list[p];
    const uint32_t k = key_idx[i];
    const uint32_t* row = bmid + (uint64_t)(early ? i : p) * row_words;
    uint32_t ea[8];
#pragma unroll
    for (int q = 0; q < 8; q++) ea[q] = row[hd_word + q];
    const uint32_t* tab = table + (uint64_t)k * ED_TAB_WORDS;
    ge_p2 r;
    ge_p1p1 t;
    ge_p3 u;
    ge_cached ca;
    auto a_digit = [&]() -> int {
        const int d = (int)(ea[7] >> 28) - 8;
        shl256(ea, 4);
        return d;
    };
    auto a_add = [&]() {   // u = 16 r, then t = u + d (-A)
#pragma unroll 1
        for (int q = 0; q < 3; q++) {
            ge_p2_dbl(t, r);
            ge_p1p1_to_p2(r, t);
        }
        ge_p2_dbl(t, r);
        ge_p1p1_to_p3(u, t);
        const int d = a_digit();
        ed_load_row_signed(ca, tab + 40 * (uint32_t)(d < 0 ? -d : d), d < 0);
        ge_add_row<false>(t, u, ca, (uint32_t)(d >> 31));
    };
    {   // window 63 from the identity
        const int d = a_digit();
        ed_load_row_signed(ca, tab + 40 * (uint32_t)(d < 0 ? -d : d), d < 0);
        fe_sub(t.X, ca.YpX, ca.YmX);
        fe_add(t.Y, ca.YpX, ca.YmX);
        fe_add(t.Z, ca.Z, ca.Z);
        t.T = t.Z;
        ge_p1p1_to_p2(r, t);
    }
#pragma unroll 1
    for (int w = 62; w > 0; w--) {
        a_add();
        ge_p1p1_to_p2(r, t);
    }
    a_add();   // window 0
    // + [S]B: the row's completed point to extended, then cached
    ge_p3 acc;
    ge_p1p1_to_p3(acc, t);
    {
        ge_p1p1 sb;
#pragma unroll
        for (int q = 0; q < 10; q++) {
            sb.X.v[q] = row[q];
            sb.Y.v[q] = row[10 + q];
            sb.Z.v[q] = row[20 + q];
            sb.T.v[q] = row[30 + q];
        }
        ge_p1p1_to_p3(u, sb);
    }
    ge_p3_to_cached(ca, u);
    ge_add_cached(t, acc, ca, false);
    fe X, Y, Z;
    fe_mul(X, t.X, t.T);
    fe_mul(Y, t.Z, t.Y);
    fe_mul(Z, t.Z, t.T);
#pragma unroll
    for (int q = 0; q < 10; q++) {
        xyz[(uint64_t)q * cap + p] = X.v[q];
        xyz[(uint64_t)(10 + q) * cap + p] = Y.v[q];
        xyz[(uint64_t)(20 + q) * cap + p] = Z.v[q];
    }
}

void launch_ed25519_verify_a(hipStream_t st, uint64_t n, const uint32_t* list, const uint32_t* count,
                             const uint32_t* key_idx, const uint32_t* table, const uint32_t* bmid, uint32_t row_words,
                             uint32_t hd_word, uint32_t* xyz, bool early) {
    if (!n) return;
    // 3 waves per SIMD (168 VGPRs, 32 B of scratch outside the window loop): cold keys 55.2-55.8M vs 53.7-55.2M at the
    // compiler's 178 VGPRs and 53.5-53.7M at 4 waves (spills in the loop; profiles/r06/ab_straus_split.txt)
    static const int occ = [] {
        const char* e = getenv("CHIP_ED_SPLIT_OCC");
        return e ? atoi(e) : 3;
    }();
    auto kern = occ == 4 ? k_ed25519_verify_a<4> : (occ == 3 ? k_ed25519_verify_a<3> : k_ed25519_verify_a<1>);
    hipLaunchKernelGGL(kern, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, list, count, key_idx, table, bmid,
                       row_words, hd_word, xyz, n, early ? 1u : 0u);
}

// ---- Crypto.decodePublicKey of an Ed25519 SPKI (i2p GroupElement(curve, bytes)) for the Kryo front end:
// ok = the point decodes; kind 1 also requires the canonical encoding EdDSAPublicKey re-encodes (A.toByteArray:
// y < p, the sign bit = parity of x)
__global__ void __launch_bounds__(256) k_ed25519_key_check(uint64_t n, const uint8_t* __restrict__ pool,
                                                           const uint64_t* __restrict__ off,
                                                           const uint32_t* __restrict__ len,
                                                           const uint8_t* __restrict__ kind, uint8_t* __restrict__ ok) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || len[i] != 44) return;
    const uint8_t* p = pool + off[i];
    bool is_ed = true;
#pragma unroll
    for (int j = 0; j < 12; j++) is_ed = is_ed && (p[j] == SPKI_ED[j]);
    if (!is_ed) return;
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = ld_le32(p + 12 + 4 * j);
    ge_p3 A;
    bool good = ge_frombytes(A, w);
    if (good && kind[i]) {
        uint32_t ab[8];
        fe_tobytes(ab, A.Y);
        ab[7] |= fe_isnegative(A.X) << 31;
#pragma unroll
        for (int j = 0; j < 8; j++) good = good && ab[j] == w[j];
    }
    ok[i] = good ? 1 : 0;
}

void launch_ed25519_key_check(hipStream_t st, uint64_t n, const uint8_t* pool, const uint64_t* off, const uint32_t* len,
                              const uint8_t* kind, uint8_t* ok) {
    if (!n) return;
    hipLaunchKernelGGL(k_ed25519_key_check, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, n, pool, off, len, kind,
                       ok);
}

// ---------------------------------------------------------------------------------------
void launch_ed25519_key_prep(hipStream_t st, uint64_t n_keys, const uint8_t* key_data, const uint64_t* key_off,
                             const uint32_t* key_len, KeyMeta* meta, uint32_t* abytes, uint32_t* table,
                             uint32_t* nega, const uint32_t* skip) {
    if (!n_keys) return;
    const uint32_t blocks = (uint32_t)((n_keys + 255) / 256);
    static const int occ = [] {
        const char* e = getenv("CHIP_ED_KEYPREP_OCC");
        return e ? atoi(e) : 1;
    }();
    if (table) {
        auto kern = occ == 4 ? k_ed25519_key_prep<true, 4> : (occ == 3 ? k_ed25519_key_prep<true, 3>
                                                                         : k_ed25519_key_prep<true, 1>);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, st, n_keys, key_data, key_off, key_len, meta, abytes, table,
                           nega, skip);
    }
    else
        hipLaunchKernelGGL(k_ed25519_key_prep<false>, dim3(blocks), dim3(256), 0, st, n_keys, key_data, key_off, key_len,
                           meta, abytes, table, nega, skip);
}

void launch_ed25519_verify(hipStream_t st, uint64_t n, const uint32_t* list, const uint32_t* count,
                           const chip_sig_batch* b, const uint32_t* abytes, const uint32_t* table, uint8_t* status) {
    if (!n) return;
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    static const int occ = [] {
        const char* e = getenv("CHIP_ED_STRAUS_OCC");
        return e ? atoi(e) : ED_STRAUS_OCC;
    }();
    if (occ == 3)
        hipLaunchKernelGGL(k_ed25519_verify<3>, dim3(blocks), dim3(256), 0, st, list, count, b->key_idx, b->msg_idx,
                           b->sig_data, b->sig_off, b->msg_data, b->msg_off, b->msg_len, abytes, table, status);
    else
        hipLaunchKernelGGL(k_ed25519_verify<1>, dim3(blocks), dim3(256), 0, st, list, count, b->key_idx, b->msg_idx,
                           b->sig_data, b->sig_off, b->msg_data, b->msg_off, b->msg_len, abytes, table, status);
}
