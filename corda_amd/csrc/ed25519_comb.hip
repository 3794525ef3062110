// ed25519_comb.hip — K1c: Ed25519 batch verification with per-key comb tables, for keys that sign
// several signatures of a batch (every Corda party / notary key does).
//
// Semantics are those of k_ed25519_verify (ed25519.hip; i2p eddsa 0.2.0 EdDSAEngine.engineVerify as
// reached from Crypto.isValid, core/.../crypto/Crypto.kt:615-625, through X509EdDSAEngine.kt:40):
//   h = SHA-512(R || Abyte || M) mod L;  S not range checked, slide() carry drop for S >= 2^255;
//   R' = [h](-A) + [S]B;  accept iff canonical encode(R') == R bytewise.
// R' is a group element, so any exact schedule gives the same bytes.  This one has no doublings:
//   [h](-A) = sum_w d_w (2^(W w) (-A)),  d_w the signed radix-2^W digits of h, read from a per-key
//             table of ED_COMB_AWIN windows x (2^(W-1)+1) cached multiples built for the batch by
//             k_ed_comb_chain (the W-fold doubling chain, one lane per key) and k_ed_comb_fill
//             (the multiples, one lane per key x window);
//   [S]B    = sum_w e_w (2^(16 w) B),    e_w the signed radix-2^16 digits of S, read from the fixed
//             table built per context by k_ed_bcomb16_build (16 x 32,769 affine Niels rows, 67 MB).
// 43 + 16 additions per signature (W = 6: ~460 field multiplications) instead of 252 doublings + 96
// additions (2,766).  The projective R' is inverted in batches of ED_FIN_G by k_ed_comb_finish
// (Montgomery's trick: ~21 instead of 265 multiplications per signature).
//
// Work list: k_ed_comb_partition groups the signatures of one key contiguously (counting sort on
// the key index), and k_ed_comb_ahalf maps consecutive blocks of the list onto one XCD, so a key's
// 227 KB table (W = 6) is read through one XCD's L2.  Keys with fewer than min_sigs signatures (or beyond the
// table budget) keep the Straus kernel.
#include "ed_common_dev.hpp"
#include <cstdlib>
#include "runtime.hpp"
#include "comb_tables.hpp"

#define ED_COMB_ABIAS (1 << (ED_COMB_W - 1))
#define ED_COMB_ADW ((ED_COMB_AWIN + 3) / 4)   // digit words, 4 biased digits per word

// signed radix-2^W digits of a (< 2^253), each biased by 2^(W-1) into one byte, NDIG digits
template <int W, int NDIG>
CHIP_DEV void recode_bytes(uint32_t out[(NDIG + 3) / 4], const uint32_t a[8]) {
    int carry = 0;
#pragma unroll
    for (int q = 0; q < (NDIG + 3) / 4; q++) out[q] = 0;
#pragma unroll
    for (int d = 0; d < NDIG; d++) {
        const int bit = d * W, wi = bit >> 5, sh = bit & 31;
        const uint64_t two = ((uint64_t)(wi + 1 < 8 ? a[wi + 1] : 0u) << 32) | (wi < 8 ? a[wi] : 0u);
        int v = (int)((uint32_t)(two >> sh) & ((1u << W) - 1)) + carry;
        carry = (v + (1 << (W - 1))) >> W;
        v -= carry << W;
        out[d >> 2] |= (uint32_t)(v + (1 << (W - 1))) << (8 * (d & 3));
    }
}

CHIP_DEV void ed_load_niels(ge_niels& q, const uint32_t* __restrict__ src) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint4 x = s4[k];
        const uint32_t vals[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int idx = 4 * k + e;
            if (idx < 10) q.ypx.v[idx] = vals[e];
            else if (idx < 20) q.ymx.v[idx - 10] = vals[e];
            else if (idx < 30) q.xy2d.v[idx - 20] = vals[e];
        }
    }
}

// ---- work list: key slots, counting sort by key ----
// A key gets a comb slot when it is a valid Ed25519 key with at least min_sigs signatures in the
// batch and the table budget allows; its signatures then occupy comb_list[base, base + count).
// Eager mode (many signatures per key): every valid Ed25519 key's table was built at slot = key
// index on the second stream while classify ran, so only the work list is assigned here.
CHIP_DEV bool ed_key_ok(const KeyMeta* meta, uint32_t k) {
    const KeyMeta m = meta[k];
    return m.scheme == CHIP_SCHEME_ED25519 && m.ok;
}
__global__ void __launch_bounds__(256) k_ed_comb_slots(uint64_t n_keys, const KeyMeta* __restrict__ meta,
                                                       const uint32_t* __restrict__ key_count, uint32_t min_sigs,
                                                       uint32_t max_slots, uint32_t eager, int32_t* __restrict__ key_slot,
                                                       uint32_t* __restrict__ key_base, uint32_t* __restrict__ slot_key,
                                                       uint32_t* __restrict__ ctr) {
    // slot and list-range claims: one atomic per workgroup on each counter (block prefix sums)
    __shared__ uint32_t s_wave[4], s_base[2];
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t c = k < n_keys ? key_count[k] : 0u;
    // eager: every valid key has its table, so every one of its signatures takes the comb (no Straus table is
    // built then)
    const bool want = k < n_keys && ed_key_ok(meta, (uint32_t)k) && c > 0 && (eager || c >= min_sigs);
    uint32_t tot;
    const uint32_t ex0 = block_scan_excl(want && !eager ? 1u : 0u, s_wave, tot);
    if (threadIdx.x == 0) s_base[0] = tot ? atomicAdd(&ctr[0], tot) : 0u;
    __syncthreads();
    const uint32_t s = eager ? (uint32_t)k : s_base[0] + ex0;
    const bool got = want && s < max_slots;
    const uint32_t ex1 = block_scan_excl(got ? c : 0u, s_wave, tot);
    if (threadIdx.x == 0) s_base[1] = tot ? atomicAdd(&ctr[1], tot) : 0u;
    __syncthreads();
    if (k >= n_keys) return;
    if (got) {
        slot_key[s] = (uint32_t)k;
        key_base[k] = s_base[1] + ex1;
    }
    key_slot[k] = got ? (int32_t)s : -1;
}

// The comb path only pays when enough signatures take it: its table chain is a fixed serial latency
// (~0.5 ms) that a few thousand hot-key signatures do not amortise, so below `min_total` comb-bound
// signatures the whole list goes to the Straus kernel.  The gated counts (ctr[ED_CTR_NCOMB],
// ctr[ED_CTR_NSLOTS]) are what every later comb kernel reads; ctr[0..1] stay the raw assignment.
#define ED_CTR_NCOMB 8
#define ED_CTR_NSLOTS 9
__global__ void __launch_bounds__(256) k_ed_comb_partition(const uint32_t* __restrict__ ed_list,
                                                           const uint32_t* __restrict__ ed_count,
                                                           const uint32_t* __restrict__ key_idx,
                                                           const int32_t* __restrict__ key_slot,
                                                           const uint32_t* __restrict__ key_base,
                                                           const uint32_t* __restrict__ key_rank, uint32_t* __restrict__ comb_list,
                                                           uint32_t* __restrict__ straus_list, uint32_t* __restrict__ ctr,
                                                           uint32_t min_total, uint32_t max_slots) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    const bool on = ctr[1] >= min_total;
    if (g == 0) {
        ctr[ED_CTR_NCOMB] = on ? ctr[1] : 0u;
        ctr[ED_CTR_NSLOTS] = on ? min(ctr[0], max_slots) : 0u;
    }
    bool straus = false, comb = false;
    uint32_t i = 0, k = 0;
    if (g < *ed_count) {
        i = ed_list[g];
        k = key_idx[i];
        comb = on && key_slot[k] >= 0;
        straus = !comb;
    }
    // the slot inside the key's range: the signature's key rank from k_classify (no atomics)
    if (comb) comb_list[key_base[k] + key_rank[i]] = i;
    // Straus list: one atomic per workgroup (block prefix sum)
    __shared__ uint32_t s_wave[4], s_base;
    uint32_t tot;
    const uint32_t ex = block_scan_excl(straus ? 1u : 0u, s_wave, tot);
    if (!tot) return;   // workgroup-uniform
    if (threadIdx.x == 0) s_base = atomicAdd(&ctr[2], tot);
    __syncthreads();
    if (straus) straus_list[s_base + ex] = i;
}

// ---- per-key tables ----
// chain: P_w = 2^(W w) (-A) for every window, stashed (extended form, 40 words) in the window's last row
// (affine rows: from row 1 on).  One lane per key: W doublings per window, the only serial part of the comb path.
#define ED_COMB_STASH_C (ED_COMB_AENT - 1)   // cached rows: P_w in the window's last row until the fill reads it
#define ED_COMB_STASH_A 1                    // affine rows: from row 1 on
CHIP_DEV uint32_t ed_stash_at(uint32_t w, uint32_t aff) {   // word offset of window w's stashed P_w
    return aff ? (w * ED_COMB_AENT + ED_COMB_STASH_A) * ED_COMB_ROW_A : (w * ED_COMB_AENT + ED_COMB_STASH_C) * ED_COMB_ROW_C;
}
#ifndef ED_CHAIN_PAIR
#define ED_CHAIN_PAIR 0   // 1: the doubling chain on lane pairs (k_ed_comb_chain2): chain 0.60 -> 0.44 ms, but the
                          // [S]B kernel beside it slowed by as much (0.76 -> 1.2 ms): 263-265M vs 265-269M
                          // (profiles/r04/ab_chain_pair.txt); the step is issue-bound on its total work
#endif
__global__ void __launch_bounds__(64) k_ed_comb_chain(const uint32_t* __restrict__ ctr, uint32_t max_slots,
                                                      uint32_t eager, const KeyMeta* __restrict__ meta,
                                                      const uint32_t* __restrict__ slot_key,
                                                      const uint32_t* __restrict__ nega, uint32_t* __restrict__ ctab,
                                                      const uint32_t* __restrict__ skip, uint32_t aff) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nslots = eager ? max_slots : ctr[ED_CTR_NSLOTS];
    if (s >= nslots || (skip && *skip)) return;
    // the serial critical path of the comb path: its few waves win VALU arbitration against the batch-wide
    // kernels of the main stream that share their SIMDs
#if !ED_NO_PRIO
    __builtin_amdgcn_s_setprio(3);
#endif
    if (eager && !ed_key_ok(meta, s)) return;
    const uint32_t k = eager ? s : slot_key[s];
    ge_p3 P;
    ed_load_p3(P, nega + (uint64_t)k * 40);
    uint32_t* tab = ctab + (uint64_t)s * (aff ? ED_COMB_KEY_WORDS_A : ED_COMB_KEY_WORDS_C);
    for (int w = 0; w < ED_COMB_AWIN; w++) {
        ed_store_p3(tab + ed_stash_at((uint32_t)w, aff), P);
        if (w + 1 == ED_COMB_AWIN) break;
        ge_p2 r;
        ge_p3_to_p2(r, P);
        ge_p1p1 t;
#pragma unroll 1
        for (int b = 0; b < ED_COMB_W - 1; b++) {
            ge_p2_dbl(t, r);
            ge_p1p1_to_p2(r, t);
        }
        ge_p2_dbl(t, r);
        ge_p1p1_to_p3(P, t);
    }
}

// The same chain with two lanes per key (adjacent lanes of a wave): each doubling's four squarings and the
// three / four multiplications of its conversion are split between the pair and the halves exchanged through
// DPP quad permutes (one v_mov_dpp per word), so the serial chain per key — the critical path of the step
// once the challenge hash runs beside it — carries about half the field operations per doubling.
CHIP_DEV uint32_t pair_swap(uint32_t v) {   // the partner lane's v (lanes 2i <-> 2i+1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
}
CHIP_DEV void fe_swap_in(fe& out, const fe& mine) {
#pragma unroll
    for (int i = 0; i < 10; i++) out.v[i] = pair_swap(mine.v[i]);
}
CHIP_DEV void fe_sel(fe& r, uint32_t m, const fe& a, const fe& b) {   // m all-ones: a, else b
#pragma unroll
    for (int i = 0; i < 10; i++) r.v[i] = bit_select(m, a.v[i], b.v[i]);
}
// one doubling p2 -> p1p1 on a lane pair; odd = all-ones on the odd lane
CHIP_DEV void ge_p2_dbl_pair(ge_p1p1& r, const ge_p2& p, uint32_t odd) {
    fe in1, in2, s1, s2, o1, o2, XX, YY, A, Z2, B, t;
    fe_add(t, p.X, p.Y);
    fe_sel(in1, odd, p.Y, p.X);   // even: X^2, (X+Y)^2; odd: Y^2, Z^2
    fe_sel(in2, odd, p.Z, t);
    fe_sq(s1, in1);
    fe_sq(s2, in2);
    fe_swap_in(o1, s1);
    fe_swap_in(o2, s2);
    fe_sel(XX, odd, o1, s1);
    fe_sel(YY, odd, s1, o1);
    fe_sel(A, odd, o2, s2);
    fe_sel(Z2, odd, s2, o2);
    fe_add(B, Z2, Z2);            // 2 Z^2 (loose; r.T is carried below)
    fe_add(r.Y, YY, XX);
    fe_sub(r.Z, YY, XX);
    fe_sub4(r.X, A, r.Y);
    fe_carry(r.X);
    fe_add(t, B, XX);
    fe_sub(r.T, t, YY);
    fe_carry(r.T);
}
// p1p1 -> p2 on a lane pair: even computes X, odd Z, both Y
CHIP_DEV void ge_p1p1_to_p2_pair(ge_p2& r, const ge_p1p1& p, uint32_t odd) {
    fe m1, in_a, o;
    fe_sel(in_a, odd, p.Z, p.X);   // even: X T; odd: Z T
    fe_mul(m1, in_a, p.T);
    fe_mul(r.Y, p.Z, p.Y);
    fe_swap_in(o, m1);
    fe_sel(r.X, odd, o, m1);
    fe_sel(r.Z, odd, m1, o);
}
// p1p1 -> p3 on a lane pair: even X and Y, odd Z and T
CHIP_DEV void ge_p1p1_to_p3_pair(ge_p3& r, const ge_p1p1& p, uint32_t odd) {
    fe a1, b1, a2, b2, m1, m2, o1, o2;
    fe_sel(a1, odd, p.Z, p.X);     // even: X T, Z Y;  odd: Z T, X Y
    fe_sel(b1, odd, p.T, p.T);
    fe_sel(a2, odd, p.X, p.Z);
    fe_sel(b2, odd, p.Y, p.Y);
    fe_mul(m1, a1, b1);
    fe_mul(m2, a2, b2);
    fe_swap_in(o1, m1);
    fe_swap_in(o2, m2);
    fe_sel(r.X, odd, o1, m1);
    fe_sel(r.Y, odd, o2, m2);
    fe_sel(r.Z, odd, m1, o1);
    fe_sel(r.T, odd, m2, o2);
}
__global__ void __launch_bounds__(64) k_ed_comb_chain2(const uint32_t* __restrict__ ctr, uint32_t max_slots,
                                                       uint32_t eager, const KeyMeta* __restrict__ meta,
                                                       const uint32_t* __restrict__ slot_key,
                                                       const uint32_t* __restrict__ nega, uint32_t* __restrict__ ctab,
                                                       const uint32_t* __restrict__ skip, uint32_t aff) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t s = g >> 1;
    const uint32_t odd = (g & 1u) ? ~0u : 0u;
    const uint32_t nslots = eager ? max_slots : ctr[ED_CTR_NSLOTS];
    // both lanes of a pair take the same exits (same key), so the pair stays whole for the DPP exchanges
    if (s >= nslots || (skip && *skip)) return;
    if (eager && !ed_key_ok(meta, s)) return;
#if !ED_NO_PRIO
    __builtin_amdgcn_s_setprio(3);
#endif
    const uint32_t k = eager ? s : slot_key[s];
    ge_p3 P;
    ed_load_p3(P, nega + (uint64_t)k * 40);
    uint32_t* tab = ctab + (uint64_t)s * (aff ? ED_COMB_KEY_WORDS_A : ED_COMB_KEY_WORDS_C);
    for (int w = 0; w < ED_COMB_AWIN; w++) {
        if (!odd) ed_store_p3(tab + ed_stash_at((uint32_t)w, aff), P);
        if (w + 1 == ED_COMB_AWIN) break;
        ge_p2 r;
        ge_p3_to_p2(r, P);
        ge_p1p1 t;
#pragma unroll 1
        for (int b = 0; b < ED_COMB_W - 1; b++) {
            ge_p2_dbl_pair(t, r, odd);
            ge_p1p1_to_p2_pair(r, t, odd);
        }
        ge_p2_dbl_pair(t, r, odd);
        ge_p1p1_to_p3_pair(P, t, odd);
    }
}

// fill: rows j = 0..2^(W-1) of window w: j * P_w as [Y+X, Y-X, 2Z, 2dT] (2Z stored, so the addition needs no
// doubling of its column sums; row 0: the identity [1, 1, 2, 0]).  A negative digit reads the same row with
// Y+X and Y-X swapped by address (-Q = (-x, y)) and negates the 2dT term.
CHIP_DEV void ed_store_row(uint32_t* __restrict__ dst, const ge_cached& c) {
    fe z2;
    fe_add(z2, c.Z, c.Z);            // loose: even limbs < 2^27, odd < 2^26
#pragma unroll
    for (int i = 0; i < 10; i++) {
        dst[i] = c.YpX.v[i];
        dst[10 + i] = c.YmX.v[i];
        dst[20 + i] = z2.v[i];
        dst[30 + i] = c.T2d.v[i];
    }
}
// Two lanes per key x window (adjacent lanes of one wave): rows 0..16 from P_w, rows 17..32 from 17 P_w (4
// doublings + 1 addition first), so the serial chain of additions per lane halves.  Both read the stash in the
// last row before either writes a row (same wave, the load precedes the divergence); the second writes the
// last row last.
#define ED_FILL_SPLIT 2
#define ED_FILL_ROWS ((ED_COMB_AENT - 1) / ED_FILL_SPLIT)
#ifndef ED_FILL_WAVES
#define ED_FILL_WAVES 1   // waves per SIMD the cached-row fill's registers must leave room for (1: the compiler's 231 VGPRs)
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ED_FILL_WAVES))) k_ed_comb_fill(const uint32_t* __restrict__ ctr, uint32_t max_slots,
                                                      uint32_t eager, const KeyMeta* __restrict__ meta,
                                                      uint32_t* __restrict__ ctab, const uint32_t* __restrict__ skip) {
    constexpr uint32_t ED_COMB_ROW = ED_COMB_ROW_C, ED_COMB_KEY_WORDS = ED_COMB_KEY_WORDS_C;
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t s = g / (ED_COMB_AWIN * ED_FILL_SPLIT), r = g % (ED_COMB_AWIN * ED_FILL_SPLIT);
    const uint32_t w = r / ED_FILL_SPLIT, h = r % ED_FILL_SPLIT;
    if (s >= (eager ? max_slots : ctr[ED_CTR_NSLOTS]) || (skip && *skip)) return;
    if (eager && !ed_key_ok(meta, s)) return;
    uint32_t* e = ctab + (uint64_t)s * ED_COMB_KEY_WORDS + (uint64_t)w * ED_COMB_AENT * ED_COMB_ROW;
    ge_p3 P;
    ed_load_p3(P, e + ED_COMB_STASH_C * ED_COMB_ROW);   // P_w, stashed by the chain
    ge_cached c1, c;
    ge_p3_to_cached(c1, P);
    ge_p3 Q = P;
    ge_p1p1 t;
    const uint32_t j0 = 1 + h * ED_FILL_ROWS;
    if (h == 0) {
        fe_1(c.YpX);
        fe_1(c.YmX);
        fe_1(c.Z);
        fe_0(c.T2d);
        ed_store_row(e, c);   // the identity
    } else {
        // Q = j0 P = 2^k P + P (j0 - 1 a power of two)
        ge_p2 q2;
        ge_p3_to_p2(q2, P);
        for (uint32_t m = ED_FILL_ROWS * h; m > 2; m >>= 1) {
            ge_p2_dbl(t, q2);
            ge_p1p1_to_p2(q2, t);
        }
        ge_p2_dbl(t, q2);
        ge_p1p1_to_p3(Q, t);
        ge_add_cached(t, Q, c1, false);
        ge_p1p1_to_p3(Q, t);
    }
    for (uint32_t j = j0; j < j0 + ED_FILL_ROWS; j++) {
        if (j > j0) {
            ge_add_cached(t, Q, c1, false);
            ge_p1p1_to_p3(Q, t);
        }
        ge_p3_to_cached(c, Q);
        ed_store_row(e + ED_COMB_ROW * j, c);
    }
}
// Affine rows in three steps (one lane per key x window in a and b):
//   a: j P_w for j = 1..2^(W-1) by additions; row j holds (X_j Z_1..Z_{j-1}, Y_j Z_1..Z_{j-1}, Z_j), so that step
//      b needs no prefix array: with inv = 1 / (Z_1..Z_j), x_j = row.X inv and the next inv = inv Z_j;
//      fz[lane] = Z_1..Z_{2^(W-1)}
//   zinv: one lane per ED_COMB_ZG fill lanes inverts their products together (Montgomery's trick again:
//      one inversion per group instead of per lane; a serial latency on the second stream)
//   b: rows to affine Niels [y+x, y-x, 2dxy], row 0 the identity [1, 1, 0]
CHIP_DEV bool ed_fill_lane(uint32_t g, const uint32_t* __restrict__ ctr, uint32_t max_slots, uint32_t eager,
                           const KeyMeta* __restrict__ meta, uint32_t& s, uint32_t& w, bool& skip) {
    s = g / ED_COMB_AWIN;
    w = g % ED_COMB_AWIN;
    if (s >= (eager ? max_slots : ctr[ED_CTR_NSLOTS])) return false;
    skip = eager && !ed_key_ok(meta, s);
    return true;
}
CHIP_DEV void ed_store_fe(uint32_t* __restrict__ dst, const fe& f) {
#pragma unroll
    for (int i = 0; i < 10; i++) dst[i] = f.v[i];
}
CHIP_DEV void ed_load_fe(fe& f, const uint32_t* __restrict__ src) {
#pragma unroll
    for (int i = 0; i < 10; i++) f.v[i] = src[i];
}
__global__ void __launch_bounds__(256) k_ed_comb_fill_a(const uint32_t* __restrict__ ctr, uint32_t max_slots,
                                                        uint32_t eager, const KeyMeta* __restrict__ meta,
                                                        uint32_t* __restrict__ ctab, uint32_t* __restrict__ fz,
                                                        const uint32_t* __restrict__ cached) {
    constexpr uint32_t ED_COMB_ROW = ED_COMB_ROW_A, ED_COMB_KEY_WORDS = ED_COMB_KEY_WORDS_A;
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t s, w;
    bool skip = false;
    if (!ed_fill_lane(g, ctr, max_slots, eager, meta, s, w, skip) || (cached && *cached)) return;
    fe acc;
    fe_1(acc);
    if (!skip) {
        uint32_t* e = ctab + (uint64_t)s * ED_COMB_KEY_WORDS + (uint64_t)w * ED_COMB_AENT * ED_COMB_ROW;
        ge_p3 P;
        ed_load_p3(P, e + ED_COMB_ROW);   // P_w, stashed from row 1 on by the chain
        ge_cached c1;
        ge_p3_to_cached(c1, P);
        ge_p3 Q = P;
        ge_p1p1 t;
        for (int j = 1; j < ED_COMB_AENT; j++) {
            uint32_t* r = e + j * ED_COMB_ROW;
            if (j == 1) {
                ed_store_fe(r, Q.X);
                ed_store_fe(r + 10, Q.Y);
                acc = Q.Z;
            } else {
                fe x, y;
                fe_mul(x, Q.X, acc);
                fe_mul(y, Q.Y, acc);
                ed_store_fe(r, x);
                ed_store_fe(r + 10, y);
                fe_mul(acc, acc, Q.Z);
            }
            ed_store_fe(r + 20, Q.Z);
            if (j + 1 < ED_COMB_AENT) {
                ge_add_cached(t, Q, c1, false);
                ge_p1p1_to_p3(Q, t);
            }
        }
    }
    ed_store_fe(fz + (uint64_t)g * 10, acc);   // 1 for a skipped lane
}
__global__ void __launch_bounds__(64) k_ed_comb_zinv(const uint32_t* __restrict__ ctr, uint32_t max_slots, uint32_t eager,
                                                     const uint32_t* __restrict__ zprod, uint32_t* __restrict__ zinv,
                                                     const uint32_t* __restrict__ cached) {
    const uint32_t nl = (eager ? max_slots : ctr[ED_CTR_NSLOTS]) * ED_COMB_AWIN;
    const uint32_t g0 = (blockIdx.x * blockDim.x + threadIdx.x) * ED_COMB_ZG;
    if (g0 >= nl || (cached && *cached)) return;
    const uint32_t m = min((uint32_t)ED_COMB_ZG, nl - g0);
    fe acc, z, inv, t;
    fe_1(acc);
    for (uint32_t i = 0; i < m; i++) {   // zinv[i] = the product of the group's values before i
        ed_store_fe(zinv + (uint64_t)(g0 + i) * 10, acc);
        ed_load_fe(z, zprod + (uint64_t)(g0 + i) * 10);
        fe_mul(acc, acc, z);
    }
    fe_invert(inv, acc);
    for (uint32_t i = m; i-- > 0;) {
        ed_load_fe(t, zinv + (uint64_t)(g0 + i) * 10);
        ed_load_fe(z, zprod + (uint64_t)(g0 + i) * 10);
        fe_mul(t, inv, t);
        fe_mul(inv, inv, z);
        ed_store_fe(zinv + (uint64_t)(g0 + i) * 10, t);
    }
}
__global__ void __launch_bounds__(256) k_ed_comb_fill_b(const uint32_t* __restrict__ ctr, uint32_t max_slots,
                                                        uint32_t eager, const KeyMeta* __restrict__ meta,
                                                        uint32_t* __restrict__ ctab, const uint32_t* __restrict__ zinv,
                                                        const uint32_t* __restrict__ cached) {
    constexpr uint32_t ED_COMB_ROW = ED_COMB_ROW_A, ED_COMB_KEY_WORDS = ED_COMB_KEY_WORDS_A;
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t s, w;
    bool skip = false;
    if (!ed_fill_lane(g, ctr, max_slots, eager, meta, s, w, skip) || skip || (cached && *cached)) return;
    uint32_t* e = ctab + (uint64_t)s * ED_COMB_KEY_WORDS + (uint64_t)w * ED_COMB_AENT * ED_COMB_ROW;
    fe inv, d2;
    ed_load_fe(inv, zinv + (uint64_t)g * 10);
    fe_from_c(d2, ED_D2);
    for (int j = ED_COMB_AENT - 1; j >= 1; j--) {
        uint32_t* r = e + j * ED_COMB_ROW;
        fe X, Y, Z, x, y, xy;
        ed_load_fe(X, r);
        ed_load_fe(Y, r + 10);
        ed_load_fe(Z, r + 20);
        fe_mul(x, X, inv);
        fe_mul(y, Y, inv);
        fe_mul(inv, inv, Z);
        ge_niels n;
        fe_add(n.ypx, y, x);
        fe_carry(n.ypx);
        fe_sub(n.ymx, y, x);
        fe_carry(n.ymx);
        fe_mul(xy, x, y);
        fe_mul(n.xy2d, xy, d2);
        ed_store_fe(r, n.ypx);
        ed_store_fe(r + 10, n.ymx);
        ed_store_fe(r + 20, n.xy2d);
        r[30] = 0;
        r[31] = 0;
    }
#pragma unroll
    for (int i = 0; i < ED_COMB_ROW; i++) e[i] = (i == 0 || i == 10) ? 1u : 0u;   // identity
}

// ---- verify: one lane per comb-list position ----
// blocks b, b+8, b+16, ... are dispatched to one XCD: give them consecutive work.  `used` = blocks
// that hold list positions (the comb count is on the device; the grid covers the whole batch):
// each XCD takes ceil(used / 8) consecutive blocks, so a short list still spreads over all 8 XCDs.
CHIP_DEV uint32_t xcd_block(uint32_t b, uint32_t used) {
    const uint32_t share = (used + 7) >> 3;
    return (b & 7u) * share + (b >> 3);
}

// ---- fixed-base comb of B, radix 2^16 (built once per context, 67 MB, Infinity-Cache resident) ----
// ED_B16[w][j] = j * 2^(16 w) * B for w < 16, j = 0..2^15 (+ padding to whole 64-entry chunks),
// affine Niels rows of 30 limbs padded to 32 words (one 128-B line per entry).  [S]B then takes 16
// mixed additions from signed radix-2^16 digits of s instead of 32 from the L2-resident radix-256
// table: 112 fewer field multiplications per signature for one 128-B gather per window.
// Build: one lane per (window, chunk of 64 consecutive multiples): j0 * P by double-and-add, then 63
// additions, the 64 Z inverted together (Montgomery's trick; prefix products in `scratch`).
CHIP_DEV void ed_niels_to_p3(ge_p3& r, const uint32_t* __restrict__ e) {
    ge_niels q;
    ed_load_niels(q, e);
    fe two, inv2, s, d;
    fe_0(two);
    two.v[0] = 2;
    fe_invert(inv2, two);
    fe_sub(d, q.ypx, q.ymx);
    fe_carry(d);
    fe_add(s, q.ypx, q.ymx);
    fe_carry(s);
    fe_mul(r.X, d, inv2);
    fe_mul(r.Y, s, inv2);
    fe_1(r.Z);
    fe_mul(r.T, r.X, r.Y);
}

__global__ void __launch_bounds__(64) k_ed_bcomb16_build(uint32_t* __restrict__ tab, uint32_t* __restrict__ scratch) {
    const uint32_t* b8 = ED_B_COMB;   // device symbol (its host-side name is not a device address)
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ED_B16_WIN * ED_B16_CHUNKS) return;
    const uint32_t w = g / ED_B16_CHUNKS, chunk = g % ED_B16_CHUNKS, j0 = chunk * 64;
    // P = 2^(16 w) B = 256^(2w) B: entry 1 of window 2w of the radix-256 table
    ge_p3 P, Q;
    ed_niels_to_p3(P, b8 + ((2 * w) * ED_COMB_BENT + 1) * ED_COMB_BSTRIDE);
    ge_cached pc;
    ge_p3_to_cached(pc, P);
    ge_p3_0(Q);
    ge_p1p1 t;
    for (int b = 15; b >= 0; b--) {   // Q = j0 * P
        ge_p3_dbl(t, Q);
        ge_p1p1_to_p3(Q, t);
        if ((j0 >> b) & 1u) {
            ge_add_cached(t, Q, pc, false);
            ge_p1p1_to_p3(Q, t);
        }
    }
    uint32_t* out = tab + ((uint64_t)w * ED_B16_ENT + j0) * 32;
    uint32_t* zp = scratch + (uint64_t)g * 64 * 10;
    fe acc;
    for (int j = 0; j < 64; j++) {   // X, Y, Z of (j0 + j) P into the entry, prefix products of Z
        uint32_t* e = out + j * 32;
#pragma unroll
        for (int q = 0; q < 10; q++) {
            e[q] = Q.X.v[q];
            e[10 + q] = Q.Y.v[q];
            e[20 + q] = Q.Z.v[q];
        }
        if (j == 0) acc = Q.Z;
        else fe_mul(acc, acc, Q.Z);
#pragma unroll
        for (int q = 0; q < 10; q++) zp[j * 10 + q] = acc.v[q];
        ge_add_cached(t, Q, pc, false);
        ge_p1p1_to_p3(Q, t);
    }
    fe inv, d2;
    fe_invert(inv, acc);
    fe_from_c(d2, ED_D2);
    for (int j = 63; j >= 0; j--) {
        uint32_t* e = out + j * 32;
        fe X, Y, Z, zi, x, y;
#pragma unroll
        for (int q = 0; q < 10; q++) {
            X.v[q] = e[q];
            Y.v[q] = e[10 + q];
            Z.v[q] = e[20 + q];
        }
        if (j > 0) {
            fe prev;
#pragma unroll
            for (int q = 0; q < 10; q++) prev.v[q] = zp[(j - 1) * 10 + q];
            fe_mul(zi, inv, prev);
            fe_mul(inv, inv, Z);
        } else {
            zi = inv;
        }
        fe_mul(x, X, zi);
        fe_mul(y, Y, zi);
        ge_niels n;
        fe_add(n.ypx, y, x);
        fe_carry(n.ypx);
        fe_sub(n.ymx, y, x);
        fe_carry(n.ymx);
        fe xy;
        fe_mul(xy, x, y);
        fe_mul(n.xy2d, xy, d2);
#pragma unroll
        for (int q = 0; q < 10; q++) {
            e[q] = n.ypx.v[q];
            e[10 + q] = n.ymx.v[q];
            e[20 + q] = n.xy2d.v[q];
        }
        e[30] = 0;
        e[31] = 0;
    }
}

void launch_ed_bcomb16_build(hipStream_t st, uint32_t* tab, uint32_t* scratch) {
    const uint32_t lanes = ED_B16_WIN * ED_B16_CHUNKS;
    hipLaunchKernelGGL(k_ed_bcomb16_build, dim3((lanes + 63) / 64), dim3(64), 0, st, tab, scratch);
}
uint64_t ed_bcomb16_words() { return (uint64_t)ED_B16_WIN * ED_B16_ENT * 32; }
uint64_t ed_bcomb16_scratch_words() { return (uint64_t)ED_B16_WIN * ED_B16_CHUNKS * 64 * 10; }

// signed radix-2^16 digits of a (< 2^253), two per word as int16
CHIP_DEV void recode16(uint32_t out[8], const uint32_t a[8]) {
    int carry = 0;
#pragma unroll
    for (int d = 0; d < 16; d++) {
        int v = (int)((a[d >> 1] >> (16 * (d & 1))) & 0xffffu) + carry;
        carry = (v + 0x8000) >> 16;
        v -= carry << 16;
        if (d & 1) out[d >> 1] |= (uint32_t)(v & 0xffff) << 16;
        else out[d >> 1] = (uint32_t)(v & 0xffff);
    }
}

// The verify runs in two kernels so that the part that needs no per-key table overlaps the table
// build on the second stream:
//   k_ed_comb_hash   h = SHA-512(R || Abyte || M) mod L and the effective S, recoded
//   k_ed_comb_bhalf  [S]B from the fixed comb (16 madds)
//   k_ed_comb_ahalf  + [h](-A) from the key's table, projective R' to xyz
// hand-off rows (AoS, ED_BMID_W words per slot): [S]B extended (40) | h's biased digit bytes (ED_COMB_ADW
// words, read one word per 4 windows by the table half) | S's radix-2^16 digits (8).  A slot is the comb-list
// position, or with `early` (eager tables, device entry) the signature index: then hash and [S]B run over the
// whole batch before the key prep has finished (it runs on the second stream with the tables), and the table
// half reads row list[p] — one 240-B row per lane, 16-byte loads.
#define ED_BMID_HD 40                                  // h digits
#define ED_BMID_SD (40 + ED_COMB_ADW)                   // S digits
#define ED_BMID_W ((ED_BMID_SD + 8 + 3) & ~3)           // W = 6: 60 words (16-byte aligned rows)
#ifndef ED_BHALF_MINW
#define ED_BHALF_MINW 2   // the [S]B additions allocate 165 VGPRs: 3 waves per SIMD (a bound of 3 spills)
#endif
#ifndef ED_AHALF_MINW
#define ED_AHALF_MINW 3   // waves per SIMD: 134 VGPRs, no scratch (a bound of 4 spills the table offset into the
                          // loop; measured 1.81 vs 1.82-1.87 ms, profiles/r04/ab_early_hash.txt)
#endif
// i2p's Abyte = A.toByteArray() (k_ed25519_key_prep) from the SPKI bytes alone, for a key that decodes: the
// canonical y (the low 255 bits mod p) and the encoding's sign bit, cleared for x = 0 (y = +-1), whose negation
// is itself.  For a key that does not decode the value is never used (its signatures are KEY_INVALID).
CHIP_DEV void ed_abyte_canonical(uint32_t ab[8], const uint8_t* __restrict__ raw) {
    uint32_t y[8];
#pragma unroll
    for (int q = 0; q < 8; q++) y[q] = ld_le32(raw + 4 * q);
    uint32_t bit = y[7] >> 31;
    y[7] &= 0x7fffffffu;
    // y >= p = 2^255 - 19 <=> y[7] = 0x7fffffff, y[1..6] all ones, y[0] >= 0xffffffed: then y - p = y + 19 - 2^255
    bool ones = y[7] == 0x7fffffffu;
#pragma unroll
    for (int q = 1; q < 7; q++) ones = ones && y[q] == 0xffffffffu;
    if (ones && y[0] >= 0xffffffedu) {
        y[0] -= 0xffffffedu;
#pragma unroll
        for (int q = 1; q < 8; q++) y[q] = 0;
    }
    bool pm1 = y[7] == 0x7fffffffu && y[0] == 0xffffffecu;   // p - 1
#pragma unroll
    for (int q = 1; q < 7; q++) pm1 = pm1 && y[q] == 0xffffffffu;
    bool one = y[0] == 1u;
#pragma unroll
    for (int q = 1; q < 8; q++) one = one && y[q] == 0u;
    if (one || pm1) bit = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) ab[q] = y[q];
    ab[7] |= bit << 31;
}
// DIG16 (the split Straus path, k_ed25519_verify_a): h's signed radix-16 digits (8 words) in the row's digit words
template <bool EARLY, bool DIG16 = false>
__global__ void __launch_bounds__(256) k_ed_comb_hash(const uint32_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                                                      uint64_t n, const uint32_t* __restrict__ key_idx,
                                                      const uint32_t* __restrict__ msg_idx,
                                                      const uint8_t* __restrict__ sig_data,
                                                      const uint64_t* __restrict__ sig_off,
                                                      const uint32_t* __restrict__ sig_len,
                                                      const uint8_t* __restrict__ msg_data,
                                                      const uint64_t* __restrict__ msg_off,
                                                      const uint32_t* __restrict__ msg_len, uint64_t n_keys,
                                                      uint64_t n_msgs, const uint8_t* __restrict__ key_data,
                                                      const uint64_t* __restrict__ key_off,
                                                      const uint32_t* __restrict__ key_len,
                                                      const uint32_t* __restrict__ abytes, uint32_t* __restrict__ bmid) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t i, Ab[8];
    if (EARLY) {
        // every signature that can take the Ed25519 path (the bounds k_classify checks before any of its reads)
        if (p >= n) return;
        i = p;
        const uint32_t k = key_idx[i];
        if (k >= n_keys || msg_idx[i] >= n_msgs || sig_len[i] != 64 || key_len[k] != 44) return;
        ed_abyte_canonical(Ab, key_data + key_off[k] + 12);
    } else {
        if (p >= *cnt) return;
        i = list[p];
        const uint32_t k = key_idx[i];
#pragma unroll
        for (int q = 0; q < 8; q++) Ab[q] = abytes[(uint64_t)k * 8 + q];
    }
    const uint32_t mi = msg_idx[i];
    const uint8_t* sig = sig_data + sig_off[i];
    uint32_t R[8], S[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        R[q] = ld_le32(sig + 4 * q);
        S[q] = ld_le32(sig + 32 + 4 * q);
    }
    uint32_t hx[16], h[8], s[8];
    ed_challenge(hx, R, Ab, msg_data + msg_off[mi], msg_len[mi], sig);
    sc_reduce512(h, hx);
    ed_effective_s(s, S);
    uint32_t db[8];
    recode16(db, s);
    uint32_t* row = bmid + (uint64_t)p * ED_BMID_W;
    if (DIG16) {
        uint32_t ea[8];
        sc_recode16(ea, h);
#pragma unroll
        for (int q = 0; q < 8; q++) row[ED_BMID_HD + q] = ea[q];
    } else {
        uint32_t da[ED_COMB_ADW];
        recode_bytes<ED_COMB_W, ED_COMB_AWIN>(da, h);
#pragma unroll
        for (int q = 0; q < ED_COMB_ADW; q++) row[ED_BMID_HD + q] = da[q];
    }
#pragma unroll
    for (int q = 0; q < 8; q++) row[ED_BMID_SD + q] = db[q];
}

// k_ed_comb_bhalf: [S]B from the fixed radix-2^16 comb, 16 mixed additions; [S]B (extended) into the row's words 0..39
__global__ void __launch_bounds__(256, ED_BHALF_MINW) k_ed_comb_bhalf(const uint32_t* __restrict__ cnt, uint64_t n_early,
                                                                      const uint32_t* __restrict__ b16,
                                                                      uint32_t* __restrict__ bmid) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    // early: every slot of the batch (a slot the hash skipped holds stale digits: any int16 digit stays inside
    // the radix-2^16 table, and the row is never read back)
    if (p >= (n_early ? n_early : (uint64_t)*cnt)) return;
    uint32_t* row = bmid + (uint64_t)p * ED_BMID_W;
    const uint32_t* sdig = row + ED_BMID_SD;   // digit word j at sdig[j]
    // [S]B: one mixed (affine Niels) addition per radix-2^16 window.  Window 0 from the identity needs no
    // multiplication: identity + q = (q+ - q-, q+ + q-, 2, 2) in completed form.  The loop carries only t.
    ge_p1p1 t;
    fe qp, qm, xy2d, z2;
    uint32_t cur = sdig[0];
    {
        const int d = (int)(int16_t)cur;
        const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
        ed_load_niels_signed(qp, qm, xy2d, b16 + (uint64_t)ad * 32, d < 0);
        fe_sub(t.X, qp, qm);
        fe_add(t.Y, qp, qm);
        fe_0(t.Z);
        t.Z.v[0] = 2;
        t.T = t.Z;
    }
    ge_p3 u;
    // window w: the signed digit d of S, entry |d| of the window's table; the accumulator carries 2Z
    auto window = [&](uint32_t w, int d) {
        const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
        ed_load_niels_signed(qp, qm, xy2d, b16 + ((uint64_t)w * ED_B16_ENT + ad) * 32, d < 0);
        fe_mul(u.X, t.X, t.T);
        fe_mul(u.Y, t.Z, t.Y);
        fe_mul2(z2, t.Z, t.T);
        fe_mul(u.T, t.X, t.Y);
        ge_madd_signed(t, u, z2, qp, qm, xy2d, (uint32_t)(d >> 31));
    };
    window(1, (int)(int16_t)(cur >> 16));
#pragma unroll 1
    for (uint32_t wd = 1; wd < ED_B16_WIN / 2; wd++) {   // two windows per digit word, read as it is needed
        cur = sdig[wd];
        window(2 * wd, (int)(int16_t)cur);
        window(2 * wd + 1, (int)(int16_t)(cur >> 16));
    }
    // handed over completed (X, Y, Z, T): the table half's first window converts it like every other
#pragma unroll
    for (int q = 0; q < 10; q++) {
        row[q] = t.X.v[q];
        row[10 + q] = t.Y.v[q];
        row[20 + q] = t.Z.v[q];
        row[30 + q] = t.T.v[q];
    }
}

// AFF: the key's rows are affine Niels (ED_COMB_ROW_A, tables kept across batches) instead of cached ones
template <bool AFF>
__global__ void __launch_bounds__(256, ED_AHALF_MINW) k_ed_comb_ahalf(const uint32_t* __restrict__ list,
                                                                      const uint32_t* __restrict__ ctr,
                                                       const uint32_t* __restrict__ key_idx,
                                                       const int32_t* __restrict__ key_slot,
                                                       const uint32_t* __restrict__ ctab,
                                                       const uint32_t* __restrict__ bmid, uint32_t* __restrict__ xyz,
                                                       uint64_t cap, uint32_t early, uint32_t base,
                                                       uint32_t* __restrict__ flist) {
    const uint32_t ncomb = ctr[ED_CTR_NCOMB];
    const uint32_t p = xcd_block(blockIdx.x, (ncomb + 255) / 256) * blockDim.x + threadIdx.x;
    if (p >= ncomb) return;
    const uint32_t i = list[p];
    const uint32_t k = key_idx[i];
    // digit d of window w reads row |d| of the window, signed
    // the key's table as a 32-bit word offset from the uniform base (<= 2^32 words of tables): one VGPR, not two
    constexpr uint32_t ED_COMB_ROW = AFF ? ED_COMB_ROW_A : ED_COMB_ROW_C;
    const uint32_t toff = (uint32_t)key_slot[k] * (uint32_t)(AFF ? ED_COMB_KEY_WORDS_A : ED_COMB_KEY_WORDS_C);
    // the row as a 32-bit word offset from the uniform base (slot * ED_BMID_W < 2^32): one VGPR through the loop;
    // p itself is rebuilt after the loop from the wave's first position (an SGPR) and the lane id
    const uint32_t ro = (early ? i : p) * (uint32_t)ED_BMID_W;
    const uint32_t pwave = __builtin_amdgcn_readfirstlane(p & ~63u);
    // + [h](-A): one addition per window from the key's signed-multiple rows (extended coordinates, unified =
    // complete formulas), starting from [S]B in completed form; the loop carries only the completed point t
    ge_p1p1 t;
    {
        const uint32_t* r = bmid + ro;
#pragma unroll
        for (int q = 0; q < 10; q++) {
            t.X.v[q] = r[q];
            t.Y.v[q] = r[10 + q];
            t.Z.v[q] = r[20 + q];
            t.T.v[q] = r[30 + q];
        }
    }
    // h's digit words parked in LDS ([word][thread]): the loop reads one every 4 windows at an address rebuilt
    // from the wave's base (an SGPR) and the lane id, so no per-lane offset stays live through the loop
    __shared__ uint32_t s_hd[ED_COMB_ADW][256];
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u);
#pragma unroll
    for (int q = 0; q < ED_COMB_ADW; q++) s_hd[q][wbase + lane] = bmid[ro + ED_BMID_HD + q];
    auto hd_word = [&](uint32_t j) {
        uint32_t l;   // the lane id recomputed at each use (volatile: not hoisted into a register kept live)
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
        return s_hd[j][wbase + l];
    };
    ge_p3 u;
    uint32_t cur = 0;
    if constexpr (AFF) {
    // affine Niels rows: a mixed addition (3 multiplications) after a conversion that yields 2Z directly
    fe qp, qm, xy2d, z2;
#pragma unroll 1
    for (uint32_t w = 0; w < ED_COMB_AWIN; w++) {
        if ((w & 3u) == 0) cur = hd_word(w >> 2);
        const int d = (int)((cur >> (8 * (w & 3u))) & 0xffu) - ED_COMB_ABIAS;
        fe_mul(u.X, t.X, t.T);
        fe_mul(u.Y, t.Z, t.Y);
        fe_mul2(z2, t.Z, t.T);
        fe_mul(u.T, t.X, t.Y);
        ed_load_niels_signed(qp, qm, xy2d, ctab + (toff + (w * ED_COMB_AENT + (uint32_t)(d < 0 ? -d : d)) * ED_COMB_ROW),
                             d < 0);
        ge_madd_signed(t, u, z2, qp, qm, xy2d, (uint32_t)(d >> 31));
    }
    } else {
    ge_cached ca;
#pragma unroll 1
    for (uint32_t w = 0; w < ED_COMB_AWIN; w++) {
        if ((w & 3u) == 0) cur = hd_word(w >> 2);
        const int d = (int)((cur >> (8 * (w & 3u))) & 0xffu) - ED_COMB_ABIAS;
        ge_p1p1_to_p3(u, t);
        ed_load_row_signed(ca, ctab + (toff + (w * ED_COMB_AENT + (uint32_t)(d < 0 ? -d : d)) * ED_COMB_ROW), d < 0);
        ge_add_row(t, u, ca, (uint32_t)(d >> 31));
    }
    }
    // projective R' = (X : Y : Z), stored structure-of-arrays for the finish kernel
    fe X, Y, Z;
    fe_mul(X, t.X, t.T);
    fe_mul(Y, t.Z, t.Y);
    fe_mul(Z, t.Z, t.T);
    const uint32_t pe = pwave + __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) + base;
    if (flist) flist[pe] = base + list[pe - base];   // deferred finish: the position's signature in the whole batch
#pragma unroll
    for (int q = 0; q < 10; q++) {
        xyz[(uint64_t)q * cap + pe] = X.v[q];
        xyz[(uint64_t)(10 + q) * cap + pe] = Y.v[q];
        xyz[(uint64_t)(20 + q) * cap + pe] = Z.v[q];
    }
}

// ---- finish: batched inversion of Z, canonical encoding, compare with R ----
// Lane l owns positions l, l + lanes, l + 2 lanes, ... (coalesced SoA reads).  Z != 0 always: the
// unified Edwards formulas are complete for a = -1, d non-square, and A, B are curve points.
CHIP_DEV void ld_fe_soa(fe& f, const uint32_t* __restrict__ base, uint64_t cap, uint64_t p) {
#pragma unroll
    for (int q = 0; q < 10; q++) f.v[q] = base[(uint64_t)q * cap + p];
}
#ifndef ED_FINISH_WAVES
#define ED_FINISH_WAVES 4   // waves per SIMD the finish's registers must leave room for: 4 (128 VGPRs, 10 spilled; the
                            // compiler's 136 = 3 waves): cfg2 263.4-266.2 vs 260.5-263.2M in 3 same-box rounds
                            // (profiles/r05/ab_r05l.txt; [S]B at 3 waves was slower, 250-256M)
#endif
// ALL (the deferred finish of a chunked host batch): positions [0, nall) over every chunk's R', list = flist (the
// signature of each position in the whole batch, ~0 where a chunk left the position empty: skipped, its Z counted as 1)
template <bool ALL>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ED_FINISH_WAVES))) k_ed_comb_finish(const uint32_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                                                        const uint8_t* __restrict__ sig_data,
                                                        const uint64_t* __restrict__ sig_off,
                                                        const uint32_t* __restrict__ xyz, uint32_t* __restrict__ zpre,
                                                        uint64_t cap, uint8_t* __restrict__ status, uint32_t g,
                                                        uint32_t nall) {
    const uint32_t n = ALL ? nall : *cnt;
    const uint32_t lanes = (n + g - 1) / g;
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= lanes) return;
    const uint32_t ne = min(g, (n - l + lanes - 1) / lanes);
    const uint32_t* Zs = xyz + 20 * cap;
    fe acc, z;
    bool any = false;
    for (uint32_t e = 0; e < ne; e++) {
        const uint64_t p = l + (uint64_t)e * lanes;
        if (ALL) {
            if (list[p] != 0xffffffffu) {
                ld_fe_soa(z, Zs, cap, p);
                if (!any) acc = z;
                else fe_mul(acc, acc, z);
                any = true;
            } else if (!any) {
                fe_1(acc);
            }
        } else {
            ld_fe_soa(z, Zs, cap, p);
            if (e == 0) acc = z;
            else fe_mul(acc, acc, z);
        }
#pragma unroll
        for (int q = 0; q < 10; q++) zpre[(uint64_t)q * cap + p] = acc.v[q];
    }
    if (ALL && !any) return;
    fe inv;
    fe_invert(inv, acc);
    for (int e = (int)ne - 1; e >= 0; e--) {
        const uint64_t p = l + (uint64_t)e * lanes;
        if (ALL && list[p] == 0xffffffffu) continue;
        fe zi;
        if (e > 0) {
            fe prev;
            ld_fe_soa(prev, zpre, cap, p - lanes);
            fe_mul(zi, inv, prev);
            ld_fe_soa(z, Zs, cap, p);
            fe_mul(inv, inv, z);
        } else {
            zi = inv;
        }
        fe X, Y, x, y;
        ld_fe_soa(X, xyz, cap, p);
        ld_fe_soa(Y, xyz + 10 * cap, cap, p);
        fe_mul(x, X, zi);
        fe_mul(y, Y, zi);
        uint32_t enc[8];
        fe_tobytes(enc, y);
        enc[7] |= fe_isnegative(x) << 31;
        const uint32_t i = list[p];
        const uint8_t* sig = sig_data + sig_off[i];
        bool eq = true;
#pragma unroll
        for (int q = 0; q < 8; q++) eq = eq && (enc[q] == ld_le32(sig + 4 * q));
        status[i] = eq ? CHIP_VALID : CHIP_INVALID;
    }
}

// ---------------------------------------------------------------------------------------
static inline uint32_t nblk(uint64_t n, uint32_t bs) { return (uint32_t)((n + bs - 1) / bs); }

void launch_ed_comb_plan(hipStream_t st, uint64_t n, uint64_t n_keys, const uint32_t* ed_list,
                         const uint32_t* ed_count, const chip_sig_batch* b, const KeyMeta* meta, const EdCombWs& w,
                         bool partition) {
    if (!n || !n_keys) return;
    if (!partition) {
        hipLaunchKernelGGL(k_ed_comb_slots, dim3(nblk(n_keys, 256)), dim3(256), 0, st, n_keys, meta, w.key_count,
                           w.min_sigs, w.max_slots, w.eager, w.key_slot, w.key_base, w.slot_key, w.ctr);
        return;
    }
    hipLaunchKernelGGL(k_ed_comb_partition, dim3(nblk(n, 256)), dim3(256), 0, st, ed_list, ed_count, b->key_idx,
                       w.key_slot, w.key_base, w.key_rank, w.comb_list, w.straus_list, w.ctr,
                       w.eager ? 0u : w.min_total, w.max_slots);
}

void launch_ed_comb_build(hipStream_t st, uint64_t n, uint64_t n_keys, const KeyMeta* meta, const EdCombWs& w) {
    if (!n || !n_keys || !w.max_slots) return;
#if ED_CHAIN_PAIR
    hipLaunchKernelGGL(k_ed_comb_chain2, dim3(nblk((uint64_t)w.max_slots * 2, 64)), dim3(64), 0, st, w.ctr, w.max_slots,
                       w.eager, meta, w.slot_key, w.nega, w.ctab, w.skip, w.affine);
#else
    hipLaunchKernelGGL(k_ed_comb_chain, dim3(nblk(w.max_slots, 64)), dim3(64), 0, st, w.ctr, w.max_slots, w.eager, meta,
                       w.slot_key, w.nega, w.ctab, w.skip, w.affine);
#endif
    if (!w.affine) {
        hipLaunchKernelGGL(k_ed_comb_fill, dim3(nblk((uint64_t)w.max_slots * ED_COMB_AWIN * ED_FILL_SPLIT, 256)), dim3(256),
                           0, st, w.ctr, w.max_slots, w.eager, meta, w.ctab, w.skip);
        return;
    }
    const uint64_t lanes = (uint64_t)w.max_slots * ED_COMB_AWIN;
    uint32_t* zprod = w.fz;
    uint32_t* zinv = w.fz + lanes * 10;
    hipLaunchKernelGGL(k_ed_comb_fill_a, dim3(nblk(lanes, 256)), dim3(256), 0, st, w.ctr, w.max_slots, w.eager, meta,
                       w.ctab, zprod, w.skip);
    hipLaunchKernelGGL(k_ed_comb_zinv, dim3(nblk((lanes + ED_COMB_ZG - 1) / ED_COMB_ZG, 64)), dim3(64), 0, st, w.ctr,
                       w.max_slots, w.eager, zprod, zinv, w.skip);
    hipLaunchKernelGGL(k_ed_comb_fill_b, dim3(nblk(lanes, 256)), dim3(256), 0, st, w.ctr, w.max_slots, w.eager, meta,
                       w.ctab, zinv, w.skip);
}

uint64_t ed_comb_bmid_words() { return ED_BMID_W; }

void launch_ed_comb_bhalf(hipStream_t st, uint64_t n, const chip_sig_batch* b, const uint32_t* abytes,
                          const EdCombWs& w, int part) {
    if (!n || !w.max_slots) return;
    if (part & 2) {   // [S]B only (its hash launched before)
        hipLaunchKernelGGL(k_ed_comb_bhalf, dim3(nblk(n, 256)), dim3(256), 0, st, w.ctr + ED_CTR_NCOMB, w.early ? n : 0,
                           w.bcomb16, w.bmid);
        return;
    }
    if (w.early)
        hipLaunchKernelGGL(k_ed_comb_hash<true>, dim3(nblk(n, 256)), dim3(256), 0, st, w.comb_list, w.ctr + ED_CTR_NCOMB, n,
                           b->key_idx,
                           b->msg_idx, b->sig_data, b->sig_off, b->sig_len, b->msg_data, b->msg_off, b->msg_len,
                           b->n_keys, b->n_msgs, b->key_data, b->key_off, b->key_len, abytes, w.bmid);
    else
        hipLaunchKernelGGL(k_ed_comb_hash<false>, dim3(nblk(n, 256)), dim3(256), 0, st, w.comb_list, w.ctr + ED_CTR_NCOMB, n,
                           b->key_idx, b->msg_idx, b->sig_data, b->sig_off, b->sig_len, b->msg_data, b->msg_off,
                           b->msg_len, b->n_keys, b->n_msgs, b->key_data, b->key_off, b->key_len, abytes, w.bmid);
    if (part & 1) return;   // the hash only
    hipLaunchKernelGGL(k_ed_comb_bhalf, dim3(nblk(n, 256)), dim3(256), 0, st, w.ctr + ED_CTR_NCOMB, w.early ? n : 0,
                       w.bcomb16, w.bmid);
}
void launch_ed_comb_ahalf(hipStream_t st, uint64_t n, const chip_sig_batch* b, const EdCombWs& w) {
    if (!n || !w.max_slots) return;
    const uint32_t blocks = (nblk(n, 256) + 7) & ~7u;   // multiple of 8 for the XCD remap
    auto kern = w.affine ? k_ed_comb_ahalf<true> : k_ed_comb_ahalf<false>;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, st, w.comb_list, w.ctr, b->key_idx, w.key_slot, w.ctab, w.bmid,
                       w.xyz, w.xyz_cap ? w.xyz_cap : (uint64_t)n, w.early, w.flist ? w.xyz_base : 0u, w.flist);
}

void launch_ed_comb_finish(hipStream_t st, uint64_t n, const chip_sig_batch* b, const EdCombWs& w, uint8_t* status) {
    if (!n || !w.max_slots) return;
    // signatures per inversion: ED_FIN_G (16) for 2^20-signature batches; fewer for smaller ones (the chunks of
    // a host batch), whose lanes would otherwise be too few to fill the chip (each lane's chain is serial):
    // at least min_lanes lanes (g halves below that), 4 <= g <= ED_FIN_G
    uint32_t g = ED_FIN_G;
    // 32768 (CHIP_FINISH_MIN_LANES overrides): the host pipeline's ~292k-signature chunks take g = 8 (g = 4 at 49152):
    // pinned cfg2 172.0-172.5 -> 174.6-176.5M, pageable 169.8-170.9 -> 171.9-172.4M (profiles/r05/ab_r05s.txt)
    static const uint32_t min_lanes = [] {
        const char* e = getenv("CHIP_FINISH_MIN_LANES");
        return e ? (uint32_t)strtoul(e, nullptr, 10) : 32768u;
    }();
    while (g > 4 && n / g < min_lanes) g >>= 1;
    hipLaunchKernelGGL(k_ed_comb_finish<false>, dim3(nblk((n + g - 1) / g, 256)), dim3(256), 0, st, w.comb_list,
                       w.ctr + ED_CTR_NCOMB, b->sig_data, b->sig_off, w.xyz, w.zpre, w.xyz_cap ? w.xyz_cap : (uint64_t)n, status, g, 0u);
}
void launch_ed_comb_finish_all(hipStream_t st, uint64_t n, const uint8_t* sig_data, const uint64_t* sig_off,
                               const EdCombWs& w, uint8_t* status) {
    if (!n || !w.flist) return;
    const uint32_t g = ED_FIN_G;
    hipLaunchKernelGGL(k_ed_comb_finish<true>, dim3(nblk((n + g - 1) / g, 256)), dim3(256), 0, st, w.flist, w.ctr + ED_CTR_NCOMB,
                       sig_data, sig_off, w.xyz, w.zpre, w.xyz_cap, status, g, (uint32_t)n);
}

// The split Straus path (cold keys: few signatures per key, no per-key comb): the table-free work of the comb path —
// the challenge hash with h's signed radix-16 digits and [S]B from the radix-2^16 comb of B (16 mixed additions instead
// of the 32 radix-256 ones that ride on the Straus doublings) — then k_ed25519_verify_a's 252 doublings + 64 additions
// of h (-A) from the key's radix-16 table, + [S]B, and the batched-inversion finish (one inversion per g signatures
// instead of one per signature).  Positions p < *cnt of `list`; rows, R' and prefix products are this path's own.
void launch_ed_straus_front(hipStream_t st, uint64_t n, const chip_sig_batch* b, const uint32_t* bcomb16, uint32_t* bmid) {
    if (!n) return;
    auto hash = k_ed_comb_hash<true, true>;
    hipLaunchKernelGGL(hash, dim3(nblk(n, 256)), dim3(256), 0, st, nullptr, nullptr, n, b->key_idx, b->msg_idx,
                       b->sig_data, b->sig_off, b->sig_len, b->msg_data, b->msg_off, b->msg_len, b->n_keys, b->n_msgs,
                       b->key_data, b->key_off, b->key_len, nullptr, bmid);
    hipLaunchKernelGGL(k_ed_comb_bhalf, dim3(nblk(n, 256)), dim3(256), 0, st, nullptr, n, bcomb16, bmid);
}
void launch_ed_straus_split(hipStream_t st, uint64_t n, const uint32_t* list, const uint32_t* cnt, const chip_sig_batch* b,
                            const uint32_t* abytes, const uint32_t* table, const uint32_t* bcomb16, uint32_t* bmid,
                            uint32_t* xyz, uint32_t* zpre, uint8_t* status, bool early) {
    if (!n) return;
    if (!early) {
        auto hash = k_ed_comb_hash<false, true>;
        hipLaunchKernelGGL(hash, dim3(nblk(n, 256)), dim3(256), 0, st, list, cnt, n, b->key_idx, b->msg_idx,
                           b->sig_data, b->sig_off, b->sig_len, b->msg_data, b->msg_off, b->msg_len, b->n_keys, b->n_msgs,
                           b->key_data, b->key_off, b->key_len, abytes, bmid);
        hipLaunchKernelGGL(k_ed_comb_bhalf, dim3(nblk(n, 256)), dim3(256), 0, st, cnt, (uint64_t)0, bcomb16, bmid);
    }
    launch_ed25519_verify_a(st, n, list, cnt, b->key_idx, table, bmid, ED_BMID_W, ED_BMID_HD, xyz, early);
    uint32_t g = ED_FIN_G;
    while (g > 4 && n / g < 32768u) g >>= 1;
    hipLaunchKernelGGL(k_ed_comb_finish<false>, dim3(nblk((n + g - 1) / g, 256)), dim3(256), 0, st, list, cnt,
                       b->sig_data, b->sig_off, xyz, zpre, n, status, g, 0u);
}
