// txid.hip — K3: WireTransaction.id recomputation (SHA-256 Merkle root over component groups).
//
//   id          = MerkleRoot(groupHashes)                         WireTransaction.kt:63,139
//   groupHashes = g in 0..maxGroup: present ? MerkleRoot(leaves of g) : allOnesHash   :146-155
//   leaf(g,i)   = SHA256(SHA256(nonce(g,i) || bytes))             CryptoUtils.kt:220
//   nonce(g,i)  = SHA256(SHA256(salt || BE32 g || BE32 i))         CryptoUtils.kt:233
//   MerkleRoot  = pad with zeroHash to 2^k; 1 leaf -> the leaf; nodes SHA256(l || r)  MerkleTree.kt:27-66
//
// One lane per transaction (the unit the caller batches; no cross-lane divergence for
// same-shaped transactions).  Fast path (groups in ascending ordinal order, ordinals < 16, <= 16 components each
// (TX_LEVELS): what createComponentGroups produces for ordinary transactions): every tree is reduced in LDS stacks as its
// leaves arrive (a binary-counter stack per tree, padding subtrees from the constant zero-hash chain), so
// nothing but the id is written.  Otherwise the leaf and group-root levels are reduced in place in a
// per-tx scratch slab in HBM (64 slots x 32 B; group ordinals must be < 64).
#include <algorithm>
#include "sha2_dev.hpp"
#include "runtime.hpp"

#define TX_MAX_GROUPS 64

// N big-endian words from p (any alignment): N (+1 when unaligned) independent aligned dword loads,
// funnel-shifted — one batch of loads per block instead of a dependent chain of byte gathers.  The
// extra word shares its aligned dword with the last wanted byte, so it never crosses a page.
template <int N>
CHIP_DEV void load_be_words(uint32_t* w, const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t sh = (uint32_t)(a & 3u);
    const uint32_t* ap = reinterpret_cast<const uint32_t*>(a - sh);
    uint32_t d[N + 1];
#pragma unroll
    for (int k = 0; k < N; k++) d[k] = ap[k];
    d[N] = sh ? ap[N] : 0u;
#pragma unroll
    for (int k = 0; k < N; k++) w[k] = __builtin_bswap32(__builtin_amdgcn_alignbyte(d[k + 1], d[k], sh));
}

// SHA256(SHA256(prefix32 || bytes[0:len]))  (componentHash with prefix = nonce)
CHIP_DEV void sha256d_prefixed(uint32_t out[8], const uint32_t pre[8], const uint8_t* p, uint32_t len) {
    uint32_t H[8], w[16];
    sha256_init(H);
    const uint64_t total = 32ull + len;
    const uint32_t nblocks = (uint32_t)((total + 9 + 63) / 64);
    for (uint32_t b = 0; b < nblocks; b++) {
        const int64_t q0 = (int64_t)b * 64 - 32;   // first component byte of this block
        if (b > 0 && q0 + 64 <= (int64_t)len) {
            load_be_words<16>(w, p + q0);           // whole block inside the component
        } else if (b == 0 && len >= 32) {
#pragma unroll
            for (int j = 0; j < 8; j++) w[j] = pre[j];
            load_be_words<8>(w + 8, p);
        } else {
#pragma unroll
            for (int j = 0; j < 16; j++) {
                if (b == 0 && j < 8) w[j] = pre[j];
                else w[j] = comp_word(p, len, q0 + 4 * j);
            }
        }
        if (b == nblocks - 1) {
            w[14] = (uint32_t)((total * 8) >> 32);
            w[15] = (uint32_t)(total * 8);
        }
        sha256_compress(H, w);
    }
    // second hash over the 32-byte digest: one block
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = H[j];
    w[8] = 0x80000000u;
#pragma unroll
    for (int j = 9; j < 15; j++) w[j] = 0;
    w[15] = 256;
    sha256_init(out);
    sha256_compress(out, w);
}

// computeNonce: SHA256(SHA256(salt || BE32 g || BE32 i))
CHIP_DEV void compute_nonce(uint32_t out[8], const uint32_t salt_be[8], uint32_t g, uint32_t i) {
    uint32_t H[8], w[16];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = salt_be[j];
    w[8] = g;
    w[9] = i;
    w[10] = 0x80000000u;
#pragma unroll
    for (int j = 11; j < 15; j++) w[j] = 0;
    w[15] = 40 * 8;
    sha256_init(H);
    sha256_compress(H, w);
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = H[j];
    w[8] = 0x80000000u;
#pragma unroll
    for (int j = 9; j < 15; j++) w[j] = 0;
    w[15] = 256;
    sha256_init(out);
    sha256_compress(out, w);
}

// hashConcat: SHA256(l || r)
CHIP_DEV void hash_concat(uint32_t out[8], const uint32_t l[8], const uint32_t r[8]) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        w[j] = l[j];
        w[8 + j] = r[j];
    }
    sha256_init(out);
    sha256_compress(out, w);
    w[0] = 0x80000000u;
#pragma unroll
    for (int j = 1; j < 15; j++) w[j] = 0;
    w[15] = 512;
    sha256_compress(out, w);
}

CHIP_DEV void ld8(uint32_t v[8], const uint32_t* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
CHIP_DEV void st8(uint32_t* p, const uint32_t v[8]) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(v[0], v[1], v[2], v[3]);
    q[1] = make_uint4(v[4], v[5], v[6], v[7]);
}

// in-place Merkle root over slots[0..n) (MerkleTree.getMerkleTree): leaves are padded with
// zeroHash to m = 2^ceil(log2 n); a node whose whole subtree is padding equals Z_k (Z_0 = zeroHash,
// Z_{k+1} = SHA256(Z_k || Z_k)) and is produced without re-hashing the padding.  For the top
// tree (top=true) a leaf j < n whose group is absent is allOnesHash (WireTransaction.kt:146-155).
CHIP_DEV void merkle_inplace(uint32_t root[8], uint32_t* slots, uint32_t n, uint32_t present_mask_lo,
                             uint32_t present_mask_hi, bool top) {
    if (n == 1) {
        if (top && !(present_mask_lo & 1u)) {
#pragma unroll
            for (int j = 0; j < 8; j++) root[j] = 0xffffffffu;
        } else {
            ld8(root, slots);
        }
        return;
    }
    uint32_t m = 1;
    while (m < n) m <<= 1;
    uint32_t cnt = n;   // nodes at this level with at least one real leaf below them
    uint32_t z[8];      // Z_k for the current level
#pragma unroll
    for (int q = 0; q < 8; q++) z[q] = 0;
    bool first = true;
    while (m > 1) {
        const uint32_t half = m >> 1;
        const uint32_t live = (cnt + 1) >> 1;
        for (uint32_t j = 0; j < live; j++) {
            uint32_t l[8], r[8], h[8];
            const uint32_t a = 2 * j, b = 2 * j + 1;
            // a < cnt always
            const bool pa = !(top && first) || ((a < 32 ? (present_mask_lo >> a) : (present_mask_hi >> (a - 32))) & 1u);
            if (pa) ld8(l, slots + 8 * a);
            else {
#pragma unroll
                for (int q = 0; q < 8; q++) l[q] = 0xffffffffu;
            }
            if (b < cnt) {
                const bool pb = !(top && first) || ((b < 32 ? (present_mask_lo >> b) : (present_mask_hi >> (b - 32))) & 1u);
                if (pb) ld8(r, slots + 8 * b);
                else {
#pragma unroll
                    for (int q = 0; q < 8; q++) r[q] = 0xffffffffu;
                }
            } else {
#pragma unroll
                for (int q = 0; q < 8; q++) r[q] = z[q];
            }
            hash_concat(h, l, r);
            st8(slots + 8 * j, h);
        }
        if (live < half) {   // next level's padding value
            uint32_t h[8];
            hash_concat(h, z, z);
#pragma unroll
            for (int q = 0; q < 8; q++) z[q] = h[q];
        }
        cnt = live;
        m = half;
        first = false;
    }
    ld8(root, slots);
}

// Z_k: the root of a subtree of 2^k zeroHash padding leaves (Z_0 = zeroHash, Z_{k+1} = SHA256(Z_k || Z_k))
__constant__ uint32_t k_zhash[8][8] = {
    {0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u},
    {0xf5a5fd42u, 0xd16a2030u, 0x2798ef6eu, 0xd309979bu, 0x43003d23u, 0x20d9f0e8u, 0xea9831a9u, 0x2759fb4bu},
    {0xdb56114eu, 0x00fdd4c1u, 0xf85c892bu, 0xf35ac9a8u, 0x9289aaecu, 0xb1ebd0a9u, 0x6cde606au, 0x748b5d71u},
    {0xc78009fdu, 0xf07fc56au, 0x11f12237u, 0x0658a353u, 0xaaa542edu, 0x63e44c4bu, 0xc15ff4cdu, 0x105ab33cu},
    {0x536d9883u, 0x7f2dd165u, 0xa55d5eeau, 0xe9148595u, 0x4472d56fu, 0x246df256u, 0xbf3cae19u, 0x352a123cu},
    {0x9efde052u, 0xaa15429fu, 0xae05bad4u, 0xd0b1d7c6u, 0x4da64d03u, 0xd7a1854au, 0x588c2cb8u, 0x430c0d30u},
    {0xd88ddfeeu, 0xd400a875u, 0x5596b219u, 0x42c1497eu, 0x114c302eu, 0x6118290fu, 0x91e67729u, 0x76041fa1u},
    {0x87eb0ddbu, 0xa57e35f6u, 0xd2866738u, 0x02a4af59u, 0x75e22506u, 0xc7cf4c64u, 0xbb6be5eeu, 0x11527f2cu}};

// A Merkle tree built as its leaves arrive (MerkleTree.getMerkleTree over leaves padded with zeroHash to a
// power of two): stack level l holds the root of a complete subtree of 2^l leaves when bit l of `count` is
// set.  The stack lives in LDS, word q of level l at s[(8 l + q) * TX_BLOCK] (this lane's column: no bank
// conflicts), so one hash call site serves every level and nothing but the id reaches HBM.
#define TX_BLOCK 64   // k_txid's block: one wave (the LDS stacks below are per lane)
#define TX_LEVELS 4   // fast path: <= 16 components per group, group ordinals < 16 (stacks of 5 levels)
struct MerkleLds {
    uint32_t* s;
    uint32_t count;
    CHIP_DEV void init(uint32_t* base) {
        s = base;
        count = 0;
    }
    CHIP_DEV void ld(uint32_t v[8], uint32_t l) const {
#pragma unroll
        for (int q = 0; q < 8; q++) v[q] = s[(8 * l + q) * TX_BLOCK];
    }
    CHIP_DEV void st(uint32_t l, const uint32_t v[8]) {
#pragma unroll
        for (int q = 0; q < 8; q++) s[(8 * l + q) * TX_BLOCK] = v[q];
    }
    CHIP_DEV void push(const uint32_t leaf[8]) {
        uint32_t node[8], left[8];
#pragma unroll
        for (int q = 0; q < 8; q++) node[q] = leaf[q];
        uint32_t l = 0;
        while ((count >> l) & 1u) {
            ld(left, l);
            hash_concat(node, left, node);
            l++;
        }
        st(l, node);
        count++;
    }
    // the root (count >= 1): a single leaf is the root itself; otherwise the partial subtrees are closed with
    // padding subtrees of zeroHash leaves (Z_l from the constant chain)
    CHIP_DEV void root(uint32_t out[8]) const {
        const uint32_t n = count;
        uint32_t d = 0;
        while ((1u << d) < n) d++;
        if (n == (1u << d)) {
            ld(out, d);
            return;
        }
        bool have = false;
        uint32_t left[8], right[8];
        for (uint32_t l = 0; l < d; l++) {
            const bool bit = (n >> l) & 1u;
            if (!have && !bit) continue;
            if (bit) {
                ld(left, l);
                if (!have) {
#pragma unroll
                    for (int q = 0; q < 8; q++) right[q] = k_zhash[l][q];
                } else {
#pragma unroll
                    for (int q = 0; q < 8; q++) right[q] = out[q];
                }
            } else {
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    left[q] = out[q];
                    right[q] = k_zhash[l][q];
                }
            }
            hash_concat(out, left, right);
            have = true;
        }
    }
};
#define TX_FAST_GROUP_LEAVES (1u << TX_LEVELS)
#define TX_FAST_TOP (1u << TX_LEVELS)

// the fast path's precondition: groups in strictly ascending ordinal order, ordinals < 16, each of <= 16 components
// (TX_FAST_GROUP_LEAVES = TX_FAST_TOP = 2^TX_LEVELS)
CHIP_DEV bool txid_fast_ok(const uint32_t* __restrict__ grp, uint64_t a, uint64_t e) {
    uint32_t prev = 0xffffffffu, run = 0;
    for (uint64_t k = a; k < e; k++) {
        const uint32_t g = grp[k];
        if (g == prev) {
            if (++run > TX_FAST_GROUP_LEAVES) return false;
        } else {
            if ((prev != 0xffffffffu && g <= prev) || g >= TX_FAST_TOP) return false;
            prev = g;
            run = 1;
        }
    }
    return true;
}

__global__ void __launch_bounds__(TX_BLOCK) k_txid(uint64_t ntx, const uint8_t* __restrict__ salts,
                                              const uint64_t* __restrict__ start, const uint32_t* __restrict__ grp,
                                              const uint32_t* __restrict__ internal, const uint8_t* __restrict__ data,
                                              const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
                                              uint8_t* __restrict__ ids, uint32_t* __restrict__ leafbuf,
                                              uint32_t* __restrict__ slots_all) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx) return;
    const uint64_t a = start[t], e = start[t + 1];
    uint32_t* slots = slots_all + t * (TX_MAX_GROUPS * 8);
    uint32_t id[8];
    if (a == e) {
#pragma unroll
        for (int j = 0; j < 8; j++) id[j] = 0;
    } else {
        uint32_t salt[8];
        const uint8_t* sp = salts + 32 * t;
#pragma unroll
        for (int j = 0; j < 8; j++) salt[j] = ld_be32(sp + 4 * j);
        if (txid_fast_ok(grp, a, e)) {
            __shared__ uint32_t lds[2 * (TX_LEVELS + 1) * 8 * TX_BLOCK];   // two stacks per lane, 20 KB per block
            MerkleLds top, grp_tree;
            top.init(lds + threadIdx.x);
            uint64_t k = a;
            while (k < e) {
                const uint32_t g = grp[k];
                while (top.count < g) {   // absent ordinals below g: allOnesHash
                    uint32_t ones[8];
#pragma unroll
                    for (int q = 0; q < 8; q++) ones[q] = 0xffffffffu;
                    top.push(ones);
                }
                grp_tree.init(lds + (TX_LEVELS + 1) * 8 * TX_BLOCK + threadIdx.x);
                for (; k < e && grp[k] == g; k++) {
                    uint32_t nonce[8], leaf[8];
                    compute_nonce(nonce, salt, g, internal[k]);
                    sha256d_prefixed(leaf, nonce, data + off[k], len[k]);
                    grp_tree.push(leaf);
                }
                uint32_t root[8];
                grp_tree.root(root);
                top.push(root);
            }
            top.root(id);
            goto out;
        }
        uint32_t pm_lo = 0, pm_hi = 0, maxg = 0;
        uint64_t k = a;
        while (k < e) {
            const uint32_t g = grp[k];
            uint64_t kend = k;
            while (kend < e && grp[kend] == g) kend++;
            // leaves of group g into leafbuf[k .. kend)
            for (uint64_t c = k; c < kend; c++) {
                uint32_t nonce[8], leaf[8];
                compute_nonce(nonce, salt, g, internal[c]);
                sha256d_prefixed(leaf, nonce, data + off[c], len[c]);
                st8(leafbuf + 8 * c, leaf);
            }
            uint32_t root[8];
            merkle_inplace(root, leafbuf + 8 * k, (uint32_t)(kend - k), 0xffffffffu, 0xffffffffu, false);
            st8(slots + 8 * g, root);
            if (g < 32) pm_lo |= 1u << g;
            else pm_hi |= 1u << (g - 32);
            maxg = g > maxg ? g : maxg;
            k = kend;
        }
        merkle_inplace(id, slots, maxg + 1, pm_lo, pm_hi, true);
    }
out:
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t v = id[j];
        ids[32 * t + 4 * j + 0] = (uint8_t)(v >> 24);
        ids[32 * t + 4 * j + 1] = (uint8_t)(v >> 16);
        ids[32 * t + 4 * j + 2] = (uint8_t)(v >> 8);
        ids[32 * t + 4 * j + 3] = (uint8_t)v;
    }
}

void launch_txid(hipStream_t st, const chip_tx_batch* b, uint8_t* ids, uint32_t* scratch, uint64_t scratch_words) {
    if (!b->ntx) return;
    (void)scratch_words;
    // scratch layout: [ntx][64 slots][8 words] group roots, then [ncomp][8 words] leaves
    uint32_t* slots = scratch;
    uint32_t* leaves = scratch + b->ntx * TX_MAX_GROUPS * 8;
    const uint32_t blocks = (uint32_t)((b->ntx + TX_BLOCK - 1) / TX_BLOCK);
    hipLaunchKernelGGL(k_txid, dim3(blocks), dim3(TX_BLOCK), 0, st, b->ntx, b->salts, b->tx_comp_start, b->comp_group,
                       b->comp_internal, b->data, b->comp_off, b->comp_len, ids, leaves, slots);
}

// ---------------------------------------------------------------------------------------
// K3b: FilteredTransaction.verify() + checkAllComponentsVisible() (the non-validating notary's
// check, NonValidatingNotaryFlow.kt:27-29), one lane per filtered transaction:
//   groupHashes non-empty (reason 1); MerkleTree(groupHashes).hash == id (2)   MerkleTransaction.kt:176-179
//   per filtered group: groupIndex < |groupHashes| (3); partial-tree root == groupHashes[groupIndex] (4);
//   the IncludedLeaf hashes == componentHash(nonce_i, component_i) as multisets (5)  :185-190,
//   PartialMerkleTree.kt:133-160; a partial tree whose post-order encoding is not one tree (9)
//   checkAllComponentsVisible(ordinal)                                         MerkleTransaction.kt:218-234
//     group absent: ordinal >= |groupHashes| or groupHashes[ordinal] == allOnesHash (6);
//     present: index in range (7), MerkleTree(all visible component hashes) == groupHashes[index] (8)
// Per-lane scratch slab in HBM: 64 group-hash slots | 64-deep tree stack | 256 component hashes.
#define FTX_MAX_STACK 64
#define FTX_MAX_COMPS 256
#define FTX_SLOTS (TX_MAX_GROUPS + FTX_MAX_STACK + FTX_MAX_COMPS)

CHIP_DEV void ld8_be(uint32_t v[8], const uint8_t* p) {
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = ld_be32(p + 4 * j);
}
CHIP_DEV bool eq8(const uint32_t* a, const uint32_t* b) {
    uint32_t d = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) d |= a[j] ^ b[j];
    return d == 0;
}

// FilteredTransaction.checkAllComponentsVisible(ord) (MerkleTransaction.kt:218-234) for filtered tx t
CHIP_DEV void ftx_visible(const chip_ftx_batch& b, uint64_t t, uint64_t g0, uint64_t ngh, uint32_t ord,
                          uint32_t* __restrict__ comps, uint32_t (&h)[8], uint8_t& st, uint8_t& rs) {
    int64_t found = -1;
    for (uint64_t g = b.fg_start[t]; g < b.fg_start[t + 1]; g++)
        if (b.fg_index[g] == ord) { found = (int64_t)g; break; }
    if (found < 0) {
        bool ok = (uint64_t)ord >= ngh;
        if (!ok) {
            ld8_be(h, b.group_hashes + 32 * (g0 + ord));
            ok = true;
#pragma unroll
            for (int j = 0; j < 8; j++) ok = ok && h[j] == 0xffffffffu;
        }
        if (!ok) { st = 2; rs = 6; }
        return;
    }
    const uint32_t gi = b.fg_index[found];
    const uint64_t c0 = b.comp_start[found], nc = b.comp_start[found + 1] - c0;
    if (gi >= ngh) { st = 2; rs = 7; return; }
    if (nc == 0 || nc > FTX_MAX_COMPS) { st = 2; rs = 8; return; }
    for (uint64_t c = 0; c < nc; c++) {
        uint32_t nonce[8], leaf[8];
        ld8_be(nonce, b.nonces + 32 * (c0 + c));
        sha256d_prefixed(leaf, nonce, b.comp_data + b.comp_off[c0 + c], b.comp_len[c0 + c]);
        st8(comps + 8 * c, leaf);
    }
    uint32_t want[8];
    merkle_inplace(h, comps, (uint32_t)nc, 0xffffffffu, 0xffffffffu, false);
    ld8_be(want, b.group_hashes + 32 * (g0 + gi));
    if (!eq8(h, want)) { st = 2; rs = 8; }
}

__global__ void __launch_bounds__(256) k_ftx_verify(chip_ftx_batch b, uint8_t* __restrict__ status,
                                                    uint8_t* __restrict__ reason, uint32_t* __restrict__ scratch) {
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
    uint32_t* top = scratch + lane * (FTX_SLOTS * 8);
    uint32_t* stk = top + TX_MAX_GROUPS * 8;
    uint32_t* comps = stk + FTX_MAX_STACK * 8;
    for (uint64_t t = lane; t < b.ntx; t += lanes) {
        uint8_t st = 0, rs = 0;
        const uint64_t g0 = b.gh_start[t], ngh = b.gh_start[t + 1] - g0;
        uint32_t id[8], h[8];
        ld8_be(id, b.ids + 32 * t);
        if (ngh == 0) { st = 1; rs = 1; }
        else if (ngh > TX_MAX_GROUPS) { st = 1; rs = 9; }
        if (!st) {
            for (uint64_t k = 0; k < ngh; k++) {
                ld8_be(h, b.group_hashes + 32 * (g0 + k));
                st8(top + 8 * k, h);
            }
            merkle_inplace(h, top, (uint32_t)ngh, 0xffffffffu, 0xffffffffu, false);
            if (!eq8(h, id)) { st = 1; rs = 2; }
        }
        for (uint64_t g = b.fg_start[t]; !st && g < b.fg_start[t + 1]; g++) {
            const uint32_t gi = b.fg_index[g];
            if (gi >= ngh) { st = 1; rs = 3; break; }
            const uint64_t c0 = b.comp_start[g], nc = b.comp_start[g + 1] - c0;
            if (nc > FTX_MAX_COMPS) { st = 1; rs = 9; break; }
            for (uint64_t c = 0; c < nc; c++) {
                uint32_t nonce[8], leaf[8];
                ld8_be(nonce, b.nonces + 32 * (c0 + c));
                sha256d_prefixed(leaf, nonce, b.comp_data + b.comp_off[c0 + c], b.comp_len[c0 + c]);
                st8(comps + 8 * c, leaf);
            }
            // post-order evaluation (rootAndUsedHashes); IncludedLeaf hashes matched against the
            // component hashes one-to-one (multiset equality, PartialMerkleTree.verify's groupBy)
            uint32_t matched[FTX_MAX_COMPS / 32];
#pragma unroll
            for (int q = 0; q < FTX_MAX_COMPS / 32; q++) matched[q] = 0;
            uint32_t sp = 0, nused = 0;
            bool bad_tree = false, unmatched = false;
            for (uint64_t k = b.pt_start[g]; k < b.pt_start[g + 1]; k++) {
                const uint8_t tag = b.pt_tag[k];
                if (tag == 2) {
                    if (sp < 2) { bad_tree = true; break; }
                    uint32_t l[8], r[8];
                    ld8(r, stk + 8 * (sp - 1));
                    ld8(l, stk + 8 * (sp - 2));
                    hash_concat(h, l, r);
                    sp -= 2;
                } else if (tag <= 1) {
                    ld8_be(h, b.pt_hash + 32 * k);
                    if (tag == 0) {
                        nused++;
                        bool hit = false;
                        for (uint64_t c = 0; c < nc && !hit; c++) {
                            if ((matched[c >> 5] >> (c & 31)) & 1u) continue;
                            if (eq8(comps + 8 * c, h)) {
                                matched[c >> 5] |= 1u << (c & 31);
                                hit = true;
                            }
                        }
                        unmatched = unmatched || !hit;
                    }
                } else {
                    bad_tree = true;
                    break;
                }
                if (sp >= FTX_MAX_STACK) { bad_tree = true; break; }
                st8(stk + 8 * sp, h);
                sp++;
            }
            if (bad_tree || sp != 1) { st = 1; rs = 9; break; }
            uint32_t want[8];
            ld8(h, stk);
            ld8_be(want, b.group_hashes + 32 * (g0 + gi));
            if (!eq8(h, want)) { st = 1; rs = 4; break; }
            if (unmatched || nused != nc) { st = 1; rs = 5; break; }
        }
        // checkAllComponentsVisible(check_visible[t]), then once per bit of visible_mask[t] in ascending ordinal
        // (NonValidatingNotaryFlow.kt:27-29: INPUTS_GROUP, then TIMEWINDOW_GROUP); the first failure decides
        const int32_t cv = b.check_visible ? b.check_visible[t] : -1;
        uint64_t vis = (b.visible_mask ? (uint64_t)b.visible_mask[t] << 1 : 0ull) | (cv >= 0 ? 1ull : 0ull);
        while (!st && vis) {
            const uint32_t bit = (uint32_t)__builtin_ctzll(vis);
            vis &= vis - 1;
            const uint32_t ord = bit == 0 ? (uint32_t)cv : bit - 1;
            ftx_visible(b, t, g0, ngh, ord, comps, h, st, rs);
        }
        status[t] = st;
        if (reason) reason[t] = rs;
    }
}

uint64_t ftx_scratch_words(uint64_t ntx) {
    const uint64_t blocks = std::min<uint64_t>((ntx + 255) / 256, 256);
    return blocks * 256 * FTX_SLOTS * 8;
}

void launch_ftx_verify(hipStream_t st, const chip_ftx_batch* b, uint8_t* status, uint8_t* reason, uint32_t* scratch) {
    if (!b->ntx) return;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((b->ntx + 255) / 256, 256);
    hipLaunchKernelGGL(k_ftx_verify, dim3(blocks), dim3(256), 0, st, *b, status, reason, scratch);
}
