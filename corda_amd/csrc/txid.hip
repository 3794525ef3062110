// txid.hip — K3: WireTransaction.id recomputation (SHA-256 Merkle root over component groups).
//
//   id          = MerkleRoot(groupHashes)                         WireTransaction.kt:63,139
//   groupHashes = g in 0..maxGroup: present ? MerkleRoot(leaves of g) : allOnesHash   :146-155
//   leaf(g,i)   = SHA256(SHA256(nonce(g,i) || bytes))             CryptoUtils.kt:220
//   nonce(g,i)  = SHA256(SHA256(salt || BE32 g || BE32 i))         CryptoUtils.kt:233
//   MerkleRoot  = pad with zeroHash to 2^k; 1 leaf -> the leaf; nodes SHA256(l || r)  MerkleTree.kt:27-66
//
// One lane per transaction (the unit the caller batches; no cross-lane divergence for
// same-shaped transactions).  Leaf and group-root levels are reduced in place in a per-tx
// scratch slab in HBM (64 slots x 32 B; group ordinals must be < 64).
#include "sha2_dev.hpp"
#include "runtime.hpp"

#define TX_MAX_GROUPS 64

// SHA256(SHA256(prefix32 || bytes[0:len]))  (componentHash with prefix = nonce)
CHIP_DEV void sha256d_prefixed(uint32_t out[8], const uint32_t pre[8], const uint8_t* p, uint32_t len) {
    uint32_t H[8], w[16];
    sha256_init(H);
    const uint64_t total = 32ull + len;
    const uint32_t nblocks = (uint32_t)((total + 9 + 63) / 64);
    for (uint32_t b = 0; b < nblocks; b++) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
            if (b == 0 && j < 8) w[j] = pre[j];
            else w[j] = comp_word(p, len, (int64_t)b * 64 + 4 * j - 32);
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

__global__ void __launch_bounds__(256) k_txid(uint64_t ntx, const uint8_t* __restrict__ salts,
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
    const uint32_t blocks = (uint32_t)((b->ntx + 255) / 256);
    hipLaunchKernelGGL(k_txid, dim3(blocks), dim3(256), 0, st, b->ntx, b->salts, b->tx_comp_start, b->comp_group,
                       b->comp_internal, b->data, b->comp_off, b->comp_len, ids, leaves, slots);
}
