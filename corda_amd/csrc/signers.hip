// signers.hip — required-signer check of a batch of transactions on the device (cordahip.h
// chip_required_signers*, chip_verify_signed_tx_batch*): the part of
//   TransactionWithSignatures.verifySignaturesExcept   core/.../transactions/TransactionWithSignatures.kt:44-50
// that follows the signature statuses:
//   checkSignaturesAreValid  :62-66   first non-VALID signature in list order
//   getMissingSigners        :79-85   requiredSigningKeys.filter { !it.isFulfilledBy(sigKeys) }
//   PublicKey.isFulfilledBy           core/.../crypto/CryptoUtils.kt:103-105 (plain key: set membership)
//   CompositeKey.checkFulfilledBy     core/.../crypto/CompositeKey.kt:175-185 (weighted thresholds)
//   needed = missing - allowedToBeMissing
//
// One lane per transaction (a transaction has a handful of signatures and required keys; the kernel
// reads a few coalesced-per-wave index ranges and is a negligible part of the fused pipeline).  A key
// tree is evaluated in post-order with a small per-lane stack of pending child contributions
// (`weight` when the child is fulfilled, else 0): a leaf pushes its contribution, a composite node
// pops its children's, compares their sum with its threshold and pushes its own.  Key equality is
// SPKI byte equality: equal pool indices, or (for a pool that is not de-duplicated) equal lengths and
// bytes.  Every index is range-checked on the device; a violation makes the transaction MALFORMED
// instead of reading out of bounds.
#include "runtime.hpp"

namespace {

CHIP_DEV bool key_bytes_eq(uint32_t a, uint32_t b, const uint8_t* __restrict__ kd, const uint64_t* __restrict__ ko,
                           const uint32_t* __restrict__ kl, uint64_t key_bytes) {
    const uint32_t n = kl[a];
    if (n != kl[b]) return false;
    const uint64_t oa = ko[a], ob = ko[b];
    if (oa + n > key_bytes || ob + n > key_bytes) return false;
    for (uint32_t i = 0; i < n; i++)
        if (kd[oa + i] != kd[ob + i]) return false;
    return true;
}

}  // namespace

__global__ void __launch_bounds__(256) k_required_signers(
    uint64_t ntx, const uint64_t* __restrict__ sig_start, const uint64_t* __restrict__ req_start, uint64_t nreq,
    const uint64_t* __restrict__ node_start, const uint8_t* __restrict__ allowed, uint64_t n_nodes,
    const uint32_t* __restrict__ node_val, const uint32_t* __restrict__ node_nkids,
    const uint32_t* __restrict__ node_weight, uint64_t nsig, const uint32_t* __restrict__ key_idx,
    const uint32_t* __restrict__ tx_idx, uint64_t n_keys, const uint8_t* __restrict__ key_data,
    const uint64_t* __restrict__ key_off, const uint32_t* __restrict__ key_len, uint64_t key_bytes,
    const uint8_t* __restrict__ status, uint8_t* __restrict__ verdict, uint32_t* __restrict__ arg,
    uint8_t* __restrict__ missing) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx) return;
    const uint64_t s0 = sig_start[t], s1 = sig_start[t + 1];
    const uint64_t r0 = req_start[t], r1 = req_start[t + 1];
    const bool req_ok = r0 <= r1 && r1 <= nreq;
    if (missing && req_ok)
        for (uint64_t r = r0; r < r1; r++) missing[r] = 0;
    if (s0 > s1 || s1 > nsig || !req_ok) {
        verdict[t] = CHIP_TXV_MALFORMED;
        arg[t] = 0;
        return;
    }
    // checkSignaturesAreValid: the first failing signature in list order
    for (uint64_t j = s0; j < s1; j++) {
        if ((tx_idx && tx_idx[j] != (uint32_t)t) || key_idx[j] >= n_keys) {
            verdict[t] = CHIP_TXV_MALFORMED;
            arg[t] = 0;
            return;
        }
    }
    for (uint64_t j = s0; j < s1; j++) {
        if (status[j] != CHIP_VALID) {
            verdict[t] = CHIP_TXV_SIGNATURE;
            arg[t] = (uint32_t)j;
            return;
        }
    }
    // getMissingSigners - allowedToBeMissing
    uint32_t needed = 0;
    uint32_t stack[CHIP_REQ_MAX_PENDING];
    for (uint64_t r = r0; r < r1; r++) {
        const uint64_t a = node_start[r], b = node_start[r + 1];
        if (a >= b || b > n_nodes) {
            verdict[t] = CHIP_TXV_MALFORMED;
            arg[t] = 0;
            return;
        }
        int sp = 0;
        bool bad = false;
        for (uint64_t j = a; j < b && !bad; j++) {
            const uint32_t nk = node_nkids[j];
            const uint32_t w = (j + 1 == b) ? 1u : node_weight[j];   // the root contributes "fulfilled"
            uint32_t ful;
            if (nk == 0) {
                const uint32_t k = node_val[j];
                if (k == CHIP_REQ_NO_SIGNER) {
                    ful = 0;
                    goto push;
                }
                if (k >= n_keys) {
                    bad = true;
                    break;
                }
                bool hit = false;
                for (uint64_t q = s0; q < s1 && !hit; q++) hit = key_idx[q] == k;
                for (uint64_t q = s0; q < s1 && !hit; q++)
                    hit = key_bytes_eq(key_idx[q], k, key_data, key_off, key_len, key_bytes);
                ful = hit;
            } else {
                if ((int)nk > sp) {
                    bad = true;
                    break;
                }
                uint64_t sum = 0;
                for (uint32_t c = 0; c < nk; c++) sum += stack[--sp];
                ful = sum >= (uint64_t)node_val[j];
            }
        push:
            if (sp >= CHIP_REQ_MAX_PENDING) {
                bad = true;
                break;
            }
            stack[sp++] = ful ? w : 0u;
        }
        if (bad || sp != 1) {
            verdict[t] = CHIP_TXV_MALFORMED;
            arg[t] = 0;
            if (missing)
                for (uint64_t q = r0; q < r1; q++) missing[q] = 0;
            return;
        }
        const bool miss = stack[0] == 0 && !(allowed && allowed[r]);
        if (missing) missing[r] = miss;
        needed += miss;
    }
    verdict[t] = needed ? CHIP_TXV_MISSING : CHIP_TXV_OK;
    arg[t] = needed;
}

void launch_required_signers(hipStream_t st, const chip_req_batch* q, uint64_t nsig, const uint32_t* key_idx,
                             const uint32_t* tx_idx, uint64_t n_keys, const uint8_t* key_data, const uint64_t* key_off,
                             const uint32_t* key_len, uint64_t key_bytes, const uint8_t* status, uint8_t* verdict,
                             uint32_t* arg, uint8_t* missing) {
    if (!q->ntx) return;
    hipLaunchKernelGGL(k_required_signers, dim3((uint32_t)((q->ntx + 255) / 256)), dim3(256), 0, st, q->ntx,
                       q->sig_start, q->req_start, q->nreq, q->node_start, q->allowed, q->n_nodes, q->node_val,
                       q->node_nkids, q->node_weight, nsig, key_idx, tx_idx, n_keys, key_data, key_off, key_len,
                       key_bytes, status, verdict, arg, missing);
}
