#include "../../corda_amd/csrc/txid.hip"
#include <cstdio>
__global__ void k(uint32_t* out, const uint8_t* data) {
    uint32_t salt[8];
    for (int j = 0; j < 8; j++) salt[j] = 0x01020304u * (j + 1);
    uint32_t nonce[8], leaf[8];
    compute_nonce(nonce, salt, 1, 0);
    for (int j = 0; j < 8; j++) out[j] = nonce[j];
    sha256d_prefixed(leaf, nonce, data, 100);
    for (int j = 0; j < 8; j++) out[8 + j] = leaf[j];
    sha256d_prefixed(leaf, nonce, data + 1, 100);
    for (int j = 0; j < 8; j++) out[16 + j] = leaf[j];
    uint32_t h[8];
    hash_concat(h, nonce, leaf);
    for (int j = 0; j < 8; j++) out[24 + j] = h[j];
}
int main() {
    uint32_t* d; uint8_t* dd; hipMalloc(&d, 256); hipMalloc(&dd, 256);
    uint8_t hd[256]; for (int i = 0; i < 256; i++) hd[i] = (uint8_t)(i * 7 + 3);
    hipMemcpy(dd, hd, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(1), 0, 0, d, dd);
    uint32_t h[32]; hipMemcpy(h, d, 128, hipMemcpyDeviceToHost);
    for (int r = 0; r < 4; r++) { for (int j = 0; j < 8; j++) printf("%08x", h[8*r+j]); printf("\n"); }
}
