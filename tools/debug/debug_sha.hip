#include "../../corda_amd/csrc/sha2_dev.hpp"
#include <cstdio>
__global__ void k(uint32_t* out) {
    uint32_t H[8], w[16];
    // "abc"
    for (int j = 0; j < 16; j++) w[j] = 0;
    w[0] = 0x61626380u; w[15] = 24;
    sha256_init(H); sha256_compress(H, w);
    for (int j = 0; j < 8; j++) out[j] = H[j];
}
int main() {
    uint32_t* d; hipMalloc(&d, 64);
    hipLaunchKernelGGL(k, dim3(1), dim3(1), 0, 0, d);
    uint32_t h[8]; hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
    for (int j = 0; j < 8; j++) printf("%08x", h[j]);
    printf("\nexpect ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad\n");
}
