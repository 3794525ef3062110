// ec_field_test.hip — test harness (not part of libcordahip): runs the device field / scalar
// arithmetic of corda_amd/csrc/ec_dev.hpp on host-supplied operands so tests/test_gpu_ec_field.py
// can compare every result with Python integers, including the rare carry / borrow paths that
// random signatures almost never reach (operands near 0, p, K = 2^256 - p and 2^256).
#include "../corda_amd/csrc/ec_dev.hpp"

enum { OP_MUL = 0, OP_SQR = 1, OP_ADD = 2, OP_SUB = 3, OP_INV = 4, OP_MN_MUL = 5, OP_CANON = 6, OP_MN_INV = 7 };

template <int C>
__global__ void k_field(int op, uint64_t n, const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                        uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u256 x, y, r;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        x.w[k] = a[i * 8 + k];
        y.w[k] = b[i * 8 + k];
    }
    switch (op) {
        case OP_MUL: fp_mul<C>(r, x, y); break;
        case OP_SQR: fp_sqr<C>(r, x); break;
        case OP_ADD: fp_add<C>(r, x, y); break;
        case OP_SUB: fp_sub<C>(r, x, y); break;
        case OP_INV: fp_inv<C>(r, x); break;
        case OP_MN_MUL: mn_mul<C>(r, x, y); break;
        case OP_MN_INV: mn_inv<C>(r, x); break;
        default: fp_canon<C>(r, x); break;
    }
#pragma unroll
    for (int k = 0; k < 8; k++) out[i * 8 + k] = r.w[k];
}

extern "C" int ec_field_run(int curve, int op, uint64_t n, const uint32_t* a, const uint32_t* b, uint32_t* out) {
    uint32_t *da = nullptr, *db = nullptr, *dout = nullptr;
    const size_t bytes = n * 32;
    if (hipMalloc(&da, bytes) || hipMalloc(&db, bytes) || hipMalloc(&dout, bytes)) return -1;
    (void)hipMemcpy(da, a, bytes, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, b, bytes, hipMemcpyHostToDevice);
    const uint32_t blocks = (uint32_t)((n + 63) / 64);
    if (curve == 0) hipLaunchKernelGGL(k_field<CURVE_R1>, dim3(blocks), dim3(64), 0, 0, op, n, da, db, dout);
    else hipLaunchKernelGGL(k_field<CURVE_K1>, dim3(blocks), dim3(64), 0, 0, op, n, da, db, dout);
    int rc = hipDeviceSynchronize() == hipSuccess ? 0 : -2;
    (void)hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(da);
    (void)hipFree(db);
    (void)hipFree(dout);
    return rc;
}
