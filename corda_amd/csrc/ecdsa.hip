// ecdsa.hip — K2 placeholder (first build): ECDSA keys stay unmarked (CHIP_UNSUPPORTED).
#include "runtime.hpp"
void launch_ecdsa_key_prep(hipStream_t, uint64_t, const uint8_t*, const uint64_t*, const uint32_t*, KeyMeta*, uint32_t*) {}
void launch_ecdsa_verify(hipStream_t, int, uint64_t, const uint32_t*, const uint32_t*, const chip_sig_batch*,
                         const uint32_t*, uint8_t*) {}
