#include "runtime.hpp"
extern "C" {
int chip_uniq_open(chip_ctx*, uint64_t, chip_uniq** out) { if (out) *out = nullptr; return CHIP_E_ARG; }
void chip_uniq_close(chip_uniq*) {}
uint64_t chip_uniq_size(const chip_uniq*) { return 0; }
int chip_uniq_rebuild(chip_uniq*, uint64_t, const uint8_t*, const uint8_t*, const uint32_t*, const uint32_t*) { return CHIP_E_ARG; }
int chip_uniq_commit_batch(chip_uniq*, uint64_t, const uint64_t*, const uint8_t*, const uint8_t*, const uint32_t*,
                           uint8_t*, chip_conflict*, uint64_t, uint64_t*) { return CHIP_E_ARG; }
}
