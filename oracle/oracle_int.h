/* oracle_int.h — internal helpers shared by the oracle translation units (test infrastructure). */
#ifndef CORDA_ORACLE_INT_H
#define CORDA_ORACLE_INT_H
#include "oracle.h"

typedef struct { uint32_t h[8]; uint64_t len; size_t fill; uint8_t buf[64]; } orc_sha256_ctx;
typedef struct { uint64_t h[8]; uint64_t len; size_t fill; uint8_t buf[128]; } orc_sha512_ctx;
void orc_sha256_init(orc_sha256_ctx*);
void orc_sha256_update(orc_sha256_ctx*, const uint8_t*, size_t);
void orc_sha256_final(orc_sha256_ctx*, uint8_t out[32]);
void orc_sha512_init(orc_sha512_ctx*);
void orc_sha512_update(orc_sha512_ctx*, const uint8_t*, size_t);
void orc_sha512_final(orc_sha512_ctx*, uint8_t out[64]);
void orc_sha256_block(uint32_t h[8], const uint8_t b[64]);

typedef unsigned __int128 u128;
#endif
