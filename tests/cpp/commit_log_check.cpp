// C++ PersistentUniquenessProvider over a commit log written by the Python provider (same 76-byte row
// format): prints the rebuilt size, then commits two transactions — one spending an already committed
// StateRef (argv[2..3]), one spending a fresh StateRef — and prints their statuses.
#include <cstdio>
#include <string>

#include "corda/verify.hpp"

using namespace corda;

static SecureHash hash_hex(const char* h) {
    SecureHash s;
    for (int i = 0; i < 32; i++) s.bytes[i] = (uint8_t)std::stoi(std::string(h + 2 * i, 2), nullptr, 16);
    return s;
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    Engine e(0);
    PersistentUniquenessProvider p(e, 1 << 14, argv[1]);
    std::printf("%llu\n", (unsigned long long)p.size());
    StateRef spent{hash_hex(argv[2]), (uint32_t)std::stoul(argv[3])};
    StateRef fresh{hash_hex(argv[2]), 1000u};
    SecureHash t1, t2;
    t1.bytes[0] = 0xA1;
    t2.bytes[0] = 0xA2;
    auto r = p.commitBatch({{{spent}, t1, 9}, {{fresh, fresh}, t2, 9}});
    std::printf("%d %d %llu\n", r[0].status, r[1].status, (unsigned long long)p.size());
    return 0;
}
