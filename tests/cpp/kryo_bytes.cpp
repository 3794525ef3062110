// Prints kryo::signableData(id = 0,1,..,31, SignatureMetadata(pv, scheme)) as hex for the metadata
// values given on the command line (pairs), to compare with corda_amd/kryo.py (tests/test_kryo_cpu.py).
#include <cstdio>
#include <cstdlib>

#include "corda/verify.hpp"

int main(int argc, char** argv) {
    uint8_t id[32];
    for (int i = 0; i < 32; i++) id[i] = (uint8_t)i;
    for (int a = 1; a + 1 < argc; a += 2) {
        corda::SignatureMetadata m{std::atoi(argv[a]), std::atoi(argv[a + 1])};
        const corda::Bytes b = corda::kryo::signableData(id, m);
        for (uint8_t c : b) std::printf("%02x", c);
        std::printf("\n");
    }
    return 0;
}
