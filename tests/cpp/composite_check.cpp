// CompositeKey in the C++ mirror (include/corda/verify.hpp) against the Python one: reads leaf SPKIs
// (hex, one per argument), builds the CompositeKeyTests.kt trees and prints, one per line, each tree's
// DER encoding (hex) and its fulfilment by a fixed list of signer sets.  No GPU call.
#include <cstdio>
#include <string>

#include "corda/verify.hpp"

using namespace corda;

static PublicKey from_hex(const char* h) {
    PublicKey k;
    for (size_t i = 0; h[i] && h[i + 1]; i += 2) k.encoded.push_back((uint8_t)std::stoi(std::string(h + i, 2), nullptr, 16));
    return k;
}
static void hex(const PublicKey& k) {
    for (uint8_t b : k.encoded) std::printf("%02x", b);
    std::printf("\n");
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const PublicKey a = from_hex(argv[1]), b = from_hex(argv[2]), c = from_hex(argv[3]);
    const PublicKey two_of_three = CompositeKey::build({{a, 1}, {b, 1}, {c, 1}}, 2);
    const PublicKey ab = CompositeKey::build({{a, 1}, {b, 1}});
    const PublicKey ab_or_c = CompositeKey::build({{ab, 1}, {c, 1}}, 1);
    const PublicKey ab2 = CompositeKey::build({{a, 2}, {b, 1}}, 2);
    const PublicKey weighted = CompositeKey::build({{ab2, 3}, {c, 2}}, 3);
    const PublicKey trees[] = {two_of_three, ab_or_c, weighted};
    const std::set<PublicKey> sets[] = {{a}, {b}, {c}, {a, b}, {a, c}, {b, c}, {a, b, c}, {c, ab}};
    for (const auto& t : trees) {
        hex(t);
        if (CompositeKey::encoded_roundtrip_ok(t) != true) return 3;
        for (const auto& s : sets) std::printf("%d", isFulfilledBy(t, s) ? 1 : 0);
        std::printf("\n");
    }
    const auto leaves = CompositeKey::decode(ab_or_c).leafKeys();
    std::printf("%zu\n", leaves.size());
    // constraints (CompositeKeyTests.kt:177-216)
    int thrown = 0;
    try { CompositeKey::build({{a, 0}}); } catch (const IllegalArgumentException&) { thrown++; }
    try { CompositeKey::build({{a, 2}, {b, 2}}, 5); } catch (const IllegalArgumentException&) { thrown++; }
    try { CompositeKey::build({{a, 3}}, 2); } catch (const IllegalArgumentException&) { thrown++; }
    try { CompositeKey::build({{a, INT32_MAX}, {b, INT32_MAX}}); } catch (const IllegalArgumentException&) { thrown++; }
    try { CompositeKey::build({{a, 1}, {b, 1}, {a, 1}}); } catch (const IllegalArgumentException&) { thrown++; }
    std::printf("%d\n", thrown);
    return 0;
}
