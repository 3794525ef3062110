"""The C++ mirror's CompositeKey (include/corda/verify.hpp) against corda_amd.composite: identical DER
encodings and fulfilment answers for the CompositeKeyTests.kt trees; constraint failures.  CPU only
(no engine call), compiled with g++ -Wall -Werror."""
import os
import subprocess

import cordagen as G
from cash_workload import entropy_seed
from corda_amd.composite import CompositeKey, is_fulfilled_by

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_composite_matches_python(tmp_path):
    exe = str(tmp_path / "composite_check")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           "-o", exe, os.path.join(ROOT, "tests", "cpp", "composite_check.cpp")])
    a, b, c = [G.spki_ed25519(G.ed25519_pub(entropy_seed(v))) for v in (20, 30, 40)]
    out = subprocess.run([exe, a.hex(), b.hex(), c.hex()], check=True, capture_output=True, text=True).stdout.split()
    B = CompositeKey.Builder
    ab = B().add_keys(a, b).build()
    trees = [B().add_keys(a, b, c).build(threshold=2),
             B().add_keys(ab, c).build(threshold=1),
             B().add_key(B().add_key(a, 2).add_key(b, 1).build(threshold=2), 3).add_key(c, 2).build(threshold=3)]
    sets = [[a], [b], [c], [a, b], [a, c], [b, c], [a, b, c], [c, ab]]
    for i, t in enumerate(trees):
        assert out[2 * i] == t.encoded.hex()
        assert out[2 * i + 1] == "".join("1" if is_fulfilled_by(t, s) else "0" for s in sets)
    assert out[6] == "3"    # leaf keys of ((a and b) or c)
    assert out[7] == "5"    # every constraint case threw IllegalArgumentException
