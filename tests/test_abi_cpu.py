"""CPU: the C-ABI library loads and exports every function include/cordahip.h declares; the C++
reference-API mirror compiles; no compute call needs a GPU here."""
import ctypes
import os
import re
import subprocess

import pytest

import corda_amd
from corda_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "cordahip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(chip_[a-z_]+)\s*\(", src)))


def test_library_exports_every_header_function():
    lib = corda_amd.load()
    names = header_functions()
    assert len(names) >= 16
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) <= set(native.EXPORTS) | {"chip_reset_stats"}
    out = subprocess.run(["nm", "-D", "--defined-only", native.lib_path()], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (chip_\w+)", out))
    assert set(names) <= exported


def test_abi_version_and_device_count():
    lib = corda_amd.load()
    assert lib.chip_abi_version() == 10
    assert lib.chip_device_count() >= 0


def test_init_fails_loudly_without_gpu():
    lib = corda_amd.load()
    if lib.chip_device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(corda_amd.NativeUnavailable):
        corda_amd.Context(0)


def test_null_arguments_rejected():
    lib = corda_amd.load()
    assert lib.chip_verify_batch(None, None, None, None) == -1
    assert lib.chip_init(None, None) == -1
    lib.chip_shutdown(None)   # no-op


def test_cpp_mirror_compiles(tmp_path):
    exe = tmp_path / "mirror"
    r = subprocess.run(["g++", "-std=c++17", "-O0", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                        "-o", str(exe), os.path.join(ROOT, "tests", "cpp", "test_verify_mirror.cpp"),
                        "-L", os.path.join(ROOT, "corda_amd"), "-lcordahip", "-lcrypto"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


def test_struct_layouts_match_header():
    # ctypes mirrors of the ABI structs (offsets the C compiler would produce)
    assert ctypes.sizeof(native.ChipSigBatch) == 8 * 18   # 17 words + schemes hint / pad
    assert ctypes.sizeof(native.ChipTxBatch) == 8 * 10
    assert ctypes.sizeof(native.ChipConflict) == 8 + 4 + 4 + 32 + 4 + 4
    src = r'''
#include "cordahip.h"
#include <stdio.h>
#include <stddef.h>
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(chip_sig_batch), sizeof(chip_tx_batch), sizeof(chip_conflict),
         sizeof(chip_stats), offsetof(chip_stats, kernel_ms_total), offsetof(chip_stats, key_cache_checks),
         sizeof(chip_group_stats), offsetof(chip_group_stats, exchange_bytes_max));
  return 0; }
'''
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, c])
        vals = [int(x) for x in subprocess.check_output([exe]).split()]
    assert vals[0] == ctypes.sizeof(native.ChipSigBatch)
    assert vals[1] == ctypes.sizeof(native.ChipTxBatch)
    assert vals[2] == ctypes.sizeof(native.ChipConflict)
    assert vals[3] == ctypes.sizeof(native.ChipStats)
    assert vals[4] == native.ChipStats.kernel_ms_total.offset
    assert vals[5] == native.ChipStats.key_cache_checks.offset
    assert vals[6] == ctypes.sizeof(native.ChipGroupStats)
    assert vals[7] == native.ChipGroupStats.exchange_bytes_max.offset


def test_kryo_registry_defaults_match_the_restatement():
    """The registry defaults of cordahip.h / runtime.hip are the ids corda_amd/kryo.py derives from
    DefaultKryoCustomizer.kt's registration order."""
    from corda_amd import kryo as K
    src = open(os.path.join(ROOT, "corda_amd", "csrc", "runtime.hip")).read()
    m = re.search(r"chip_kryo_registry kreg\{(\d+), (\d+), (\d+), (\d+), (\d+), (\d+), \{([\d, ]+)\}\}", src)
    vals = [int(x) for x in m.groups()[:6]]
    keys = [int(x) for x in m.group(7).split(",")][:vals[5]]
    r = K.DEFAULT_REGISTRY
    assert vals[:5] == [r.arrays_aslist, r.signed_tx, r.wire_tx, r.serialized_bytes, r.privacy_salt]
    assert keys == list(r.public_key)
    assert ctypes.sizeof(native.ChipKryoRegistry) == 4 * 14
