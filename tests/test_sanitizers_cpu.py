"""CPU: AddressSanitizer + UndefinedBehaviorSanitizer over the native host code that runs without a GPU
(SURVEY.md §5): the C restatement in oracle/ (rebuilt with -fsanitize=address,undefined and loaded
into a child Python with libasan preloaded; the oracle tests rerun against it) and the C++
reference-API mirror's CPU-side code (CompositeKey DER, Kryo SignableData bytes).  Any sanitizer
report fails the child process, and so the test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g", "-O1"]
SAN_ENV = {"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=0:halt_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}


def _libasan():
    p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not p or not os.path.isabs(p) or not os.path.exists(p):
        pytest.skip("libasan not available")
    return p


def test_oracle_under_asan_ubsan():
    """The oracle's golden-vector, X.509 and FilteredTransaction / uniqueness tests, with every call into
    the C restatement running sanitized."""
    libasan = _libasan()
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"])
    env = dict(os.environ, **SAN_ENV)
    env["CORDA_ORACLE_LIB"] = os.path.join(ROOT, "oracle", "_asan", "liboracle.so")
    env["LD_PRELOAD"] = libasan + ((":" + os.environ["LD_PRELOAD"]) if os.environ.get("LD_PRELOAD") else "")
    files = ["test_oracle_golden.py", "test_ref_x509_cpu.py", "test_ftx_cpu.py", "test_commit_log_cpu.py",
             "test_uniq_sharded_cpu.py", "test_cfg1_cash_cpu.py", "test_kryo_oracle_cpu.py"]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu"]
                       + [os.path.join(ROOT, "tests", f) for f in files],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, tail


def _composite_args():
    import cordagen as G
    from cash_workload import entropy_seed
    return [G.spki_ed25519(G.ed25519_pub(entropy_seed(v))).hex() for v in (20, 30, 40)]


@pytest.mark.parametrize("src", ["composite_check.cpp", "kryo_bytes.cpp"])
def test_cpp_mirror_cpu_code_under_asan_ubsan(tmp_path, src):
    args = _composite_args() if src == "composite_check.cpp" else ["1", "4", "2", "3", "-1", "2"]
    exe = str(tmp_path / src.replace(".cpp", ""))
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror"] + SAN + ["-I", os.path.join(ROOT, "include"), "-o", exe,
                        os.path.join(ROOT, "tests", "cpp", src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([exe] + args, capture_output=True, text=True, env=dict(os.environ, **SAN_ENV), timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-2000:]
    assert "runtime error:" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-2000:]
