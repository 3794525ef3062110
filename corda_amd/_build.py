"""In-tree build of libcordahip.so for gfx950 (hipcc; no JIT cache, the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libcordahip.so")
SOURCES = ["runtime.hip", "ed25519.hip", "ed25519_comb.hip", "ecdsa.hip", "txid.hip", "uniq.hip", "signers.hip", "kryo.hip", "group.hip"]
HEADERS = ["common.hpp", "fe25519_dev.hpp", "scalar_dev.hpp", "sha2_dev.hpp", "runtime.hpp", "curve_consts.hpp",
           "ec_dev.hpp", "ed_common_dev.hpp", "comb_tables.hpp", "host_threads.hpp"]
GEN = os.path.join(ROOT, "tools", "gen_constants.py")
CONSTS = os.path.join(CSRC, "curve_consts.hpp")
COMB = os.path.join(CSRC, "comb_tables.hpp")   # generated, git-ignored (3 MB of fixed-base tables)


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


def sources():
    return [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def _obj(src):
    return os.path.join(PKG, "build", os.path.basename(src) + ".o")


def _hdr_mtime():
    return max([_mtime(os.path.join(CSRC, h)) for h in HEADERS] + [_mtime(os.path.join(ROOT, "include", "cordahip.h"))])


def _stale(src, hdr):
    # an object older than its source or any header (a source edited while a build compiled it stays stale)
    return _mtime(_obj(src)) <= max(_mtime(src), hdr)


def needs_rebuild() -> bool:
    if not os.path.exists(LIB):
        return True
    hdr = _hdr_mtime()
    lm = _mtime(LIB)
    return any(_stale(s, hdr) or _mtime(_obj(s)) > lm for s in sources()) or _mtime(GEN) > lm


def build(force: bool = False, verbose: bool = False) -> str:
    if _mtime(CONSTS) < _mtime(GEN):
        subprocess.check_call([sys.executable, GEN, CONSTS])
    if _mtime(COMB) < _mtime(GEN):
        subprocess.check_call([sys.executable, GEN, "--comb", COMB])
    if not force and not needs_rebuild():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs = []
    procs = []
    os.makedirs(os.path.join(PKG, "build"), exist_ok=True)
    hdr = _hdr_mtime()
    for src in sources():
        obj = _obj(src)
        objs.append(obj)
        if not force and not _stale(src, hdr):   # object newer than its source and every header
            continue
        cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj,
               "-I", os.path.join(ROOT, "include")]
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError("hipcc failed: %s\n%s" % (" ".join(cmd), out.decode(errors="replace")))
    tmp = LIB + ".tmp"
    subprocess.check_call([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
