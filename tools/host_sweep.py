#!/usr/bin/env python3
"""chip_verify_batch (host buffers, PCIe-inclusive) on the cfg2 batch for CHIP_HOST_CHUNKS = 1, 2, 4, 6, 8:
pageable and pinned sources, ms per call (best of 3).  One JSON line per setting."""
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np
import cordagen as G
import corda_amd

FIELDS = ("key_idx", "msg_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off", "key_len", "msg_data",
          "msg_off", "msg_len")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ks = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 6, 8]
    ctx = corda_amd.Context(0)
    b = G.ed25519_batch(n, n_keys=4096, seed=0x5EED0002, threads=16)
    pb = copy.copy(b)
    for f in FIELDS:
        setattr(pb, f, ctx.pinned_copy(getattr(b, f)))
    for k in ks:
        os.environ["CHIP_HOST_CHUNKS"] = str(k)
        out = {"chunks": k, "n": n}
        for name, x in (("pageable", b), ("pinned", pb)):
            ctx.verify_batch(x)
            best = 1e9
            for _ in range(3):
                t = time.perf_counter()
                st, _ = ctx.verify_batch(x)
                best = min(best, time.perf_counter() - t)
            out[name + "_ms"] = best * 1e3
            out[name + "_msigs_per_s"] = n / best / 1e6
            out[name + "_correct"] = bool(np.array_equal(st, b.expected))
        print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
