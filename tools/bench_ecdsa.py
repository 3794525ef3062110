#!/usr/bin/env python3
"""Experiment driver for the cfg3 ECDSA leg alone (not the judged bench): one mixed r1/k1 batch
resident in HBM, timed steps through chip_verify_batch_device, labels checked.  Prints one JSON line.
Usage: bench_ecdsa.py [--n 500000] [--keys 4096] [--steps 5] [--p256-only | --ed25519 --n 1000000]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500_000)
    ap.add_argument("--keys", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--p256-only", action="store_true")
    ap.add_argument("--ed25519", action="store_true", help="the cfg2 shape instead (1M Ed25519, schemes hint)")
    ap.add_argument("--no-hint", action="store_true", help="no schemes hint (bench.py's cfg3 leg sets EC_HINT)")
    a = ap.parse_args()
    import torch
    import corda_amd
    from corda_amd import native
    import cordagen as G
    import bench as B
    dev = torch.device("cuda", 0)
    ctx = corda_amd.Context(0)
    stream = torch.cuda.current_stream(dev)
    if a.ed25519:
        eb = G.ed25519_batch(a.n, n_keys=a.keys, seed=0x5EED0002, threads=16)
    else:
        eb = G.ecdsa_batch(a.n, n_keys=a.keys, seed=0x5EED0003, threads=16,
                           schemes=(G.SCHEME_R1,) if a.p256_only else (G.SCHEME_R1, G.SCHEME_K1))
    de = B.upload(eb, B.SIG_FIELDS, torch, dev)
    if not a.no_hint:
        de.schemes_hint = B.ED_HINT if a.ed25519 else (1 << 3 if a.p256_only else B.EC_HINT)
    est = torch.empty(eb.n, dtype=torch.uint8, device=dev)
    ebm = torch.empty((eb.n + 63) // 64, dtype=torch.int64, device=dev)
    for _ in range(a.warmup):
        ctx.verify_batch_device(de, est, ebm, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    ok = bool(np.array_equal(est.cpu().numpy(), eb.expected))
    ctx.reset_stats()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ctx.verify_batch_device(de, est, ebm, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    s = ctx.stats()
    print(json.dumps({"sigs_per_s": eb.n * a.steps / el, "ms_per_step": el / a.steps * 1e3, "correct": ok,
                      "n": eb.n, "p256_only": a.p256_only,
                      "r1_ms": s.kernel_ms_total[native.K_ECDSA_R1] / max(1, s.kernel_launches[native.K_ECDSA_R1]),
                      "k1_ms": s.kernel_ms_total[native.K_ECDSA_K1] / max(1, s.kernel_launches[native.K_ECDSA_K1]),
                      "tables_ms": s.kernel_ms_total[native.K_EC_TABLES] / max(1, s.kernel_launches[native.K_EC_TABLES]),
                      "front_ms": s.kernel_ms_total[native.K_EC_FRONT] / max(1, s.kernel_launches[native.K_EC_FRONT]),
                      "env": {k: v for k, v in os.environ.items() if k.startswith("CHIP_")}}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
