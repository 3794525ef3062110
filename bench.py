#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X batch verification engine.

Workload (BASELINE.json configs[1], "cfg2"): a batch of 1,000,000 Ed25519 (EDDSA_ED25519_SHA512)
signatures, 2 per transaction over a shared 200-byte SignableData-shaped message, 4,096 signing
keys, 10% corrupted across the 8 classes of SURVEY.md §8(d) (R flip, S flip, message flip, wrong
key, 63-byte signature, S+L [reference-valid], non-canonical R, small-order-key forgery
[reference-valid]).  Synthetic data generated with OpenSSL (tools/cordagen.c), resident in HBM
before the timed region.

One step = the full verify pipeline on the batch through the C-ABI's device entry point
(chip_verify_batch_device): key decode + per-key tables -> classify/compact -> Ed25519 verify ->
status bytes -> accept bitmap, plus (N > 1) the RCCL all-gather of the per-rank bitmaps.
Scaling is weak: every rank verifies its own 1M-signature batch.

Prints ONE JSON line (rank 0).  `roofline` is for the dominant kernel (k_ed25519_verify), whose
average device duration comes from HIP events the library records around each launch on the
launch stream; `cpu_baseline` times the oracle (oracle/, the C restatement) on the host.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

# Fixed algorithmic work per unit (pinned from the algorithm each kernel runs)
ED25519_OPS_PER_VERIFY = 2.4e5        # SURVEY §8d canonical count (~3,400 field mults x 64 + 3 SHA-512 blocks)
# k_ed_comb_verify: 32x32->64 multiply-accumulates (v_mad_u64_u32) per signature, counted from the
# schedule: 64 cached adds (4 mults) + 63 p1p1->p3 (4) + 1 conversion (4) + 32 Niels adds (3) + 31
# conversions (4) + 3 final = 735 GF(2^255-19) multiplications x 100 limb products (radix 2^25.5)
ED_COMB_MACS_PER_VERIFY = 73_500
TXID_OPS_PER_COMPRESSION = 3.3e3      # SHA-256 compression (64 rounds + schedule)
# VALU issue peak: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6e12 lane-ops/s (= FP32 vector 157.3 TFLOPS / 2,
# MI355X_MICROARCH.md chip table).  v_mad_u64_u32 issues at a quarter of that: 19.66e12 MACs/s
# (tools/microbench_mul.hip measures 18.0e12 including a dependent xor per MAC).
INT32_PEAK_TOPS = 78.6
MAC_PEAK_T = 78.6 / 4
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=1_000_000, help="signatures per rank")
    ap.add_argument("--keys", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=32768)
    ap.add_argument("--no-txid", action="store_true", help="skip the secondary tx-id measurement")
    ap.add_argument("--txid-n", type=int, default=1_000_000)
    ap.add_argument("--no-ecdsa", action="store_true", help="skip the secondary ECDSA measurement")
    ap.add_argument("--ecdsa-n", type=int, default=500_000, help="cfg3 share per GPU (4M over 8 GPUs)")
    return ap.parse_args()


def to_dev(arr, torch, dev):
    return torch.from_numpy(np.ascontiguousarray(arr)).to(dev)


class DevBatch:
    pass


def upload_sig_batch(b, torch, dev):
    d = DevBatch()
    for f in ("key_idx", "msg_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off", "key_len",
              "msg_data", "msg_off", "msg_len"):
        a = getattr(b, f)
        if a.dtype == np.uint64:
            a = a.view(np.int64)
        elif a.dtype == np.uint32:
            a = a.view(np.int32)
        setattr(d, f, to_dev(a, torch, dev))
    return d


def upload_tx_batch(t, torch, dev):
    d = DevBatch()
    d.ntx = t.ntx
    for f in ("salts", "tx_comp_start", "comp_group", "comp_internal", "data", "comp_off", "comp_len"):
        a = getattr(t, f)
        if a.dtype == np.uint64:
            a = a.view(np.int64)
        elif a.dtype == np.uint32:
            a = a.view(np.int32)
        setattr(d, f, to_dev(a, torch, dev))
    return d


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import corda_amd
    from corda_amd import native
    import cordagen as G

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ctx = corda_amd.Context(local)

    # ---- inputs (outside the timed region) ----
    threads = min(16, os.cpu_count() or 1)
    t_gen = time.time()
    batch = G.ed25519_batch(args.n, n_keys=args.keys, seed=0x5EED0002 + rank, threads=threads)
    gen_s = time.time() - t_gen
    db = upload_sig_batch(batch, torch, dev)
    n = batch.n
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    bitmap = torch.empty((n + 63) // 64, dtype=torch.int64, device=dev)
    gathered = torch.empty(world * bitmap.numel(), dtype=torch.int64, device=dev) if world > 1 else None
    stream = torch.cuda.current_stream(dev)

    def step():
        ctx.verify_batch_device(db, status, bitmap, stream=stream.cuda_stream)
        if world > 1:
            dist.all_gather_into_tensor(gathered, bitmap)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    st = status.cpu().numpy()
    correct = bool(np.array_equal(st, batch.expected))
    n_arith = int(((st == 0) | (st == 1)).sum())

    ctx.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        c = torch.tensor([int(correct)], dtype=torch.int32, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.MIN)
        correct = bool(c.item())
    s = ctx.stats()

    def kms(k):
        return s.kernel_ms_total[k] / max(1, s.kernel_launches[k])
    comb_ms, fin_ms, tab_ms, straus_ms, kp_ms = (kms(native.K_ED_COMB), kms(native.K_ED_FINISH),
                                                 kms(native.K_ED_TABLES), kms(native.K_ED25519),
                                                 kms(native.K_KEYPREP))
    ms_per_step = elapsed / args.steps * 1e3
    value = world * n * args.steps / elapsed
    # signatures on the comb path: arithmetic-needing signatures of keys with >= 4 of them (default policy)
    arith = (batch.expected == 0) | (batch.expected == 1)
    per_key = np.bincount(batch.key_idx[arith], minlength=len(batch.key_off))
    n_comb = int(per_key[per_key >= 4].sum())
    achieved = ED_COMB_MACS_PER_VERIFY * n_comb / (comb_ms * 1e-3) / 1e12

    # ---- secondary: tx ids/s on cfg4-shaped transactions (1 GPU per rank, same weak scaling) ----
    secondary = {}
    if not args.no_txid:
        tb = G.tx_batch(args.txid_n, seed=0x5EED0004 + rank)
        dt = upload_tx_batch(tb, torch, dev)
        ids = torch.empty(tb.ntx * 32, dtype=torch.uint8, device=dev)
        for _ in range(2):
            ctx.txid_batch_device(dt, ids, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        ctx.reset_stats()
        ts = max(2, args.steps)
        t1 = time.perf_counter()
        for _ in range(ts):
            ctx.txid_batch_device(dt, ids, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        tel = time.perf_counter() - t1
        if world > 1:
            e = torch.tensor([tel], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            tel = float(e.item())
        s2 = ctx.stats()
        tx_ms = s2.kernel_ms_total[native.K_TXID] / max(1, s2.kernel_launches[native.K_TXID])
        comp_per_tx = 105  # cfg4 profile: SHA-256 compressions per transaction
        secondary = {
            "txids_per_s": world * tb.ntx * ts / tel,
            "txid_workload": "cfg4 profile: %d tx x 8 components (groups 0-5, 2.1 KB/tx)" % tb.ntx,
            "txid_kernel_ms": tx_ms,
            "txid_roofline_frac": (comp_per_tx * TXID_OPS_PER_COMPRESSION * tb.ntx / (tx_ms * 1e-3) / 1e12) / INT32_PEAK_TOPS,
        }
        del dt, ids

    # ---- secondary: cfg3 mixed ECDSA r1/k1 (500k per GPU = 4M over 8 GPUs) ----
    if not args.no_ecdsa:
        eb = G.ecdsa_batch(args.ecdsa_n, n_keys=args.keys, seed=0x5EED0003 + rank, threads=threads)
        de = upload_sig_batch(eb, torch, dev)
        est = torch.empty(eb.n, dtype=torch.uint8, device=dev)
        ebm = torch.empty((eb.n + 63) // 64, dtype=torch.int64, device=dev)
        for _ in range(2):
            ctx.verify_batch_device(de, est, ebm, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        ecorrect = bool(np.array_equal(est.cpu().numpy(), eb.expected))
        ctx.reset_stats()
        ts = max(2, args.steps)
        t1 = time.perf_counter()
        for _ in range(ts):
            ctx.verify_batch_device(de, est, ebm, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        eel = time.perf_counter() - t1
        if world > 1:
            e = torch.tensor([eel], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            eel = float(e.item())
        s3 = ctx.stats()
        r1_ms = s3.kernel_ms_total[native.K_ECDSA_R1] / max(1, s3.kernel_launches[native.K_ECDSA_R1])
        k1_ms = s3.kernel_ms_total[native.K_ECDSA_K1] / max(1, s3.kernel_launches[native.K_ECDSA_K1])
        n_r1 = int((eb.scheme == G.SCHEME_R1).sum())
        secondary.update({
            "ecdsa_mixed_sigs_per_s": world * eb.n * ts / eel,
            "ecdsa_workload": "cfg3 share: %d ECDSA sigs per GPU (r1/k1 interleaved, 10%% corrupted)" % eb.n,
            "ecdsa_correct_vs_labels": ecorrect,
            "ecdsa_p256_kernel_ms": r1_ms, "ecdsa_k1_kernel_ms": k1_ms,
            "ecdsa_p256_sigs_per_s_kernel": world * n_r1 / (r1_ms * 1e-3),
            "ecdsa_roofline_frac": (ED25519_OPS_PER_VERIFY * eb.n / ((r1_ms + k1_ms) * 1e-3) / 1e12) / INT32_PEAK_TOPS,
        })
        del de, est, ebm

    # ---- CPU baseline (rank 0, N = 1 only): the oracle restatement on host cores ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle_bind as O
        m = min(args.cpu_sample, n)
        sub = G.SigBatch()
        sub.key_idx, sub.msg_idx = batch.key_idx[:m], batch.msg_idx[:m]
        sub.sig_data, sub.sig_off, sub.sig_len = batch.sig_data, batch.sig_off[:m], batch.sig_len[:m]
        sub.key_data, sub.key_off, sub.key_len = batch.key_data, batch.key_off, batch.key_len
        sub.msg_data, sub.msg_off, sub.msg_len = batch.msg_data, batch.msg_off, batch.msg_len
        t2 = time.perf_counter()
        ref = O.verify_batch(sub, threads=threads)
        cel = time.perf_counter() - t2
        cpu = {"value": m / cel, "unit": "verified sigs/s", "cores": threads, "kind": "port",
               "sample": "first %d signatures of the same cfg2 batch through oracle/ (C restatement of "
                         "i2p eddsa 0.2.0 semantics), %d threads" % (m, threads),
               "agrees_with_gpu": bool(np.array_equal(ref, st[:m]))}

    if rank == 0:
        out = {
            "metric": "verified sigs/sec (Ed25519, ECDSA P-256) at 1/2/4/8 MI355X; tx ids/sec",
            "value": value,
            "unit": "verified Ed25519 sigs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (radix-2^25.5 GF(2^255-19) limbs, 32x32->64 MACs)",
            "data": "synthetic (OpenSSL-signed, seeded; SURVEY.md §8d cfg2 corruption mix)",
            "config": {"workload": "cfg2: %d-signature EDDSA_ED25519_SHA512 batch per GPU, %d keys, 200-B messages, "
                                   "10%% corrupted" % (n, args.keys),
                       "sigs_per_gpu": n, "keys": args.keys, "msg_len": 200, "corrupt": 0.10,
                       "parallelism": "dp%d (batch sharded by transaction, RCCL bitmap all-gather)" % world},
            "correct_vs_labels": correct,
            "roofline": {"bound": "valu", "achieved": achieved, "peak": MAC_PEAK_T,
                         "unit": "T MAC/s (v_mad_u64_u32 32x32->64)", "frac": achieved / MAC_PEAK_T,
                         "traffic": None, "kernel": "k_ed_comb_verify", "kernel_ms": comb_ms,
                         "units_per_launch": n_comb, "macs_per_unit": ED_COMB_MACS_PER_VERIFY,
                         "pipeline_ms": {"keyprep": kp_ms, "comb_tables": tab_ms, "comb_verify": comb_ms,
                                         "comb_finish": fin_ms, "straus_verify": straus_ms},
                         "canonical_tops": ED25519_OPS_PER_VERIFY * n_arith / (ms_per_step * 1e-3) / 1e12 / world},
            "cpu_baseline": cpu,
            "secondary": secondary,
            "gen_s": gen_s,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
