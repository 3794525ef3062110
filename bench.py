#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X batch verification engine.

Headline workload (BASELINE.json configs[1], "cfg2"): a batch of 1,000,000 Ed25519
(EDDSA_ED25519_SHA512) signatures, 2 per transaction over a shared 200-byte SignableData-shaped
message, 4,096 signing keys, 10% corrupted across the 8 classes of SURVEY.md §8(d) (R flip, S flip,
message flip, wrong key, 63-byte signature, S+L [reference-valid], non-canonical R, small-order-key
forgery [reference-valid]).  Synthetic data generated with OpenSSL (tools/cordagen.c), resident in
HBM before the timed region.

One step = the full verify pipeline on the batch through the C-ABI's device entry point
(chip_verify_batch_device): key decode + per-key tables -> classify/compact -> Ed25519 verify ->
status bytes -> accept bitmap, plus (N > 1) the RCCL all-gather of the per-rank bitmaps.
Scaling is weak: every rank verifies its own 1M-signature batch.

Secondary legs (same JSON line, "secondary"): cfg3 share (500k mixed ECDSA r1/k1 per GPU), cfg4
(1M WireTransactions: tx ids alone, and ids + 2M required-signer verifications fused on the device),
cfg5 (notary batch: ~10M input StateRefs against a 10M-row commit log + one notary Ed25519 signature
per transaction; the commit log is key-sharded across the ranks when N > 1).

Prints ONE JSON line (rank 0).  `roofline` is for the dominant kernel (k_ed_comb_verify), whose
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
ECDSA_OPS_PER_VERIFY = 2.4e5          # SURVEY §8d canonical count (~3,500 field mults x 64 + scalar mults + 4 SHA-256)
# k_ed_comb_verify: 32x32->64 multiply-accumulates (v_mad_u64_u32) per signature, counted from the
# schedule: 64 cached adds (4 mults) + 63 p1p1->p3 (4) + 1 conversion (4) + 32 Niels adds (3) + 31
# conversions (4) + 3 final = 735 GF(2^255-19) multiplications x 100 limb products (radix 2^25.5)
ED_COMB_MACS_PER_VERIFY = 73_500
# SHA-256 compression as the gfx950 compiler issues it: k_txid's SQ_INSTS_VALU x 64 lanes per
# (tx x compression), measured with rocprofv3 (profiles/r01c/pmc_sq.csv: 2.331e9 wave-instructions
# for 1M cfg4 transactions of 89 compressions) — includes the loads and tree bookkeeping
TXID_OPS_PER_COMPRESSION = 1_676
# HBM traffic per launch comes from the committed PMC passes of the same command (tools/profile.sh):
# FETCH_SIZE + WRITE_SIZE (KiB) of the launch with the same grid
PROFILE_DIR = os.path.join(ROOT, "profiles", "r01d")
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
    ap.add_argument("--sigs", "--n", dest="n", type=int, default=1_000_000, help="cfg2 signatures per rank")
    ap.add_argument("--keys", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=32768)
    ap.add_argument("--no-txid", action="store_true", help="skip the cfg4 legs")
    ap.add_argument("--txid-n", type=int, default=1_000_000)
    ap.add_argument("--no-ecdsa", action="store_true", help="skip the cfg3 leg")
    ap.add_argument("--ecdsa-n", type=int, default=500_000, help="cfg3 share per GPU (4M over 8 GPUs)")
    ap.add_argument("--no-notary", action="store_true", help="skip the cfg5 leg")
    ap.add_argument("--notary-tx", type=int, default=4_000_000, help="cfg5 transactions (~2.5 inputs each)")
    ap.add_argument("--notary-pre", type=int, default=10_000_000, help="cfg5 pre-committed StateRefs")
    return ap.parse_args()


def to_dev(arr, torch, dev):
    a = np.ascontiguousarray(arr)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).to(dev)


class DevBatch:
    pass


def upload(obj, fields, torch, dev):
    d = DevBatch()
    for f in fields:
        setattr(d, f, to_dev(getattr(obj, f), torch, dev))
    return d


SIG_FIELDS = ("key_idx", "msg_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off", "key_len", "msg_data",
              "msg_off", "msg_len")
TX_FIELDS = ("salts", "tx_comp_start", "comp_group", "comp_internal", "data", "comp_off", "comp_len")


# The driver launches N ranks over RCCL ("nccl").  CORDA_BENCH_BACKEND=gloo rehearses the N > 1 code
# path on a one-GPU box (every rank on device 0, collectives staged through host memory); its
# timings are not scaling numbers.
BACKEND = os.environ.get("CORDA_BENCH_BACKEND", "nccl")


def all_reduce(t, op, dist):
    if BACKEND == "nccl" or not t.is_cuda:
        dist.all_reduce(t, op=op)
        return t
    c = t.cpu()
    dist.all_reduce(c, op=op)
    t.copy_(c)
    return t


def max_over_ranks(x, world, torch, dev, dist):
    if world == 1:
        return x
    e = torch.tensor([x], dtype=torch.float64, device=dev)
    all_reduce(e, dist.ReduceOp.MAX, dist)
    return float(e.item())


def kernel_base(name):
    """'void k_foo<1>(unsigned int const*, ...)' -> 'k_foo<1>' (rocprofv3 CSVs carry full signatures)."""
    name = name.split("(", 1)[0].strip()
    return name[5:] if name.startswith("void ") else name


def profile_traffic(kernel, grid):
    """HBM bytes of one launch of `kernel` with `grid` threads from the committed rocprofv3 PMC
    passes (FETCH_SIZE + WRITE_SIZE, KiB), or None when the profile has no such launch.  FETCH_SIZE is
    uncalibrated for gathers on gfx950 (MI355X_MICROARCH.md §HBM), so this is reported as measured."""
    import csv
    tot = 0.0
    for name, ctr in (("pmc_fetch_size.csv", "FETCH_SIZE"), ("pmc_write_size.csv", "WRITE_SIZE")):
        path = os.path.join(PROFILE_DIR, name)
        if not os.path.exists(path):
            return None
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
                if kernel_base(r["Kernel_Name"]) == kernel and int(r["Grid_Size"]) == grid and r["Counter_Name"] == ctr]
        if not vals:
            return None
        tot += sum(vals) / len(vals) * 1024.0
    return tot


def sha256_compressions(tb):
    """Exact SHA-256 compressions WireTransaction.id costs for each tx of a TxBatch (the kernel's
    all-zero padding subtrees Z_k are counted as the reference computes them, i.e. hashed)."""
    lens = tb.comp_len.astype(np.int64)
    per_comp = 2 + (32 + lens + 9 + 63) // 64 + 1          # nonce (2) + leaf (ceil) + outer (1)
    total = 0
    start = tb.tx_comp_start.astype(np.int64)
    for t in range(min(tb.ntx, 1)):                          # the cfg4 profile is uniform: one tx stands for all
        a, e = start[t], start[t + 1]
        total += int(per_comp[a:e].sum())
        groups = {}
        for g in tb.comp_group[a:e]:
            groups[int(g)] = groups.get(int(g), 0) + 1
        for cnt in groups.values():
            m = 1 << (cnt - 1).bit_length()
            total += 2 * (m - 1) if cnt > 1 else 0
        top = max(groups) + 1
        m = 1 << (top - 1).bit_length()
        total += 2 * (m - 1) if top > 1 else 0
    return total


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import corda_amd
    from corda_amd import native
    from corda_amd import distributed as D
    import cordagen as G

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(BACKEND, rank=rank, world_size=world)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ctx = corda_amd.Context(local)
    threads = min(16, os.cpu_count() or 1)
    stream = torch.cuda.current_stream(dev)

    # ---- headline: cfg2 Ed25519 (inputs generated and uploaded outside the timed region) ----
    t_gen = time.time()
    batch = G.ed25519_batch(args.n, n_keys=args.keys, seed=0x5EED0002 + rank, threads=threads)
    gen_s = time.time() - t_gen
    db = upload(batch, SIG_FIELDS, torch, dev)
    n = batch.n
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    bitmap = torch.empty((n + 63) // 64, dtype=torch.int64, device=dev)
    gathered = torch.empty(world * bitmap.numel(), dtype=torch.int64, device=dev) if world > 1 else None

    def step():
        ctx.verify_batch_device(db, status, bitmap, stream=stream.cuda_stream)
        if world > 1:
            if BACKEND == "nccl":
                dist.all_gather_into_tensor(gathered, bitmap)
            else:
                parts = [torch.empty_like(bitmap, device="cpu") for _ in range(world)]
                dist.all_gather(parts, bitmap.cpu())
                gathered.copy_(torch.cat(parts))

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
    elapsed = max_over_ranks(time.perf_counter() - t0, world, torch, dev, dist)
    if world > 1:
        c = torch.tensor([int(correct)], dtype=torch.int32, device=dev)
        all_reduce(c, dist.ReduceOp.MIN, dist)
        correct = bool(c.item())
    s = ctx.stats()

    def kms(stats, k):
        return stats.kernel_ms_total[k] / max(1, stats.kernel_launches[k])
    comb_ms, fin_ms, tab_ms, straus_ms, kp_ms = (kms(s, native.K_ED_COMB), kms(s, native.K_ED_FINISH),
                                                 kms(s, native.K_ED_TABLES), kms(s, native.K_ED25519),
                                                 kms(s, native.K_KEYPREP))
    plan_ms = kms(s, native.K_ED_PLAN)
    ms_per_step = elapsed / args.steps * 1e3
    value = world * n * args.steps / elapsed
    # signatures on the comb path: arithmetic-needing signatures of keys with >= 4 of them (default policy)
    arith = (batch.expected == 0) | (batch.expected == 1)
    per_key = np.bincount(batch.key_idx[arith], minlength=len(batch.key_off))
    n_comb = int(per_key[per_key >= 4].sum())
    achieved = ED_COMB_MACS_PER_VERIFY * n_comb / (comb_ms * 1e-3) / 1e12
    comb_grid = (((n + 255) // 256 + 7) & ~7) * 256
    traffic = profile_traffic("k_ed_comb_verify", comb_grid)
    del db, status, bitmap, gathered

    secondary = {}
    # ---- cfg4: tx ids alone, then ids + required signers fused (1M tx, 2M Ed25519 signers) ----
    if not args.no_txid:
        tb, tm, sb, ids_ref, _msgs = G.cfg4_workload(args.txid_n, n_keys=args.keys, seed=0x5EED0004 + rank,
                                                    threads=threads)
        del _msgs
        dt = upload(tb, TX_FIELDS, torch, dev)
        dt.ntx = tb.ntx
        ids = torch.empty(tb.ntx * 32, dtype=torch.uint8, device=dev)
        for _ in range(2):
            ctx.txid_batch_device(dt, ids, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        ids_ok = bool(np.array_equal(ids.cpu().numpy().reshape(-1, 32), ids_ref))
        ctx.reset_stats()
        ts = max(2, args.steps)
        t1 = time.perf_counter()
        for _ in range(ts):
            ctx.txid_batch_device(dt, ids, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        tel = max_over_ranks(time.perf_counter() - t1, world, torch, dev, dist)
        s2 = ctx.stats()
        tx_ms = kms(s2, native.K_TXID)
        comp_per_tx = sha256_compressions(tb)
        secondary.update({
            "txids_per_s": world * tb.ntx * ts / tel,
            "txid_workload": "cfg4 profile: %d tx x 8 components (groups 0-5, 2.1 KB/tx), %d SHA-256 compressions/tx"
                             % (tb.ntx, comp_per_tx),
            "txid_correct": ids_ok,
            "txid_kernel_ms": tx_ms,
            "txid_roofline_frac": (comp_per_tx * TXID_OPS_PER_COMPRESSION * tb.ntx / (tx_ms * 1e-3) / 1e12)
                                  / INT32_PEAK_TOPS,
            "txid_traffic": profile_traffic("k_txid", (tb.ntx + 255) // 256 * 256),
            "txid_algorithmic_bytes": int(tb.data.nbytes + tb.salts.nbytes + 32 * tb.ntx + 20 * len(tb.comp_len)),
        })
        # fused: ids -> SignableData messages -> 2 signers per tx
        dm = upload(tm, ("data", "off", "len", "id_at"), torch, dev)
        dm.max_len = tm.max_len
        ds = upload(sb, ("tx_idx", "tmpl_idx", "key_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off",
                         "key_len"), torch, dev)
        fst = torch.empty(sb.n, dtype=torch.uint8, device=dev)
        fbm = torch.empty((sb.n + 63) // 64, dtype=torch.int64, device=dev)
        for _ in range(2):
            ctx.verify_tx_batch_device(dt, dm, ds, ids, fst, fbm, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        fused_ok = bool(np.array_equal(fst.cpu().numpy(), sb.expected)) and \
            bool(np.array_equal(ids.cpu().numpy().reshape(-1, 32), ids_ref))
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        for _ in range(ts):
            ctx.verify_tx_batch_device(dt, dm, ds, ids, fst, fbm, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        fel = max_over_ranks(time.perf_counter() - t1, world, torch, dev, dist)
        secondary.update({
            "cfg4_verified_tx_per_s": world * tb.ntx * ts / fel,
            "cfg4_signers_per_s": world * sb.n * ts / fel,
            "cfg4_ms_per_batch": fel / ts * 1e3,
            "cfg4_workload": "%d WireTransactions: id recomputed + %d Ed25519 required signers (owner of %d keys + "
                             "notary) verified against it, 1%% corrupted" % (tb.ntx, sb.n, args.keys),
            "cfg4_correct": fused_ok,
        })
        del dt, ids, dm, ds, fst, fbm, tb, tm, sb

    # ---- cfg3 share: mixed ECDSA r1/k1 (500k per GPU = 4M over 8 GPUs) ----
    if not args.no_ecdsa:
        eb = G.ecdsa_batch(args.ecdsa_n, n_keys=args.keys, seed=0x5EED0003 + rank, threads=threads)
        de = upload(eb, SIG_FIELDS, torch, dev)
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
        eel = max_over_ranks(time.perf_counter() - t1, world, torch, dev, dist)
        s3 = ctx.stats()
        r1_ms, k1_ms = kms(s3, native.K_ECDSA_R1), kms(s3, native.K_ECDSA_K1)
        n_r1 = int((eb.scheme == G.SCHEME_R1).sum())
        secondary.update({
            "ecdsa_mixed_sigs_per_s": world * eb.n * ts / eel,
            "ecdsa_workload": "cfg3 share: %d ECDSA sigs per GPU (r1/k1 interleaved, 10%% corrupted)" % eb.n,
            "ecdsa_correct_vs_labels": ecorrect,
            "ecdsa_p256_kernel_ms": r1_ms, "ecdsa_k1_kernel_ms": k1_ms,
            "ecdsa_p256_sigs_per_s_kernel": world * n_r1 / (r1_ms * 1e-3),
            "ecdsa_roofline_frac": (ECDSA_OPS_PER_VERIFY * eb.n / ((r1_ms + k1_ms) * 1e-3) / 1e12) / INT32_PEAK_TOPS,
        })
        del de, est, ebm, eb

    # ---- cfg5: notary batch (uniqueness against a 10M-row log + one notary signature per tx) ----
    if not args.no_notary:
        secondary.update(notary_leg(args, ctx, world, rank, torch, dev, dist, D, G, native, threads, stream))

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
                         "traffic": traffic,
                         "traffic_note": "FETCH_SIZE+WRITE_SIZE bytes per launch, %s (same grid); vs ~%d B/sig "
                                         "algorithmic (sig 64 + shared msg 100 + Abyte 32 + indices 16 + R' 120)"
                                         % (os.path.relpath(PROFILE_DIR, ROOT), 332),
                         "kernel": "k_ed_comb_verify", "kernel_ms": comb_ms,
                         "units_per_launch": n_comb, "macs_per_unit": ED_COMB_MACS_PER_VERIFY,
                         "pipeline_ms": {"keyprep": kp_ms, "comb_plan": plan_ms, "comb_tables_aux_stream": tab_ms,
                                         "comb_verify": comb_ms, "comb_finish": fin_ms, "straus_verify": straus_ms},
                         "canonical_tops": ED25519_OPS_PER_VERIFY * n_arith / (ms_per_step * 1e-3) / 1e12 / world},
            "cpu_baseline": cpu,
            "secondary": secondary,
            "gen_s": gen_s,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def notary_leg(args, ctx, world, rank, torch, dev, dist, D, G, native, threads, stream):
    """cfg5: every rank builds the same global batch (same seed).  Uniqueness: N = 1 commits through
    chip_uniq_commit_batch_device; N > 1 runs the key-sharded protocol (each rank owns a slice of the
    commit log, one RCCL all-reduce MAX of per-tx votes per ordered-commit round).  The commit log is
    rebuilt from the pre-committed rows before each step, outside the timing.  The notary's Ed25519
    signature over each tx id is verified by the rank owning the tx range (strong scaling)."""
    t_gen = time.time()
    pre, ub = G.uniq_workload(args.notary_tx, args.notary_pre, seed=0x5EED0005)
    ntx, nref = ub.ntx, int(ub.tx_ref_start[-1])
    refs, txs, idx, caller = pre
    if world > 1:
        rows = D.route_rows(refs, world)[rank]
        pre = (refs.reshape(-1, 36)[rows].reshape(-1).copy(), txs.reshape(-1, 32)[rows].reshape(-1).copy(),
               idx[rows].copy(), caller[rows].copy())
    n_pre_local = len(pre[2])
    table = ctx.uniq_open(2 * (n_pre_local + nref // world) + 1024)
    ts = 2
    times, rounds, st_sum = [], 0, None
    if world == 1:
        d_start, d_refs = to_dev(ub.tx_ref_start, torch, dev), to_dev(ub.refs, torch, dev)
        d_ids, d_call = to_dev(ub.tx_ids, torch, dev), to_dev(ub.callers, torch, dev)
        d_st = torch.empty(ntx, dtype=torch.uint8, device=dev)
        cap = nref + 1
        d_out = torch.empty(cap * 56, dtype=torch.uint8, device=dev)
        for _ in range(ts + 1):
            table.close()
            table = ctx.uniq_open(2 * (n_pre_local + nref) + 1024)
            table.rebuild(*pre)
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            nout = table.commit_batch_device(d_start, nref, d_refs, d_ids, d_call, d_st, d_out, cap,
                                             stream=stream.cuda_stream)
            torch.cuda.synchronize(dev)
            times.append(time.perf_counter() - t1)
        st = d_st.cpu().numpy()
        del d_start, d_refs, d_ids, d_call, d_st, d_out
    else:
        eng = native.UniqShardEngine(table)
        shard = D.route_uniq_batch(ub.tx_ref_start, ub.refs, world)[rank]
        dshard = eng.upload(shard, ub.tx_ids, ub.callers)
        for _ in range(ts + 1):
            table.close()
            table = ctx.uniq_open(2 * (n_pre_local + shard.nref) + 1024)
            table.rebuild(*pre)
            eng = native.UniqShardEngine(table)
            torch.cuda.synchronize(dev)
            dist.barrier()
            t1 = time.perf_counter()
            st, recs, rounds = D.commit_sharded(eng, ub, shard=dshard)
            torch.cuda.synchronize(dev)
            times.append(time.perf_counter() - t1)
            nout = len(recs)
        del dshard
    table.close()
    uel = max_over_ranks(min(times[1:]), world, torch, dev, dist)
    counts = np.bincount(st, minlength=3)
    # notary signature over every tx id (one key: the per-key comb path)
    lo, hi = ntx * rank // world, ntx * (rank + 1) // world
    keys = np.zeros((hi - lo, 1), dtype=np.int64)
    sb, tm, msgs = G.ed25519_signers(ub.tx_ids.reshape(-1, 32)[lo:hi], keys, 0, corrupt=0.0, seed=0x5EED0015,
                                     threads=threads, extra_key_seeds=(G.NOTARY_SEED,))
    gen_s = time.time() - t_gen
    sbb = G.signer_sig_batch(sb, msgs)
    del msgs
    dsb = upload(sbb, SIG_FIELDS, torch, dev)
    nst = torch.empty(sbb.n, dtype=torch.uint8, device=dev)
    nbm = torch.empty((sbb.n + 63) // 64, dtype=torch.int64, device=dev)
    for _ in range(2):
        ctx.verify_batch_device(dsb, nst, nbm, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    sig_ok = bool((nst.cpu().numpy() == 0).all())
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    for _ in range(ts):
        ctx.verify_batch_device(dsb, nst, nbm, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    sel = max_over_ranks((time.perf_counter() - t1) / ts, world, torch, dev, dist)
    del dsb, nst, nbm
    return {
        "notary_staterefs_per_s": nref / uel,
        "notary_tx_per_s": ntx / uel,
        "notary_commit_ms": uel * 1e3,
        "notary_rounds": rounds if world > 1 else None,
        "notary_status_counts": {"committed": int(counts[0]), "idempotent": int(counts[1]),
                                 "conflict": int(counts[2]), "records": int(nout)},
        "notary_sig_verify_ms": sel * 1e3,
        "notary_batch_tx_per_s": ntx / (uel + sel),
        "notary_sigs_valid": sig_ok,
        "notary_workload": "cfg5: %d tx, %d input StateRefs vs a %d-row commit log (1%% pre-committed hits, 0.5%% "
                           "intra-batch double spends, 0.1%% re-submissions) + %d notary Ed25519 signatures; "
                           "log sharded by key over %d GPU(s)" % (ntx, nref, args.notary_pre, ntx, world),
        "notary_gen_s": gen_s,
    }


if __name__ == "__main__":
    main()
