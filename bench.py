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

Secondary legs (same JSON line, "secondary"): cfg2 through the host-buffer entry (PCIe included);
cold keys (every signature its own key: the windowed Straus kernel); cfg3 (4M mixed ECDSA r1/k1
sharded by transaction over the ranks, RCCL bitmap all-gather; plus a P-256-only batch); cfg4
(1M WireTransactions: tx ids alone, and ids + 2M required-signer verifications fused on the device);
cfg5 (notary batch: ~10M input StateRefs against a 10M-row commit log + one notary Ed25519 signature
per transaction; checked against the oracle at full size; the log is key-sharded when N > 1).

Prints ONE JSON line (rank 0).  `roofline` is for the dominant kernel (k_ed_comb_ahalf), whose
average device duration comes from HIP events the library records around each launch on the
launch stream; `cpu_baseline` times the oracle (oracle/, the C restatement) on the host, and
`cpu_baseline_openssl` OpenSSL EVP_DigestVerify on the same sample.
"""
import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

_T0 = time.time()
HOST_ITERS = 5          # host-buffer legs: timed calls, the median is reported


def progress(msg):
    """One stderr line per finished leg (long profiler passes keep writing while they run)."""
    print("[bench %7.1fs] %s" % (time.time() - _T0, msg), file=sys.stderr, flush=True)


def cgroup_cpu():
    """(quota in CPUs or None, throttled periods, throttled ms) of this process's cgroup: the host-buffer legs
    copy on host threads, and a CFS quota that runs out mid-copy stalls the process for the rest of the period."""
    quota, n, ms = None, None, None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else int(q) / int(p)
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()
            if k == "nr_throttled":
                n = int(v)
            elif k == "throttled_usec":
                ms = int(v) / 1e3
    except (OSError, ValueError):
        pass
    return quota, n, ms

# Fixed algorithmic work per unit (pinned from the algorithm each kernel runs).
# 32x32->64 multiply-accumulates (v_mad_u64_u32) per signature:
#   Ed25519 comb, radix 2^25.5 (100 limb products per GF(2^255-19) multiplication):
#     k_ed_comb_bhalf: [S]B from the radix-2^16 fixed-base comb: 16 Niels adds (3 mults) + 15
#                      conversions (4) + 1 final conversion (4) = 112 mults (+ SHA-512, not counted)
#     k_ed_comb_ahalf: [h](-A) from the per-key radix-64 comb (ED_COMB_W = 6): 43 cached adds (4 mults) +
#                      42 conversions (4) + 3 final = 343 mults
ED_COMB_MACS_B = 11_200
ED_COMB_MACS_A = 34_300
ED_COMB_MACS_PER_VERIFY = ED_COMB_MACS_A + ED_COMB_MACS_B          # 45,500
#   Ed25519 windowed Straus (k_ed25519_verify): 252 doublings (4 squarings each) + the encode
#   inversion (254 squarings) = 1,262 squarings x 55 limb products, and 1,504 multiplications x 100
#   (doubling-chain conversions 819, 64 cached A-adds 256 + conversions 192, 32 B-madds 224, 11 + 2
#   inversion/encode)
ED_STRAUS_MACS_PER_VERIFY = 1_262 * 55 + 1_504 * 100                # 219,810
#   the split Straus path (round 6, default): the kernel time of the cold leg's K_ED25519 bracket is
#   k_ed25519_verify_a + the batched finish (the hash and [S]B run beside the key prep, outside it):
#   verify_a 252 doublings (1,008 squarings) + 63 A-adds with their conversions (1,260 mults) + 19 for
#   the first window and + [S]B; the finish at 4 signatures per inversion 254 / 4 squarings + ~8 mults
ED_STRAUS_SPLIT_MACS_PER_VERIFY = (1_008 + 64) * 55 + (1_279 + 8) * 100   # 187,660
#   ECDSA comb (P-256 / secp256k1, 8 x 32-bit limbs): a mixed addition = 7 mults (64 products) +
#   4 squarings (36) = 592; 17 G windows (radix 2^16) + 65 Q windows (radix 16) = 82 additions;
#   17 scalar Montgomery mults (128 each: s R, 12 wave-scan, 2 finalize, u1, u2) + the x(R) check (100)
ECDSA_COMB_MACS_PER_VERIFY = 82 * 592 + 17 * 128 + 100              # 50,820 (P-256)
ECDSA_Q_MACS_PER_VERIFY = 65 * 592 + 100                            # k_ecdsa_comb_q: 38,580 (P-256)
#   secp256k1 with GLV (round 6, CHIP_EC_GLV): u2 Q = a1 Q + a2 (lambda Q) with 128-bit halves over radix-32
#   tables, 52 additions instead of 65, + the split (2 x 64 products for the rounding, 3 Montgomery mults);
#   cfg3 interleaves the curves 1:1, so its per-signature figures are the mean of the two
ECDSA_K1_SPLIT_MACS = 2 * 64 + 3 * 128
ECDSA_MIXED_MACS_PER_VERIFY = (82 + 69) * 592 // 2 + 17 * 128 + 100 + ECDSA_K1_SPLIT_MACS // 2    # 47,228
ECDSA_MIXED_Q_MACS_PER_VERIFY = (65 + 52) * 592 // 2 + 100 + ECDSA_K1_SPLIT_MACS // 2             # 34,988
# SHA-256 compression, canonical 32-bit operations (rotates as one funnel shift): 64 rounds x 24
# (Sigma1 5, Ch 3, T1 adds 4, Sigma0 5, Maj 4, 3 state adds) + 48 schedule words x 13 + 8 = 2,168
SHA256_OPS_PER_COMPRESSION = 2_168
# HBM traffic per launch comes from the committed PMC passes of the same command (tools/profile.sh):
# FETCH_SIZE + WRITE_SIZE (KiB) of the launch with the same grid
PROFILE_DIR = os.path.join(ROOT, "profiles", os.environ.get("CORDA_PROFILE_DIR", "r06"))
# VALU rooflines (profiles/r04/microbench_valu*.txt, tools/microbench_valu.hip):
#   a wave64 VALU instruction issues in 2 cycles per SIMD only for the dual-issue opcodes (v_add/sub/and/or/xor/
#   mov/lshrrev_b32, v_bitop3_b32, v_fma_f32: 2.3-2.6 cycles measured at 2-8 waves); every other opcode —
#   v_mad_u64_u32, mul_lo/hi, add3, lshl_add, alignbit, 64-bit shifts, add_co/addc, cndmask_e64, bfi, perm —
#   issues in ~4.2 cycles, and a MAC does not co-issue with the simple ops.
#   INT32_PEAK_TOPS  the guide's VALU lane-op peak: 256 CU x 4 SIMD x 64 lanes / 2 cycles x 2.4 GHz = 78.6 T
#   MAC_SPEC_T       v_mad_u64_u32 at one per 4 cycles per SIMD and 2.4 GHz = 39.3 T (BASELINE.md's figure)
#   MAC_MEASURED_T   the microbench's v_mad_u64_u32 rate, 8 independent chains x 8 waves per SIMD: 36.5 T at the
#                    2.38 GHz the in-kernel clock showed; a real kernel runs at the clock its GRBM pass shows
#                    (~2.0-2.1 GHz under the cfg2 load), so frac_measured rescales the rate to that clock
INT32_PEAK_TOPS = 78.6
MAC_SPEC_T = 39.3
MAC_PEAK_T = MAC_SPEC_T
MAC_MEASURED_T = 36.5
MAC_MEASURED_CLOCK_GHZ = 2.38
VALU_MEASURED_T = 37.3          # the ~4.2-cycle opcodes at 8 waves (add3, lshl_add, alignbit, mul_lo ...)
VALU_ISSUE_CYCLES = 4.2         # cycles per non-dual-issue VALU wave-instruction per SIMD (issue-bound kernels)
HBM_PEAK_GBS = 8000.0
# uniqueness: 36 B key read + 64 B slot probe + 64 B slot write per input StateRef
UNIQ_BYTES_PER_REF = 164


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sigs", "--n", dest="n", type=int, default=1_000_000, help="cfg2 signatures per rank")
    ap.add_argument("--keys", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=32768)
    ap.add_argument("--no-full-oracle", action="store_true", help="skip the full-size cfg2 oracle comparison")
    ap.add_argument("--no-host-path", action="store_true", help="skip the host-buffer (PCIe-inclusive) cfg2 leg")
    ap.add_argument("--no-key-cache", action="store_true", help="skip the CHIP_FLAG_KEY_CACHE legs")
    ap.add_argument("--cold-n", type=int, default=200_000, help="cold-key leg: signatures = keys (0 = skip)")
    ap.add_argument("--no-txid", action="store_true", help="skip the cfg4 legs")
    ap.add_argument("--txid-n", type=int, default=1_000_000)
    ap.add_argument("--no-ecdsa", action="store_true", help="skip the cfg3 legs")
    ap.add_argument("--ecdsa-n", type=int, default=4_000_000, help="cfg3 global batch (sharded over the ranks)")
    ap.add_argument("--no-notary", action="store_true", help="skip the cfg5 leg")
    ap.add_argument("--no-group", action="store_true", help="skip the device-group legs (chip_group_*, N = 1 only)")
    ap.add_argument("--notary-tx", type=int, default=4_000_000, help="cfg5 transactions (~2.5 inputs each)")
    ap.add_argument("--notary-pre", type=int, default=10_000_000, help="cfg5 pre-committed StateRefs")
    ap.add_argument("--no-notary-check", action="store_true", help="skip the full-size oracle check of cfg5")
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
ED_HINT = 1 << 4
EC_HINT = (1 << 2) | (1 << 3)


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


def all_gather_bitmap(gathered, bitmap, world, dist):
    if world == 1:
        return
    if BACKEND == "nccl":
        dist.all_gather_into_tensor(gathered, bitmap)
    else:
        import torch
        parts = [torch.empty_like(bitmap, device="cpu") for _ in range(world)]
        dist.all_gather(parts, bitmap.cpu())
        gathered.copy_(torch.cat(parts))


def max_over_ranks(x, world, torch, dev, dist):
    if world == 1:
        return x
    e = torch.tensor([x], dtype=torch.float64, device=dev)
    all_reduce(e, dist.ReduceOp.MAX, dist)
    return float(e.item())


def min_over_ranks_bool(ok, world, torch, dev, dist):
    if world == 1:
        return ok
    c = torch.tensor([int(ok)], dtype=torch.int32, device=dev)
    all_reduce(c, dist.ReduceOp.MIN, dist)
    return bool(c.item())


def kernel_base(name):
    """'void k_foo<1>(unsigned int const*, ...)' -> 'k_foo<1>' (rocprofv3 CSVs carry full signatures)."""
    name = name.strip()
    if name.startswith("void "):
        name = name[5:]
    return name.replace("(anonymous namespace)::", "").split("(", 1)[0].strip()


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


def profile_issue(kernel, grid):
    """The issue-model row of `kernel` with `grid` threads (tools/issue_summary.py over the committed
    SQ_INSTS_VALU + GRBM_GUI_ACTIVE pass): duration, VALU wave-instructions per launch, effective clock,
    cycles per VALU instruction per SIMD; or None."""
    import csv
    path = os.path.join(PROFILE_DIR, "issue_model.csv")
    if not os.path.exists(path):
        return None
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"] == kernel and int(r["Grid_Size"]) == grid:
            return {"duration_ms": float(r["Duration_ms"]), "valu_per_launch": float(r["VALU_per_launch"]),
                    "eff_clock_ghz": float(r["Eff_clock_GHz"]), "cyc_per_valu": float(r["Cyc_per_VALU_per_SIMD"])}
    return None


def stx_traffic(ntx, nsig, ncomp):
    """FETCH_SIZE + WRITE_SIZE of one Kryo front-end call from the committed PMC profile, or None: pass 1 (the fused
    walk since round 5), pass 2 when it ran (only blobs past pass 1's rows: 0 for cfg4), the post-dechunk pass
    (duplicate inputs + required-key walk), the de-chunk copies, the row transposes, the key interning and the
    required-key passes (the pool copy is a DMA, not counted)."""
    grid_tx, grid_sig = (ntx + 255) // 256 * 256, (nsig + 255) // 256 * 256

    def first(*cands):   # the first (kernel, grid) the profile holds: kernel names of this round, then older ones
        for k, g in cands:
            v = profile_traffic(k, g)
            if v is not None:
                return v
        return None
    parts = [first(("k_stx_parse<false, 1>", grid_tx), ("k_stx_parse<false>", grid_tx)),
             first(("k_stx_post", grid_tx), ("k_stx_req_tail", grid_tx)),
             first(("k_stx_dechunk<16>", (ntx * 16 + 255) // 256 * 256), ("k_stx_dechunk", (ntx * 64 + 255) // 256 * 256)),
             profile_traffic("k_stx_required", grid_tx)]
    parts += [profile_traffic(k, grid_sig) for k in ("k_stx_key_insert", "k_stx_key_flag", "k_stx_key_assign",
                                                      "k_stx_req_entry<false>", "k_stx_req_entry<true>")]
    if any(p is None for p in parts):
        return None
    # launched only when needed / present in the profile: pass 2, the transposes
    opt = [profile_traffic("k_stx_parse<true, 0>", grid_tx) or profile_traffic("k_stx_parse<true>", grid_tx),
           profile_traffic("k_stx_lm_comps", (ncomp + 255) // 256 * 256),
           profile_traffic("k_stx_lm_sigs", grid_sig)]
    return sum(parts) + sum(p for p in opt if p)


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


def cpu_share():
    """Threads for the CPU baselines: the CPUs this process may use, capped by the share the GPU box
    grants one GPU (OMP_NUM_THREADS is set to it there; nproc shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(n, share) if share > 0 else n), n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def sub_batch(G, b, m):
    sub = G.SigBatch()
    sub.key_idx, sub.msg_idx = b.key_idx[:m], b.msg_idx[:m]
    sub.sig_data, sub.sig_off, sub.sig_len = b.sig_data, b.sig_off[:m], b.sig_len[:m]
    sub.key_data, sub.key_off, sub.key_len = b.key_data, b.key_off, b.key_len
    sub.msg_data, sub.msg_off, sub.msg_len = b.msg_data, b.msg_off, b.msg_len
    return sub


def kms(stats, k):
    return stats.kernel_ms_total[k] / max(1, stats.kernel_launches[k])


def timed_steps(fn, steps, world, torch, dev, dist):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    return max_over_ranks(time.perf_counter() - t0, world, torch, dev, dist)


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
    threads, nproc = cpu_share()
    gen_threads = max(1, threads)
    stream = torch.cuda.current_stream(dev)

    # ---- headline: cfg2 Ed25519 (inputs generated and uploaded outside the timed region) ----
    t_gen = time.time()
    batch = G.ed25519_batch(args.n, n_keys=args.keys, seed=0x5EED0002 + rank, threads=gen_threads)
    gen_s = time.time() - t_gen
    db = upload(batch, SIG_FIELDS, torch, dev)
    db.schemes_hint = ED_HINT
    n = batch.n
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    bitmap = torch.empty((n + 63) // 64, dtype=torch.int64, device=dev)
    gathered = torch.empty(world * bitmap.numel(), dtype=torch.int64, device=dev) if world > 1 else None

    def step():
        ctx.verify_batch_device(db, status, bitmap, stream=stream.cuda_stream)
        all_gather_bitmap(gathered, bitmap, world, dist)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    st = status.cpu().numpy()
    correct = min_over_ranks_bool(bool(np.array_equal(st, batch.expected)), world, torch, dev, dist)
    n_arith = int(((st == 0) | (st == 1)).sum())

    ctx.reset_stats()
    elapsed = timed_steps(step, args.steps, world, torch, dev, dist)
    s = ctx.stats()
    a_ms, b_ms, fin_ms, tab_ms, straus_ms, kp_ms, plan_ms = (
        kms(s, native.K_ED_COMB), kms(s, native.K_ED_COMB_B), kms(s, native.K_ED_FINISH), kms(s, native.K_ED_TABLES),
        kms(s, native.K_ED25519), kms(s, native.K_KEYPREP), kms(s, native.K_ED_PLAN))

    ms_per_step = elapsed / args.steps * 1e3
    value = world * n * args.steps / elapsed
    # signatures on the comb path: arithmetic-needing signatures of keys with >= 4 of them (default policy)
    arith = (batch.expected == 0) | (batch.expected == 1)
    per_key = np.bincount(batch.key_idx[arith], minlength=len(batch.key_off))
    n_comb = int(per_key[per_key >= 4].sum())
    achieved = ED_COMB_MACS_A * n_comb / (a_ms * 1e-3) / 1e12
    comb_grid = (((n + 255) // 256 + 7) & ~7) * 256
    # (k_ed_comb_ahalf<false> since the row format became a template parameter in round 6; the plain name in
    # profiles taken before)
    traffic = profile_traffic("k_ed_comb_ahalf<false>", comb_grid) or profile_traffic("k_ed_comb_ahalf", comb_grid)
    ahalf_issue = profile_issue("k_ed_comb_ahalf<false>", comb_grid) or profile_issue("k_ed_comb_ahalf", comb_grid)

    secondary = {}
    progress("cfg2 headline done")
    # ---- cfg2 with the key state kept across batches (CHIP_FLAG_KEY_CACHE, a context of its own): every step
    # verifies the whole batch again, but the key pool equals the previous step's, so the key prep and the per-key
    # comb tables are reused (the headline builds them inside every step) ----
    if not args.no_key_cache:
        kctx = corda_amd.Context(local, flags=native.FLAG_KEY_CACHE)

        def kstep():
            kctx.verify_batch_device(db, status, bitmap, stream=stream.cuda_stream)
            all_gather_bitmap(gathered, bitmap, world, dist)

        for _ in range(max(2, args.warmup)):   # the first call builds the key state
            kstep()
        torch.cuda.synchronize(dev)
        kst = status.cpu().numpy()
        kctx.reset_stats()
        kel = timed_steps(kstep, args.steps, world, torch, dev, dist)
        ks = kctx.stats()
        secondary.update({
            "cfg2_key_cache_sigs_per_s": world * n * args.steps / kel,
            "cfg2_key_cache_ms_per_step": kel / args.steps * 1e3,
            "cfg2_key_cache_correct": min_over_ranks_bool(bool(np.array_equal(kst, batch.expected)), world, torch,
                                                          dev, dist),
            "cfg2_key_cache_pipeline_ms": {"keyprep": kms(ks, native.K_KEYPREP), "comb_tables_aux_stream":
                                           kms(ks, native.K_ED_TABLES), "comb_bhalf": kms(ks, native.K_ED_COMB_B),
                                           "comb_ahalf": kms(ks, native.K_ED_COMB), "comb_finish": kms(ks, native.K_ED_FINISH)},
            "cfg2_key_cache_note": "the cfg2 batch re-verified with CHIP_FLAG_KEY_CACHE: statuses recomputed every "
                                   "step; the key pool is compared on the device and the key state reused",
        })
        kctx.close()
        progress("cfg2 key cache done")
    del db, status, bitmap, gathered
    # ---- cfg2 through the host-buffer entry (staging H2D + pipeline + D2H, blocking) ----
    if not args.no_host_path:
        ctx.verify_batch(batch)
        quota, thr_n0, thr_ms0 = cgroup_cpu()
        it_ms = []
        for _ in range(HOST_ITERS):
            t1 = time.perf_counter()
            hst, _bm = ctx.verify_batch(batch)
            it_ms.append((time.perf_counter() - t1) * 1e3)
        _, thr_n1, thr_ms1 = cgroup_cpu()
        hel = max_over_ranks(float(np.median(it_ms)) / 1e3, world, torch, dev, dist)
        secondary.update({
            "cfg2_host_path_sigs_per_s": world * n / hel,
            "cfg2_host_path_ms": hel * 1e3,
            "cfg2_host_path_bytes_in": int(batch.sig_data.nbytes + batch.msg_data.nbytes + batch.key_data.nbytes +
                                           16 * n),
            "cfg2_host_path_note": "chip_verify_batch from pageable host buffers: H2D of every pool + index array "
                                   "in signature chunks, each chunk's copy beside the previous chunk's kernels "
                                   "(key tables built once), D2H of status + bitmap",
            "cfg2_host_path_correct": bool(np.array_equal(hst, batch.expected)),
            "cfg2_host_path_iter_ms": [round(x, 3) for x in it_ms],
            "cfg2_host_path_cgroup": {"cpu_quota": quota,
                                      "throttled_periods": None if thr_n0 is None else thr_n1 - thr_n0,
                                      "throttled_ms": None if thr_ms0 is None else round(thr_ms1 - thr_ms0, 3)},
            "cfg2_host_path_staging": "library pinned ring (CHIP_STAGING_RING=1)"
                                      if os.environ.get("CHIP_STAGING_RING", "0") not in ("", "0")
                                      else "HIP runtime pageable path (the default; the ring is opt-in)",
        })
        # the same from page-locked host buffers (chip_alloc_pinned: the JNI layer's direct ByteBuffers)
        pb = copy.copy(batch)
        for f in SIG_FIELDS:
            setattr(pb, f, ctx.pinned_copy(getattr(batch, f)))
        ctx.verify_batch(pb)
        pit_ms = []
        for _ in range(HOST_ITERS):
            t1 = time.perf_counter()
            pst, _bm = ctx.verify_batch(pb)
            pit_ms.append((time.perf_counter() - t1) * 1e3)
        pel = max_over_ranks(float(np.median(pit_ms)) / 1e3, world, torch, dev, dist)
        secondary.update({
            "cfg2_host_path_pinned_sigs_per_s": world * n / pel,
            "cfg2_host_path_pinned_ms": pel * 1e3,
            "cfg2_host_path_pinned_correct": bool(np.array_equal(pst, batch.expected)),
            "cfg2_host_path_pinned_iter_ms": [round(x, 3) for x in pit_ms],
        })
        if world == 1 and not args.no_group:
            secondary["group_cfg2_host_pinned"] = group_cfg2_leg(native, local, batch, pb, pel)
            progress("cfg2 device-group leg done")
        del pb
        ctx.free_pinned()

    progress("cfg2 host path done")
    # ---- cold keys: every signature its own key (the split Straus path; CHIP_ED_STRAUS_SPLIT=0 the fused kernel) ----
    if args.cold_n:
        cb = G.ed25519_batch(args.cold_n, n_keys=args.cold_n, seed=0x5EED0012 + rank, threads=gen_threads)
        dc = upload(cb, SIG_FIELDS, torch, dev)
        dc.schemes_hint = ED_HINT
        cst = torch.empty(cb.n, dtype=torch.uint8, device=dev)
        cbm = torch.empty((cb.n + 63) // 64, dtype=torch.int64, device=dev)
        for _ in range(2):
            ctx.verify_batch_device(dc, cst, cbm, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        cok = bool(np.array_equal(cst.cpu().numpy(), cb.expected))
        ctx.reset_stats()
        cel = timed_steps(lambda: ctx.verify_batch_device(dc, cst, cbm, stream=stream.cuda_stream), max(2, args.steps),
                          world, torch, dev, dist)
        sc = ctx.stats()
        st_ms = kms(sc, native.K_ED25519)
        cold_split = os.environ.get("CHIP_ED_STRAUS_SPLIT", "1") != "0"
        c_arith = int(((cb.expected == 0) | (cb.expected == 1)).sum())
        secondary.update({
            "ed25519_cold_sigs_per_s": world * cb.n * max(2, args.steps) / cel,
            "ed25519_cold_workload": "%d Ed25519 signatures, every one by its own key (key decode + Straus "
                                     "schedule, 10%% corrupted)" % cb.n,
            "ed25519_cold_correct": cok,
            "ed25519_cold_ms_per_batch": cel / max(2, args.steps) * 1e3,
            "ed25519_cold_keyprep_ms": kms(sc, native.K_KEYPREP),
            "ed25519_cold_straus_ms": st_ms,
            "ed25519_cold_roofline_frac": (ED_STRAUS_SPLIT_MACS_PER_VERIFY if cold_split else ED_STRAUS_MACS_PER_VERIFY)
            * c_arith / (st_ms * 1e-3) / 1e12 / MAC_PEAK_T,
            "ed25519_cold_schedule": "split Straus: hash + [S]B comb beside the key prep, k_ed25519_verify_a + batched "
                                     "finish" if cold_split else "fused k_ed25519_verify",
        })
        del dc, cst, cbm, cb

    progress("cold-key leg done")
    # ---- cfg4: tx ids alone, then ids + required signers fused (1M tx, 2M Ed25519 signers) ----
    if not args.no_txid:
        tb, tm, sb, ids_ref, _msgs = G.cfg4_workload(args.txid_n, n_keys=args.keys, seed=0x5EED0004 + rank,
                                                    threads=gen_threads)
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
        tel = timed_steps(lambda: ctx.txid_batch_device(dt, ids, stream=stream.cuda_stream), ts, world, torch, dev,
                          dist)
        s2 = ctx.stats()
        tx_ms = kms(s2, native.K_TXID)
        comp_per_tx = sha256_compressions(tb)
        secondary.update({
            "txids_per_s": world * tb.ntx * ts / tel,
            "txid_workload": "cfg4 profile: %d tx x 8 components (groups 0-5, 2.1 KB/tx), %d SHA-256 compressions/tx"
                             % (tb.ntx, comp_per_tx),
            "txid_correct": ids_ok,
            "txid_kernel_ms": tx_ms,
            "txid_roofline_frac": (comp_per_tx * SHA256_OPS_PER_COMPRESSION * tb.ntx / (tx_ms * 1e-3) / 1e12)
                                  / INT32_PEAK_TOPS,
            "txid_roofline_note": "canonical %d int32 ops per SHA-256 compression x %d compressions/tx vs the %.1f T "
                                  "VALU lane-op peak" % (SHA256_OPS_PER_COMPRESSION, comp_per_tx, INT32_PEAK_TOPS),
            "txid_traffic": profile_traffic("k_txid", (tb.ntx + 63) // 64 * 64),   # TX_BLOCK 64
            # the instructions it issues (SQ_INSTS_VALU of the committed profile; fused add3 / bitop3 / alignbit
            # instructions do two or three canonical ops) and the cycles each took per SIMD at the profiled clock
            # (2.3-2.6 = dual-issue bound, ~4.2 = single-issue bound, more = waiting on memory / dependencies)
            "txid_issue": profile_issue("k_txid", (tb.ntx + 63) // 64 * 64),
            "txid_algorithmic_bytes": int(tb.data.nbytes + tb.salts.nbytes + 32 * tb.ntx + 20 * len(tb.comp_len)),
        })
        # fused: ids -> SignableData messages -> 2 signers per tx -> required signers (verifySignaturesExcept)
        q = G.cfg4_required(sb, tb.ntx, args.keys, seed=0x5EED0006 + rank)
        dm = upload(tm, ("data", "off", "len", "id_at"), torch, dev)
        dm.max_len = tm.max_len
        ds = upload(sb, ("tx_idx", "tmpl_idx", "key_idx", "sig_data", "sig_off", "sig_len", "key_data", "key_off",
                         "key_len"), torch, dev)
        dq = upload(q, ("sig_start", "req_start", "node_start", "node_val", "node_nkids", "node_weight"), torch, dev)
        dq.ntx = q.ntx
        fst = torch.empty(sb.n, dtype=torch.uint8, device=dev)
        fv = torch.empty(tb.ntx, dtype=torch.uint8, device=dev)
        fa = torch.empty(tb.ntx, dtype=torch.int32, device=dev)
        fm = torch.empty(len(q.node_start) - 1, dtype=torch.uint8, device=dev)

        def fused():
            ctx.verify_signed_tx_batch_device(dt, dm, ds, dq, ids, fst, fv, fa, fm, stream=stream.cuda_stream)
        for _ in range(2):
            fused()
        torch.cuda.synchronize(dev)
        fused_ok = bool(np.array_equal(fst.cpu().numpy(), sb.expected)) and \
            bool(np.array_equal(ids.cpu().numpy().reshape(-1, 32), ids_ref)) and \
            bool(np.array_equal(fv.cpu().numpy(), q.expected_verdict)) and \
            bool(np.array_equal(fa.cpu().numpy().view(np.uint32), q.expected_arg))
        vcounts = np.bincount(fv.cpu().numpy(), minlength=4)
        ctx.reset_stats()
        fel = timed_steps(fused, ts, world, torch, dev, dist)
        s3 = ctx.stats()
        secondary.update({
            "cfg4_verified_tx_per_s": world * tb.ntx * ts / fel,
            "cfg4_signers_per_s": world * sb.n * ts / fel,
            "cfg4_ms_per_batch": fel / ts * 1e3,
            "cfg4_required_kernel_ms": kms(s3, native.K_REQ),
            "cfg4_workload": "%d SignedTransactions, verifySignaturesExcept: id recomputed + %d Ed25519 signatures "
                             "(owner of %d keys + notary) verified against it (1%% corrupted) + requiredSigningKeys "
                             "check on the device (2%% CompositeKey 1-of-2, 1%% with a party that did not sign)"
                             % (tb.ntx, sb.n, args.keys),
            "cfg4_verdicts": {"ok": int(vcounts[0]), "signature_exception": int(vcounts[1]),
                              "signatures_missing": int(vcounts[2]), "malformed": int(vcounts[3])},
            "cfg4_correct": fused_ok,
        })
        del dq, fv, fa, fm, q
        del dt, ids, dm, ds, fst, tb, tm, sb

        # verifySignaturesExcept from the bytes alone (§8f-2): 1M SignedTransaction blobs (Kryo) whose command /
        # notary components are real Command / Party objects; the device parses them, derives
        # requiredSigningKeys, recomputes the ids and verifies -- no host-built batch at all
        tb, tm, sb, ids_ref, want_v, want_a = G.cfg4_workload_commands(args.txid_n, n_keys=args.keys,
                                                                       seed=0x5EED0014 + rank, threads=gen_threads)
        bdata, boff, blen = G.stx_uniform(tb, sb, 2)
        # two blob buffers (the pipelined leg alternates them), each with room for the de-chunked runs behind
        # the blobs: chip_stx_parse_device parses in place (data_capacity), no copy of the 3 GB of blobs
        nbytes = int(bdata.nbytes)
        bcap = nbytes + nbytes // 2 + (1 << 20)
        bbs = []
        for _ in range(2):
            x = torch.empty(bcap, dtype=torch.uint8, device=dev)
            x[:nbytes].copy_(torch.from_numpy(bdata))
            bbs.append(x)
        bb = bbs[0]
        bo, bl = torch.from_numpy(boff).to(dev), torch.from_numpy(blen).to(dev)
        # the host-buffer leg's blobs: page-locked, what the JNI binding hands chip_stx_verify
        hb = ctx.pinned_copy(bdata) if not args.no_host_path else None
        del bdata
        dm = upload(tm, ("data", "off", "len", "id_at"), torch, dev)
        dm.max_len = tm.max_len
        ids = torch.empty(tb.ntx * 32, dtype=torch.uint8, device=dev)
        fst = torch.empty(sb.n, dtype=torch.uint8, device=dev)
        fv = torch.empty(tb.ntx, dtype=torch.uint8, device=dev)
        fa = torch.empty(tb.ntx, dtype=torch.int32, device=dev)
        fm = torch.empty(2 * tb.ntx + 16, dtype=torch.uint8, device=dev)
        bst = torch.empty(tb.ntx, dtype=torch.uint8, device=dev)
        meta = np.array([[1, 4]], dtype=np.int32)
        holder = {}

        def from_bytes():
            holder["p"] = ctx.stx_parse_device(bb, bo, bl, nbytes, meta, bst, stream=stream.cuda_stream,
                                               required=True, data_capacity=bcap)
            ctx.verify_signed_tx_parsed_device(holder["p"], dm, None, ids, fst, fv, fa, fm, stream=stream.cuda_stream)
        for _ in range(2):
            from_bytes()
        torch.cuda.synchronize(dev)
        bytes_ok = bool(int((bst != 0).sum()) == 0) and bool(np.array_equal(fst.cpu().numpy(), sb.expected)) and \
            bool(np.array_equal(ids.cpu().numpy().reshape(-1, 32), ids_ref)) and \
            bool(np.array_equal(fv.cpu().numpy(), want_v)) and \
            bool(np.array_equal(fa.cpu().numpy().view(np.uint32), want_a))
        bvc = np.bincount(fv.cpu().numpy(), minlength=4)
        ctx.reset_stats()
        bel_serial = timed_steps(from_bytes, ts, world, torch, dev, dist)
        s4 = ctx.stats()
        parse_ms = kms(s4, native.K_STX)
        # pipelined: batch k + 1 is parsed on a second stream while batch k is verified (the front end's
        # two buffer sets alternate; the parse of batch k + 2 waits for the verification of batch k)
        # the parse stream at a higher priority (CORDA_PARSE_PRIORITY, torch convention: lower = higher; 0 = equal):
        # the verify kernels fill every wave slot, so at equal priority the parse's workgroups wait for them to drain,
        # while the latency-bound parse slots in beside the issue-bound verify at a higher one (73.3-74.1M at equal
        # priority vs 78.7-78.8M, profiles/r05/ab_r05q.txt)
        s_parse = torch.cuda.Stream(dev, priority=int(os.environ.get("CORDA_PARSE_PRIORITY", "-1")))
        evs = [None, None]

        def from_bytes_pipelined():
            k = holder.get("k", 0)
            if evs[k % 2] is not None:
                s_parse.wait_event(evs[k % 2])
            holder["p"] = ctx.stx_parse_device(bbs[k % 2], bo, bl, nbytes, meta, bst, stream=s_parse.cuda_stream,
                                               required=True, data_capacity=bcap)
            ctx.verify_signed_tx_parsed_device(holder["p"], dm, None, ids, fst, fv, fa, fm, stream=stream.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(stream)
            evs[k % 2] = ev
            holder["k"] = k + 1
        for _ in range(3):
            from_bytes_pipelined()
        torch.cuda.synchronize(dev)
        bytes_ok = bytes_ok and bool(np.array_equal(fv.cpu().numpy(), want_v)) and \
            bool(np.array_equal(fst.cpu().numpy(), sb.expected))
        bel = timed_steps(from_bytes_pipelined, ts, world, torch, dev, dist)
        p = holder["p"]
        blob_bytes = nbytes
        host_bytes = {}
        if hb is not None:
            # host-buffer entry (PCIe-inclusive): the blobs in page-locked host memory through chip_stx_verify,
            # which copies transaction chunks beside the previous chunk's parse and verification
            hres = {}

            def from_bytes_host():
                hres["r"] = ctx.stx_verify(hb, boff, blen, tm, meta)
            from_bytes_host()
            hst_, hv, ha, _ = hres["r"]
            host_ok = bool(not hst_.any() and np.array_equal(hv, want_v) and np.array_equal(ha, want_a))
            hsteps = max(2, ts // 2)
            hel = timed_steps(from_bytes_host, hsteps, world, torch, dev, dist)
            # the PCIe bound of this leg: the same bytes copied alone (pinned -> device, one copy)
            hdst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            hsrc = torch.from_numpy(hb)
            torch.cuda.synchronize(dev)
            t_h = time.perf_counter()
            hdst.copy_(hsrc, non_blocking=True)
            torch.cuda.synchronize(dev)
            h2d_gbs = nbytes / (time.perf_counter() - t_h) / 1e9
            del hdst, hsrc
            host_bytes = {
                "cfg4_from_bytes_host_tx_per_s": world * tb.ntx * hsteps / hel,
                "cfg4_from_bytes_host_ms_per_batch": hel / hsteps * 1e3,
                "cfg4_from_bytes_host_correct": host_ok,
                "cfg4_from_bytes_host_h2d_GBps": h2d_gbs,
                "cfg4_from_bytes_host_pcie_bound_tx_per_s": world * tb.ntx / (nbytes / (h2d_gbs * 1e9)),
                "cfg4_from_bytes_host_note": "chip_stx_verify from page-locked host blobs (PCIe included): transaction "
                                             "chunks, chunk j+1's blobs copied on a second stream beside chunk j's "
                                             "parse + verify; the pcie bound is the blob bytes / the measured "
                                             "pinned H2D rate",
            }
        # algorithmic bytes of one parse: the blobs read once, the index arrays written (components 20 B,
        # signatures 40 B incl. the key interning, required keys 16 B, tx 56 B)
        alg = blob_bytes + 20 * int(p.txs.ncomp) + 40 * int(p.sigs.n) + 16 * int(p.req.nreq) + 56 * tb.ntx
        secondary.update({
            "cfg4_from_bytes_verified_tx_per_s": world * tb.ntx * ts / bel,
            "cfg4_from_bytes_ms_per_batch": bel / ts * 1e3,
            "cfg4_from_bytes_serial_verified_tx_per_s": world * tb.ntx * ts / bel_serial,
            "cfg4_from_bytes_note": "value = parse of batch k+1 on a second, higher-priority HIP stream overlapping "
                                    "the verification of batch k (steady state over the timed steps); serial = "
                                    "parse then verify on one stream",
            "cfg4_from_bytes_correct": bytes_ok,
            **host_bytes,
            "cfg4_from_bytes_verdicts": {"ok": int(bvc[0]), "signature_exception": int(bvc[1]),
                                         "signatures_missing": int(bvc[2]), "malformed": int(bvc[3])},
            "cfg4_from_bytes_workload": "%d SignedTransaction blobs (Kryo, %d B each, %.2f GB resident): parse + "
                                        "requiredSigningKeys from the Command / notary components + ids + "
                                        "SignableData messages + 2 Ed25519 signatures/tx + required-signer check, "
                                        "all on the device (1%% corrupted signatures, 1%% commands naming a "
                                        "non-signing party)" % (tb.ntx, int(blen[0]), blob_bytes / 1e9),
            "stx_parse_ms": parse_ms,
            "stx_parse_tx_per_s": world * tb.ntx / (parse_ms * 1e-3),
            "stx_parse_roofline": {"bound": "hbm", "achieved": alg / (parse_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": alg / (parse_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                   "algorithmic_bytes": alg,
                                   "traffic": stx_traffic(tb.ntx, sb.n, int(tb.comp_len.size)),
                                   "note": "one launch = the fused pass 1 (pass 2 only for blobs past its rows), "
                                           "scans, de-chunk copies, row transposes, key interning and the "
                                           "required-key passes with their 3 host syncs"},
        })
        del bb, bbs, bo, bl, bst, holder, p, dm, ids, fst, fv, fa, fm, tb, tm, sb, evs, s_parse, hb
    progress("cfg4 legs done")
    # ---- cfg3: mixed ECDSA r1/k1, one global batch sharded by transaction, RCCL bitmap all-gather ----
    if not args.no_ecdsa:
        secondary.update(ecdsa_leg(args, ctx, world, rank, torch, dev, dist, D, G, native, gen_threads, stream))

    progress("cfg3 legs done")
    # ---- cfg5: notary batch (uniqueness against a 10M-row log + one notary signature per tx) ----
    if not args.no_notary:
        secondary.update(notary_leg(args, ctx, world, rank, torch, dev, dist, D, G, native, gen_threads, stream))

    progress("cfg5 leg done")
    # ---- CPU baselines (rank 0, N = 1 only): the oracle restatement and OpenSSL on host cores ----
    cpu = cpu_ossl = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle_bind as O
        m = min(args.cpu_sample, n)
        sub = sub_batch(G, batch, m)
        t2 = time.perf_counter()
        ref = O.verify_batch(sub, threads=threads)
        cel = time.perf_counter() - t2
        share_note = "%d threads = this process's CPU share (nproc %d; %s)" % (threads, nproc, cpu_model())
        cpu = {"value": m / cel, "unit": "verified sigs/s", "cores": threads, "kind": "port",
               "sample": "first %d signatures of the same cfg2 batch through oracle/ (C restatement of i2p eddsa 0.2.0 "
                         "semantics); %s" % (m, share_note),
               "nproc": nproc, "cpu_model": cpu_model(),
               "agrees_with_gpu": bool(np.array_equal(ref, st[:m]))}
        if not args.no_full_oracle:
            # parity at full size: every status byte of the timed cfg2 batch against the oracle (untimed)
            t2 = time.perf_counter()
            ref_full = O.verify_batch(batch, threads=threads)
            cpu["oracle_full_batch"] = {"sigs": int(n), "agrees_with_gpu": bool(np.array_equal(ref_full, st)),
                                        "mismatches": int((ref_full != st).sum()),
                                        "seconds": time.perf_counter() - t2}
            del ref_full
        # OpenSSL EVP_DigestVerify (BASELINE.md substitute B): Ed25519 on the cfg2 sample, ECDSA on a
        # P-256 and a secp256k1 sample; keys decoded once per thread
        mo = min(4 * args.cpu_sample, n)
        subo = sub_batch(G, batch, mo)
        t2 = time.perf_counter()
        ok = G.ossl_verify_batch(subo, threads=threads)
        oel = time.perf_counter() - t2
        s1 = sub_batch(G, batch, min(8192, n))
        t2 = time.perf_counter()
        G.ossl_verify_batch(s1, threads=1)
        one_thread = len(s1.key_idx) / (time.perf_counter() - t2)
        eb = G.ecdsa_batch(8192, n_keys=256, seed=0x5EED0023, threads=gen_threads)
        ec_rates = {}
        for name, sch in (("p256", G.SCHEME_R1), ("secp256k1", G.SCHEME_K1)):
            sel = np.nonzero(eb.scheme == sch)[0]
            se = G.SigBatch()
            se.key_idx, se.msg_idx, se.sig_off, se.sig_len = (eb.key_idx[sel], eb.msg_idx[sel], eb.sig_off[sel],
                                                              eb.sig_len[sel])
            se.sig_data, se.key_data, se.key_off, se.key_len = eb.sig_data, eb.key_data, eb.key_off, eb.key_len
            se.msg_data, se.msg_off, se.msg_len = eb.msg_data, eb.msg_off, eb.msg_len
            reps = 4
            t2 = time.perf_counter()
            for _ in range(reps):
                G.ossl_verify_batch(se, threads=threads)
            ec_rates[name] = reps * len(sel) / (time.perf_counter() - t2)
        cpu_ossl = {"value": mo / oel, "unit": "verified Ed25519 sigs/s", "cores": threads, "kind": "openssl",
                    "sample": "first %d signatures of the cfg2 batch, OpenSSL %s EVP_DigestVerify; %s"
                              % (mo, "3.x", share_note),
                    "single_thread_sigs_per_s": one_thread,
                    "thread_scaling": (mo / oel) / one_thread,
                    "ecdsa_p256_sigs_per_s": ec_rates["p256"], "ecdsa_secp256k1_sigs_per_s": ec_rates["secp256k1"],
                    "note": "OpenSSL rejects the i2p-specific reference-valid classes (S+L, small-order forgeries): "
                            "%d of %d accepted vs %d reference-valid" % (int(ok.sum()), mo,
                                                                        int((batch.expected[:mo] == 0).sum()))}

    # CPU baselines of the secondary legs (rank 0, N = 1): the reference-semantics restatement (oracle/) on
    # bounded samples of each workload shape, threads = this process's CPU share (north_star: the
    # reference path timed beside each run; the JVM path itself cannot run here)
    cpu_legs = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle_bind as O
        share_note = "%d threads = this process's CPU share (nproc %d; %s)" % (threads, nproc, cpu_model())
        cpu_legs = {}
        if not args.no_ecdsa:
            m3 = 4096
            eb3 = G.ecdsa_batch(m3, n_keys=4096, corrupt=0.10, seed=0x5EED0033, threads=gen_threads)
            t2 = time.perf_counter()
            ref3 = O.verify_batch(eb3, threads=threads)
            el3 = time.perf_counter() - t2
            t2 = time.perf_counter()
            G.ossl_verify_batch(eb3, threads=threads)
            elo3 = time.perf_counter() - t2
            cpu_legs["cfg3"] = {"value": m3 / el3, "unit": "verified ECDSA sigs/s (r1/k1 mixed)", "cores": threads,
                                "kind": "port", "openssl_sigs_per_s": m3 / elo3,
                                "agrees_with_labels": bool(np.array_equal(ref3, eb3.expected)),
                                "sample": "%d signatures of the cfg3 shape (4,096 keys per curve, 10%% corrupted) "
                                          "through oracle/ (BC 1.57 semantics) and OpenSSL EVP_DigestVerify; %s"
                                          % (m3, share_note)}
        if not args.no_txid:
            m4 = 4096
            tb4, tm4, sb4, ids4, msgs4 = G.cfg4_workload(m4, n_keys=args.keys, seed=0x5EED0034, threads=gen_threads)
            q4 = G.cfg4_required(sb4, m4, args.keys, seed=0x5EED0036)
            b4 = G.signer_sig_batch(sb4, msgs4)
            t2 = time.perf_counter()
            oid = O.txid_batch(tb4, threads=threads)
            st4 = O.verify_batch(b4, threads=threads)
            v4, a4, _m4 = O.required_signers(q4, b4, st4)
            el4 = time.perf_counter() - t2
            cpu_legs["cfg4"] = {"value": m4 / el4, "unit": "fully verified tx/s (verifySignaturesExcept)",
                                "cores": threads, "kind": "port",
                                "agrees": bool(np.array_equal(oid, ids4)) and
                                          bool(np.array_equal(v4, q4.expected_verdict)),
                                "sample": "%d cfg4 transactions: tx id (oracle/txid_ref.c) + 2 Ed25519 signatures "
                                          "(oracle/ed25519_ref.c) + required signers (oracle/required_ref.c); %s"
                                          % (m4, share_note)}
        chk = secondary.get("notary_oracle_check")
        if chk and chk.get("oracle_commit_s"):
            cpu_legs["cfg5"] = {"value": chk["nref"] / chk["oracle_commit_s"], "unit": "input StateRefs/s",
                                "cores": 1, "kind": "port",
                                "sample": "the whole cfg5 batch (%d input StateRefs against the 10M-row log) through "
                                          "oracle/uniq_ref.c's ordered commit, one thread: the reference commits "
                                          "under one global lock (PersistentUniquenessProvider.kt:56-60), so its "
                                          "parallelism is one" % chk["nref"]}

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
            "roofline": {"bound": "valu", "achieved": achieved, "peak": MAC_SPEC_T,
                         "unit": "T MAC/s (v_mad_u64_u32 32x32->64)", "frac": achieved / MAC_SPEC_T,
                         "traffic": traffic,
                         "traffic_note": "FETCH_SIZE+WRITE_SIZE bytes per launch, %s (same grid); vs ~%d B/sig "
                                         "algorithmic (h 32 + [S]B 160 in, key table entries read from L2, R' 120 out)"
                                         % (os.path.relpath(PROFILE_DIR, ROOT), 312),
                         "peak_note": "v_mad_u64_u32 issues once per 4 cycles per SIMD: 256 CU x 4 SIMD x 64 lanes "
                                      "/ 4 x 2.4 GHz = 39.3 T; frac_spec_dual_issue prices against the guide's 78.6 T "
                                      "VALU lane-op peak (2-cycle issue, which only the simple 32-bit opcodes reach); "
                                      "frac_measured against the microbench MAC rate (36.5 T at 2.38 GHz) rescaled to "
                                      "the kernel's own clock from its GRBM_GUI_ACTIVE pass",
                         "frac_spec_dual_issue": achieved / INT32_PEAK_TOPS,
                         "frac_measured": (achieved / (MAC_MEASURED_T * ahalf_issue["eff_clock_ghz"] /
                                                       MAC_MEASURED_CLOCK_GHZ)) if ahalf_issue else None,
                         "effective_clock_ghz": ahalf_issue["eff_clock_ghz"] if ahalf_issue else None,
                         "issue_model": ({
                             "valu_instr_per_sig": ahalf_issue["valu_per_launch"] * 64 / comb_grid,
                             "macs_per_sig": ED_COMB_MACS_A,
                             "cyc_per_valu_profiled": ahalf_issue["cyc_per_valu"],
                             "predicted_ms": ahalf_issue["valu_per_launch"] / 1024 * VALU_ISSUE_CYCLES /
                                             (ahalf_issue["eff_clock_ghz"] * 1e6),
                             "frac": ahalf_issue["valu_per_launch"] / 1024 * VALU_ISSUE_CYCLES /
                                     (ahalf_issue["eff_clock_ghz"] * 1e6) / a_ms,
                             "note": "time >= VALU wave-instructions / 1024 SIMDs x %.1f cycles / effective clock "
                                     "(SQ_INSTS_VALU and GRBM_GUI_ACTIVE of the committed pass, tools/"
                                     "issue_summary.py); the MACs are %.0f%% of the instructions, the rest are "
                                     "carries, reductions, table selects and loads' address arithmetic"
                                     % (VALU_ISSUE_CYCLES, 100.0 * ED_COMB_MACS_A * comb_grid / 64 /
                                        ahalf_issue["valu_per_launch"])} if ahalf_issue else None),
                         "kernel": "k_ed_comb_ahalf", "kernel_ms": a_ms,
                         "units_per_launch": n_comb, "macs_per_unit": ED_COMB_MACS_A,
                         "both_halves_frac": ED_COMB_MACS_PER_VERIFY * n_comb / ((a_ms + b_ms) * 1e-3) / 1e12 / MAC_SPEC_T,
                         "comb_share_of_step": (a_ms + b_ms) / ms_per_step,
                         "pipeline_ms": {"keyprep": kp_ms, "comb_plan": plan_ms, "comb_tables_aux_stream": tab_ms,
                                         "comb_bhalf": b_ms, "comb_ahalf": a_ms, "comb_finish": fin_ms,
                                         "straus_verify": straus_ms}},
            "cpu_baseline": cpu,
            "cpu_baseline_openssl": cpu_ossl,
            "cpu_baselines_secondary": cpu_legs,
            "secondary": secondary,
            "gen_s": gen_s,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def ecdsa_leg(args, ctx, world, rank, torch, dev, dist, D, G, native, threads, stream):
    """cfg3: a global mixed r1/k1 batch (2 signatures per transaction) sharded by transaction across
    the ranks: each rank verifies its own contiguous tx range of args.ecdsa_n / 8 signatures (the
    4M / 8-GPU share) and the per-rank bitmaps are all-gathered over RCCL.  The per-GPU
    work is the same at every N (weak scaling; the global batch is the full 4M at N = 8).  Plus a
    P-256-only batch of the same size."""
    share = args.ecdsa_n // 8
    share -= share % 2
    eb = G.ecdsa_batch(share, n_keys=args.keys, seed=0x5EED0003 + rank, threads=threads)
    de = upload(eb, SIG_FIELDS, torch, dev)
    de.schemes_hint = EC_HINT
    est = torch.empty(eb.n, dtype=torch.uint8, device=dev)
    ebm = torch.empty((eb.n + 63) // 64, dtype=torch.int64, device=dev)
    gath = torch.empty(world * ebm.numel(), dtype=torch.int64, device=dev) if world > 1 else None

    def step():
        ctx.verify_batch_device(de, est, ebm, stream=stream.cuda_stream)
        all_gather_bitmap(gath, ebm, world, dist)

    for _ in range(2):
        step()
    torch.cuda.synchronize(dev)
    ecorrect = min_over_ranks_bool(bool(np.array_equal(est.cpu().numpy(), eb.expected)), world, torch, dev, dist)
    ctx.reset_stats()
    ts = max(2, args.steps)
    eel = timed_steps(step, ts, world, torch, dev, dist)
    s3 = ctx.stats()
    r1_ms, k1_ms, front_ms, tab_ms = (kms(s3, native.K_ECDSA_R1), kms(s3, native.K_ECDSA_K1),
                                      kms(s3, native.K_EC_FRONT), kms(s3, native.K_EC_TABLES))
    n_arith = int(((eb.expected == 0) | (eb.expected == 1)).sum())
    step_ms = eel / ts * 1e3
    out = {
        "ecdsa_mixed_sigs_per_s": world * eb.n * ts / eel,
        "ecdsa_workload": "cfg3: %d mixed ECDSA sigs (r1/k1 interleaved, 10%% corrupted, %d keys per curve), %d per "
                          "GPU, sharded by transaction, RCCL bitmap all-gather" % (world * eb.n, args.keys, eb.n),
        "ecdsa_correct_vs_labels": ecorrect,
        "ecdsa_ms_per_step": step_ms,
        "ecdsa_front_ms": front_ms, "ecdsa_tables_aux_ms": tab_ms,
        "ecdsa_q_kernel_ms": r1_ms + k1_ms,   # k_ecdsa_comb_q: low + high table half, both curves per launch
        "ecdsa_roofline_frac": ECDSA_MIXED_MACS_PER_VERIFY * n_arith / (step_ms * 1e-3) / 1e12 / MAC_PEAK_T,
        "ecdsa_q_roofline_frac": ECDSA_MIXED_Q_MACS_PER_VERIFY * n_arith / ((r1_ms + k1_ms) * 1e-3) / 1e12 / MAC_PEAK_T,
        "ecdsa_roofline_note": "%d MACs/signature (mean of P-256's 82 mixed additions and secp256k1's 69 with GLV, x "
                               "592, + scalar work) over the whole step; q kernels %d MACs/signature over their own time"
                               % (ECDSA_MIXED_MACS_PER_VERIFY, ECDSA_MIXED_Q_MACS_PER_VERIFY),
    }
    # the same batch with the key state kept across batches (CHIP_FLAG_KEY_CACHE, a context of its own): the
    # per-key comb tables (ecdsa_tables_aux_ms above) are reused from the previous step
    if not args.no_key_cache:
        import corda_amd
        kctx = corda_amd.Context(torch.cuda.current_device(), flags=native.FLAG_KEY_CACHE)

        def kstep():
            kctx.verify_batch_device(de, est, ebm, stream=stream.cuda_stream)
            all_gather_bitmap(gath, ebm, world, dist)

        for _ in range(2):
            kstep()
        torch.cuda.synchronize(dev)
        kok = min_over_ranks_bool(bool(np.array_equal(est.cpu().numpy(), eb.expected)), world, torch, dev, dist)
        kel = timed_steps(kstep, ts, world, torch, dev, dist)
        out.update({"ecdsa_key_cache_sigs_per_s": world * eb.n * ts / kel, "ecdsa_key_cache_ms_per_step": kel / ts * 1e3,
                    "ecdsa_key_cache_correct": kok})
        kctx.close()
    del de, est, ebm, gath, eb
    # P-256 only (ECDSA_SECP256R1_SHA256): the same share size, every signature on secp256r1
    pb = G.ecdsa_batch(share, n_keys=args.keys, seed=0x5EED0013 + rank, threads=threads, schemes=(G.SCHEME_R1,))
    dp = upload(pb, SIG_FIELDS, torch, dev)
    dp.schemes_hint = 1 << 3
    pst = torch.empty(pb.n, dtype=torch.uint8, device=dev)
    pbm = torch.empty((pb.n + 63) // 64, dtype=torch.int64, device=dev)
    for _ in range(2):
        ctx.verify_batch_device(dp, pst, pbm, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    pok = min_over_ranks_bool(bool(np.array_equal(pst.cpu().numpy(), pb.expected)), world, torch, dev, dist)
    ctx.reset_stats()
    pel = timed_steps(lambda: ctx.verify_batch_device(dp, pst, pbm, stream=stream.cuda_stream), ts, world, torch, dev,
                      dist)
    sp = ctx.stats()
    p_arith = int(((pb.expected == 0) | (pb.expected == 1)).sum())
    out.update({
        "ecdsa_p256_sigs_per_s": world * pb.n * ts / pel,
        "ecdsa_p256_workload": "%d ECDSA_SECP256R1_SHA256 signatures per GPU, %d keys, 10%% corrupted" % (pb.n,
                                                                                                        args.keys),
        "ecdsa_p256_correct": pok,
        "ecdsa_p256_ms_per_step": pel / ts * 1e3,
        "ecdsa_p256_q_kernel_ms": kms(sp, native.K_ECDSA_R1) + kms(sp, native.K_ECDSA_K1),
        "ecdsa_p256_front_ms": kms(sp, native.K_EC_FRONT),
        "ecdsa_p256_roofline_frac": ECDSA_COMB_MACS_PER_VERIFY * p_arith / (pel / ts) / 1e12 / MAC_PEAK_T,
    })
    del dp, pst, pbm, pb
    return out


def group_cfg2_leg(native, local, batch, pb, single_s):
    """cfg2 through the device-group entry (chip_group_verify_batch, the path a Corda JVM reaches N GPUs by) from
    page-locked host buffers, on device lists [d] and [d, d] (two member contexts sharing this one GPU: the split,
    rebasing, member threads and the per-member table builds, not a speed-up).  Each call's split and host times
    come from chip_group_last_stats."""
    out = {"single_context_ms": single_s * 1e3}
    for devs in ([local], [local, local]):
        g = native.Group(devs)
        try:
            g.verify_batch(pb)
            its, stats = [], []
            for _ in range(HOST_ITERS):
                t1 = time.perf_counter()
                st, _bm = g.verify_batch(pb)
                its.append((time.perf_counter() - t1) * 1e3)
                stats.append(g.last_stats())
            med = float(np.median(its))
            out["x".join(str(d) for d in devs)] = {
                "members": len(devs), "sigs_per_s": batch.n / med * 1e3, "ms": med,
                "iter_ms": [round(x, 3) for x in its], "correct": bool(np.array_equal(st, batch.expected)),
                "stats": stats[int(np.argsort(its)[len(its) // 2])]}
        finally:
            g.close()
    one = out["x".join([str(local)])]
    one["vs_single_context"] = (single_s * 1e3) / one["ms"]
    out["note"] = ("chip_group_verify_batch on pinned host buffers; %s = one member (the single-context entry through "
                   "the group), %s = two member contexts on this one GPU, each verifying half the transactions and "
                   "building its own per-key tables" % (str(local), "x".join([str(local)] * 2)))
    return out


def notary_group_legs(native, ctx, local, pre, ub, st_ref, recs_ref):
    """cfg5 from page-locked host buffers: the single-context host entry (chip_uniq_commit_batch) beside the
    device-group commit (chip_group_uniq_commit_batch) on [d] and [d, d].  Each commit is timed alone after an
    untimed rebuild of the 10M-row log; statuses and every conflict record must equal the device-resident commit's,
    which bench.py compares with the oracle at full size.  The group's own split (per-member H2D bytes, the members'
    input exchange, rounds and their on-device vote exchange) comes from chip_group_uniq_last_stats."""
    ntx, nref = ub.ntx, int(ub.tx_ref_start[-1])
    pin = [ctx.pinned_copy(a) for a in (ub.tx_ref_start, ub.refs, ub.tx_ids, ub.callers)]
    whole = int(sum(a.nbytes for a in pin))
    cap = len(pre[2]) + nref + 1024
    out = {"batch_bytes_in": whole}

    def leg(name, opener, stats_of):
        times, stats, res = [], [], None
        for _ in range(3):
            t = opener()
            try:
                t.rebuild(*pre)
                t1 = time.perf_counter()
                res = t.commit_batch_raw(*pin)
                times.append((time.perf_counter() - t1) * 1e3)
                stats.append(stats_of(t))
            finally:
                t.close()
        st, raw, n = res
        ok = bool(np.array_equal(st, st_ref)) and n * 56 == len(recs_ref) and bool(np.array_equal(raw, recs_ref))
        best = int(np.argmin(times[1:])) + 1
        out[name] = {"ms": times[best], "staterefs_per_s": nref / (times[best] * 1e-3), "iter_ms": [round(x, 3) for x in times],
                     "equal_to_device_commit": ok, "stats": stats[best]}

    leg("single_context", lambda: ctx.uniq_open(cap), lambda t: {"rounds": t.last_rounds()})
    for devs in ([local], [local, local]):
        g = native.Group(devs)
        try:
            leg("group_" + "x".join(str(d) for d in devs), lambda: g.uniq_open(cap), lambda t: t.last_stats())
        finally:
            g.close()
    one = out["group_" + str(local)]
    one["vs_single_context"] = out["single_context"]["ms"] / one["ms"]
    two = out["group_" + "x".join([str(local)] * 2)]
    s2 = two["stats"]
    two["h2d_bytes_max_frac_of_batch"] = s2["h2d_bytes_max"] / whole
    two["ms_per_round_incl_vote_exchange"] = s2["rounds_ms"] / max(1, s2["rounds"])
    out["note"] = ("chip_group_uniq_commit_batch from pinned host buffers (%d tx, %d input StateRefs, %d B in): "
                   "the group of one is the single-context entry; on two members (both on this one GPU) each stages "
                   "only its slice from the host, the members exchange owned inputs and ids device to device, and the "
                   "rounds exchange votes on the devices" % (ntx, nref, whole))
    ctx.free_pinned()
    return out


def notary_leg(args, ctx, world, rank, torch, dev, dist, D, G, native, threads, stream):
    """cfg5: every rank builds the same global batch (same seed).  Uniqueness: N = 1 commits through
    chip_uniq_commit_batch_device; N > 1 runs the key-sharded protocol (each rank owns a slice of the
    commit log, one RCCL all-reduce MAX of per-tx votes per ordered-commit round).  The commit log is
    rebuilt from the pre-committed rows before each step, outside the timing.  At N = 1 the statuses
    and the conflict records are compared with the oracle (oracle/uniq_ref.c) at full size.  The
    notary's Ed25519 signature over each tx id is verified by the rank owning the tx range."""
    t_gen = time.time()
    pre, ub = G.uniq_workload(args.notary_tx, args.notary_pre, seed=0x5EED0005)
    ntx, nref = ub.ntx, int(ub.tx_ref_start[-1])
    refs, txs, idx, caller = pre
    pre_all = pre
    if world > 1:
        rows = D.route_rows(refs, world)[rank]
        pre = (refs.reshape(-1, 36)[rows].reshape(-1).copy(), txs.reshape(-1, 32)[rows].reshape(-1).copy(),
               idx[rows].copy(), caller[rows].copy())
    n_pre_local = len(pre[2])
    table = ctx.uniq_open(n_pre_local + nref // world + 1024)
    ts = 2
    times, rounds, st_sum = [], 0, None
    recs_gpu = None
    if world == 1:
        d_start, d_refs = to_dev(ub.tx_ref_start, torch, dev), to_dev(ub.refs, torch, dev)
        d_ids, d_call = to_dev(ub.tx_ids, torch, dev), to_dev(ub.callers, torch, dev)
        d_st = torch.empty(ntx, dtype=torch.uint8, device=dev)
        cap = nref + 1
        d_out = torch.empty(cap * 56, dtype=torch.uint8, device=dev)
        for _ in range(ts + 1):
            table.close()
            table = ctx.uniq_open(n_pre_local + nref + 1024)   # entries; the table keeps load <= 1/2
            table.rebuild(*pre)
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            nout = table.commit_batch_device(d_start, nref, d_refs, d_ids, d_call, d_st, d_out, cap,
                                             stream=stream.cuda_stream)
            torch.cuda.synchronize(dev)
            times.append(time.perf_counter() - t1)
        st = d_st.cpu().numpy()
        recs_gpu = d_out[:nout * 56].cpu().numpy()
        rounds = table.last_rounds()
        del d_start, d_refs, d_ids, d_call, d_st, d_out
    else:
        eng = native.UniqShardEngine(table)
        shard = D.route_uniq_batch(ub.tx_ref_start, ub.refs, world)[rank]
        dshard = eng.upload(shard, ub.tx_ids, ub.callers)
        for _ in range(ts + 1):
            table.close()
            table = ctx.uniq_open(n_pre_local + shard.nref + 1024)
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
    group = None
    if world == 1 and not args.no_group:
        group = notary_group_legs(native, ctx, dev.index, pre_all, ub, st, recs_gpu)
    counts = np.bincount(st, minlength=3)
    # full-size correctness: the oracle's ordered commit over the same log and batch (host, untimed)
    check = None
    if world == 1 and not args.no_notary_check:
        import oracle_bind as O
        t_chk = time.time()
        u = O.Uniq(capacity=2 * (len(pre_all[2]) + nref) + 1024)
        u.preload(*pre_all)
        ost = np.zeros(ntx, dtype=np.uint8)
        ocap = nref + 1
        obuf = (O.OrcConflict * ocap)()
        onout = O.ctypes.c_uint64()
        t_commit = time.perf_counter()
        O.lib().orc_uniq_commit_batch(u.h, O.ctypes.c_uint64(ntx), O._p(ub.tx_ref_start), O._p(ub.refs),
                                      O._p(ub.tx_ids), O._p(ub.callers), O._p(ost), obuf, O.ctypes.c_uint64(ocap),
                                      O.ctypes.byref(onout))
        commit_s = time.perf_counter() - t_commit
        orecs = np.frombuffer(obuf, dtype=np.uint8, count=int(onout.value) * 56)
        check = {"statuses_equal": bool(np.array_equal(st, ost)), "records_gpu": int(nout),
                 "records_oracle": int(onout.value), "records_equal": bool(np.array_equal(recs_gpu, orecs)),
                 "oracle_s": time.time() - t_chk, "oracle_commit_s": commit_s, "nref": int(nref)}
        del u, obuf, orecs
    # notary signature over every tx id (one key: the per-key comb path)
    lo, hi = ntx * rank // world, ntx * (rank + 1) // world
    keys = np.zeros((hi - lo, 1), dtype=np.int64)
    sb, tm, msgs = G.ed25519_signers(ub.tx_ids.reshape(-1, 32)[lo:hi], keys, 0, corrupt=0.0, seed=0x5EED0015,
                                     threads=threads, extra_key_seeds=(G.NOTARY_SEED,))
    gen_s = time.time() - t_gen
    sbb = G.signer_sig_batch(sb, msgs)
    del msgs
    dsb = upload(sbb, SIG_FIELDS, torch, dev)
    dsb.schemes_hint = ED_HINT
    nst = torch.empty(sbb.n, dtype=torch.uint8, device=dev)
    nbm = torch.empty((sbb.n + 63) // 64, dtype=torch.int64, device=dev)
    for _ in range(2):
        ctx.verify_batch_device(dsb, nst, nbm, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    sig_ok = bool((nst.cpu().numpy() == 0).all())
    sel = timed_steps(lambda: ctx.verify_batch_device(dsb, nst, nbm, stream=stream.cuda_stream), ts, world, torch, dev,
                      dist) / ts
    del dsb, nst, nbm
    achieved_gbs = UNIQ_BYTES_PER_REF * nref / uel / 1e9
    return {
        "notary_staterefs_per_s": nref / uel,
        "notary_tx_per_s": ntx / uel,
        "notary_commit_ms": uel * 1e3,
        "notary_roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": achieved_gbs / HBM_PEAK_GBS,
                            "note": "%d B/StateRef algorithmic (SURVEY §8d) x %d input StateRefs / commit time"
                                    % (UNIQ_BYTES_PER_REF, nref)},
        "notary_rounds": rounds,
        "notary_group_host_pinned": group,
        "notary_status_counts": {"committed": int(counts[0]), "idempotent": int(counts[1]),
                                 "conflict": int(counts[2]), "records": int(nout)},
        "notary_oracle_check": check,
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
