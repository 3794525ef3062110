#!/usr/bin/env python3
"""Kryo front-end micro-bench (one GPU): 1M cfg4 SignedTransaction blobs with real Command / Party
components, parsed with CHIP_STX_REQUIRED `--steps` times (and optionally verified).  Prints one JSON line
with the parse time per call (host clock and the library's per-kernel-kind events); run it under
`rocprofv3 --kernel-trace` for the per-kernel breakdown (tools/timeline.py --marker k_stx_parse)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np
import torch

import cordagen as G
import corda_amd
from corda_amd import native


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--verify", action="store_true")
    ap.add_argument("--no-required", action="store_true", help="parse without CHIP_STX_REQUIRED")
    ap.add_argument("--copy", action="store_true", help="no data_capacity: the blobs are copied into the context")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    ctx = corda_amd.Context(0)
    t0 = time.time()
    tb, tm, sb, ids_ref, want_v, want_a = G.cfg4_workload_commands(a.n, n_keys=4096, seed=0x5EED0014, threads=16)
    bdata, boff, blen = G.stx_uniform(tb, sb, 2)
    gen_s = time.time() - t0
    # the blobs in a buffer with room for the de-chunked runs behind them: the parse runs in place
    cap = bdata.nbytes + bdata.nbytes // 2 + (1 << 20)
    bb = torch.empty(cap, dtype=torch.uint8, device=dev)
    bb[:bdata.nbytes].copy_(torch.from_numpy(bdata))
    nbytes = int(bdata.nbytes)
    if a.copy:
        cap = 0
    bo, bl = torch.from_numpy(boff).to(dev), torch.from_numpy(blen).to(dev)
    bst = torch.empty(a.n, dtype=torch.uint8, device=dev)
    meta = np.array([[1, 4]], dtype=np.int32)
    stream = torch.cuda.current_stream(dev)
    for _ in range(2):
        p = ctx.stx_parse_device(bb, bo, bl, nbytes, meta, bst, stream=stream.cuda_stream, required=not a.no_required, data_capacity=cap)
    torch.cuda.synchronize(dev)
    ok = int((bst != 0).sum()) == 0
    ctx.reset_stats()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for _ in range(a.steps):
        p = ctx.stx_parse_device(bb, bo, bl, nbytes, meta, bst, stream=stream.cuda_stream, required=not a.no_required, data_capacity=cap)
    torch.cuda.synchronize(dev)
    host_ms = (time.perf_counter() - t) / a.steps * 1e3
    s = ctx.stats()
    out = {"n": a.n, "blob_bytes": nbytes, "in_place": cap > 0, "parse_host_ms": host_ms,
           "parse_kernel_ms": s.kernel_ms_total[native.K_STX] / max(s.kernel_launches[native.K_STX], 1),
           "ncomp": int(p.txs.ncomp), "nsig": int(p.sigs.n), "n_keys": int(p.sigs.n_keys), "nreq": int(p.req.nreq),
           "status_ok": ok, "gen_s": gen_s}
    if a.verify:
        dm = G.Templates()
        dm.data, dm.off, dm.len, dm.id_at = (torch.from_numpy(np.ascontiguousarray(x)).to(dev)
                                             for x in (tm.data, tm.off, tm.len, tm.id_at))
        dm.max_len = tm.max_len
        ids = torch.empty(a.n * 32, dtype=torch.uint8, device=dev)
        fst = torch.empty(sb.n, dtype=torch.uint8, device=dev)
        fv = torch.empty(a.n, dtype=torch.uint8, device=dev)
        fa = torch.empty(a.n, dtype=torch.int32, device=dev)
        fm = torch.empty(2 * a.n + 16, dtype=torch.uint8, device=dev)
        ctx.verify_signed_tx_parsed_device(p, dm, None, ids, fst, fv, fa, fm, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        ids_ok = np.all(ids.cpu().numpy().reshape(-1, 32) == ids_ref, axis=1)
        fv_ok = fv.cpu().numpy() == want_v
        out["verify_correct"] = bool(fv_ok.all()) and \
            bool(np.array_equal(fa.cpu().numpy().view(np.uint32), want_a)) and bool(ids_ok.all())
        out["ids_wrong"] = int((~ids_ok).sum())
        out["verdicts_wrong"] = int((~fv_ok).sum())
        out["sigs_wrong"] = int((fst.cpu().numpy() != sb.expected).sum())
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
