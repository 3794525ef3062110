"""GPU: the Kryo front end with its blobs beyond 2 GiB of the data buffer (and so an extra region of
de-chunked runs there too): every 64-bit offset the parse, k_stx_dechunk and the key interning carry
must survive the upper half of a 32-bit word.  A batch verified from those bytes must give the same
ids, signature statuses and required-signer verdicts as the generator's labels (the structured
batch the bytes were serialised from); a 32-bit or sign-extended offset anywhere breaks every one."""
import numpy as np
import pytest
import torch

import cordagen as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("base", [(1 << 31) + 12, (1 << 32) + 4])
def test_verify_from_bytes_beyond_2gib(ctx, base):
    n = 2000
    tb, tm, sb, ids_ref, want_v, want_a = G.cfg4_workload_commands(n, n_keys=64, seed=0x5EED0031, threads=4)
    bdata, boff, blen = G.stx_uniform(tb, sb, 2)
    nbytes = base + int(bdata.nbytes)
    cap = nbytes + int(bdata.nbytes) + (1 << 20)
    dev = torch.device(DEV)
    bb = torch.empty(cap, dtype=torch.uint8, device=dev)
    bb[base:base + bdata.nbytes].copy_(torch.from_numpy(bdata))
    bo = torch.from_numpy((boff.astype(np.uint64) + np.uint64(base)).astype(boff.dtype)).to(dev)
    bl = torch.from_numpy(blen).to(dev)
    bst = torch.empty(n, dtype=torch.uint8, device=dev)
    meta = np.array([[1, 4]], dtype=np.int32)
    stream = torch.cuda.current_stream(dev)
    for in_place in (True, False):
        p = ctx.stx_parse_device(bb, bo, bl, nbytes, meta, bst, stream=stream.cuda_stream, required=True,
                                 data_capacity=cap if in_place else 0)
        dm = G.Templates()
        dm.data, dm.off, dm.len, dm.id_at = (torch.from_numpy(np.ascontiguousarray(x)).to(dev)
                                             for x in (tm.data, tm.off, tm.len, tm.id_at))
        dm.max_len = tm.max_len
        ids = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        fst = torch.empty(sb.n, dtype=torch.uint8, device=dev)
        fv = torch.empty(n, dtype=torch.uint8, device=dev)
        fa = torch.empty(n, dtype=torch.int32, device=dev)
        fm = torch.empty(2 * n + 16, dtype=torch.uint8, device=dev)
        ctx.verify_signed_tx_parsed_device(p, dm, None, ids, fst, fv, fa, fm, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        assert int((bst != 0).sum()) == 0
        assert np.array_equal(ids.cpu().numpy().reshape(-1, 32), ids_ref), in_place
        assert np.array_equal(fst.cpu().numpy(), sb.expected), in_place
        assert np.array_equal(fv.cpu().numpy(), want_v), in_place
        assert np.array_equal(fa.cpu().numpy().view(np.uint32), want_a), in_place
    del bb
    torch.cuda.empty_cache()
