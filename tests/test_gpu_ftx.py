"""GPU parity: FilteredTransaction.verify + checkAllComponentsVisible (k_ftx_verify through
chip_ftx_verify_batch) vs the oracle and the Kotlin-semantics labels."""
import numpy as np
import pytest

import oracle_bind as O
from ftx_build import FtxBatch, notary_workload
from test_ftx_cpu import COMPS, _one_group_ftx

pytestmark = pytest.mark.gpu


def test_ftx_notary_workload_matches_oracle(ctx):
    ftxs, want = notary_workload(5000, seed=3)
    b = FtxBatch(ftxs)
    st, rs = ctx.ftx_verify_batch(b)
    ost, ors = O.ftx_verify_batch(b)
    assert np.array_equal(st, ost) and np.array_equal(rs, ors)
    assert list(zip(st.tolist(), rs.tolist())) == want


def test_ftx_notary_flow_mask_matches_oracle(ctx):
    """The notary flow's two checks (visible_mask = INPUTS_GROUP | TIMEWINDOW_GROUP): device == oracle ==
    the Kotlin-semantics labels, including hidden time-window components."""
    ftxs, want = notary_workload(5000, seed=0x5EED0017, flow=True)
    b = FtxBatch(ftxs)
    st, rs = ctx.ftx_verify_batch(b)
    ost, ors = O.ftx_verify_batch(b)
    assert np.array_equal(st, ost) and np.array_equal(rs, ors)
    assert list(zip(st.tolist(), rs.tolist())) == want
    assert sum(1 for w in want if w == (2, 6)) > 100


def test_ftx_scenarios(ctx):
    fs = [_one_group_ftx(COMPS, inc, vis, chk) for inc, vis, chk in
          [([3, 5], None, -1), ([], None, -1), ([0, 1, 2, 3, 4, 5], None, 1), ([3, 5], [3, 5, 0], -1),
           ([3, 5, 0], [3, 5], -1), ([3, 5], [3, 5, 5], -1), ([3, 5], [2, 4], -1), ([0, 1], None, 1)]]
    b = FtxBatch(fs)
    st, rs = ctx.ftx_verify_batch(b)
    assert list(zip(st.tolist(), rs.tolist())) == [(0, 0), (0, 0), (0, 0), (1, 5), (1, 5), (1, 5), (1, 5), (2, 8)]


def test_ftx_device_entry(ctx):
    import torch
    from corda_amd import native
    ftxs, want = notary_workload(2000, seed=8)
    b = FtxBatch(ftxs)
    dev = torch.device("cuda", 0)

    class D:
        pass
    d = D()
    d.ntx = b.ntx
    for f in native.FTX_FIELDS:
        a = np.ascontiguousarray(getattr(b, f))
        if a.dtype == np.uint64:
            a = a.view(np.int64)
        elif a.dtype == np.uint32:
            a = a.view(np.int32)
        setattr(d, f, torch.from_numpy(a).to(dev))
    st = torch.empty(b.ntx, dtype=torch.uint8, device=dev)
    rs = torch.empty(b.ntx, dtype=torch.uint8, device=dev)
    ctx.ftx_verify_batch_device(d, st, rs)
    torch.cuda.synchronize()
    assert list(zip(st.cpu().tolist(), rs.cpu().tolist())) == want
