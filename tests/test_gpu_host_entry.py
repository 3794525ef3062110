"""GPU: chip_verify_batch's argument checks (now on the device, before any verify kernel) and its status
counters.  An out-of-range key / message index or an (offset, length) outside its pool is CHIP_E_ARG and
nothing is verified; a valid call afterwards is unaffected and chip_stats counts its statuses."""
import copy

import numpy as np
import pytest

import cordagen as G
from corda_amd import native

pytestmark = pytest.mark.gpu


def test_bad_arguments_rejected_then_valid_call(ctx):
    b = G.ed25519_batch(512, n_keys=8, corrupt=0.25, seed=77)
    cases = []
    x = copy.copy(b)
    x.key_idx = b.key_idx.copy()
    x.key_idx[3] = len(b.key_off) + 5
    cases.append((x, "key_idx"))
    x = copy.copy(b)
    x.msg_idx = b.msg_idx.copy()
    x.msg_idx[-1] = len(b.msg_off)
    cases.append((x, "msg_idx"))
    x = copy.copy(b)
    x.sig_off = b.sig_off.copy()
    x.sig_off[100] = len(b.sig_data) - 10
    cases.append((x, "sig pool"))
    x = copy.copy(b)
    x.key_len = b.key_len.copy()
    x.key_len[0] = 10 ** 6
    cases.append((x, "key pool"))
    x = copy.copy(b)
    x.msg_off = b.msg_off.copy()
    x.msg_off[0] = 2 ** 64 - 4                       # offset + length wraps around
    cases.append((x, "msg pool"))
    for bad, what in cases:
        with pytest.raises(native.ChipError) as e:
            ctx.verify_batch(bad)
        assert "range" in str(e.value) or "outside" in str(e.value), what
    ctx.reset_stats()
    st, _bm = ctx.verify_batch(b)
    assert np.array_equal(st, b.expected)
    s = ctx.stats()
    assert [int(s.status_count[k]) for k in range(8)] == list(np.bincount(st, minlength=8))
