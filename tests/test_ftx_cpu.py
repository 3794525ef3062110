"""CPU: FilteredTransaction.verify + checkAllComponentsVisible restatement (oracle/ftx_ref.c) on
filtered transactions built the reference's way (tests/ftx_build.py), including the
PartialMerkleTreeTest.kt:153-225 scenarios expressed as filtered groups."""
import numpy as np
import pytest

import oracle_bind as O
from ftx_build import (Ftx, FtxBatch, ZERO, build_filtered, component_hash, compute_nonce, merkle_root,
                       merkle_tree, notary_workload, partial_merkle_tree, post_order, MerkleTreeException)


def run(ftxs):
    st, rs = O.ftx_verify_batch(FtxBatch(ftxs))
    return list(zip(st.tolist(), rs.tolist()))


def test_notary_workload_labels():
    ftxs, want = notary_workload(1500)
    got = run(ftxs)
    assert got == want
    assert sum(1 for s, _ in got if s == 0) > 500
    assert {r for _, r in got} >= {0, 1, 2, 3, 4, 5, 6, 8, 9}


def test_notary_flow_two_visibility_checks():
    """NonValidatingNotaryFlow.kt:26-31: verify(), then checkAllComponentsVisible(INPUTS_GROUP), then
    (TIMEWINDOW_GROUP), as visible_mask bits 0 and 5: a hidden time-window component is (2, 6) when the
    inputs are all visible, and the inputs' failure wins when both fail."""
    ftxs, want = notary_workload(1500, seed=0x5EED0016, flow=True)
    got = run(ftxs)
    assert got == want
    tw_only = [i for i, f in enumerate(ftxs) if want[i] == (2, 6) and f.groups and f.groups[0][0] == 0
               and 5 not in [g for g, *_ in f.groups]]
    assert len(tw_only) > 20
    # the same filtered transactions through check_visible = INPUTS_GROUP alone pass those
    for i in tw_only[:5]:
        f = ftxs[i]
        f.visible_mask, f.check_visible = 0, 0
        assert run([f]) == [(0, 0)]
    # ascending-ordinal order: a mask bit below check_visible still runs after it
    f = _one_group_ftx(COMPS, [0, 1], check=-1)
    f.visible_mask = (1 << 1) | (1 << 7)
    assert run([f]) == [(2, 8)]


def _one_group_ftx(comps, include_idx, visible_comps=None, check=-1):
    salt = bytes(range(1, 33))
    nonces = [compute_nonce(salt, 1, i) for i in range(len(comps))]
    hashes = [component_hash(n, c) for n, c in zip(nonces, comps)]
    tree = merkle_tree(hashes)
    pt = partial_merkle_tree(tree, [hashes[i] for i in include_idx])
    gh = [b"\xff" * 32, tree[1]]
    if visible_comps is None:
        visible_comps = include_idx
    group = (1, [comps[i] for i in visible_comps], [nonces[i] for i in visible_comps], post_order(pt))
    return Ftx(merkle_root(gh), gh, [group], check)


COMPS = [bytes([c]) * 20 for c in b"abcdef"]


@pytest.mark.parametrize("include,visible,want", [
    ([3, 5], None, (0, 0)),            # only left nodes branch (PartialMerkleTreeTest.kt:155)
    ([], None, (0, 0)),                # include zero leaves (:162)
    ([0, 1, 2, 3, 4, 5], None, (0, 0)),  # include all leaves (:168)
    ([3, 5], [3, 5, 0], (1, 5)),       # too many leaves (:188)
    ([3, 5, 0], [3, 5], (1, 5)),       # too little leaves (:196)
    ([3, 5], [3, 5, 5], (1, 5)),       # duplicate leaves (:204)
    ([3, 5], [2, 4], (1, 5)),          # different leaves (:213)
])
def test_partial_tree_scenarios(include, visible, want):
    assert run([_one_group_ftx(COMPS, include, visible)]) == [want]


def test_wrong_root_and_nothing_filtered():
    f = _one_group_ftx(COMPS, [3, 5])
    f.group_hashes = [b"\xff" * 32, merkle_root([ZERO])]            # advertised root differs
    f.id = merkle_root(f.group_hashes)
    assert run([f]) == [(1, 4)]
    blind = _one_group_ftx(COMPS, [3])
    blind.groups = []                                                 # "nothing filtered" (:141): blind sign
    assert run([blind]) == [(0, 0)]


def test_visibility():
    full = _one_group_ftx(COMPS, [0, 1, 2, 3, 4, 5], check=1)
    part = _one_group_ftx(COMPS, [0, 1], check=1)
    absent_empty = _one_group_ftx(COMPS, [0], check=0)                # group 0 hash is allOnes: fine
    absent_past = _one_group_ftx(COMPS, [0], check=7)                 # ordinal >= groupHashes.size: fine
    hidden = _one_group_ftx(COMPS, [0], check=1)
    hidden.groups = []
    assert run([full, part, absent_empty, absent_past, hidden]) == [(0, 0), (2, 8), (0, 0), (0, 0), (2, 6)]


def test_builder_rejects_like_the_reference():
    with pytest.raises(MerkleTreeException):
        merkle_tree([])
    t = merkle_tree([bytes([i]) * 32 for i in range(1, 7)])
    with pytest.raises(MerkleTreeException):
        partial_merkle_tree(t, [bytes([9]) * 32])                     # not in the tree
    with pytest.raises(ValueError):
        partial_merkle_tree(t, [ZERO])
