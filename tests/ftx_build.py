"""Builds FilteredTransactions the way the reference's client side does (TEST INFRASTRUCTURE):
  WireTransaction.buildFilteredTransaction / filterWithFun   MerkleTransaction.kt:95-165
  PartialMerkleTree.build / buildPartialTree / checkFull     PartialMerkleTree.kt:61-124
  MerkleTree.getMerkleTree                                   MerkleTree.kt:27-66
in plain Python over hashlib, and packs them into the chip_ftx_batch layout (partial trees
flattened in post-order).  Independent of oracle/ and of the GPU path."""
import hashlib
import struct

import numpy as np

ZERO = bytes(32)
ONES = b"\xff" * 32


class MerkleTreeException(Exception):
    pass


def sha256(b):
    return hashlib.sha256(b).digest()


def sha256d(b):
    return sha256(sha256(b))


def compute_nonce(salt, g, i):
    return sha256d(salt + struct.pack(">ii", g, i))


def component_hash(nonce, comp):
    return sha256d(nonce + comp)


# MerkleTree: ("leaf", h) | ("node", h, left, right)
def merkle_tree(leaves):
    if not leaves:
        raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
    m = 1
    while m < len(leaves):
        m <<= 1
    level = [("leaf", h) for h in leaves] + [("leaf", ZERO)] * (m - len(leaves))
    while len(level) > 1:
        level = [("node", sha256(level[2 * k][1] + level[2 * k + 1][1]), level[2 * k], level[2 * k + 1])
                 for k in range(len(level) // 2)]
    return level[0]


def merkle_root(leaves):
    return merkle_tree(leaves)[1]


def _check_full(t, level=0):
    if t[0] == "leaf":
        return level
    a, b = _check_full(t[2], level + 1), _check_full(t[3], level + 1)
    if a != b:
        raise MerkleTreeException("Got not full binary tree.")
    return a


def _build_partial(t, include, used):
    if t[0] == "leaf":
        if t[1] in include:
            used.append(t[1])
            return True, ("incl", t[1])
        return False, ("leaf", t[1])
    lf, lt = _build_partial(t[2], include, used)
    rf, rt = _build_partial(t[3], include, used)
    if lf or rf:
        return True, ("node", lt, rt)
    return False, ("leaf", t[1])


def partial_merkle_tree(tree, include):
    """PartialMerkleTree.build(merkleRoot, includeHashes)."""
    if ZERO in include:
        raise ValueError("Zero hashes shouldn't be included in partial tree.")
    _check_full(tree)
    used = []
    _, pt = _build_partial(tree, include, used)
    if len(include) != len(used):
        raise MerkleTreeException("Some of the provided hashes are not in the tree.")
    return pt


def post_order(pt, out=None):
    """[(tag, hash)] with tag 0 IncludedLeaf, 1 Leaf, 2 Node."""
    out = [] if out is None else out
    if pt[0] == "incl":
        out.append((0, pt[1]))
    elif pt[0] == "leaf":
        out.append((1, pt[1]))
    else:
        post_order(pt[1], out)
        post_order(pt[2], out)
        out.append((2, ZERO))
    return out


class Ftx:
    """One FilteredTransaction: id, groupHashes, filtered groups [(index, comps, nonces, post-order)]."""

    def __init__(self, id, group_hashes, groups, check_visible=-1, visible_mask=0):
        self.id = id
        self.group_hashes = group_hashes
        self.groups = groups
        self.check_visible = check_visible
        self.visible_mask = visible_mask


def build_filtered(salt, component_groups, predicate, check_visible=-1):
    """WireTransaction(componentGroups, salt).buildFilteredTransaction(predicate(g, i, comp))."""
    groups = dict(component_groups)
    maxg = max(groups)
    hashes, nonces, roots = {}, {}, {}
    for g, comps in groups.items():
        nonces[g] = [compute_nonce(salt, g, i) for i in range(len(comps))]
        hashes[g] = [component_hash(n, c) for n, c in zip(nonces[g], comps)]
        roots[g] = merkle_root(hashes[g])
    group_hashes = [roots.get(g, ONES) for g in range(maxg + 1)]
    tx_id = merkle_root(group_hashes)
    filtered = []
    for g in sorted(groups):
        sel = [i for i, c in enumerate(groups[g]) if predicate(g, i, groups[g][i])]
        if not sel:
            continue
        pt = partial_merkle_tree(merkle_tree(hashes[g]), [hashes[g][i] for i in sel])
        filtered.append((g, [groups[g][i] for i in sel], [nonces[g][i] for i in sel], post_order(pt)))
    return Ftx(tx_id, group_hashes, filtered, check_visible)


class FtxBatch:
    """chip_ftx_batch layout."""

    def __init__(self, ftxs):
        self.ntx = len(ftxs)
        self.ids = np.frombuffer(b"".join(f.id for f in ftxs), dtype=np.uint8).copy()
        gh_start, gh = [0], []
        fg_start, fg_index, comp_start, pt_start = [0], [], [0], [0]
        comps, nonces, tags, phash = [], [], [], []
        for f in ftxs:
            gh += f.group_hashes
            gh_start.append(len(gh))
            for g, cs, ns, po in f.groups:
                fg_index.append(g)
                comps += cs
                nonces += ns
                comp_start.append(len(comps))
                tags += [t for t, _ in po]
                phash += [h for _, h in po]
                pt_start.append(len(tags))
            fg_start.append(len(fg_index))
        self.gh_start = np.array(gh_start, dtype=np.uint64)
        self.group_hashes = np.frombuffer(b"".join(gh) or ZERO, dtype=np.uint8).copy()
        self.fg_start = np.array(fg_start, dtype=np.uint64)
        self.fg_index = np.array(fg_index or [0], dtype=np.uint32)
        self.comp_start = np.array(comp_start, dtype=np.uint64)
        lens = np.array([len(c) for c in comps] or [0], dtype=np.uint32)
        off = np.zeros(len(lens), dtype=np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        self.comp_off, self.comp_len = off, lens
        self.comp_data = np.frombuffer(b"".join(comps) or b"\x00", dtype=np.uint8).copy()
        self.nonces = np.frombuffer(b"".join(nonces) or ZERO, dtype=np.uint8).copy()
        self.pt_start = np.array(pt_start, dtype=np.uint64)
        self.pt_tag = np.array(tags or [0], dtype=np.uint8)
        self.pt_hash = np.frombuffer(b"".join(phash) or ZERO, dtype=np.uint8).copy()
        self.check_visible = np.array([f.check_visible for f in ftxs], dtype=np.int32)
        self.visible_mask = np.array([f.visible_mask for f in ftxs], dtype=np.uint32)


NOTARY_FLOW_MASK = (1 << 0) | (1 << 5)   # NonValidatingNotaryFlow.kt:27-29: INPUTS_GROUP, then TIMEWINDOW_GROUP


def notary_workload(n, seed=0x5EED0006, corrupt=0.2, flow=False):
    """Non-validating-notary shaped FilteredTransactions (inputs, notary, time-window visible;
    outputs / commands / attachments hidden) plus corrupted variants, with the expected
    (status, reason) from the Kotlin semantics.  flow=False: checkAllComponentsVisible(INPUTS_GROUP) through
    check_visible; flow=True: the notary flow's two checks (INPUTS_GROUP, then TIMEWINDOW_GROUP) through
    visible_mask, with the time-window component hidden in some transactions.  Returns ([Ftx], [(status, reason)])."""
    rng = np.random.Generator(np.random.PCG64(seed))
    ftxs, want = [], []
    for t in range(n):
        salt = bytes(rng.integers(1, 256, size=32, dtype=np.uint8))
        groups = [(0, [rng.bytes(36) for _ in range(int(rng.integers(1, 5)))]),
                  (1, [rng.bytes(int(rng.integers(50, 300))) for _ in range(int(rng.integers(1, 4)))]),
                  (2, [rng.bytes(120)]), (4, [rng.bytes(96)])]
        if rng.random() < 0.5:
            groups.append((5, [rng.bytes(40)]))
        if rng.random() < 0.2:
            groups.append((3, [rng.bytes(32) for _ in range(int(rng.integers(1, 3)))]))
        if rng.random() < 0.05:
            groups.append((int(rng.integers(6, 30)), [rng.bytes(10)]))    # unknown group ordinal
        hide_tw = flow and rng.random() < 0.15
        vis = lambda g, i, c: g in (0, 4) or (g == 5 and not hide_tw)          # noqa: E731
        if rng.random() < 0.1:
            vis = lambda g, i, c, s=int(rng.integers(0, 1 << 30)): g == 4 or (g == 5 and not hide_tw) or (g == 0 and (i + s) % 2 == 0)  # noqa: E731
        if flow:
            f = build_filtered(salt, groups, vis)
            f.visible_mask = NOTARY_FLOW_MASK
        else:
            f = build_filtered(salt, groups, vis, check_visible=0)
        exp = (0, 0)
        n_inputs = len(dict(groups)[0])
        visible_inputs = len(f.groups[0][1]) if f.groups and f.groups[0][0] == 0 else 0
        if visible_inputs != n_inputs:
            exp = (2, 8) if visible_inputs else (2, 6)
        elif flow and hide_tw and 5 in dict(groups):
            exp = (2, 6)   # "Did not receive components for group 5 ..." (its group hash is not allOnesHash)
        u = rng.random()
        if u < corrupt:
            kind = int(rng.integers(0, 6))
            if kind == 0:     # wrong id
                f.id = sha256(f.id)
                exp = (1, 2)
            elif kind == 1:   # a visible component altered
                g, cs, ns, po = f.groups[0]
                cs = [bytes([cs[0][0] ^ 1]) + cs[0][1:]] + cs[1:]
                f.groups[0] = (g, cs, ns, po)
                exp = (1, 5)
            elif kind == 2:   # a hidden subtree hash altered -> partial root mismatch
                g, cs, ns, po = f.groups[0]
                k = [j for j, (tg, _) in enumerate(po) if tg != 2]
                j = k[-1]
                po = list(po)
                po[j] = (po[j][0], sha256(po[j][1]))
                f.groups[0] = (g, cs, ns, po)
                exp = (1, 4) if po[j][0] == 1 else (1, 4)
            elif kind == 3:   # group hashes emptied
                f.group_hashes = []
                exp = (1, 1)
            elif kind == 4:   # filtered group index past the group hashes (and the id recomputed)
                g, cs, ns, po = f.groups[-1]
                f.groups[-1] = (len(f.group_hashes) + 3, cs, ns, po)
                exp = (1, 3)
            else:             # malformed post-order: a dangling node
                g, cs, ns, po = f.groups[0]
                f.groups[0] = (g, cs, ns, list(po) + [(2, ZERO)])
                exp = (1, 9) if len(po) < 2 else (1, 9)
        ftxs.append(f)
        want.append(exp)
    return ftxs, want
