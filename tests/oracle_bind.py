"""ctypes binding of oracle/liboracle.so — the CPU restatement (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# CORDA_ORACLE_LIB: an alternative build of the same sources (the sanitizer build, oracle/_asan/)
LIB_PATH = os.environ.get("CORDA_ORACLE_LIB") or os.path.join(ORACLE_DIR, "liboracle.so")
_lib = None

VALID, INVALID, SIG_DECODE, EMPTY_SIG, EMPTY_CLEAR, UNSUPPORTED, KEY_INVALID = range(7)


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.orc_uniq_new.restype = ctypes.c_void_p
        _lib.orc_uniq_size.restype = ctypes.c_uint64
        _lib.orc_uniq_size.argtypes = [ctypes.c_void_p]
        _lib.orc_uniq_free.argtypes = [ctypes.c_void_p]
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def sha256(b: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_sha256(b, ctypes.c_size_t(len(b)), out)
    return out.raw


def sha512(b: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    lib().orc_sha512(b, ctypes.c_size_t(len(b)), out)
    return out.raw


def do_verify(spki: bytes, sig: bytes, msg: bytes) -> int:
    return lib().orc_do_verify(spki, ctypes.c_size_t(len(spki)), sig, ctypes.c_size_t(len(sig)), msg,
                               ctypes.c_size_t(len(msg)))


def ed25519_verify(a: bytes, sig: bytes, msg: bytes) -> int:
    return lib().orc_ed25519_verify(a, sig, ctypes.c_size_t(len(sig)), msg, ctypes.c_size_t(len(msg)))


def ed25519_decode_key(a: bytes):
    out = ctypes.create_string_buffer(32)
    r = lib().orc_ed25519_decode_key(a, out)
    return out.raw if r == 0 else None


def ed25519_slide(s: bytes):
    r = (ctypes.c_int8 * 256)()
    drops = lib().orc_ed25519_slide(s, r)
    return list(r), drops


def ed25519_scalarmult_base(s: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_ed25519_scalarmult_base(s, out)
    return out.raw


def ed25519_double_scalarmult_plain(p: bytes, a: bytes, b: bytes):
    out = ctypes.create_string_buffer(32)
    r = lib().orc_ed25519_double_scalarmult_plain(p, a, b, out)
    return out.raw if r == 0 else None


def sc_reduce64(b: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_ed25519_sc_reduce64(b, out)
    return out.raw


def der_decode(sig: bytes):
    r = ctypes.create_string_buffer(32)
    s = ctypes.create_string_buffer(32)
    ro, so = ctypes.c_int(), ctypes.c_int()
    rc = lib().orc_der_decode(sig, ctypes.c_size_t(len(sig)), r, s, ctypes.byref(ro), ctypes.byref(so))
    if rc != 0:
        return None
    return r.raw, s.raw, ro.value, so.value


def ecdsa_scalarmult_base(scheme: int, k: bytes):
    out = ctypes.create_string_buffer(64)
    r = lib().orc_ecdsa_scalarmult_base(scheme, k, out)
    return out.raw if r == 0 else None


def ecdsa_decode_key(scheme: int, pt: bytes):
    out = ctypes.create_string_buffer(64)
    r = lib().orc_ecdsa_decode_key(scheme, pt, ctypes.c_size_t(len(pt)), out)
    return out.raw if r == 0 else None


def verify_batch(b, threads: int = 1, is_valid: bool = False) -> np.ndarray:
    """Crypto.doVerify statuses (is_valid=False) or Crypto.isValid statuses (no empty-input checks)."""
    st = np.zeros(b.n, dtype=np.uint8)
    lib().orc_verify_batch_mode(ctypes.c_uint64(b.n), _p(b.key_idx), _p(b.msg_idx), _p(b.sig_data), _p(b.sig_off),
                                _p(b.sig_len), _p(b.key_data), _p(b.key_off), _p(b.key_len), _p(b.msg_data),
                                _p(b.msg_off), _p(b.msg_len), _p(st), threads, int(is_valid))
    return st


def compute_nonce(salt: bytes, g: int, i: int) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_compute_nonce(salt, ctypes.c_uint32(g), ctypes.c_uint32(i), out)
    return out.raw


def merkle_root(leaves) -> bytes:
    buf = b"".join(leaves)
    out = ctypes.create_string_buffer(32)
    lib().orc_merkle_root(buf, ctypes.c_uint32(len(leaves)), out)
    return out.raw


def txid_batch(tb, threads: int = 1) -> np.ndarray:
    ids = np.zeros(tb.ntx * 32, dtype=np.uint8)
    lib().orc_txid_batch(ctypes.c_uint64(tb.ntx), _p(tb.salts), _p(tb.tx_comp_start), _p(tb.comp_group),
                         _p(tb.comp_internal), _p(tb.data), _p(tb.comp_off), _p(tb.comp_len), _p(ids), threads)
    return ids.reshape(tb.ntx, 32)


class OrcConflict(ctypes.Structure):
    _fields_ = [("tx", ctypes.c_uint64), ("input_index", ctypes.c_uint32), ("consumed_index", ctypes.c_uint32),
                ("consuming_tx", ctypes.c_uint8 * 32), ("consuming_caller", ctypes.c_uint32),
                ("pad", ctypes.c_uint32)]


class Uniq:
    """PersistentUniquenessProvider restatement with batch commit."""

    def __init__(self, capacity: int = 1024):
        self.h = ctypes.c_void_p(lib().orc_uniq_new(ctypes.c_uint64(capacity)))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_uniq_free(self.h)
            self.h = None

    def size(self) -> int:
        return lib().orc_uniq_size(self.h)

    def preload(self, refs36, tx32, idx, caller):
        n = len(idx)
        lib().orc_uniq_preload(self.h, ctypes.c_uint64(n), _p(refs36), _p(tx32), _p(idx), _p(caller))

    def commit_batch(self, tx_ref_start, refs36, tx_ids, callers, cap=None):
        ntx = len(tx_ref_start) - 1
        st = np.zeros(ntx, dtype=np.uint8)
        if cap is None:
            cap = int(tx_ref_start[-1]) + 1
        out = (OrcConflict * max(cap, 1))()
        nout = ctypes.c_uint64()
        lib().orc_uniq_commit_batch(self.h, ctypes.c_uint64(ntx), _p(tx_ref_start), _p(refs36), _p(tx_ids),
                                    _p(callers), _p(st), out, ctypes.c_uint64(cap), ctypes.byref(nout))
        recs = [(c.tx, c.input_index, c.consumed_index, bytes(c.consuming_tx), c.consuming_caller)
                for c in out[:min(nout.value, cap)]]
        return st, recs


def ftx_verify_batch(f):
    """FilteredTransaction.verify + checkAllComponentsVisible over the chip_ftx_batch layout."""
    st = np.zeros(f.ntx, dtype=np.uint8)
    rs = np.zeros(f.ntx, dtype=np.uint8)
    lib().orc_ftx_verify_batch(ctypes.c_uint64(f.ntx), _p(f.ids), _p(f.gh_start), _p(f.group_hashes), _p(f.fg_start),
                               _p(f.fg_index), _p(f.comp_start), _p(f.comp_data), _p(f.comp_off), _p(f.comp_len),
                               _p(f.nonces), _p(f.pt_start), _p(f.pt_tag), _p(f.pt_hash), _p(f.check_visible),
                               _p(getattr(f, "visible_mask", None)), _p(st), _p(rs))
    return st, rs


def required_signers(q, b, status, tx_idx=None):
    """TransactionWithSignatures.verifySignaturesExcept after the statuses (chip_req_batch layout over
    the signatures / key pool of `b`) -> (verdict u8[ntx], arg u32[ntx], missing u8[nreq])."""
    ntx = int(q.ntx)
    nreq = max(len(q.node_start) - 1, 0)
    verdict = np.zeros(ntx, dtype=np.uint8)
    arg = np.zeros(ntx, dtype=np.uint32)
    missing = np.zeros(max(nreq, 1), dtype=np.uint8)
    allowed = getattr(q, "allowed", None)
    lib().orc_required_signers(
        ctypes.c_uint64(ntx), _p(q.sig_start), _p(q.req_start), ctypes.c_uint64(nreq), _p(q.node_start),
        _p(allowed), ctypes.c_uint64(len(q.node_val)), _p(q.node_val), _p(q.node_nkids), _p(q.node_weight),
        ctypes.c_uint64(len(b.key_idx)), _p(b.key_idx), _p(tx_idx), ctypes.c_uint64(len(b.key_off)), _p(b.key_data),
        _p(b.key_off), _p(b.key_len), ctypes.c_uint64(int(b.key_data.nbytes)),
        _p(np.ascontiguousarray(status, dtype=np.uint8)), _p(verdict), _p(arg), _p(missing))
    return verdict, arg, missing[:nreq]


# ---- Kryo front end (oracle/kryo_ref.c) ----
class KryoRegistry(ctypes.Structure):
    _fields_ = [("arrays_aslist", ctypes.c_int32), ("signed_tx", ctypes.c_int32), ("wire_tx", ctypes.c_int32),
                ("serialized_bytes", ctypes.c_int32), ("privacy_salt", ctypes.c_int32),
                ("n_public_key", ctypes.c_uint32), ("public_key", ctypes.c_int32 * 8)]


def kryo_registry(reg) -> KryoRegistry:
    """orc_kryo_registry of a corda_amd.kryo.Registry."""
    r = KryoRegistry(reg.arrays_aslist, reg.signed_tx, reg.wire_tx, reg.serialized_bytes, reg.privacy_salt,
                     len(reg.public_key))
    for i, v in enumerate(reg.public_key):
        r.public_key[i] = v
    return r


def _decode_stx_record(b: bytes, want_required: bool):
    """One orc_stx_parse record -> (parse status, final status, groups, salt, sigs, trees) in the shapes of
    corda_amd.kryo.stx_parse / required_key_trees (None where absent)."""
    import struct
    pst, fst = b[0], b[1]
    if pst != 0:
        return pst, fst, None, None, None, None
    at = 2

    def u32():
        nonlocal at
        v = struct.unpack_from("<I", b, at)[0]
        at += 4
        return v

    def raw(n):
        nonlocal at
        v = bytes(b[at:at + n])
        at += n
        return v

    groups = []
    for _ in range(u32()):
        g, i, n = u32(), u32(), u32()
        c = raw(n)
        if i == 0:
            groups.append((g, [c]))
        else:
            groups[-1][1].append(c)
    salt = raw(32)
    sigs = []
    for _ in range(u32()):
        pv, sch = struct.unpack("<ii", raw(8))
        s = raw(u32())
        k = raw(u32())
        sigs.append((s, k, pv, sch))
    trees = None
    if want_required and fst == 0:
        trees = []
        for _ in range(u32()):
            nodes = []
            for _ in range(u32()):
                nk, w, thr, ln = u32(), u32(), u32(), u32()
                nodes.append((raw(ln) if nk == 0 else None, thr, nk, w))
            trees.append(nodes)
    return pst, fst, groups, salt, sigs, trees


def stx_parse(blobs, reg, want_required: bool = False):
    """oracle/kryo_ref.c over a list of SignedTransaction blobs -> one decoded record per blob."""
    data, off, ln = _pools(blobs)
    r = kryo_registry(reg)
    cap = 4 * int(data.nbytes) + 4096 * len(blobs) + 4096
    out = np.zeros(cap, dtype=np.uint8)
    rec_off = np.zeros(len(blobs) + 1, dtype=np.uint64)
    rc = lib().orc_stx_parse_batch(ctypes.c_uint64(len(blobs)), _p(data), _p(off), _p(ln), ctypes.byref(r),
                                   int(want_required), _p(out), ctypes.c_uint64(cap), _p(rec_off))
    if rc != 0:
        raise RuntimeError("orc_stx_parse_batch: output too small")
    return [_decode_stx_record(out[int(rec_off[t]):int(rec_off[t + 1])].tobytes(), want_required)
            for t in range(len(blobs))]


def _pools(blobs):
    ln = np.array([len(b) for b in blobs], dtype=np.uint32)
    off = np.zeros(len(blobs), dtype=np.uint64)
    if len(blobs) > 1:
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    data = np.frombuffer(b"".join(bytes(b) for b in blobs) or b"\0", dtype=np.uint8).copy()
    return data, off, ln
