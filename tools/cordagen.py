"""Python front-end of tools/libcordagen.so (OpenSSL-backed synthetic workload generator).

Used by bench.py (input generation, outside the timed region) and by the fixture scripts in
tests/golden/.  Independent of oracle/: OpenSSL is the third party whose verdicts pin the
oracle on canonical inputs.  Workload shapes follow SURVEY.md §8(d).
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import struct
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libcordagen.so")
_lib = None

SCHEME_K1, SCHEME_R1, SCHEME_ED25519 = 2, 3, 4

# SubjectPublicKeyInfo prefixes (what PublicKey.encoded yields for the three schemes)
SPKI_ED25519 = bytes.fromhex("302a300506032b6570032100")
SPKI_R1 = bytes.fromhex("3059301306072a8648ce3d020106082a8648ce3d030107034200")
SPKI_K1 = bytes.fromhex("3056301006072a8648ce3d020106052b8104000a034200")

L_ED = 2**252 + 27742317777372353535851937790883648493
N_R1 = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
N_K1 = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "cordagen.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-Wall", "-o", _LIB_PATH, src,
                               "-lcrypto", "-lpthread"])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def ed25519_pub(seed: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    if lib().gen_ed25519_pub(seed, out) != 0:
        raise RuntimeError("ed25519 keygen failed")
    return out.raw


def ed25519_sign(seed: bytes, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    if lib().gen_ed25519_sign(seed, msg, ctypes.c_size_t(len(msg)), out) != 0:
        raise RuntimeError("ed25519 sign failed")
    return out.raw


def ec_pub(scheme: int, d: bytes) -> bytes:
    out = ctypes.create_string_buffer(65)
    if lib().gen_ec_pub(scheme, d, out) != 0:
        raise RuntimeError("ec keygen failed")
    return out.raw


def ec_sign(scheme: int, d: bytes, k: bytes, msg: bytes):
    der = ctypes.create_string_buffer(72)
    r = ctypes.create_string_buffer(32)
    s = ctypes.create_string_buffer(32)
    n = lib().gen_ec_sign(scheme, d, k, msg, ctypes.c_size_t(len(msg)), der, r, s)
    if n < 0:
        raise RuntimeError("ec sign failed")
    return der.raw[:n], r.raw, s.raw


def ossl_verify(spki: bytes, sig: bytes, msg: bytes) -> int:
    return lib().ossl_verify_spki(spki, ctypes.c_size_t(len(spki)), sig, ctypes.c_size_t(len(sig)),
                                  msg, ctypes.c_size_t(len(msg)))


def ossl_verify_batch(b, threads: int = 8) -> np.ndarray:
    """OpenSSL EVP_DigestVerify over a SigBatch (CPU baseline): uint8[n], 1 = valid."""
    n = len(b.key_idx)
    ok = np.zeros(n, dtype=np.uint8)
    lib().ossl_verify_many(ctypes.c_uint64(n), _p(b.key_idx), _p(b.msg_idx), _p(b.sig_data), _p(b.sig_off),
                           _p(b.sig_len), ctypes.c_uint64(len(b.key_off)), _p(b.key_data), _p(b.key_off),
                           _p(b.key_len), _p(b.msg_data), _p(b.msg_off), _p(b.msg_len), _p(ok), int(threads))
    return ok


def spki_ed25519(a: bytes) -> bytes:
    return SPKI_ED25519 + a


def spki_ec(scheme: int, pub65: bytes) -> bytes:
    return (SPKI_R1 if scheme == SCHEME_R1 else SPKI_K1) + pub65


def der_encode_int(v: int) -> bytes:
    """Minimal DER INTEGER (two's complement) of a non-negative int."""
    b = v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big")
    while len(b) > 1 and b[0] == 0 and not (b[1] & 0x80):
        b = b[1:]
    return b"\x02" + bytes([len(b)]) + b


def der_sig(r: int, s: int) -> bytes:
    body = der_encode_int(r) + der_encode_int(s)
    return b"\x30" + bytes([len(body)]) + body


class PRNG:
    """Counter-mode SHA-256 stream: deterministic bytes from a seed."""

    def __init__(self, seed: int, label: bytes = b""):
        self.key = struct.pack("<Q", seed) + label
        self.ctr = 0

    def bytes(self, n: int) -> bytes:
        out = bytearray()
        while len(out) < n:
            out += hashlib.sha256(self.key + struct.pack("<Q", self.ctr)).digest()
            self.ctr += 1
        return bytes(out[:n])

    def np_bytes(self, n: int) -> np.ndarray:
        # fast bulk stream: numpy generator seeded from the SHA-256 stream (deterministic)
        seed = int.from_bytes(self.bytes(16), "little")
        return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, size=n, dtype=np.uint8)


def key_seed(i: int) -> bytes:
    return hashlib.sha256(b"cordahip-key" + struct.pack("<Q", i)).digest()


class SigBatch:
    """SoA signature batch in the chip_sig_batch layout of include/cordahip.h."""

    def __init__(self):
        self.key_idx = None   # u32[n]
        self.msg_idx = None   # u32[n]
        self.sig_data = None  # u8 pool
        self.sig_off = None   # u64[n]
        self.sig_len = None   # u32[n]
        self.key_data = None  # u8 pool (SPKI)
        self.key_off = None   # u64[k]
        self.key_len = None   # u32[k]
        self.msg_data = None
        self.msg_off = None
        self.msg_len = None
        self.expected = None  # u8[n] intended outcome (generator's label, not a verdict)
        self.kind = None      # u8[n] corruption class

    @property
    def n(self):
        return len(self.key_idx)


def pools_from_list(items, stride=None):
    """Pack a list of bytes into (data u8, off u64, len u32)."""
    lens = np.fromiter((len(x) for x in items), dtype=np.uint32, count=len(items))
    off = np.zeros(len(items), dtype=np.uint64)
    if len(items):
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    data = np.frombuffer(b"".join(items), dtype=np.uint8).copy() if items else np.zeros(0, np.uint8)
    return data, off, lens


def signable_message(rng_bytes: bytes, tx_id: bytes, scheme_id: int, platform_version: int = 1) -> bytes:
    """SignableData-shaped message (~200 B): Kryo header 'corda\\0\\0\\1' (SerializationScheme.kt:251),
    class-name-like filler, txId and SignatureMetadata(platformVersion, schemeNumberID)."""
    return (b"corda\x00\x00\x01" + rng_bytes[:150] + tx_id + struct.pack(">ii", platform_version, scheme_id))[:200]


# Corruption classes of cfg2
ED_KINDS = ["valid", "r_flip", "s_flip", "msg_flip", "wrong_key", "len63", "s_plus_l", "noncanon_r",
            "small_order_forgery"]


def ed25519_batch(n: int, n_keys: int = 4096, msg_len: int = 200, corrupt: float = 0.10,
                  seed: int = 0x5EED0002, threads: int = 8) -> SigBatch:
    """cfg2: n Ed25519 signatures, 2 per tx (one shared SignableData message per tx),
    `corrupt` fraction spread evenly over the 8 corruption classes."""
    rng = np.random.Generator(np.random.PCG64(seed))
    seeds = b"".join(key_seed(i) for i in range(n_keys))
    seeds_np = np.frombuffer(seeds, dtype=np.uint8).copy()
    pubs = np.zeros(n_keys * 32, dtype=np.uint8)
    if lib().gen_pubs_many(SCHEME_ED25519, ctypes.c_uint64(n_keys), _p(seeds_np), _p(pubs)) != 0:
        raise RuntimeError("keygen failed")
    # extra key: the identity point (small-order key, i2p accepts forged R = [S]B)
    ident = bytes([1] + [0] * 31)
    key_items = [spki_ed25519(pubs[32 * i:32 * i + 32].tobytes()) for i in range(n_keys)] + [spki_ed25519(ident)]
    ntx = (n + 1) // 2
    body = PRNG(seed, b"msg").np_bytes(ntx * msg_len).reshape(ntx, msg_len)
    body[:, :8] = np.frombuffer(b"corda\x00\x00\x01", dtype=np.uint8)
    msgs = body.reshape(-1)
    msg_off = (np.arange(ntx, dtype=np.uint64) * msg_len)
    msg_lenv = np.full(ntx, msg_len, dtype=np.uint32)
    msg_idx = (np.arange(n, dtype=np.uint32) // 2)
    key_of = rng.integers(0, n_keys, size=n, dtype=np.uint32)
    # second signer of a tx differs from the first
    same = (np.arange(n) % 2 == 1) & (key_of == np.roll(key_of, 1))
    key_of[same] = (key_of[same] + 1) % n_keys
    kind = np.zeros(n, dtype=np.uint8)
    ncor = int(n * corrupt)
    cidx = rng.choice(n, size=ncor, replace=False)
    kind[cidx] = 1 + (np.arange(ncor) % 8)
    # msg_flip: sign a flipped copy of the message; append those messages to the pool
    mf = np.nonzero(kind == 3)[0]
    sign_msg = msg_idx.copy()
    if len(mf):
        extra = msgs.reshape(ntx, msg_len)[msg_idx[mf]].copy()
        bitpos = rng.integers(0, msg_len * 8, size=len(mf))
        extra[np.arange(len(mf)), bitpos // 8] ^= (1 << (bitpos % 8)).astype(np.uint8)
        sign_msg[mf] = ntx + np.arange(len(mf), dtype=np.uint32)
        msgs_all = np.concatenate([msgs, extra.reshape(-1)])
        msg_off_all = np.concatenate([msg_off, (ntx + np.arange(len(mf), dtype=np.uint64)) * msg_len])
        msg_len_all = np.concatenate([msg_lenv, np.full(len(mf), msg_len, np.uint32)])
    else:
        msgs_all, msg_off_all, msg_len_all = msgs, msg_off, msg_lenv
    sigs = np.zeros(n * 64, dtype=np.uint8)
    sig_len = np.zeros(n, dtype=np.uint32)
    err = lib().gen_sign_many(SCHEME_ED25519, ctypes.c_uint64(n), _p(seeds_np), _p(key_of), _p(msgs_all),
                              _p(msg_off_all), _p(msg_len_all), _p(sign_msg), None, _p(sigs), _p(sig_len),
                              ctypes.c_uint32(64), threads)
    if err:
        raise RuntimeError("signing failed")
    sigs = sigs.reshape(n, 64)
    expected = np.zeros(n, dtype=np.uint8)
    key_idx = key_of.copy()
    # apply corruptions
    for i in np.nonzero(kind)[0]:
        k = kind[i]
        if k == 1:    # R bit flip
            b = int(rng.integers(0, 256)); sigs[i, b // 8] ^= 1 << (b % 8); expected[i] = 1
        elif k == 2:  # S bit flip (low 252 bits so S stays < 2^253: reference rejects by arithmetic)
            b = int(rng.integers(0, 252)); sigs[i, 32 + b // 8] ^= 1 << (b % 8); expected[i] = 1
        elif k == 3:  # signature over a different message
            expected[i] = 1
        elif k == 4:  # wrong key
            key_idx[i] = (key_of[i] + 1 + int(rng.integers(0, n_keys - 1))) % n_keys; expected[i] = 1
        elif k == 5:  # 63-byte signature -> "signature length is wrong"
            sig_len[i] = 63; expected[i] = 2
        elif k == 6:  # S + L: i2p 0.2.0 has no S < L check -> reference-VALID
            S = int.from_bytes(sigs[i, 32:].tobytes(), "little") + L_ED
            sigs[i, 32:] = np.frombuffer(S.to_bytes(32, "little"), dtype=np.uint8); expected[i] = 0
        elif k == 7:  # non-canonical R: identity encoded as y = 1 + p, identity key, S = 0 -> INVALID
            key_idx[i] = n_keys
            sigs[i, :32] = np.frombuffer(bytes([0xee] + [0xff] * 30 + [0x7f]), dtype=np.uint8)
            sigs[i, 32:] = 0; expected[i] = 1
        elif k == 8:  # identity key, R = [S]B with S = clamp(SHA512(seed)) -> reference-VALID forgery
            s_seed = key_seed(1_000_000 + i)
            h = hashlib.sha512(s_seed).digest()
            a = bytearray(h[:32]); a[0] &= 248; a[31] &= 127; a[31] |= 64
            key_idx[i] = n_keys
            sigs[i, :32] = np.frombuffer(ed25519_pub(s_seed), dtype=np.uint8)
            sigs[i, 32:] = np.frombuffer(bytes(a), dtype=np.uint8); expected[i] = 0
    b = SigBatch()
    b.key_idx = key_idx.astype(np.uint32)
    b.msg_idx = msg_idx.astype(np.uint32)
    b.sig_data = sigs.reshape(-1)
    b.sig_off = np.arange(n, dtype=np.uint64) * 64
    b.sig_len = sig_len
    b.key_data, b.key_off, b.key_len = pools_from_list(key_items)
    b.msg_data, b.msg_off, b.msg_len = msgs_all, msg_off_all.astype(np.uint64), msg_len_all.astype(np.uint32)
    b.expected = expected
    b.kind = kind
    return b


EC_KINDS = ["valid", "r_flip", "s_flip", "msg_flip", "wrong_key", "wrong_curve", "r_zero", "s_ge_n",
            "high_s", "der_long_len", "der_extra_elem", "der_trailing", "der_nonminimal_int"]


def ecdsa_batch(n: int, n_keys: int = 4096, msg_len: int = 200, corrupt: float = 0.10,
                seed: int = 0x5EED0003, threads: int = 8, schemes=(SCHEME_R1, SCHEME_K1)) -> SigBatch:
    """cfg3: n ECDSA signatures, r1/k1 interleaved (even index r1, odd k1), one message per tx of 2.
    schemes=(SCHEME_R1,) gives a P-256-only batch (the same keys, messages and corruption mix)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    nk = n_keys
    privs = {}
    pubs = {}
    key_items = []
    for sch in (SCHEME_R1, SCHEME_K1):
        order = N_R1 if sch == SCHEME_R1 else N_K1
        ds = []
        for i in range(nk):
            d = int.from_bytes(hashlib.sha256(b"cordahip-eckey" + struct.pack("<QB", i, sch)).digest(), "big") % (order - 1) + 1
            ds.append(d.to_bytes(32, "big"))
        privs[sch] = np.frombuffer(b"".join(ds), dtype=np.uint8).copy()
        pb = np.zeros(nk * 65, dtype=np.uint8)
        if lib().gen_pubs_many(sch, ctypes.c_uint64(nk), _p(privs[sch]), _p(pb)) != 0:
            raise RuntimeError("ec keygen failed")
        pubs[sch] = pb
        key_items += [spki_ec(sch, pb[65 * i:65 * i + 65].tobytes()) for i in range(nk)]
    # key table: [0, nk) r1, [nk, 2nk) k1
    ntx = (n + 1) // 2
    body = PRNG(seed, b"msg").np_bytes(ntx * msg_len).reshape(ntx, msg_len)
    body[:, :8] = np.frombuffer(b"corda\x00\x00\x01", dtype=np.uint8)
    msgs = body.reshape(-1)
    msg_off = np.arange(ntx, dtype=np.uint64) * msg_len
    msg_lenv = np.full(ntx, msg_len, dtype=np.uint32)
    msg_idx = (np.arange(n, dtype=np.uint32) // 2)
    if len(schemes) == 1:
        scheme = np.full(n, schemes[0], dtype=np.uint8)
    else:
        scheme = np.where(np.arange(n) % 2 == 0, SCHEME_R1, SCHEME_K1).astype(np.uint8)
    key_local = rng.integers(0, nk, size=n, dtype=np.uint32)
    kind = np.zeros(n, dtype=np.uint8)
    ncor = int(n * corrupt)
    cidx = rng.choice(n, size=ncor, replace=False)
    kind[cidx] = 1 + (np.arange(ncor) % (len(EC_KINDS) - 1))
    nonces = PRNG(seed, b"nonce").np_bytes(n * 32)
    stride = 80
    sigs = np.zeros(n * stride, dtype=np.uint8)
    sig_len = np.zeros(n, dtype=np.uint32)
    mf = np.nonzero(kind == 3)[0]
    sign_msg = msg_idx.copy()
    if len(mf):
        extra = msgs.reshape(ntx, msg_len)[msg_idx[mf]].copy()
        bitpos = rng.integers(0, msg_len * 8, size=len(mf))
        extra[np.arange(len(mf)), bitpos // 8] ^= (1 << (bitpos % 8)).astype(np.uint8)
        sign_msg[mf] = ntx + np.arange(len(mf), dtype=np.uint32)
        msgs_all = np.concatenate([msgs, extra.reshape(-1)])
        msg_off_all = np.concatenate([msg_off, (ntx + np.arange(len(mf), dtype=np.uint64)) * msg_len])
        msg_len_all = np.concatenate([msg_lenv, np.full(len(mf), msg_len, np.uint32)])
    else:
        msgs_all, msg_off_all, msg_len_all = msgs, msg_off, msg_lenv
    for sch in (SCHEME_R1, SCHEME_K1):
        sel = np.nonzero(scheme == sch)[0]
        m = len(sel)
        out = np.zeros(m * stride, dtype=np.uint8)
        ol = np.zeros(m, dtype=np.uint32)
        ko = key_local[sel].copy()
        so = sign_msg[sel].copy()
        nn = np.frombuffer(nonces, dtype=np.uint8).reshape(n, 32)[sel].copy() if isinstance(nonces, bytes) \
            else nonces.reshape(n, 32)[sel].copy()
        err = lib().gen_sign_many(sch, ctypes.c_uint64(m), _p(privs[sch]), _p(ko), _p(msgs_all), _p(msg_off_all),
                                  _p(msg_len_all), _p(so), _p(nn), _p(out), _p(ol), ctypes.c_uint32(stride), threads)
        if err:
            raise RuntimeError("ecdsa signing failed")
        sigs.reshape(n, stride)[sel] = out.reshape(m, stride)
        sig_len[sel] = ol
    sigs = sigs.reshape(n, stride)
    key_idx = np.where(scheme == SCHEME_R1, key_local, key_local + nk).astype(np.uint32)
    expected = np.zeros(n, dtype=np.uint8)

    def parse(i):
        raw = sigs[i, :sig_len[i]].tobytes()
        lr = raw[3]
        r = int.from_bytes(raw[4:4 + lr], "big")
        ls = raw[5 + lr]
        s = int.from_bytes(raw[6 + lr:6 + lr + ls], "big")
        return r, s

    def put(i, der):
        sigs[i, :] = 0
        sigs[i, :len(der)] = np.frombuffer(der, dtype=np.uint8)
        sig_len[i] = len(der)

    for i in np.nonzero(kind)[0]:
        k = int(kind[i])
        order = N_R1 if scheme[i] == SCHEME_R1 else N_K1
        r, s = parse(i)
        if k == 1:
            put(i, der_sig(r ^ (1 << int(rng.integers(0, 250))), s)); expected[i] = 1
        elif k == 2:
            put(i, der_sig(r, s ^ (1 << int(rng.integers(0, 250))))); expected[i] = 1
        elif k == 3:
            expected[i] = 1
        elif k == 4:
            key_idx[i] = (key_idx[i] // nk) * nk + (key_local[i] + 1) % nk; expected[i] = 1
        elif k == 5:  # the same scalar's key on the other curve
            key_idx[i] = (key_local[i] + nk) if scheme[i] == SCHEME_R1 else key_local[i]; expected[i] = 1
        elif k == 6:
            put(i, der_sig(0, s)); expected[i] = 1
        elif k == 7:
            put(i, der_sig(r, s + order)); expected[i] = 1
        elif k == 8:  # high-s: (r, n - s) is also valid in BC (no low-s rule)
            put(i, der_sig(r, order - s)); expected[i] = 0
        elif k == 9:  # long-form length for a short length -> DER re-encode mismatch
            der = der_sig(r, s)
            put(i, b"\x30\x81" + der[1:2] + der[2:]); expected[i] = 2
        elif k == 10:  # a third INTEGER element
            body = der_encode_int(r) + der_encode_int(s) + der_encode_int(1)
            put(i, b"\x30" + bytes([len(body)]) + body); expected[i] = 2
        elif k == 11:  # trailing byte after the SEQUENCE
            put(i, der_sig(r, s) + b"\x00"); expected[i] = 2
        elif k == 12:  # non-minimal INTEGER padding: ASN1Integer's malformed-integer check (unpinned)
            rb = b"\x00" + r.to_bytes(33, "big")
            body = b"\x02" + bytes([len(rb)]) + rb + der_encode_int(s)
            put(i, b"\x30" + bytes([len(body)]) + body); expected[i] = 2
    b = SigBatch()
    b.key_idx = key_idx
    b.msg_idx = msg_idx.astype(np.uint32)
    b.sig_data = sigs.reshape(-1)
    b.sig_off = np.arange(n, dtype=np.uint64) * stride
    b.sig_len = sig_len
    b.key_data, b.key_off, b.key_len = pools_from_list(key_items)
    b.msg_data, b.msg_off, b.msg_len = msgs_all, msg_off_all.astype(np.uint64), msg_len_all.astype(np.uint32)
    b.expected = expected
    b.kind = kind
    b.scheme = scheme
    return b


class TxBatch:
    """SoA transaction batch in the chip_tx_batch layout (include/cordahip.h)."""
    ntx = 0
    salts = None          # u8[ntx*32]
    tx_comp_start = None  # u64[ntx+1]
    comp_group = None     # u32[ncomp]
    comp_internal = None  # u32[ncomp]
    data = None           # u8 pool
    comp_off = None       # u64[ncomp]
    comp_len = None       # u32[ncomp]


# cfg4 profile: (group ordinal, [component sizes])
CFG4_PROFILE = [(0, [96, 96]), (1, [640, 640]), (2, [320]), (3, [96]), (4, [384]), (5, [96])]


def tx_batch(ntx: int, profile=CFG4_PROFILE, seed: int = 0x5EED0004, shuffle_groups: bool = False) -> TxBatch:
    """ntx WireTransaction-shaped component sets with random non-zero 32-byte salts."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = [s for _, ss in profile for s in ss]
    groups = [g for g, ss in profile for _ in ss]
    internal = [i for _, ss in profile for i in range(len(ss))]
    per_tx = len(sizes)
    tb = TxBatch()
    tb.ntx = ntx
    salts = PRNG(seed, b"salt").np_bytes(ntx * 32).reshape(ntx, 32)
    salts[:, 0] |= 1  # never all-zero (PrivacySalt invariant, Structures.kt:268-276)
    tb.salts = salts.reshape(-1).copy()
    tb.tx_comp_start = (np.arange(ntx + 1, dtype=np.uint64) * per_tx)
    tb.comp_group = np.tile(np.array(groups, dtype=np.uint32), ntx)
    tb.comp_internal = np.tile(np.array(internal, dtype=np.uint32), ntx)
    lens = np.tile(np.array(sizes, dtype=np.uint32), ntx)
    tb.comp_len = lens
    off = np.zeros(len(lens), dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    tb.comp_off = off
    tb.data = PRNG(seed, b"data").np_bytes(int(lens.sum()))
    return tb


def tx_batch_from_lists(txs) -> TxBatch:
    """txs: list of (salt32, [(group, [bytes, ...]), ...]) in component-group order."""
    tb = TxBatch()
    tb.ntx = len(txs)
    salts, start, grp, internal, items = [], [0], [], [], []
    for salt, groups in txs:
        salts.append(salt)
        for g, comps in groups:
            for i, c in enumerate(comps):
                grp.append(g)
                internal.append(i)
                items.append(c)
        start.append(len(grp))
    tb.salts = np.frombuffer(b"".join(salts), dtype=np.uint8).copy() if salts else np.zeros(0, np.uint8)
    tb.tx_comp_start = np.array(start, dtype=np.uint64)
    tb.comp_group = np.array(grp, dtype=np.uint32)
    tb.comp_internal = np.array(internal, dtype=np.uint32)
    tb.data, tb.comp_off, tb.comp_len = pools_from_list(items)
    if len(tb.data) == 0:
        tb.data = np.zeros(1, dtype=np.uint8)
    return tb


def state_ref(txhash: bytes, index: int) -> bytes:
    """StateRef (Structures.kt:143-145) as the 36-byte key of the C-ABI: txhash || LE u32 index."""
    return txhash + struct.pack("<I", index)


class UniqBatch:
    """chip_uniq_commit_batch layout: tx_ref_start u64[ntx+1], refs u8[nref*36], tx_ids u8[ntx*32], callers u32[ntx]."""
    tx_ref_start = None
    refs = None
    tx_ids = None
    callers = None

    @property
    def ntx(self):
        return len(self.tx_ref_start) - 1


def uniq_batch_from_lists(txs) -> UniqBatch:
    """txs: list of (tx_id32, [StateRef36, ...], caller)"""
    b = UniqBatch()
    start = [0]
    refs = []
    for _, ins, _ in txs:
        refs += ins
        start.append(len(refs))
    b.tx_ref_start = np.array(start, dtype=np.uint64)
    b.refs = np.frombuffer(b"".join(refs), dtype=np.uint8).copy() if refs else np.zeros(36, np.uint8)
    b.tx_ids = np.frombuffer(b"".join(t[0] for t in txs), dtype=np.uint8).copy()
    b.callers = np.array([t[2] for t in txs], dtype=np.uint32)
    return b


def uniq_workload(ntx: int, n_pre: int, seed: int = 0x5EED0005, pre_hit: float = 0.01, dbl: float = 0.005,
                  resubmit: float = 0.001, n_callers: int = 64):
    """cfg5-shaped notary batch: 1-4 inputs per tx (mean 2.5), index 0-3; a pre-committed table of
    n_pre StateRefs; `pre_hit` of inputs hit pre-committed states, `dbl` are intra-batch double
    spends (earlier tx's input reused, including chains), `resubmit` of txs are exact re-submissions
    of an earlier tx of the batch (idempotent).  Returns (pre rows, UniqBatch)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    pre_hash = PRNG(seed, b"pre").np_bytes(n_pre * 32).reshape(n_pre, 32)
    pre_idx = rng.integers(0, 4, size=n_pre, dtype=np.uint32)
    pre_refs = np.concatenate([pre_hash, pre_idx.view(np.uint8).reshape(n_pre, 4)], axis=1)
    pre_tx = PRNG(seed, b"pretx").np_bytes(n_pre * 32).reshape(n_pre, 32)
    pre_pos = rng.integers(0, 4, size=n_pre, dtype=np.uint32)
    pre_caller = rng.integers(0, n_callers, size=n_pre, dtype=np.uint32)
    nin = rng.integers(1, 5, size=ntx)
    start = np.zeros(ntx + 1, dtype=np.uint64)
    start[1:] = np.cumsum(nin)
    nref = int(start[-1])
    hashes = PRNG(seed, b"in").np_bytes(nref * 32).reshape(nref, 32)
    idx = rng.integers(0, 4, size=nref, dtype=np.uint32)
    refs = np.concatenate([hashes, idx.view(np.uint8).reshape(nref, 4)], axis=1)
    u = rng.random(nref)
    hit = np.nonzero(u < pre_hit)[0]
    refs[hit] = pre_refs[rng.integers(0, n_pre, size=len(hit))] if n_pre else refs[hit]
    dsp = np.nonzero((u >= pre_hit) & (u < pre_hit + dbl))[0]
    ref_tx = np.repeat(np.arange(ntx), nin)
    for r in dsp:                                  # reuse an input of an earlier tx (chains form naturally)
        t = ref_tx[r]
        if t == 0:
            continue
        t2 = int(rng.integers(max(0, t - 64), t))
        r2 = int(start[t2] + rng.integers(0, nin[t2]))
        refs[r] = refs[r2]
    tx_ids = PRNG(seed, b"txid").np_bytes(ntx * 32).reshape(ntx, 32)
    callers = rng.integers(0, n_callers, size=ntx, dtype=np.uint32)
    # exact re-submissions: copy an earlier tx (same id, inputs, caller) when the input counts match
    rs = np.nonzero(rng.random(ntx) < resubmit)[0]
    for t in rs:
        if t == 0:
            continue
        t2 = int(rng.integers(max(0, t - 256), t))
        if nin[t2] != nin[t]:
            continue
        refs[int(start[t]):int(start[t + 1])] = refs[int(start[t2]):int(start[t2 + 1])]
        tx_ids[t] = tx_ids[t2]
        callers[t] = callers[t2]
    b = UniqBatch()
    b.tx_ref_start = start
    b.refs = refs.reshape(-1).copy()
    b.tx_ids = tx_ids.reshape(-1).copy()
    b.callers = callers
    pre = (pre_refs.reshape(-1).copy(), pre_tx.reshape(-1).copy(), pre_pos, pre_caller)
    return pre, b


def txids(tb: TxBatch, threads: int = 8) -> np.ndarray:
    """Generator-side WireTransaction ids (OpenSSL SHA-256 in tools/cordagen.c), [ntx, 32]."""
    ids = np.zeros(tb.ntx * 32, dtype=np.uint8)
    lib().gen_txids(ctypes.c_uint64(tb.ntx), _p(tb.salts), _p(tb.tx_comp_start), _p(tb.comp_group),
                    _p(tb.comp_internal), _p(tb.data), _p(tb.comp_off), _p(tb.comp_len), _p(ids), threads)
    return ids.reshape(tb.ntx, 32)


# SignableData(txId, SignatureMetadata(platformVersion, schemeNumberID)).serialize(): the Kryo 4.0.0
# restatement of corda_amd.kryo (parity unpinned without a JVM).  `total` gives a synthetic
# SignableData-shaped template of another length instead (template-length coverage only).
_SIGNABLE_HEAD = (b"corda\x00\x00\x01" + b"\x01\x00net.corda.core.crypto.SignableData\x01\x01"
                  b"net.corda.core.crypto.SecureHash$SHA256\x01\x02net.corda.core.crypto.SignatureMetadata")


class Templates:
    """chip_msg_templates layout: data pool, off u64[n], len u32[n], id_at u32[n], max_len."""
    data = off = len = id_at = None
    max_len = 0


def signable_template(scheme_id: int, platform_version: int = 1, total: int = None):
    """(template bytes without the id, id offset): the Kryo SignableData bytes, or a `total`-byte
    SignableData-shaped message when `total` is given."""
    if total is None:
        from corda_amd import kryo
        return kryo.signable_data_template(platform_version, scheme_id)
    head = (_SIGNABLE_HEAD + bytes(200))[:total - 32 - 8]
    return head + struct.pack(">ii", platform_version, scheme_id), len(head)


def templates_from_list(items) -> Templates:
    """items: [(template_bytes, id_at)]"""
    t = Templates()
    t.data, t.off, t.len = pools_from_list([b for b, _ in items])
    t.id_at = np.array([a for _, a in items], dtype=np.uint32)
    t.max_len = int(t.len.max()) if len(items) else 0
    return t


def messages_from_templates(ids: np.ndarray, tmpl: bytes, id_at: int) -> np.ndarray:
    """[ntx, len(tmpl) + 32] messages tmpl[:id_at] || id || tmpl[id_at:] (host side, for signing)."""
    ntx = len(ids)
    t = np.frombuffer(tmpl, dtype=np.uint8)
    out = np.empty((ntx, len(tmpl) + 32), dtype=np.uint8)
    out[:, :id_at] = t[:id_at]
    out[:, id_at:id_at + 32] = ids
    out[:, id_at + 32:] = t[id_at:]
    return out


class SignerBatch:
    """chip_signer_batch layout (+ expected labels)."""
    tx_idx = tmpl_idx = key_idx = None
    sig_data = sig_off = sig_len = None
    key_data = key_off = key_len = None
    expected = None

    @property
    def n(self):
        return len(self.key_idx)


def ed25519_signers(ids: np.ndarray, signer_keys: np.ndarray, n_keys: int, corrupt: float = 0.0,
                    seed: int = 0x5EED0004, threads: int = 8, extra_key_seeds=()):
    """One Ed25519 signature per (tx, key) pair over the SignableData template of scheme 4.
    signer_keys: [ntx, s] key indices into key_seed(0..n_keys-1) followed by extra_key_seeds.
    `corrupt` of the signatures get one R bit flipped (expected INVALID)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    ntx, s = signer_keys.shape
    seeds = b"".join(key_seed(i) for i in range(n_keys)) + b"".join(extra_key_seeds)
    seeds_np = np.frombuffer(seeds, dtype=np.uint8).copy()
    nk = len(seeds_np) // 32
    pubs = np.zeros(nk * 32, dtype=np.uint8)
    if lib().gen_pubs_many(SCHEME_ED25519, ctypes.c_uint64(nk), _p(seeds_np), _p(pubs)) != 0:
        raise RuntimeError("keygen failed")
    tmpl, at = signable_template(SCHEME_ED25519)
    msgs = messages_from_templates(ids, tmpl, at)
    mlen = msgs.shape[1]
    n = ntx * s
    tx_idx = np.repeat(np.arange(ntx, dtype=np.uint32), s)
    key_of = signer_keys.reshape(-1).astype(np.uint32)
    # sign grouped by key (the generator caches one EVP key per run of equal keys)
    order = np.argsort(key_of, kind="stable")
    sig_sorted = np.zeros(n * 64, dtype=np.uint8)
    sl = np.zeros(n, dtype=np.uint32)
    err = lib().gen_sign_many(SCHEME_ED25519, ctypes.c_uint64(n), _p(seeds_np), _p(np.ascontiguousarray(key_of[order])),
                              _p(msgs.reshape(-1)), _p(np.arange(ntx, dtype=np.uint64) * mlen),
                              _p(np.full(ntx, mlen, dtype=np.uint32)), _p(np.ascontiguousarray(tx_idx[order])), None,
                              _p(sig_sorted), _p(sl), ctypes.c_uint32(64), threads)
    if err:
        raise RuntimeError("signing failed")
    sigs = np.zeros((n, 64), dtype=np.uint8)
    sigs[order] = sig_sorted.reshape(n, 64)
    expected = np.zeros(n, dtype=np.uint8)
    bad = np.nonzero(rng.random(n) < corrupt)[0]
    for i in bad:
        b = int(rng.integers(0, 256))
        sigs[i, b // 8] ^= 1 << (b % 8)
        expected[i] = 1
    sb = SignerBatch()
    sb.tx_idx = tx_idx
    sb.tmpl_idx = np.zeros(n, dtype=np.uint32)
    sb.key_idx = key_of
    sb.sig_data = sigs.reshape(-1)
    sb.sig_off = np.arange(n, dtype=np.uint64) * 64
    sb.sig_len = np.full(n, 64, dtype=np.uint32)
    sb.key_data, sb.key_off, sb.key_len = pools_from_list([spki_ed25519(pubs[32 * i:32 * i + 32].tobytes())
                                                           for i in range(nk)])
    sb.expected = expected
    return sb, templates_from_list([(tmpl, at)]), msgs


NOTARY_SEED = hashlib.sha256(b"cordahip-notary").digest()


def cfg4_workload(ntx: int, n_keys: int = 4096, seed: int = 0x5EED0004, corrupt: float = 0.01, threads: int = 8):
    """cfg4: ntx WireTransactions of the 8-component profile + 2 Ed25519 required
    signers per tx (owner from n_keys parties, the notary) signing SignableData(id)."""
    tb = tx_batch(ntx, seed=seed)
    ids = txids(tb, threads)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    keys = np.stack([rng.integers(0, n_keys, size=ntx), np.full(ntx, n_keys)], axis=1)
    sb, tm, msgs = ed25519_signers(ids, keys, n_keys, corrupt=corrupt, seed=seed + 2, threads=threads,
                                   extra_key_seeds=(NOTARY_SEED,))
    return tb, tm, sb, ids, msgs


def signer_sig_batch(sb: SignerBatch, msgs: np.ndarray) -> SigBatch:
    """The same signatures as a plain chip_sig_batch over host-built messages (oracle / cross-check)."""
    b = SigBatch()
    b.key_idx, b.sig_data, b.sig_off, b.sig_len = sb.key_idx, sb.sig_data, sb.sig_off, sb.sig_len
    b.key_data, b.key_off, b.key_len = sb.key_data, sb.key_off, sb.key_len
    ntx, ml = msgs.shape
    b.msg_idx = sb.tx_idx.astype(np.uint32)
    b.msg_data = msgs.reshape(-1)
    b.msg_off = np.arange(ntx, dtype=np.uint64) * ml
    b.msg_len = np.full(ntx, ml, dtype=np.uint32)
    b.expected = sb.expected
    return b


REQ_NO_SIGNER = 0xFFFFFFFF


class ReqBatch:
    """chip_req_batch layout (+ expected verdicts)."""
    ntx = 0
    sig_start = req_start = node_start = allowed = None
    node_val = node_nkids = node_weight = None
    expected_verdict = expected_arg = None


def cfg4_required(sb: SignerBatch, ntx: int, n_keys: int, seed: int = 0x5EED0006, p_composite: float = 0.02,
                  p_missing: float = 0.01) -> ReqBatch:
    """requiredSigningKeys of the cfg4 transactions (SURVEY.md §8d cfg4 "all required-signer
    verification"), over the signer batch of cfg4_workload (2 signatures per tx: owner, notary):
    {owner, notary} for most; {CompositeKey(1 of owner, another party), notary} for p_composite
    (fulfilled by the owner's signature); {owner, notary, a party that did not sign} for p_missing
    (-> SignaturesMissingException).  Expected verdicts follow the signature labels (a corrupted
    signature throws first) — TransactionWithSignatures.kt:44-50."""
    rng = np.random.Generator(np.random.PCG64(seed))
    kind = rng.random(ntx)
    comp = kind < p_composite
    miss = (kind >= p_composite) & (kind < p_composite + p_missing)
    owner = sb.key_idx[0::2].astype(np.int64)
    notary = sb.key_idx[1::2].astype(np.int64)
    other = (owner + 1 + rng.integers(0, n_keys - 1, size=ntx)) % n_keys
    nreq = np.where(miss, 3, 2)
    nnodes = np.where(comp, 4, np.where(miss, 3, 2))
    req_start = np.zeros(ntx + 1, dtype=np.uint64)
    req_start[1:] = np.cumsum(nreq)
    node_base = np.zeros(ntx + 1, dtype=np.int64)
    node_base[1:] = np.cumsum(nnodes)
    nn = int(node_base[-1])
    val = np.zeros(nn, dtype=np.uint32)
    nk = np.zeros(nn, dtype=np.uint32)
    w = np.ones(nn, dtype=np.uint32)
    b = node_base[:-1]
    # plain txs: [owner] [notary]; missing: + [other]; composite: [owner other C(1,2)] [notary]
    val[b] = owner
    plain = ~comp
    val[b[plain] + 1] = notary[plain]
    val[b[miss] + 2] = other[miss]
    cb = b[comp]
    val[cb + 1] = other[comp]
    val[cb + 2] = 1
    nk[cb + 2] = 2
    val[cb + 3] = notary[comp]
    # node_start per required key
    ns = []
    starts = np.zeros(int(req_start[-1]) + 1, dtype=np.uint64)
    r = req_start[:-1].astype(np.int64)
    starts[r[plain]] = b[plain]
    starts[r[plain] + 1] = b[plain] + 1
    starts[r[miss] + 2] = b[miss] + 2
    starts[r[comp]] = cb
    starts[r[comp] + 1] = cb + 3
    starts[-1] = nn
    del ns
    q = ReqBatch()
    q.ntx = ntx
    q.sig_start = (np.arange(ntx + 1, dtype=np.uint64) * 2)
    q.req_start = req_start
    q.node_start = starts
    q.allowed = None
    q.node_val, q.node_nkids, q.node_weight = val, nk, w
    bad = sb.expected.reshape(ntx, 2) != 0
    first_bad = np.where(bad[:, 0], 0, 1) + np.arange(ntx) * 2
    any_bad = bad.any(axis=1)
    q.expected_verdict = np.where(any_bad, 1, np.where(miss, 2, 0)).astype(np.uint8)
    q.expected_arg = np.where(any_bad, first_bad, np.where(miss, 1, 0)).astype(np.uint32)
    return q


# ---- Kryo SignedTransaction blobs (the §8f-2 front end's input; corda_amd/kryo.py writer) ----
def _tx_groups(tb, t):
    """[(groupIndex, [component bytes])] of transaction t of a TxBatch, in component order."""
    groups = []
    for k in range(int(tb.tx_comp_start[t]), int(tb.tx_comp_start[t + 1])):
        g = int(tb.comp_group[k])
        c = tb.data[int(tb.comp_off[k]):int(tb.comp_off[k]) + int(tb.comp_len[k])].tobytes()
        if groups and groups[-1][0] == g:
            groups[-1][1].append(c)
        else:
            groups.append((g, [c]))
    return groups


def stx_blobs_from_lists(blobs):
    """list of bytes -> (data u8, off u64, len u32)."""
    return pools_from_list(list(blobs))


def stx_signed_tx(tb, sb, t, sig_range, metas=((1, 4),), key_class_id=None):
    """SignedTransaction bytes of transaction t of (TxBatch, SignerBatch): its components, salt and the
    signatures sig_range (SignableData metadata of template sb.tmpl_idx[i] from `metas`)."""
    from corda_amd import kryo as K
    wtx = K.wire_transaction(_tx_groups(tb, t), tb.salts[32 * t:32 * t + 32].tobytes())
    sigs = []
    for i in sig_range:
        k = int(sb.key_idx[i])
        key = sb.key_data[int(sb.key_off[k]):int(sb.key_off[k]) + int(sb.key_len[k])].tobytes()
        sig = sb.sig_data[int(sb.sig_off[i]):int(sb.sig_off[i]) + int(sb.sig_len[i])].tobytes()
        pv, sch = metas[int(sb.tmpl_idx[i])]
        sigs.append(K.Sig(sig, key, pv, sch, key_class_id))
    return K.signed_transaction(wtx, sigs)


def stx_uniform(tb, sb, sigs_per_tx: int, meta=(1, 4)):
    """The SignedTransaction blobs of a uniform batch (every tx the same component lengths, sigs_per_tx
    signatures of equal lengths with equal-length keys, one metadata): the Kryo layout is then the same
    for every tx, so one template is written with corda_amd/kryo.py and each payload field's byte
    positions found by writing it all-0x00 vs all-0xFF; the batch is filled with numpy scatters.
    -> (data u8 [ntx * L], off u64, len u32)."""
    from corda_amd import kryo as K
    ntx = int(tb.ntx)
    per = int(tb.tx_comp_start[1] - tb.tx_comp_start[0])
    glist = [int(g) for g in tb.comp_group[:per]]
    clens = [int(x) for x in tb.comp_len[:per]]
    slen = int(sb.sig_len[0])
    klen = int(sb.key_len[int(sb.key_idx[0])])
    fields = [("c", k, clens[k]) for k in range(per)] + [("salt", 0, 32)] + \
             [(f, j, slen if f == "s" else klen) for j in range(sigs_per_tx) for f in ("s", "k")]

    def write(fill):
        comps = [bytes([fill.get(("c", k), 0)]) * clens[k] for k in range(per)]
        groups = []
        for k in range(per):
            if groups and groups[-1][0] == glist[k]:
                groups[-1][1].append(comps[k])
            else:
                groups.append((glist[k], [comps[k]]))
        wtx = K.wire_transaction(groups, bytes([fill.get(("salt", 0), 0)]) * 32)
        sigs = [K.Sig(bytes([fill.get(("s", j), 0)]) * slen, bytes([fill.get(("k", j), 0)]) * klen, meta[0], meta[1])
                for j in range(sigs_per_tx)]
        return np.frombuffer(K.signed_transaction(wtx, sigs), dtype=np.uint8)

    base = write({})
    pos = {}
    for f, j, n in fields:
        d = np.nonzero(base != write({(f, j): 0xFF}))[0]
        assert len(d) == n, (f, j, len(d), n)
        pos[(f, j)] = d
    L = len(base)
    out = np.tile(base, (ntx, 1))

    def put(key, src):                           # positions -> contiguous runs: slice copies, not gathers
        d = pos[key]
        cut = np.nonzero(np.diff(d) != 1)[0] + 1
        for a, b in zip(np.concatenate([[0], cut]), np.concatenate([cut, [len(d)]])):
            out[:, d[a]:d[a] + (b - a)] = src[:, a:b]
    cdat = tb.data[:ntx * sum(clens)].reshape(ntx, sum(clens))
    at = 0
    for k in range(per):
        put(("c", k), cdat[:, at:at + clens[k]])
        at += clens[k]
    put(("salt", 0), tb.salts.reshape(ntx, 32))
    sig = sb.sig_data.reshape(-1, slen).reshape(ntx, sigs_per_tx, slen)
    kpool = np.stack([sb.key_data[int(o):int(o) + klen] for o in sb.key_off])
    keys = kpool[sb.key_idx.astype(np.int64)].reshape(ntx, sigs_per_tx, klen)
    for j in range(sigs_per_tx):
        put(("s", j), sig[:, j])
        put(("k", j), keys[:, j])
    return out.reshape(-1), np.arange(ntx, dtype=np.uint64) * L, np.full(ntx, L, dtype=np.uint32)


def required_for_parsed(q, sb):
    """A ReqBatch whose leaves index the structured key pool -> the same batch over the key pool of
    chip_stx_parse_device (distinct signer keys numbered by first occurrence in the signature list;
    a key that signs nothing becomes REQ_NO_SIGNER)."""
    first = {}
    for k in sb.key_idx:
        first.setdefault(int(k), len(first))
    remap = np.array([first.get(k, REQ_NO_SIGNER) for k in range(len(sb.key_off))] + [REQ_NO_SIGNER],
                     dtype=np.uint64)
    q2 = ReqBatch()
    for f in ("ntx", "sig_start", "req_start", "node_start", "allowed", "node_nkids", "node_weight",
              "expected_verdict", "expected_arg"):
        setattr(q2, f, getattr(q, f, None))
    leaf = q.node_nkids == 0
    nv = q.node_val.astype(np.uint64).copy()
    nv[leaf] = remap[np.minimum(nv[leaf], len(remap) - 1)]
    q2.node_val = nv.astype(np.uint32)
    return q2


def ed25519_spkis(n_keys: int, extra_key_seeds=()) -> list:
    """SPKI encodings of key_seed(0..n_keys-1) followed by extra_key_seeds (ed25519_signers' key pool)."""
    seeds = b"".join(key_seed(i) for i in range(n_keys)) + b"".join(extra_key_seeds)
    seeds_np = np.frombuffer(seeds, dtype=np.uint8).copy()
    nk = len(seeds_np) // 32
    pubs = np.zeros(nk * 32, dtype=np.uint8)
    if lib().gen_pubs_many(SCHEME_ED25519, ctypes.c_uint64(nk), _p(seeds_np), _p(pubs)) != 0:
        raise RuntimeError("keygen failed")
    return [spki_ed25519(pubs[32 * i:32 * i + 32].tobytes()) for i in range(nk)]


def cfg4_workload_commands(ntx: int, n_keys: int = 4096, seed: int = 0x5EED0004, corrupt: float = 0.01,
                           p_missing: float = 0.01, threads: int = 8):
    """cfg4 with real Kryo contents where the front end reads them: the inputs are StateRef(random hash, 0 / 1)
    (176 bytes each instead of the profile's 96), the command component is Command(Cash.Commands.Move,
    [signer]) and the notary component Party(notary name, notary key) (corda_amd/kryo.py), so
    WireTransaction.requiredSigningKeys = {signer, notary}.  The owner of
    each tx signs, and so does the notary; for p_missing of the transactions the command names another
    party as its signer, which does not sign (-> SignaturesMissingException, 1 needed key).
    -> (tb, tm, sb, ids, expected_verdict, expected_arg)."""
    from corda_amd import kryo as K
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    spkis = ed25519_spkis(n_keys, (NOTARY_SEED,))
    owner = rng.integers(0, n_keys, size=ntx)
    miss = rng.random(ntx) < p_missing
    other = (owner + 1 + rng.integers(0, n_keys - 1, size=ntx)) % n_keys
    signer = np.where(miss, other, owner)
    # inputs: canonical StateRef encodings (the front end accepts no other input bytes); index 0 and 1
    sr0 = np.frombuffer(K.state_ref(bytes(32), 0), dtype=np.uint8)
    sr1 = np.frombuffer(K.state_ref(bytes(32), 1), dtype=np.uint8)
    hpos = np.nonzero(sr0 != np.frombuffer(K.state_ref(b"\xff" * 32, 0), dtype=np.uint8))[0]
    assert len(hpos) == 32 and np.all(np.diff(hpos) == 1) and len(sr0) == len(sr1)
    cmd0 = np.frombuffer(K.command([bytes(44)]), dtype=np.uint8)
    cmd1 = np.frombuffer(K.command([b"\xff" * 44]), dtype=np.uint8)
    kpos = np.nonzero(cmd0 != cmd1)[0]
    assert len(kpos) == 44 and np.all(np.diff(kpos) == 1)
    party = np.frombuffer(K.party(spkis[n_keys]), dtype=np.uint8)
    profile = [(g, [len(cmd0)] if g == 2 else [len(party)] if g == 4 else [len(sr0)] * len(ss) if g == 0 else ss)
               for g, ss in CFG4_PROFILE]
    tb = tx_batch(ntx, profile=profile, seed=seed)
    per = sum(len(ss) for _, ss in profile)
    sizes = [s for _, ss in profile for s in ss]
    groups = [g for g, ss in profile for _ in ss]
    per_bytes = sum(sizes)
    view = tb.data[:ntx * per_bytes].reshape(ntx, per_bytes)
    at = 0
    kp = np.stack([np.frombuffer(k, dtype=np.uint8) for k in spkis])
    hashes = PRNG(seed, b"inputs").np_bytes(ntx * 32 * 2).reshape(ntx, 2, 32)
    nin = 0
    for g, sz in zip(groups, sizes):
        if g == 0:
            view[:, at:at + sz] = sr0 if nin == 0 else sr1
            view[:, at + hpos[0]:at + hpos[0] + 32] = hashes[:, nin % 2]
            nin += 1
        elif g == 2:
            view[:, at:at + sz] = cmd0
            view[:, at + kpos[0]:at + kpos[0] + 44] = kp[signer]
        elif g == 4:
            view[:, at:at + sz] = party
        at += sz
    assert per == len(sizes)
    ids = txids(tb, threads)
    keys = np.stack([owner, np.full(ntx, n_keys)], axis=1)
    sb, tm, _msgs = ed25519_signers(ids, keys, n_keys, corrupt=corrupt, seed=seed + 2, threads=threads,
                                    extra_key_seeds=(NOTARY_SEED,))
    bad = sb.expected.reshape(ntx, 2) != 0
    verdict = np.where(bad.any(axis=1), 1, np.where(miss, 2, 0)).astype(np.uint8)
    first_bad = np.where(bad[:, 0], 0, 1) + np.arange(ntx) * 2          # global index of the first failing sig
    arg = np.where(bad.any(axis=1), first_bad, np.where(miss, 1, 0)).astype(np.uint32)
    return tb, tm, sb, ids, verdict, arg
