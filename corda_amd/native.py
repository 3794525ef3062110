"""ctypes binding of libcordahip.so (the C-ABI in include/cordahip.h).

The product path: every call here goes to the HIP kernels.  There is no CPU fallback — if the
library is missing or no GPU is present, calls raise NativeUnavailable.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _build

_lib = None


class NativeUnavailable(RuntimeError):
    pass


class ChipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("libcordahip error %d: %s" % (code, msg))
        self.code = code


VALID, INVALID, SIG_DECODE, EMPTY_SIG, EMPTY_CLEAR, UNSUPPORTED, KEY_INVALID = range(7)
STATUS_NAMES = ["VALID", "INVALID", "SIG_DECODE", "EMPTY_SIG", "EMPTY_CLEAR", "UNSUPPORTED", "KEY_INVALID"]
SCHEME_K1, SCHEME_R1, SCHEME_ED25519 = 2, 3, 4

# exported symbols declared in include/cordahip.h
EXPORTS = ["chip_abi_version", "chip_device_count", "chip_init", "chip_shutdown", "chip_last_error",
           "chip_verify_batch", "chip_verify_batch_device", "chip_is_valid_batch", "chip_is_valid_batch_device",
           "chip_alloc_pinned", "chip_free_pinned", "chip_txid_batch", "chip_txid_batch_device",
           "chip_uniq_open", "chip_uniq_close", "chip_uniq_size", "chip_uniq_rebuild", "chip_uniq_commit_batch",
           "chip_uniq_commit_batch_device", "chip_uniq_last_error", "chip_uniq_shard_begin", "chip_uniq_shard_vote",
           "chip_uniq_shard_apply", "chip_uniq_shard_classify", "chip_uniq_shard_finish",
           "chip_verify_tx_batch", "chip_verify_tx_batch_device", "chip_ftx_verify_batch",
           "chip_ftx_verify_batch_device", "chip_required_signers", "chip_required_signers_device",
           "chip_verify_signed_tx_batch", "chip_verify_signed_tx_batch_device",
           "chip_stx_parse_device", "chip_stx_verify", "chip_set_kryo_registry", "chip_get_kryo_registry",
           "chip_copy_to_host", "chip_get_stats", "chip_reset_stats",
           "chip_group_init", "chip_group_shutdown", "chip_group_size", "chip_group_member", "chip_group_last_error",
           "chip_group_verify_batch", "chip_group_is_valid_batch", "chip_group_txid_batch",
           "chip_group_verify_signed_tx_batch", "chip_group_stx_verify", "chip_group_ftx_verify_batch",
           "chip_group_plan_sigs", "chip_group_plan_tx", "chip_group_uniq_open", "chip_group_uniq_close",
           "chip_group_uniq_size", "chip_group_uniq_last_error", "chip_group_state_owner", "chip_group_uniq_rebuild",
           "chip_group_uniq_commit_batch", "chip_uniq_last_rounds", "chip_group_last_stats",
           "chip_group_uniq_last_stats"]

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)


class ChipKryoRegistry(ctypes.Structure):
    """chip_kryo_registry: the Kryo class ids the front end depends on (corda_amd/kryo.py Registry)."""
    _fields_ = [("arrays_aslist", ctypes.c_int32), ("signed_tx", ctypes.c_int32), ("wire_tx", ctypes.c_int32),
                ("serialized_bytes", ctypes.c_int32), ("privacy_salt", ctypes.c_int32),
                ("n_public_key", ctypes.c_uint32), ("public_key", ctypes.c_int32 * 8)]

    @classmethod
    def of(cls, reg) -> "ChipKryoRegistry":
        ks = list(reg.public_key)[:8]
        return cls(reg.arrays_aslist, reg.signed_tx, reg.wire_tx, reg.serialized_bytes, reg.privacy_salt, len(ks),
                   (ctypes.c_int32 * 8)(*(ks + [0] * (8 - len(ks)))))


class ChipConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("flags", ctypes.c_uint32), ("reserve_sigs", ctypes.c_uint64)]


class ChipSigBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("key_idx", ctypes.c_void_p), ("msg_idx", ctypes.c_void_p),
                ("sig_data", ctypes.c_void_p), ("sig_off", ctypes.c_void_p), ("sig_len", ctypes.c_void_p),
                ("n_keys", ctypes.c_uint64), ("key_data", ctypes.c_void_p), ("key_off", ctypes.c_void_p),
                ("key_len", ctypes.c_void_p), ("n_msgs", ctypes.c_uint64), ("msg_data", ctypes.c_void_p),
                ("msg_off", ctypes.c_void_p), ("msg_len", ctypes.c_void_p), ("sig_bytes", ctypes.c_uint64),
                ("key_bytes", ctypes.c_uint64), ("msg_bytes", ctypes.c_uint64), ("schemes", ctypes.c_uint32),
                ("pad", ctypes.c_uint32)]


class ChipTxBatch(ctypes.Structure):
    _fields_ = [("ntx", ctypes.c_uint64), ("salts", ctypes.c_void_p), ("tx_comp_start", ctypes.c_void_p),
                ("ncomp", ctypes.c_uint64), ("comp_group", ctypes.c_void_p), ("comp_internal", ctypes.c_void_p),
                ("data", ctypes.c_void_p), ("comp_off", ctypes.c_void_p), ("comp_len", ctypes.c_void_p),
                ("data_bytes", ctypes.c_uint64)]


class ChipMsgTemplates(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("data", ctypes.c_void_p), ("off", ctypes.c_void_p), ("len", ctypes.c_void_p),
                ("id_at", ctypes.c_void_p), ("data_bytes", ctypes.c_uint64), ("max_len", ctypes.c_uint32),
                ("pad", ctypes.c_uint32)]


class ChipSignerBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("tx_idx", ctypes.c_void_p), ("tmpl_idx", ctypes.c_void_p),
                ("key_idx", ctypes.c_void_p), ("sig_data", ctypes.c_void_p), ("sig_off", ctypes.c_void_p),
                ("sig_len", ctypes.c_void_p), ("n_keys", ctypes.c_uint64), ("key_data", ctypes.c_void_p),
                ("key_off", ctypes.c_void_p), ("key_len", ctypes.c_void_p), ("sig_bytes", ctypes.c_uint64),
                ("key_bytes", ctypes.c_uint64)]


class ChipStxBlobs(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("data", ctypes.c_void_p), ("off", ctypes.c_void_p), ("len", ctypes.c_void_p),
                ("data_bytes", ctypes.c_uint64), ("meta", ctypes.c_void_p), ("n_meta", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("data_capacity", ctypes.c_uint64)]


class ChipFtxBatch(ctypes.Structure):
    _fields_ = [("ntx", ctypes.c_uint64), ("ids", ctypes.c_void_p), ("gh_start", ctypes.c_void_p),
                ("group_hashes", ctypes.c_void_p), ("fg_start", ctypes.c_void_p), ("fg_index", ctypes.c_void_p),
                ("comp_start", ctypes.c_void_p), ("comp_data", ctypes.c_void_p), ("comp_off", ctypes.c_void_p),
                ("comp_len", ctypes.c_void_p), ("nonces", ctypes.c_void_p), ("pt_start", ctypes.c_void_p),
                ("pt_tag", ctypes.c_void_p), ("pt_hash", ctypes.c_void_p), ("check_visible", ctypes.c_void_p),
                ("comp_bytes", ctypes.c_uint64), ("visible_mask", ctypes.c_void_p)]


FTX_FIELDS = ("ids", "gh_start", "group_hashes", "fg_start", "fg_index", "comp_start", "comp_data", "comp_off",
              "comp_len", "nonces", "pt_start", "pt_tag", "pt_hash", "check_visible", "visible_mask")


def make_ftx_batch(f) -> ChipFtxBatch:
    s = ChipFtxBatch()
    s.ntx = int(f.ntx)
    for name in FTX_FIELDS:
        setattr(s, name, _ptr(getattr(f, name, None)))
    s.comp_bytes = _nbytes(f.comp_data)
    return s


class ChipReqBatch(ctypes.Structure):
    _fields_ = [("ntx", ctypes.c_uint64), ("sig_start", ctypes.c_void_p), ("req_start", ctypes.c_void_p),
                ("nreq", ctypes.c_uint64), ("node_start", ctypes.c_void_p), ("allowed", ctypes.c_void_p),
                ("n_nodes", ctypes.c_uint64), ("node_val", ctypes.c_void_p), ("node_nkids", ctypes.c_void_p),
                ("node_weight", ctypes.c_void_p)]


# required-signer verdicts (chip_tx_verdict) and the key-tree leaf of a key that signed nothing
TXV_OK, TXV_SIGNATURE, TXV_MISSING, TXV_MALFORMED = range(4)
REQ_NO_SIGNER = 0xFFFFFFFF
REQ_MAX_PENDING = 64


def make_req_batch(q) -> ChipReqBatch:
    """chip_req_batch from an object with fields ntx, sig_start, req_start, node_start, allowed (or None),
    node_val, node_nkids, node_weight (numpy arrays or torch tensors)."""
    s = ChipReqBatch()
    s.ntx = int(q.ntx)
    s.sig_start, s.req_start = _ptr(q.sig_start), _ptr(q.req_start)
    s.nreq = max(len(q.node_start) - 1, 0)
    s.node_start, s.allowed = _ptr(q.node_start), _ptr(getattr(q, "allowed", None))
    s.n_nodes = len(q.node_val)
    s.node_val, s.node_nkids, s.node_weight = _ptr(q.node_val), _ptr(q.node_nkids), _ptr(q.node_weight)
    return s


STX_REQUIRED = 0x1


class ChipStxParsed(ctypes.Structure):
    _fields_ = [("txs", ChipTxBatch), ("sigs", ChipSignerBatch), ("sig_start", ctypes.c_void_p),
                ("req", ChipReqBatch)]


class ChipUniqShardBatch(ctypes.Structure):
    _fields_ = [("ntx", ctypes.c_uint64), ("ref_start", ctypes.c_void_p), ("nref", ctypes.c_uint64),
                ("refs36", ctypes.c_void_p), ("ref_pos", ctypes.c_void_p), ("tx_ids", ctypes.c_void_p),
                ("callers", ctypes.c_void_p)]


class ChipConflict(ctypes.Structure):
    _fields_ = [("tx", ctypes.c_uint64), ("input_index", ctypes.c_uint32), ("consumed_index", ctypes.c_uint32),
                ("consuming_tx", ctypes.c_uint8 * 32), ("consuming_caller", ctypes.c_uint32),
                ("pad", ctypes.c_uint32)]


(K_ED25519, K_ECDSA_R1, K_ECDSA_K1, K_TXID, K_KEYPREP, K_UNIQ, K_ED_COMB, K_ED_FINISH, K_ED_TABLES, K_EC_TABLES,
 K_ED_PLAN, K_ED_COMB_B, K_EC_FRONT, K_REQ, K_STX) = range(15)
(STX_OK, STX_KRYO, STX_NO_SIGS, STX_INVARIANT, STX_UNSUPPORTED) = range(5)
N_KERNELS = 16
FLAG_NO_COMB, FLAG_FORCE_COMB, FLAG_EC_RETRY_ALL, FLAG_KEY_CACHE = 0x1, 0x2, 0x4, 0x8


class ChipStats(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_uint64), ("sigs", ctypes.c_uint64), ("keys_prepared", ctypes.c_uint64),
                ("status_count", ctypes.c_uint64 * 8), ("txids", ctypes.c_uint64), ("uniq_commits", ctypes.c_uint64),
                ("last_verify_kernel_ms", ctypes.c_double), ("last_txid_kernel_ms", ctypes.c_double),
                ("kernel_ms_total", ctypes.c_double * N_KERNELS), ("kernel_launches", ctypes.c_uint64 * N_KERNELS),
                ("key_cache_checks", ctypes.c_uint64)]


class ChipGroupStats(ctypes.Structure):
    """chip_group_stats (ABI 10): where the last group call's time went and how it was split."""
    _fields_ = [("members_used", ctypes.c_uint32), ("rounds", ctypes.c_uint32), ("wall_ms", ctypes.c_double),
                ("plan_ms", ctypes.c_double), ("rebase_ms", ctypes.c_double), ("member_ms_max", ctypes.c_double),
                ("member_ms_min", ctypes.c_double), ("exchange_ms", ctypes.c_double), ("rounds_ms", ctypes.c_double),
                ("finish_ms", ctypes.c_double), ("h2d_bytes_max", ctypes.c_uint64), ("h2d_bytes_total", ctypes.c_uint64),
                ("exchange_bytes_max", ctypes.c_uint64)]

    def as_dict(self):
        return {f: round(getattr(self, f), 4) if t is ctypes.c_double else int(getattr(self, f))
                for f, t in self._fields_}


def lib_path() -> str:
    # CORDAHIP_LIB: an alternative in-tree build of the same sources (A/B experiments, tools/)
    return os.environ.get("CORDAHIP_LIB") or _build.LIB


def load(build_if_missing: bool = False):
    """Load libcordahip.so.  Raises NativeUnavailable if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        if build_if_missing:
            _build.build()
        else:
            raise NativeUnavailable("libcordahip.so not built (run __graft_entry__.build())")
    # PyTorch-ROCm bundles its own HIP/HSA runtimes; when both are used in one process (device
    # tensors, streams, RCCL) torch's must initialise the GPU first or its device enumeration fails
    # after libcordahip's runtime has opened the device.  Loading torch here keeps that order.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    lib.chip_last_error.restype = ctypes.c_char_p
    lib.chip_last_error.argtypes = [ctypes.c_void_p]
    lib.chip_init.argtypes = [ctypes.POINTER(ChipConfig), ctypes.POINTER(ctypes.c_void_p)]
    lib.chip_shutdown.argtypes = [ctypes.c_void_p]
    lib.chip_verify_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipSigBatch), ctypes.c_void_p, ctypes.c_void_p]
    lib.chip_verify_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipSigBatch), ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p]
    lib.chip_is_valid_batch.argtypes = lib.chip_verify_batch.argtypes
    lib.chip_is_valid_batch_device.argtypes = lib.chip_verify_batch_device.argtypes
    lib.chip_alloc_pinned.argtypes = [ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]
    lib.chip_free_pinned.argtypes = [ctypes.c_void_p]
    lib.chip_txid_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipTxBatch), ctypes.c_void_p]
    lib.chip_txid_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipTxBatch), ctypes.c_void_p,
                                           ctypes.c_void_p]
    lib.chip_verify_tx_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipTxBatch), ctypes.POINTER(ChipMsgTemplates),
                                         ctypes.POINTER(ChipSignerBatch), ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]
    lib.chip_verify_tx_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipTxBatch),
                                                ctypes.POINTER(ChipMsgTemplates), ctypes.POINTER(ChipSignerBatch),
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.chip_ftx_verify_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipFtxBatch), ctypes.c_void_p,
                                          ctypes.c_void_p]
    lib.chip_ftx_verify_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipFtxBatch), ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p]
    lib.chip_required_signers.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipReqBatch), ctypes.POINTER(ChipSigBatch),
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.chip_required_signers_device.argtypes = lib.chip_required_signers.argtypes + [ctypes.c_void_p]
    lib.chip_verify_signed_tx_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipTxBatch),
                                                ctypes.POINTER(ChipMsgTemplates), ctypes.POINTER(ChipSignerBatch),
                                                ctypes.POINTER(ChipReqBatch), ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.chip_verify_signed_tx_batch_device.argtypes = lib.chip_verify_signed_tx_batch.argtypes + [ctypes.c_void_p]
    lib.chip_uniq_open.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]
    lib.chip_uniq_close.argtypes = [ctypes.c_void_p]
    lib.chip_uniq_size.argtypes = [ctypes.c_void_p]
    lib.chip_uniq_size.restype = ctypes.c_uint64
    lib.chip_uniq_rebuild.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p]
    lib.chip_uniq_commit_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    lib.chip_uniq_commit_batch_device.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                                  ctypes.c_void_p]
    lib.chip_uniq_last_error.restype = ctypes.c_char_p
    lib.chip_uniq_last_error.argtypes = [ctypes.c_void_p]
    lib.chip_uniq_shard_begin.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipUniqShardBatch), ctypes.c_void_p]
    lib.chip_uniq_shard_vote.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.chip_uniq_shard_apply.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    lib.chip_uniq_shard_classify.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.chip_uniq_shard_finish.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    lib.chip_stx_parse_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipStxBlobs), ctypes.c_void_p,
                                          ctypes.POINTER(ChipStxParsed), ctypes.c_void_p]
    lib.chip_stx_verify.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ChipMsgTemplates),
                                    ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p]
    lib.chip_set_kryo_registry.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipKryoRegistry)]
    lib.chip_get_kryo_registry.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipKryoRegistry)]
    lib.chip_copy_to_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    lib.chip_get_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipStats)]
    lib.chip_reset_stats.argtypes = [ctypes.c_void_p]
    # device groups (ABI 9)
    lib.chip_group_init.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ChipConfig),
                                    ctypes.POINTER(ctypes.c_void_p)]
    lib.chip_group_shutdown.argtypes = [ctypes.c_void_p]
    lib.chip_group_size.argtypes = [ctypes.c_void_p]
    lib.chip_group_member.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.chip_group_member.restype = ctypes.c_void_p
    lib.chip_group_last_error.argtypes = [ctypes.c_void_p]
    lib.chip_group_last_error.restype = ctypes.c_char_p
    lib.chip_group_verify_batch.argtypes = lib.chip_verify_batch.argtypes
    lib.chip_group_is_valid_batch.argtypes = lib.chip_verify_batch.argtypes
    lib.chip_group_txid_batch.argtypes = lib.chip_txid_batch.argtypes
    lib.chip_group_verify_signed_tx_batch.argtypes = lib.chip_verify_signed_tx_batch.argtypes
    lib.chip_group_stx_verify.argtypes = lib.chip_stx_verify.argtypes
    lib.chip_group_ftx_verify_batch.argtypes = lib.chip_ftx_verify_batch.argtypes
    lib.chip_group_plan_sigs.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]
    lib.chip_group_plan_tx.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]
    lib.chip_group_uniq_open.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]
    lib.chip_group_uniq_close.argtypes = [ctypes.c_void_p]
    lib.chip_group_uniq_size.argtypes = [ctypes.c_void_p]
    lib.chip_group_uniq_size.restype = ctypes.c_uint64
    lib.chip_group_uniq_last_error.argtypes = [ctypes.c_void_p]
    lib.chip_group_uniq_last_error.restype = ctypes.c_char_p
    lib.chip_group_state_owner.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    lib.chip_group_state_owner.restype = ctypes.c_uint32
    lib.chip_group_uniq_rebuild.argtypes = lib.chip_uniq_rebuild.argtypes
    lib.chip_group_uniq_commit_batch.argtypes = lib.chip_uniq_commit_batch.argtypes
    # ABI 10
    lib.chip_uniq_last_rounds.argtypes = [ctypes.c_void_p]
    lib.chip_uniq_last_rounds.restype = ctypes.c_uint32
    lib.chip_group_last_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipGroupStats)]
    lib.chip_group_uniq_last_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChipGroupStats)]
    _lib = lib
    return lib


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if hasattr(a, "data_ptr"):          # torch tensor (device-resident path)
        return a.data_ptr()
    return a.ctypes.data


def make_sig_batch(b) -> ChipSigBatch:
    """Build a ChipSigBatch from an object with the SoA fields (numpy arrays or torch tensors)."""
    def nbytes(a):
        if a is None:
            return 0
        if hasattr(a, "numel"):
            return int(a.numel() * a.element_size())
        return int(a.nbytes)
    s = ChipSigBatch()
    s.n = len(b.key_idx)
    s.key_idx, s.msg_idx = _ptr(b.key_idx), _ptr(b.msg_idx)
    s.sig_data, s.sig_off, s.sig_len = _ptr(b.sig_data), _ptr(b.sig_off), _ptr(b.sig_len)
    s.n_keys = len(b.key_off)
    s.key_data, s.key_off, s.key_len = _ptr(b.key_data), _ptr(b.key_off), _ptr(b.key_len)
    s.n_msgs = len(b.msg_off)
    s.msg_data, s.msg_off, s.msg_len = _ptr(b.msg_data), _ptr(b.msg_off), _ptr(b.msg_len)
    s.sig_bytes, s.key_bytes, s.msg_bytes = nbytes(b.sig_data), nbytes(b.key_data), nbytes(b.msg_data)
    s.schemes = int(getattr(b, "schemes_hint", 0) or 0)
    return s


def make_tx_batch(t) -> ChipTxBatch:
    def nbytes(a):
        if hasattr(a, "numel"):
            return int(a.numel() * a.element_size())
        return int(a.nbytes)
    s = ChipTxBatch()
    s.ntx = t.ntx
    s.salts, s.tx_comp_start = _ptr(t.salts), _ptr(t.tx_comp_start)
    s.ncomp = len(t.comp_group)
    s.comp_group, s.comp_internal = _ptr(t.comp_group), _ptr(t.comp_internal)
    s.data, s.comp_off, s.comp_len = _ptr(t.data), _ptr(t.comp_off), _ptr(t.comp_len)
    s.data_bytes = nbytes(t.data)
    return s


def _nbytes(a):
    if a is None:
        return 0
    if hasattr(a, "numel"):
        return int(a.numel() * a.element_size())
    return int(a.nbytes)


def make_templates(t) -> ChipMsgTemplates:
    """SignableData message templates: fields data, off, len, id_at (+ max_len int)."""
    s = ChipMsgTemplates()
    s.n = len(t.off)
    s.data, s.off, s.len, s.id_at = _ptr(t.data), _ptr(t.off), _ptr(t.len), _ptr(t.id_at)
    s.data_bytes = _nbytes(t.data)
    s.max_len = int(t.max_len)
    return s


def make_signers(b) -> ChipSignerBatch:
    s = ChipSignerBatch()
    s.n = len(b.key_idx)
    s.tx_idx, s.tmpl_idx, s.key_idx = _ptr(b.tx_idx), _ptr(b.tmpl_idx), _ptr(b.key_idx)
    s.sig_data, s.sig_off, s.sig_len = _ptr(b.sig_data), _ptr(b.sig_off), _ptr(b.sig_len)
    s.n_keys = len(b.key_off)
    s.key_data, s.key_off, s.key_len = _ptr(b.key_data), _ptr(b.key_off), _ptr(b.key_len)
    s.sig_bytes, s.key_bytes = _nbytes(b.sig_data), _nbytes(b.key_data)
    return s


class Context:
    """One libcordahip context = one GPU (one process per GPU)."""

    def __init__(self, device: int = 0, reserve_sigs: int = 0, flags: int = 0):
        self.lib = load()
        cfg = ChipConfig(device, flags, reserve_sigs)
        h = ctypes.c_void_p()
        rc = self.lib.chip_init(ctypes.byref(cfg), ctypes.byref(h))
        if rc != 0:
            raise NativeUnavailable("chip_init(device=%d) failed with %d (no GPU?)" % (device, rc))
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            self.lib.chip_shutdown(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise ChipError(rc, self.lib.chip_last_error(self.h).decode(errors="replace"))

    # ---- signatures ----
    def verify_batch(self, b, is_valid: bool = False):
        """Host SoA batch -> (status u8[n], bitmap u64[ceil(n/64)]).  is_valid=True gives
        Crypto.isValid semantics (no empty-input checks) instead of Crypto.doVerify's."""
        s = make_sig_batch(b)
        status = np.zeros(s.n, dtype=np.uint8)
        bitmap = np.zeros((s.n + 63) // 64, dtype=np.uint64)
        fn = self.lib.chip_is_valid_batch if is_valid else self.lib.chip_verify_batch
        self._check(fn(self.h, ctypes.byref(s), _ptr(status), _ptr(bitmap)))
        return status, bitmap

    def verify_batch_device(self, dev_batch, status, bitmap, stream=None, is_valid: bool = False):
        """Device-resident batch (torch tensors on this GPU); enqueued on `stream` (int handle) and
        returns without waiting.  A 0 / None handle means the context's own stream (NOT torch's legacy
        default stream, whose handle is also 0): pass a torch.cuda.Stream's handle and order it
        against the consumer.  An optional `schemes_hint` attribute (bit 1 << scheme per scheme
        present) is passed through."""
        s = make_sig_batch(dev_batch)
        fn = self.lib.chip_is_valid_batch_device if is_valid else self.lib.chip_verify_batch_device
        self._check(fn(self.h, ctypes.byref(s), _ptr(status), _ptr(bitmap), stream or None))

    # ---- tx ids ----
    def txid_batch(self, t) -> np.ndarray:
        s = make_tx_batch(t)
        ids = np.zeros(s.ntx * 32, dtype=np.uint8)
        self._check(self.lib.chip_txid_batch(self.h, ctypes.byref(s), _ptr(ids)))
        return ids.reshape(s.ntx, 32)

    def txid_batch_device(self, dev_tx, ids, stream=None):
        s = make_tx_batch(dev_tx)
        self._check(self.lib.chip_txid_batch_device(self.h, ctypes.byref(s), _ptr(ids), stream or None))

    # ---- fused: ids + required-signer verification against the recomputed ids ----
    def verify_tx_batch(self, t, templates, signers):
        """Host arrays -> (ids u8[ntx,32], status u8[n], bitmap u64[ceil(n/64)])."""
        tb, tm, sb = make_tx_batch(t), make_templates(templates), make_signers(signers)
        ids = np.zeros(tb.ntx * 32, dtype=np.uint8)
        status = np.zeros(sb.n, dtype=np.uint8)
        bitmap = np.zeros((sb.n + 63) // 64, dtype=np.uint64)
        self._check(self.lib.chip_verify_tx_batch(self.h, ctypes.byref(tb), ctypes.byref(tm), ctypes.byref(sb),
                                                  _ptr(ids), _ptr(status), _ptr(bitmap)))
        return ids.reshape(tb.ntx, 32), status, bitmap

    def verify_tx_batch_device(self, dev_tx, dev_templates, dev_signers, ids, status, bitmap, stream=None):
        tb, tm, sb = make_tx_batch(dev_tx), make_templates(dev_templates), make_signers(dev_signers)
        self._check(self.lib.chip_verify_tx_batch_device(self.h, ctypes.byref(tb), ctypes.byref(tm),
                                                         ctypes.byref(sb), _ptr(ids), _ptr(status), _ptr(bitmap),
                                                         stream or None))

    # ---- required signers (verifySignaturesExcept after the statuses) ----
    def required_signers(self, q, b, status):
        """Host arrays: chip_req_batch `q` over the signatures of SoA batch `b` with statuses `status`
        -> (verdict u8[ntx], arg u32[ntx], missing u8[nreq])."""
        rq, sb = make_req_batch(q), make_sig_batch(b)
        verdict = np.zeros(rq.ntx, dtype=np.uint8)
        arg = np.zeros(rq.ntx, dtype=np.uint32)
        missing = np.zeros(max(rq.nreq, 1), dtype=np.uint8)
        self._check(self.lib.chip_required_signers(self.h, ctypes.byref(rq), ctypes.byref(sb),
                                                   _ptr(np.ascontiguousarray(status, dtype=np.uint8)),
                                                   _ptr(verdict), _ptr(arg), _ptr(missing)))
        return verdict, arg, missing[:rq.nreq]

    def required_signers_device(self, dev_q, dev_b, status, verdict, arg, missing=None, stream=None):
        rq, sb = make_req_batch(dev_q), make_sig_batch(dev_b)
        self._check(self.lib.chip_required_signers_device(self.h, ctypes.byref(rq), ctypes.byref(sb), _ptr(status),
                                                          _ptr(verdict), _ptr(arg), _ptr(missing), stream or None))

    def verify_signed_tx_batch(self, t, templates, signers, q):
        """Host arrays -> (ids u8[ntx,32], status u8[n], verdict u8[ntx], arg u32[ntx], missing u8[nreq])."""
        tb, tm, sb, rq = make_tx_batch(t), make_templates(templates), make_signers(signers), make_req_batch(q)
        ids = np.zeros(tb.ntx * 32, dtype=np.uint8)
        status = np.zeros(max(sb.n, 1), dtype=np.uint8)
        verdict = np.zeros(rq.ntx, dtype=np.uint8)
        arg = np.zeros(rq.ntx, dtype=np.uint32)
        missing = np.zeros(max(rq.nreq, 1), dtype=np.uint8)
        self._check(self.lib.chip_verify_signed_tx_batch(self.h, ctypes.byref(tb), ctypes.byref(tm), ctypes.byref(sb),
                                                         ctypes.byref(rq), _ptr(ids), _ptr(status), _ptr(verdict),
                                                         _ptr(arg), _ptr(missing)))
        return ids.reshape(tb.ntx, 32), status[:sb.n], verdict, arg, missing[:rq.nreq]

    def verify_signed_tx_batch_device(self, dev_tx, dev_templates, dev_signers, dev_q, ids, status, verdict, arg,
                                      missing=None, stream=None):
        tb, tm, sb = make_tx_batch(dev_tx), make_templates(dev_templates), make_signers(dev_signers)
        rq = make_req_batch(dev_q)
        self._check(self.lib.chip_verify_signed_tx_batch_device(self.h, ctypes.byref(tb), ctypes.byref(tm),
                                                                ctypes.byref(sb), ctypes.byref(rq), _ptr(ids),
                                                                _ptr(status), _ptr(verdict), _ptr(arg), _ptr(missing),
                                                                stream or None))

    # ---- Kryo front end: SignedTransaction bytes -> batches (device) ----
    def stx_parse_device(self, data, off, lens, data_bytes, meta, tx_status, stream=None,
                         required: bool = False, data_capacity: int = 0) -> ChipStxParsed:
        """data / off / lens / tx_status: device tensors; meta: host int32 [n_meta, 2] (platformVersion,
        schemeNumberID) per message template.  Returns the chip_stx_parsed of device pointers (valid
        until the next call on this context)."""
        meta = np.ascontiguousarray(np.asarray(meta, dtype=np.int32).reshape(-1, 2))
        b = ChipStxBlobs(n=int(off.numel() if hasattr(off, "numel") else len(off)), data=_ptr(data), off=_ptr(off),
                         len=_ptr(lens), data_bytes=int(data_bytes), meta=meta.ctypes.data, n_meta=len(meta),
                         flags=STX_REQUIRED if required else 0, data_capacity=int(data_capacity))
        out = ChipStxParsed()
        self._check(self.lib.chip_stx_parse_device(self.h, ctypes.byref(b), _ptr(tx_status), ctypes.byref(out),
                                                   stream or None))
        out._meta = meta
        return out

    def set_kryo_registry(self, reg) -> None:
        """chip_set_kryo_registry from a corda_amd.kryo.Registry."""
        r = ChipKryoRegistry.of(reg)
        self._check(self.lib.chip_set_kryo_registry(self.h, ctypes.byref(r)))

    def kryo_registry(self) -> ChipKryoRegistry:
        r = ChipKryoRegistry()
        self._check(self.lib.chip_get_kryo_registry(self.h, ctypes.byref(r)))
        return r

    def stx_verify(self, data, off, lens, templates, meta, want_ids: bool = False):
        """Host arrays: SignedTransaction blobs -> (tx_status u8[n], verdict u8[n], arg u32[n], ids or None)
        through chip_stx_verify (parse + requiredSigningKeys + the fused verify, on the device)."""
        n = len(off)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        meta = np.ascontiguousarray(np.asarray(meta, dtype=np.int32).reshape(-1, 2))
        tm = make_templates(templates)
        st = np.zeros(max(n, 1), dtype=np.uint8)
        v = np.zeros(max(n, 1), dtype=np.uint8)
        a = np.zeros(max(n, 1), dtype=np.uint32)
        ids = np.zeros(max(n, 1) * 32, dtype=np.uint8) if want_ids else None
        self._check(self.lib.chip_stx_verify(self.h, n, _ptr(data), _ptr(off), _ptr(lens), len(data), ctypes.byref(tm),
                                             meta.ctypes.data, len(meta), _ptr(st), _ptr(v), _ptr(a), _ptr(ids)))
        return st[:n], v[:n], a[:n], (ids[:32 * n].reshape(n, 32) if want_ids else None)

    def pinned_copy(self, arr: np.ndarray) -> np.ndarray:
        """A copy of `arr` in page-locked host memory from chip_alloc_pinned (freed with the context);
        host entries then stage it by DMA instead of through a pageable bounce."""
        arr = np.ascontiguousarray(arr)
        nbytes = max(arr.nbytes, 1)
        p = ctypes.c_void_p()
        self._check(self.lib.chip_alloc_pinned(nbytes, ctypes.byref(p)))
        if not hasattr(self, "_pinned"):
            self._pinned = []
        self._pinned.append(p.value)
        buf = (ctypes.c_uint8 * nbytes).from_address(p.value)
        out = np.frombuffer(buf, dtype=np.uint8, count=arr.nbytes).view(arr.dtype).reshape(arr.shape)
        out[...] = arr
        return out

    def free_pinned(self):
        for p in getattr(self, "_pinned", []):
            self.lib.chip_free_pinned(p)
        self._pinned = []

    def copy_to_host(self, ptr, count: int, dtype) -> np.ndarray:
        """A library-owned device array (e.g. a chip_stx_parsed field) -> host numpy array."""
        out = np.zeros(max(count, 1), dtype=dtype)
        self._check(self.lib.chip_copy_to_host(self.h, out.ctypes.data, ptr, count * out.itemsize))
        return out[:count]

    def verify_signed_tx_parsed_device(self, parsed: ChipStxParsed, dev_templates, dev_q, ids, status, verdict, arg,
                                       missing=None, stream=None):
        """chip_verify_signed_tx_batch_device over a parsed batch (its sig_start must be dev_q's); dev_q None =
        the required keys the parse derived (required=True)."""
        tm = make_templates(dev_templates)
        rq = parsed.req if dev_q is None else make_req_batch(dev_q)
        self._check(self.lib.chip_verify_signed_tx_batch_device(self.h, ctypes.byref(parsed.txs), ctypes.byref(tm),
                                                                ctypes.byref(parsed.sigs), ctypes.byref(rq), _ptr(ids),
                                                                _ptr(status), _ptr(verdict), _ptr(arg), _ptr(missing),
                                                                stream or None))

    # ---- FilteredTransaction.verify + checkAllComponentsVisible ----
    def ftx_verify_batch(self, f):
        """Host arrays (chip_ftx_batch layout) -> (status u8[ntx], reason u8[ntx])."""
        s = make_ftx_batch(f)
        status = np.zeros(s.ntx, dtype=np.uint8)
        reason = np.zeros(s.ntx, dtype=np.uint8)
        self._check(self.lib.chip_ftx_verify_batch(self.h, ctypes.byref(s), _ptr(status), _ptr(reason)))
        return status, reason

    def ftx_verify_batch_device(self, dev_f, status, reason=None, stream=None):
        s = make_ftx_batch(dev_f)
        self._check(self.lib.chip_ftx_verify_batch_device(self.h, ctypes.byref(s), _ptr(status), _ptr(reason),
                                                          stream or None))

    def stats(self) -> ChipStats:
        st = ChipStats()
        self._check(self.lib.chip_get_stats(self.h, ctypes.byref(st)))
        return st

    def reset_stats(self):
        self._check(self.lib.chip_reset_stats(self.h))

    # ---- uniqueness ----
    def uniq_open(self, capacity: int):
        return UniqTable(self, capacity)


class UniqTable:
    """GPU-resident StateRef -> ConsumingTx table (PersistentUniquenessProvider semantics)."""

    def __init__(self, ctx: Context, capacity: int):
        self.ctx = ctx
        h = ctypes.c_void_p()
        ctx._check(ctx.lib.chip_uniq_open(ctx.h, ctypes.c_uint64(capacity), ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.chip_uniq_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self) -> int:
        return int(self.ctx.lib.chip_uniq_size(self.h))

    def _check(self, rc):
        if rc != 0:
            raise ChipError(rc, self.ctx.lib.chip_uniq_last_error(self.h).decode(errors="replace"))

    def rebuild(self, refs36, tx32, idx, caller):
        n = len(idx)
        self._check(self.ctx.lib.chip_uniq_rebuild(self.h, ctypes.c_uint64(n), _ptr(refs36), _ptr(tx32),
                                                   _ptr(idx), _ptr(caller)))

    def last_rounds(self) -> int:
        """chip_uniq_last_rounds: ordered-commit rounds of the last finished commit."""
        return int(self.ctx.lib.chip_uniq_last_rounds(self.h))

    def commit_batch_raw(self, tx_ref_start, refs36, tx_ids, callers, cap=None):
        """chip_uniq_commit_batch with the records left as raw chip_conflict bytes: (statuses, bytes, count)."""
        ntx = len(tx_ref_start) - 1
        st = np.zeros(max(ntx, 1), dtype=np.uint8)
        if cap is None:
            cap = int(tx_ref_start[-1]) + 1
        out = np.zeros(max(cap, 1) * ctypes.sizeof(ChipConflict), dtype=np.uint8)
        nout = ctypes.c_uint64()
        self._check(self.ctx.lib.chip_uniq_commit_batch(self.h, ctypes.c_uint64(ntx), _ptr(tx_ref_start),
                                                        _ptr(refs36), _ptr(tx_ids), _ptr(callers), _ptr(st),
                                                        out.ctypes.data, ctypes.c_uint64(cap), ctypes.byref(nout)))
        n = int(nout.value)
        return st[:ntx], out[:min(n, cap) * ctypes.sizeof(ChipConflict)], n

    def commit_batch_device(self, tx_ref_start, nref, refs36, tx_ids, callers, tx_status, out, cap, stream=None):
        """Device-resident commit (torch tensors on this GPU).  Returns the full conflict-record count;
        the first min(count, cap) records are in `out` (ChipConflict layout, 48 bytes each)."""
        ntx = tx_ref_start.numel() - 1
        nout = ctypes.c_uint64()
        self._check(self.ctx.lib.chip_uniq_commit_batch_device(
            self.h, ctypes.c_uint64(ntx), _ptr(tx_ref_start), ctypes.c_uint64(nref), _ptr(refs36), _ptr(tx_ids),
            _ptr(callers), _ptr(tx_status), _ptr(out), ctypes.c_uint64(cap), ctypes.byref(nout), stream or None))
        return nout.value

    def commit_batch(self, tx_ref_start, refs36, tx_ids, callers, cap=None):
        ntx = len(tx_ref_start) - 1
        st = np.zeros(ntx, dtype=np.uint8)
        if cap is None:
            cap = int(tx_ref_start[-1]) + 1
        out = (ChipConflict * max(cap, 1))()
        nout = ctypes.c_uint64()
        self._check(self.ctx.lib.chip_uniq_commit_batch(self.h, ctypes.c_uint64(ntx), _ptr(tx_ref_start),
                                                            _ptr(refs36), _ptr(tx_ids), _ptr(callers), _ptr(st),
                                                            out, ctypes.c_uint64(cap), ctypes.byref(nout)))
        recs = [(c.tx, c.input_index, c.consumed_index, bytes(c.consuming_tx), c.consuming_caller)
                for c in out[:min(nout.value, cap)]]
        return st, recs


def records_to_bytes(recs) -> bytes:
    """[(tx, input_index, consumed_index, consuming_tx, caller)] -> ChipConflict records (56 B each)."""
    arr = (ChipConflict * len(recs))()
    for a, (tx, i, ci, cid, cc) in zip(arr, recs):
        a.tx, a.input_index, a.consumed_index, a.consuming_caller, a.pad = tx, i, ci, cc, 0
        ctypes.memmove(a.consuming_tx, bytes(cid), 32)
    return bytes(arr)


def records_from_bytes(raw: bytes):
    """ChipConflict records (56 bytes each) -> [(tx, input_index, consumed_index, consuming_tx, caller)]."""
    n = len(raw) // ctypes.sizeof(ChipConflict)
    arr = (ChipConflict * n).from_buffer_copy(raw[:n * ctypes.sizeof(ChipConflict)])
    return [(c.tx, c.input_index, c.consumed_index, bytes(c.consuming_tx), c.consuming_caller) for c in arr]


class UniqShardEngine:
    """One GPU's slice of the notary table driven through the chip_uniq_shard_* phases (the
    multi-GPU protocol is corda_amd.distributed.commit_sharded).  Device buffers are torch tensors
    on the table's GPU; the phases run on the engine's own stream, ordered against torch's current
    stream (where the collectives and copies of the vote tensors run) with stream waits."""

    def __init__(self, table: UniqTable):
        self.table = table
        self.lib = table.ctx.lib
        self.device = table.ctx.device
        self._keep = None

    def upload(self, shard, tx_ids, callers):
        """Host shard arrays -> device tensors (outside any timed region)."""
        import torch
        dev = torch.device("cuda", self.device)

        def t(a, dt):
            a = np.ascontiguousarray(a)
            if a.size == 0:
                a = np.zeros(16, dtype=a.dtype)
            return torch.from_numpy(a.view(dt)).to(dev)
        ntx = len(shard.ref_start) - 1
        return {"ntx": ntx, "nref": int(shard.ref_start[-1]),
                "start": t(np.asarray(shard.ref_start, dtype=np.uint64), np.int64),
                "refs": t(np.asarray(shard.refs, dtype=np.uint8), np.uint8),
                "pos": t(np.asarray(shard.ref_pos, dtype=np.uint32), np.int32),
                "ids": t(np.asarray(tx_ids, dtype=np.uint8), np.uint8),
                "callers": t(np.asarray(callers, dtype=np.uint32), np.int32)}

    def begin(self, shard, tx_ids=None, callers=None):
        """`shard`: a host UniqShard (uploaded here) or the dict upload() returned (device-resident)."""
        import torch
        d = shard if isinstance(shard, dict) else self.upload(shard, tx_ids, callers)
        self._keep = d
        self.ntx = d["ntx"]
        dev = torch.device("cuda", self.device)
        self.vote_buf = torch.zeros(max(1, self.ntx), dtype=torch.uint8, device=dev)
        self.status = torch.zeros(max(1, self.ntx), dtype=torch.uint8, device=dev)
        b = ChipUniqShardBatch(self.ntx, d["start"].data_ptr(), d["nref"], d["refs"].data_ptr(), d["pos"].data_ptr(),
                               d["ids"].data_ptr(), d["callers"].data_ptr())
        self.stream = torch.cuda.Stream(device=dev)
        self.stream.wait_stream(torch.cuda.current_stream(dev))   # inputs / buffers written by torch
        self.table._check(self.lib.chip_uniq_shard_begin(self.table.h, ctypes.byref(b), self.stream.cuda_stream))

    def _to_torch(self):
        import torch
        torch.cuda.current_stream(torch.device("cuda", self.device)).wait_stream(self.stream)

    def _from_torch(self):
        import torch
        self.stream.wait_stream(torch.cuda.current_stream(torch.device("cuda", self.device)))

    def vote(self):
        self._from_torch()
        self.table._check(self.lib.chip_uniq_shard_vote(self.table.h, self.vote_buf.data_ptr()))
        self._to_torch()
        return self.vote_buf[:self.ntx]

    def apply(self, decision) -> int:
        self._from_torch()
        und = ctypes.c_uint64()
        self.table._check(self.lib.chip_uniq_shard_apply(self.table.h, decision.data_ptr(), ctypes.byref(und)))
        return und.value

    def classify(self):
        self._from_torch()
        self.table._check(self.lib.chip_uniq_shard_classify(self.table.h, self.vote_buf.data_ptr()))
        self._to_torch()
        return self.vote_buf[:self.ntx]

    def finish_device(self, decision):
        """-> (status u8[ntx] device tensor, this shard's ChipConflict records as a device u8 tensor of
        n * 56 bytes, ordered by (tx, input_index)); nothing leaves the GPU."""
        import torch
        cap = int(self._keep["nref"]) + 1
        out = torch.empty(cap * ctypes.sizeof(ChipConflict), dtype=torch.uint8,
                          device=torch.device("cuda", self.device))
        self._from_torch()
        nout = ctypes.c_uint64()
        self.table._check(self.lib.chip_uniq_shard_finish(self.table.h, decision.data_ptr(), self.status.data_ptr(),
                                                          out.data_ptr(), ctypes.c_uint64(cap), ctypes.byref(nout)))
        self._to_torch()
        n = min(nout.value, cap)
        self._keep = None
        return self.status[:self.ntx], out[:n * ctypes.sizeof(ChipConflict)]

    def finish(self, decision):
        """-> (status u8[ntx] numpy, this shard's conflict records)."""
        st, raw = self.finish_device(decision)
        return st.cpu().numpy(), records_from_bytes(raw.cpu().numpy().tobytes())


# ---------------------------------------------------------------------------------------
# device groups: every GPU of the process behind one handle (chip_group_*, include/cordahip.h ABI 9)
def plan_sigs(msg_idx, k: int, min_share: int = 0) -> np.ndarray:
    """chip_group_plan_sigs: the signature ranges a k-member group verifies (host-only, no GPU)."""
    lib = load()
    m = np.ascontiguousarray(msg_idx, dtype=np.uint32)
    cut = np.zeros(k + 1, dtype=np.uint64)
    rc = lib.chip_group_plan_sigs(len(m), _ptr(m) if len(m) else None, k, min_share, _ptr(cut))
    if rc:
        raise ChipError(rc, "chip_group_plan_sigs")
    return cut


def plan_tx(ntx: int, prefix, k: int, min_share: int = 0) -> np.ndarray:
    """chip_group_plan_tx: the transaction ranges of a k-member group, balanced by prefix (or one unit a tx)."""
    lib = load()
    p = None if prefix is None else np.ascontiguousarray(prefix, dtype=np.uint64)
    cut = np.zeros(k + 1, dtype=np.uint64)
    rc = lib.chip_group_plan_tx(ntx, None if p is None else _ptr(p), k, min_share, _ptr(cut))
    if rc:
        raise ChipError(rc, "chip_group_plan_tx")
    return cut


def state_owner(ref36: bytes, members: int) -> int:
    """chip_group_state_owner: the member whose table slice holds this StateRef."""
    buf = (ctypes.c_uint8 * 36).from_buffer_copy(bytes(ref36))
    return int(load().chip_group_state_owner(ctypes.addressof(buf), members))


class Group:
    """A device group: one context per entry of `devices` (an ordinal may repeat), host-buffer entries that split
    each batch by transaction ranges over the members and return the one-context results."""

    def __init__(self, devices, flags: int = 0, reserve_sigs: int = 0):
        self.lib = load()
        devs = (ctypes.c_int * len(devices))(*devices)
        cfg = ChipConfig(0, flags, reserve_sigs)
        h = ctypes.c_void_p()
        rc = self.lib.chip_group_init(devs, len(devices), ctypes.byref(cfg), ctypes.byref(h))
        if rc != 0:
            raise NativeUnavailable("chip_group_init(%s) failed with %d" % (list(devices), rc))
        self.h = h
        self.devices = list(devices)

    def close(self):
        if getattr(self, "h", None):
            self.lib.chip_group_shutdown(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self) -> int:
        return int(self.lib.chip_group_size(self.h))

    def _check(self, rc):
        if rc != 0:
            raise ChipError(rc, self.lib.chip_group_last_error(self.h).decode(errors="replace"))

    def verify_batch(self, b, is_valid: bool = False):
        s = make_sig_batch(b)
        status = np.zeros(max(s.n, 1), dtype=np.uint8)
        bitmap = np.zeros(max((s.n + 63) // 64, 1), dtype=np.uint64)
        fn = self.lib.chip_group_is_valid_batch if is_valid else self.lib.chip_group_verify_batch
        self._check(fn(self.h, ctypes.byref(s), _ptr(status), _ptr(bitmap)))
        return status[:s.n], bitmap[:(s.n + 63) // 64]

    def txid_batch(self, t) -> np.ndarray:
        s = make_tx_batch(t)
        ids = np.zeros(max(s.ntx, 1) * 32, dtype=np.uint8)
        self._check(self.lib.chip_group_txid_batch(self.h, ctypes.byref(s), _ptr(ids)))
        return ids[:32 * s.ntx].reshape(s.ntx, 32)

    def verify_signed_tx_batch(self, t, templates, signers, q, want_ids: bool = True):
        tb, tm, sb, rq = make_tx_batch(t), make_templates(templates), make_signers(signers), make_req_batch(q)
        ids = np.zeros(max(tb.ntx, 1) * 32, dtype=np.uint8) if want_ids else None
        status = np.zeros(max(sb.n, 1), dtype=np.uint8)
        verdict = np.zeros(max(rq.ntx, 1), dtype=np.uint8)
        arg = np.zeros(max(rq.ntx, 1), dtype=np.uint32)
        missing = np.zeros(max(rq.nreq, 1), dtype=np.uint8)
        self._check(self.lib.chip_group_verify_signed_tx_batch(self.h, ctypes.byref(tb), ctypes.byref(tm),
                                                               ctypes.byref(sb), ctypes.byref(rq), _ptr(ids),
                                                               _ptr(status), _ptr(verdict), _ptr(arg), _ptr(missing)))
        return ((ids[:32 * tb.ntx].reshape(tb.ntx, 32) if want_ids else None), status[:sb.n], verdict[:rq.ntx],
                arg[:rq.ntx], missing[:rq.nreq])

    def stx_verify(self, data, off, lens, templates, meta, want_ids: bool = False):
        n = len(off)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        meta = np.ascontiguousarray(np.asarray(meta, dtype=np.int32).reshape(-1, 2))
        tm = make_templates(templates)
        st = np.zeros(max(n, 1), dtype=np.uint8)
        v = np.zeros(max(n, 1), dtype=np.uint8)
        a = np.zeros(max(n, 1), dtype=np.uint32)
        ids = np.zeros(max(n, 1) * 32, dtype=np.uint8) if want_ids else None
        self._check(self.lib.chip_group_stx_verify(self.h, n, _ptr(data), _ptr(off), _ptr(lens), len(data),
                                                   ctypes.byref(tm), meta.ctypes.data, len(meta), _ptr(st), _ptr(v),
                                                   _ptr(a), _ptr(ids)))
        return st[:n], v[:n], a[:n], (ids[:32 * n].reshape(n, 32) if want_ids else None)

    def ftx_verify_batch(self, f):
        s = make_ftx_batch(f)
        status = np.zeros(max(s.ntx, 1), dtype=np.uint8)
        reason = np.zeros(max(s.ntx, 1), dtype=np.uint8)
        self._check(self.lib.chip_group_ftx_verify_batch(self.h, ctypes.byref(s), _ptr(status), _ptr(reason)))
        return status[:s.ntx], reason[:s.ntx]

    def last_stats(self) -> dict:
        """chip_group_last_stats: the last group call's split and host timings."""
        st = ChipGroupStats()
        self._check(self.lib.chip_group_last_stats(self.h, ctypes.byref(st)))
        return st.as_dict()

    def uniq_open(self, capacity: int):
        return GroupUniqTable(self, capacity)


class GroupUniqTable:
    """The notary table of a device group: member m holds the StateRefs with state_owner(ref, n) == m."""

    def __init__(self, group: Group, capacity: int):
        self.group = group
        self.lib = group.lib
        h = ctypes.c_void_p()
        group._check(self.lib.chip_group_uniq_open(group.h, ctypes.c_uint64(capacity), ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.chip_group_uniq_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self) -> int:
        return int(self.lib.chip_group_uniq_size(self.h))

    def _check(self, rc):
        if rc != 0:
            raise ChipError(rc, self.lib.chip_group_uniq_last_error(self.h).decode(errors="replace"))

    def rebuild(self, refs36, tx32, idx, caller):
        self._check(self.lib.chip_group_uniq_rebuild(self.h, ctypes.c_uint64(len(idx)), _ptr(refs36), _ptr(tx32),
                                                     _ptr(idx), _ptr(caller)))

    def last_stats(self) -> dict:
        """chip_group_uniq_last_stats: the last commit's ingest / exchange / rounds split."""
        st = ChipGroupStats()
        self._check(self.lib.chip_group_uniq_last_stats(self.h, ctypes.byref(st)))
        return st.as_dict()

    def commit_batch_raw(self, tx_ref_start, refs36, tx_ids, callers, cap=None):
        """The commit with the records left as raw chip_conflict bytes (56 B each): (statuses, bytes, count)."""
        ntx = len(tx_ref_start) - 1
        st = np.zeros(max(ntx, 1), dtype=np.uint8)
        if cap is None:
            cap = int(tx_ref_start[-1]) + 1
        out = np.zeros(max(cap, 1) * ctypes.sizeof(ChipConflict), dtype=np.uint8)
        nout = ctypes.c_uint64()
        self._check(self.lib.chip_group_uniq_commit_batch(self.h, ctypes.c_uint64(ntx), _ptr(tx_ref_start),
                                                          _ptr(refs36), _ptr(tx_ids), _ptr(callers), _ptr(st),
                                                          out.ctypes.data, ctypes.c_uint64(cap), ctypes.byref(nout)))
        n = int(nout.value)
        return st[:ntx], out[:min(n, cap) * ctypes.sizeof(ChipConflict)], n

    def commit_batch(self, tx_ref_start, refs36, tx_ids, callers, cap=None):
        ntx = len(tx_ref_start) - 1
        st = np.zeros(max(ntx, 1), dtype=np.uint8)
        if cap is None:
            cap = int(tx_ref_start[-1]) + 1
        out = (ChipConflict * max(cap, 1))()
        nout = ctypes.c_uint64()
        self._check(self.lib.chip_group_uniq_commit_batch(self.h, ctypes.c_uint64(ntx), _ptr(tx_ref_start),
                                                          _ptr(refs36), _ptr(tx_ids), _ptr(callers), _ptr(st), out,
                                                          ctypes.c_uint64(cap), ctypes.byref(nout)))
        recs = [(c.tx, c.input_index, c.consumed_index, bytes(c.consuming_tx), c.consuming_caller)
                for c in out[:min(nout.value, cap)]]
        return st[:ntx], recs
