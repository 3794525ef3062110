"""corda_amd — MI355X-native batch verification engine for Corda's signature / tx-id /
notary-uniqueness hot path.

Layers:
  include/cordahip.h        C-ABI (the drop-in boundary; see INTEGRATION.md for the JNI binding)
  corda_amd/csrc/*.hip      HIP kernels for gfx950 + the C-ABI runtime (libcordahip.so)
  corda_amd/native.py       ctypes binding of the C-ABI
  corda_amd/crypto.py       host mirror of the reference API (Crypto.doVerify, TransactionSignature,
                            SignedTransaction.verifySignaturesExcept, WireTransaction.id,
                            PersistentUniquenessProvider.commit) with the reference's exceptions
"""
from .native import (Context, ChipError, NativeUnavailable, STATUS_NAMES, VALID, INVALID, SIG_DECODE, EMPTY_SIG,
                     EMPTY_CLEAR, UNSUPPORTED, KEY_INVALID, SCHEME_K1, SCHEME_R1, SCHEME_ED25519, load)

__all__ = ["Context", "ChipError", "NativeUnavailable", "STATUS_NAMES", "VALID", "INVALID", "SIG_DECODE",
           "EMPTY_SIG", "EMPTY_CLEAR", "UNSUPPORTED", "KEY_INVALID", "SCHEME_K1", "SCHEME_R1", "SCHEME_ED25519",
           "load"]
