"""cfg1 (BASELINE.json configs[0]): finance Cash issue / move SignedTransactions,
Ed25519, checked with verifySignaturesExcept(notary).  Shapes follow Cash.kt:184-197,
CashIssueFlow.kt:37-49 and CashPaymentFlow.kt:40-69: an issue has {outputs, commands, notary} and
one signature by the issuer; a move has {inputs (1-2), outputs (2), commands, notary}, the owners'
signatures, and the notary's signature still missing (allowed).  Keys are the reference's
deterministic test keys entropyToKeyPair(20..100) (TestConstants.kt:27-72).  Labels record what the
reference's sequential verifySignaturesExcept would raise."""
import numpy as np

import cordagen as G
from corda_amd import crypto as C


def entropy_seed(v: int) -> bytes:
    b = v.to_bytes((v.bit_length() + 8) // 8, "big", signed=True)
    return (b + bytes(32))[:32]


PARTY_ENTROPY = [20, 30, 40, 50, 60, 70, 80, 90, 100]   # DUMMY_NOTARY .. (TestConstants.kt:30-72)


def cash_workload(n_tx: int = 10_000, seed: int = 0xC0DA, corrupt: float = 0.01, missing: float = 0.01):
    rng = np.random.Generator(np.random.PCG64(seed))
    seeds = [entropy_seed(v) for v in PARTY_ENTROPY]
    keys = [G.spki_ed25519(G.ed25519_pub(s)) for s in seeds]
    notary = keys[0]
    parties = list(range(1, len(keys)))
    wtxs, plans = [], []
    for t in range(n_tx):
        salt = bytes(rng.integers(0, 256, size=32, dtype=np.uint8))
        salt = bytes([salt[0] | 1]) + salt[1:]
        notary_comp = b"party:" + notary
        if t % 2 == 0:   # issue
            issuer = int(rng.choice(parties))
            groups = [(C.OUTPUTS_GROUP, [rng.bytes(int(rng.integers(200, 700)))]),
                      (C.COMMANDS_GROUP, [b"Issue" + keys[issuer]]),
                      (C.NOTARY_GROUP, [notary_comp])]
            signers = [issuer]
        else:            # move
            owners = [int(x) for x in rng.choice(parties, size=int(rng.integers(1, 3)), replace=False)]
            groups = [(C.INPUTS_GROUP, [rng.bytes(36) for _ in range(len(owners))]),
                      (C.OUTPUTS_GROUP, [rng.bytes(int(rng.integers(200, 700))) for _ in range(2)]),
                      (C.COMMANDS_GROUP, [b"Move" + b"".join(keys[o] for o in owners)]),
                      (C.NOTARY_GROUP, [notary_comp])]
            signers = owners
        wtxs.append(C.WireTransaction(groups, salt, [keys[s] for s in signers], notary))
        plans.append(signers)
    return seeds, keys, notary, wtxs, plans, rng, corrupt, missing


def sign_all(engine, seeds, keys, notary, wtxs, plans, rng, corrupt, missing):
    """Ids through `engine` (one batch), signatures with OpenSSL over SignableData(id, meta); then
    corruption (one flipped bit) and dropped signatures.  Returns (stxs, labels)."""
    ids = C.WireTransaction.ids(engine, wtxs)
    meta = C.SignatureMetadata(1, 4)
    stxs, labels = [], []
    for wtx, signers, tx_id in zip(wtxs, plans, ids):
        msg = C.signable_data_bytes(tx_id, meta)
        sigs = [C.TransactionSignature(G.ed25519_sign(seeds[s], msg), keys[s], meta) for s in signers]
        label = None
        u = rng.random()
        if u < corrupt:
            k = int(rng.integers(0, len(sigs)))
            b = bytearray(sigs[k].bytes)
            b[int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
            sigs[k] = C.TransactionSignature(bytes(b), sigs[k].by, meta)
            label = ("SignatureException", "Signature Verification failed!")
        elif u < corrupt + missing and len(sigs) > 1:
            dropped = sigs.pop(int(rng.integers(0, len(sigs))))
            label = ("SignaturesMissingException", {dropped.by})
        stxs.append(C.SignedTransaction(tx_id, sigs, wtx.required_signing_keys))
        labels.append(label)
    return stxs, labels


def outcome(exc):
    if exc is None:
        return None
    if isinstance(exc, C.SignaturesMissingException):
        return ("SignaturesMissingException", set(exc.missing))
    return (type(exc).__name__, str(exc))
