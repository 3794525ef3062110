"""Parity pin for the ECDSA oracle on the reference's own BouncyCastle-made signatures.

tests/golden/ref_x509_ecdsa.json holds every distinct SHA256withECDSA X.509 chain link of the JKS /
PEM certificate stores the reference ships (golden/make_x509_fixture.py; signed by BC through
X509Utilities, node/src/main/kotlin/net/corda/node/utilities/X509Utilities.kt:44,278).  They are
reference-produced expected outputs: Crypto.doVerify(issuerKey, sig, tbs) is true for each.
"""
import numpy as np

import cordagen as G
import golden_cases


def _batch_and_labels(oracle):
    cases = golden_cases.ref_x509_cases(corrupt=True)
    b = golden_cases.sig_batch_from_cases([dict(c, expected=c["expected"] or 0) for c in cases])
    st = oracle.verify_batch(b)
    return cases, b, st


def test_fixture_covers_both_curves_and_der_lengths():
    recs = golden_cases.ref_x509_records()
    assert len(recs) >= 6
    assert {r["curve"] for r in recs} == {"secp256r1", "secp256k1"}
    assert {len(r["sig_der"]) // 2 for r in recs} >= {70, 71, 72}


def test_oracle_accepts_every_reference_signature(oracle):
    cases = golden_cases.ref_x509_cases(corrupt=False)
    b = golden_cases.sig_batch_from_cases(cases)
    st = oracle.verify_batch(b)
    assert st.tolist() == [0] * len(cases), [(c["label"], int(s)) for c, s in zip(cases, st)]


def test_oracle_rejects_every_corruption_and_agrees_with_openssl(oracle):
    cases, b, st = _batch_and_labels(oracle)
    n0 = len(golden_cases.ref_x509_records())
    assert (st[:n0] == 0).all()
    bad = [(c["label"], int(s)) for c, s in zip(cases[n0:], st[n0:]) if s not in (1, 2)]
    assert not bad, bad[:20]
    # OpenSSL's verdict (valid or not) agrees with the oracle's on every case: its DER rules match
    # BC's strict decoder for all of these single-byte changes
    for c, s in zip(cases, st):
        ok = G.ossl_verify(bytes.fromhex(c["spki"]), bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"])) == 1
        assert ok == (s == 0), (c["label"], int(s))
