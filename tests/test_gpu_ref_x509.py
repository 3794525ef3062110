"""GPU parity on the reference's own BouncyCastle SHA256withECDSA signatures (X.509 chain links of
the JKS stores it ships; tests/golden/ref_x509_ecdsa.json, see test_ref_x509_cpu.py).  Every link is
VALID through chip_verify_batch, and every single-byte corruption / tbs flip / foreign issuer key gives
the oracle's non-VALID status, on every ECDSA schedule."""
import numpy as np
import pytest

import golden_cases

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["default", "comb", "straus", "ungated", "ec_retry"])
def test_reference_x509_links_on_gpu(ctx_modes, oracle, mode):
    cases = golden_cases.ref_x509_cases(corrupt=True)
    b = golden_cases.sig_batch_from_cases([dict(c, expected=c["expected"] or 0) for c in cases])
    st, bm = ctx_modes[mode].verify_batch(b)
    ref = oracle.verify_batch(b)
    n0 = len(golden_cases.ref_x509_records())
    assert st[:n0].tolist() == [0] * n0, [(c["label"], int(s)) for c, s in zip(cases[:n0], st[:n0])]
    assert set(np.unique(st[n0:]).tolist()) <= {1, 2}
    bad = np.nonzero(st != ref)[0]
    assert len(bad) == 0, [(cases[i]["label"], int(st[i]), int(ref[i])) for i in bad[:20]]
    valid = np.array([(int(bm[i >> 6]) >> (i & 63)) & 1 for i in range(len(st))])
    assert np.array_equal(valid, (st == 0).astype(valid.dtype))


def test_reference_x509_links_repeated_on_comb_path(ctx_modes, oracle):
    """The six links repeated 64x (hot keys -> per-key comb tables by the default policy with the
    batch-size gate off)."""
    cases = golden_cases.ref_x509_cases(corrupt=False) * 64
    b = golden_cases.sig_batch_from_cases(cases)
    st, _ = ctx_modes["ungated"].verify_batch(b)
    assert (st == 0).all()
