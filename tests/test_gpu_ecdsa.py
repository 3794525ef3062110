"""GPU parity: ECDSA secp256r1 / secp256k1 verification (K2) vs the oracle and the committed
golden vectors (BC 1.57 DER rules, range checks, high-s, r + n branch, exceptional points)."""
import numpy as np
import pytest

import cordagen as G
import golden_cases

pytestmark = pytest.mark.gpu


MODES = ["default", "comb", "straus", "ungated", "ec_retry"]


@pytest.mark.parametrize("mode", MODES)
def test_ecdsa_golden(ctx_modes, oracle, mode):
    """Every schedule (per-key comb tables / windowed) gives the golden statuses, incl. the
    exceptional-point and r + n cases."""
    ctx = ctx_modes[mode]
    b = golden_cases.ecdsa_edge_batch()
    st, _ = ctx.verify_batch(b)
    labels = [c["label"] for c in golden_cases.ecdsa_cases()]
    bad = [(labels[i], int(st[i]), int(b.expected[i])) for i in range(len(st)) if st[i] != b.expected[i]]
    assert not bad, bad
    assert np.array_equal(st, oracle.verify_batch(b))


@pytest.mark.parametrize("mode", MODES)
def test_ecdsa_mixed_batch_matches_oracle(ctx_modes, oracle, mode):
    ctx = ctx_modes[mode]
    b = G.ecdsa_batch(4000, n_keys=64, corrupt=0.4, seed=17)
    st, bm = ctx.verify_batch(b)
    ref = oracle.verify_batch(b, threads=8)
    bad = np.nonzero(st != ref)[0]
    assert len(bad) == 0, [(int(i), int(b.kind[i]), int(b.scheme[i]), int(st[i]), int(ref[i])) for i in bad[:20]]
    assert np.array_equal(st, b.expected)


def test_mixed_ed25519_and_ecdsa_one_batch(ctx, oracle):
    e = golden_cases.ed25519_cases()
    c = golden_cases.ecdsa_cases()
    b = golden_cases.sig_batch_from_cases(e + c)
    st, _ = ctx.verify_batch(b)
    assert np.array_equal(st, b.expected)
    assert np.array_equal(st, oracle.verify_batch(b))


def test_ecdsa_comb_stats_and_large_batch(ctx_modes):
    """Default policy without the batch-size gate: a batch with many signatures per key takes the
    per-key comb kernels (table build observable in the stats); 60k signatures, every corruption
    class, labels reproduced."""
    from corda_amd import native
    c = ctx_modes["ungated"]
    c.reset_stats()
    b = G.ecdsa_batch(60000, n_keys=256, corrupt=0.1, seed=23)
    st, _ = c.verify_batch(b)
    assert np.array_equal(st, b.expected)
    s = c.stats()
    assert s.kernel_launches[native.K_EC_TABLES] >= 1


def test_ecdsa_comb_without_glv_subprocess():
    """The round-5 secp256k1 schedule (CHIP_EC_GLV=0: the 65-window radix-16 table, a process-wide switch) still
    gives the labels' status bytes: a child process verifies a comb-forced r1/k1 batch with the switch off, the
    in-process contexts covering the GLV default."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "import numpy as np, corda_amd, cordagen as G\n"
            "from corda_amd import native\n"
            "c = corda_amd.Context(0, flags=native.FLAG_FORCE_COMB)\n"
            "b = G.ecdsa_batch(3000, n_keys=24, corrupt=0.3, seed=0x5EED0619)\n"
            "st, _ = c.verify_batch(b)\n"
            "c.close()\n"
            "sys.exit(0 if np.array_equal(st, b.expected) else 3)\n") % (root, os.path.join(root, "tools"))
    env = dict(os.environ, CHIP_EC_GLV="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
