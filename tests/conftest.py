import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


@pytest.fixture(scope="session")
def ctx():
    """One libcordahip context on cuda:0 for the whole GPU session."""
    import corda_amd
    c = corda_amd.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="session")
def oracle():
    import oracle_bind
    oracle_bind.lib()
    return oracle_bind


@pytest.fixture(scope="session")
def ctx_modes():
    """Contexts for each Ed25519 schedule: default policy, every key on the per-key comb, every key
    on the windowed Straus kernel, and the default policy with the batch-size gate of the comb paths
    off (CHIP_COMB_MIN_TOTAL=0: test-sized batches then take the eager-table schedules the bench
    sizes take).  Results must be identical (bit-exact status bytes)."""
    import corda_amd
    from corda_amd import native
    os.environ["CHIP_COMB_MIN_TOTAL"] = "0"
    try:
        ungated = corda_amd.Context(0)
    finally:
        del os.environ["CHIP_COMB_MIN_TOTAL"]
    cs = {"default": corda_amd.Context(0), "comb": corda_amd.Context(0, flags=native.FLAG_FORCE_COMB),
          "straus": corda_amd.Context(0, flags=native.FLAG_NO_COMB), "ungated": ungated,
          # every ECDSA comb lane finished by the exceptional-addition retry kernel (k_ecdsa_comb_retry)
          "ec_retry": corda_amd.Context(0, flags=native.FLAG_FORCE_COMB | native.FLAG_EC_RETRY_ALL)}
    yield cs
    for c in cs.values():
        c.close()
