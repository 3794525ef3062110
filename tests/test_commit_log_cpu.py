"""Notary commit log (write + rebuild at open) on the CPU oracle engine."""
from commit_log_case import run
from oracle_engine import OracleEngine


def test_commit_log_restart_equals_live_provider(tmp_path):
    assert run(OracleEngine(), tmp_path) > 0
