"""Notary commit log (write + rebuild at open) on the CPU oracle engine."""
from commit_log_case import run
from oracle_engine import OracleEngine


def test_commit_log_restart_equals_live_provider(tmp_path):
    assert run(OracleEngine(), tmp_path) > 0


def test_commit_log_failure_is_fail_stop(tmp_path):
    from commit_log_case import run_fail_stop
    assert run_fail_stop(OracleEngine(), tmp_path) > 0
