"""Pin the CPU oracle against the reference's 221 Connection* known answers.

The scenarios of plugins/policy/renderer/acl/acl_renderer_test.go:166-961 are
replayed through the renderer restatement (vpp_amd.renderer) into the oracle
engine (oracle.OracleACLEngine -> C evalACL/testConnection).  Every
expectation of the reference test must hold.
"""
import pytest

import oracle
from scenario_replay import load_scenarios, replay

SCENARIOS = load_scenarios()


def test_fixture_has_all_kats():
    n = sum(1 for t in SCENARIOS for s in t["steps"] if s["op"] == "expect_conn")
    assert len(SCENARIOS) == 7
    assert n == 221


@pytest.mark.parametrize("test", SCENARIOS, ids=[t["name"] for t in SCENARIOS])
def test_oracle_matches_reference_scenario(test):
    checked, failures = replay(test, oracle.OracleACLEngine)
    assert not failures, "\n".join(failures)
    assert checked > 0
