"""ORACLE -- test infrastructure only (see aclengine_ref.c header).

Literal restatement of MockRenderer.TestTraffic
(mock/renderer/renderer_mock.go:105-145): first match over a raw ContivRule
list, pure Python loops, for small cases.  Addresses are Go net.IP byte
strings (4 or 16 bytes); ``IPNet.contains`` is the Go 1.9 restatement in
vpp_amd/gonet.py (the data model, not the evaluator under test).

Pinning: the reference's own TestTraffic expectations (configurator_test.go,
10 tests, 115 verdicts) are replayed through the configurator restatement
(vpp_amd/configurator.py) into this evaluator from
tests/golden/configurator_scenarios.json (tests/test_configurator_cpu.py).
It is also cross-checked against the evalACL oracle: on rule lists both can
express (SrcPort 0, TCP/UDP rules) renderACL + evalACL and TestTraffic must
agree on every packet, with evalACL's default DENY standing for UNMATCHED
(tests/test_traffic_cpu.py).
"""
from __future__ import annotations

DENIED, ALLOWED, UNMATCHED = 0, 1, 2      # TrafficAction (renderer_mock.go:25-37)
ACTION_PERMIT = 1                         # renderer.ActionPermit (api.go:139-147)


def test_traffic(rules, src_ip: bytes, dst_ip: bytes, protocol: int, src_port: int, dst_port: int):
    """Returns (TrafficAction, index of the matching rule or -1)."""
    for i, rule in enumerate(rules):                                   # :122
        if len(rule.src_network.ip) > 0 and not rule.src_network.contains(src_ip):   # :123
            continue
        if len(rule.dest_network.ip) > 0 and not rule.dest_network.contains(dst_ip):  # :126
            continue
        if rule.protocol != protocol:                                  # :129
            continue
        if rule.src_port != 0 and rule.src_port != src_port:          # :132
            continue
        if rule.dest_port != 0 and rule.dest_port != dst_port:        # :135
            continue
        if rule.action == ACTION_PERMIT:                               # :139
            return ALLOWED, i
        return DENIED, i
    return UNMATCHED, -1                                               # :144


def test_traffic_batch(rules, src, dst, proto, sport, dport):
    """Batch form: src/dst are sequences of net.IP byte strings.  Returns
    (TrafficAction list, per-rule hit counts, unmatched count)."""
    verdict = []
    counts = [0] * len(rules)
    unmatched = 0
    for s, d, p, sp, dp in zip(src, dst, proto, sport, dport):
        a, i = test_traffic(rules, s, d, int(p), int(sp), int(dp))
        verdict.append(a)
        if i < 0:
            unmatched += 1
        else:
            counts[i] += 1
    return verdict, counts, unmatched
