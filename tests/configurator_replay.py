"""Replays tests/golden/configurator_scenarios.json (the reference's
configurator_test.go, 10 tests, 115 TestTraffic expectations) through the
configurator restatement (vpp_amd/configurator.py) into any renderer factory.

The fixture holds only inputs and expected outputs; the generator is
tests/golden/make_configurator_scenarios.py.
"""
import json
import os

from vpp_amd import gonet
from vpp_amd import configurator as C
from vpp_amd.renderer import traffic as T
from vpp_amd.renderer.api import TCP, UDP, PodID

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configurator_scenarios.json")

_ENUM = {"INGRESS": 0, "EGRESS": 1, "ALL": 2}
_PROTO = {"TCP": C.TCP, "UDP": C.UDP}
DIRECTION = {"INGRESS": T.INGRESS_TRAFFIC, "EGRESS": T.EGRESS_TRAFFIC}
ACTION = {"ALLOWED": T.ALLOWED_TRAFFIC, "DENIED": T.DENIED_TRAFFIC, "UNMATCHED": T.UNMATCHED_TRAFFIC}
RULE_PROTO = {"TCP": TCP, "UDP": UDP}


def load():
    with open(FIXTURE) as f:
        return json.load(f)


def _net(s):
    _, n = gonet.parse_cidr(s)
    assert n is not None, s
    return n


def policy(p):
    matches = []
    for m in p["matches"]:
        matches.append(C.Match(
            _ENUM[m["type"]],
            pods=None if m["pods"] is None else [PodID(*x) for x in m["pods"]],
            ip_blocks=None if m["ip_blocks"] is None else
            [C.IPBlock(_net(b["network"]), [_net(e) for e in b["except"]]) for b in m["ip_blocks"]],
            ports=None if m["ports"] is None else [C.Port(_PROTO[pr], n) for pr, n in m["ports"]]))
    return C.ContivPolicy(C.PolicyID(p["name"], p["namespace"]), _ENUM[p["type"]], matches)


def replay(scn, make_renderer):
    """Runs the scenario's steps; returns (renderers, [(step, got)]) where got
    is the TrafficAction or the (ip, masklen) GetPodIP result."""
    cache = {}
    renderers = {}
    conf = txn = None
    policies = {name: policy(p) for name, p in scn["policies"].items()}
    checks = []
    for st in scn["steps"]:
        op = st["op"]
        if op == "cache":
            cache[PodID(*st["pod"])] = st["ip"]
        elif op == "renderer":
            renderers[st["var"]] = make_renderer(st["name"])
        elif op == "init":
            conf = C.PolicyConfigurator(cache, parallel_rendering=st["flag"])
        elif op == "register":
            conf.register_renderer(renderers[st["renderer"]])
        elif op == "new_txn":
            txn = conf.new_txn(st["flag"])
        elif op == "configure":
            txn.configure(PodID(*st["pod"]), [policies[n] for n in st["policies"]])
        elif op == "commit":
            txn.commit()
        elif op == "pod_ip":
            checks.append((st, renderers[st["renderer"]].get_pod_ip(PodID(*st["pod"]))))
        elif op == "traffic":
            got = renderers[st["renderer"]].test_traffic(
                PodID(*st["pod"]), DIRECTION[st["dir"]], gonet.parse_ip(st["src"]), gonet.parse_ip(st["dst"]),
                RULE_PROTO[st["proto"]], st["sport"], st["dport"])
            checks.append((st, got))
        else:
            raise ValueError(op)
    return renderers, checks


def mismatches(checks):
    bad = []
    for st, got in checks:
        want = ACTION[st["expect"]] if st["op"] == "traffic" else (st["ip"], st["masklen"])
        if got != want:
            bad.append((st["line"], st, got))
    return bad


def random_policy_set(rng, n_pods=60, n_policies=25):
    """A synthetic namespace: pods with IPv4 (and some IPv6) addresses, and
    policies mixing pod peers, IP blocks with nested excepts, ports and the
    nil-peer "match anything" forms.  Returns (cache, {pod: [policies]})."""
    pods = [PodID("pod%d" % i, "ns%d" % (i % 3)) for i in range(n_pods)]
    cache = {}
    for i, p in enumerate(pods):
        if i % 11 == 10:
            continue                                  # pod without an address
        cache[p] = ("10.%d.%d.%d" % (i % 4, i // 200, 1 + i % 200) if i % 7
                    else "fd00::%x" % (i + 1))
    pols = []
    for k in range(n_policies):
        matches = []
        for _ in range(rng.randrange(1, 4)):
            mtype = rng.randrange(2)
            kind = rng.random()
            ports = None if rng.random() < 0.4 else [
                C.Port(rng.randrange(2), rng.choice([0, 22, 53, 80, 443, 8080, rng.randrange(1, 65536)]))
                for _ in range(rng.randrange(1, 4))]
            if kind < 0.15:
                matches.append(C.Match(mtype, ports=ports))
                continue
            peers = None if kind < 0.4 else rng.sample(pods, rng.randrange(0, 6))
            blocks = None
            if kind < 0.7:
                a, b = rng.randrange(4), rng.randrange(256)
                net = _net("10.%d.%d.0/%d" % (a, b, rng.choice([16, 20, 24])))
                excepts = [_net("10.%d.%d.%d/%d" % (a, b, rng.randrange(256), rng.choice([26, 28, 30, 32])))
                           for _ in range(rng.randrange(0, 3))]
                blocks = [C.IPBlock(net, excepts)]
            matches.append(C.Match(mtype, pods=peers, ip_blocks=blocks, ports=ports))
        pols.append(C.ContivPolicy(C.PolicyID("pol%d" % k, "ns%d" % (k % 3)), rng.randrange(3), matches))
    assign = {p: rng.sample(pols, rng.randrange(0, 4)) for p in pods}
    return cache, assign


def random_packets(rng, cache, n):
    """Packets between pod addresses and addresses near the policy blocks."""
    addrs = [gonet.parse_ip(ip) for ip in cache.values()]
    src, dst, proto, sport, dport = [], [], [], [], []
    for _ in range(n):
        for out in (src, dst):
            r = rng.random()
            if r < 0.5:
                out.append(rng.choice(addrs))
            else:
                out.append(bytes([10, rng.randrange(4), rng.randrange(256), rng.randrange(256)]))
        proto.append(rng.choice([TCP, UDP]))
        sport.append(rng.randrange(65536))
        dport.append(rng.choice([22, 53, 80, 443, 8080, rng.randrange(65536)]))
    return src, dst, proto, sport, dport


def gen_policy_packets(rng, n, n_blocks=1000):
    """Packets around gen-policy.py's address space: sources and destinations
    inside the block prefixes (i + 256) << 16 (block-, except- and gap-heavy),
    ports mostly from a small set so some hit the policy's ports; protocols
    TCP, UDP, ICMP and 47."""
    import numpy as np
    src = []
    dst = []
    for _ in range(n):
        for out in (src, dst):
            i = rng.randrange(n_blocks + n_blocks // 10 + 1)
            out.append((((i + 0x100) << 16) | rng.randrange(1 << 16)).to_bytes(4, "big"))
    # TCP and UDP mostly, some ICMP and a protocol outside ProtocolType (47):
    # TestTraffic's exact protocol test, evalACL's switch fall-through
    proto = [rng.choice((0, 0, 0, 1, 1, 1, 2, 47)) for _ in range(n)]
    dport = [rng.randrange(65536) for _ in range(n)]
    rows = lambda ips: np.frombuffer(b"".join(gonet.V4_IN_V6_PREFIX + x for x in ips), np.uint8).reshape(-1, 16)
    return src, dst, proto, dport, rows(src), rows(dst)
