"""Writes tests/golden/rule_list_hashes.json: the digest of the rendered ACL of
benchmark configs 2, 3 and 5, each rendered in a fresh interpreter (so that no
earlier render in the same process can influence it).

Run from the repository root: python tests/golden/make_rule_hashes.py
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r"""
import sys
sys.path[:0] = [%r, %r]
from vpp_amd import workload
from rule_hash import rule_list_digest
acl, _, _ = workload.config(int(sys.argv[1]))
print(len(acl.rules), rule_list_digest(acl.rules))
""" % (ROOT, os.path.join(ROOT, "tests"))


def main():
    out = {}
    for cfg in (2, 3, 5):
        n, d = subprocess.run([sys.executable, "-c", CHILD, str(cfg)], check=True, capture_output=True,
                              text=True).stdout.split()
        out[str(cfg)] = {"n_rules": int(n), "sha256": d}
    with open(os.path.join(ROOT, "tests", "golden", "rule_list_hashes.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(out)


if __name__ == "__main__":
    main()
