#!/usr/bin/env python3
"""Print selected fields of a JSON-lines file: tools/jl.py FILE field ...
(a.b reads a nested field)."""
import json
import sys


def get(d, k):
    for part in k.split("."):
        d = d.get(part) if isinstance(d, dict) else None
    return d


for line in open(sys.argv[1]):
    line = line.strip()
    if line.startswith("{"):
        d = json.loads(line)
        print(" ".join("%s=%s" % (k, get(d, k)) for k in sys.argv[2:]))
