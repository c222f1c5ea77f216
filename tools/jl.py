#!/usr/bin/env python3
"""Print selected fields of a JSON-lines file: tools/jl.py FILE field ..."""
import json
import sys

for line in open(sys.argv[1]):
    line = line.strip()
    if line.startswith("{"):
        d = json.loads(line)
        print(" ".join(str(d.get(k)) for k in sys.argv[2:]))
