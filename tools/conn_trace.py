"""Per-batch kernel durations and host gaps of a conn_bench rocprofv3 trace:
the last batches of each kind (uncounted: pair + connect; counted: pair +
connect + rows).  usage: python3 tools/conn_trace.py run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    n = n.replace("(anonymous namespace)::", "").split("(")[0]
    return n.split("::")[-1][:40]


prev = None
out = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    out.append((short(r["Kernel_Name"]), (e - s) / 1000, (s - prev) / 1000 if prev else 0.0))
    prev = e
# batches: a pair launch starts one
batches = []
for k, (n, d, g) in enumerate(out):
    if n.startswith("classify4_pair"):
        b = [(n, d, g)]
        for m in out[k + 1:]:
            if m[0].startswith("classify4_pair") or m[2] > 20:
                break
            b.append(m)
        batches.append(b)
kinds = {}
for b in batches:
    key = tuple(x[0] for x in b)
    kinds.setdefault(key, []).append(b)
for key, bs in kinds.items():
    last = bs[-5:]
    print(" + ".join(key), "(%d batches)" % len(bs))
    for b in last:
        print("   gap before %.1f us | " % b[0][2] + " | ".join("%.1f" % x[1] for x in b),
              "| GPU %.1f us" % sum(x[1] for x in b))
