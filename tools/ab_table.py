#!/usr/bin/env python3
"""Table of an A/B jsonl (tools/ldpass_ab.py lines): ms per pass by (shape, ncol, tag),
and whether every tag produced the same products (SHA-256) for a shape.
  python tools/ab_table.py gpurun_out/x_ab.jsonl"""
import collections
import json
import sys

d = collections.defaultdict(list)
sha = collections.defaultdict(set)
for line in open(sys.argv[1]):
    r = json.loads(line)
    r.setdefault("shape", "M=%s,bw=%s" % (r.get("M"), r.get("bw")))   # ldpass_band.py lines
    d[(r["shape"], r["ncol"], r["tag"])].append(r["ms_per_pass"])
    sha[(r["shape"], r["ncol"])].add(r["sha"])
for k in sorted(d):
    print("%-10s nc=%-3d %-28s %s" % (k[0], k[1], k[2], " ".join("%.4f" % v for v in d[k])))
print("products bitwise equal across tags:", all(len(v) == 1 for v in sha.values()))
