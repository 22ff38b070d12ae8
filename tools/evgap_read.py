"""Mean gap before each kernel of tools/evgap.hip's four patterns (trace CSV)."""
import csv
import sys
from collections import defaultdict

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(sys.argv[1])))
gaps, durs = defaultdict(list), defaultdict(list)
for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
    if n0 == n1 and "k_tick" in n1:
        gaps[n1].append((s1 - e0) / 1e3)
        durs[n1].append((e1 - s1) / 1e3)
for k in sorted(gaps):
    g = sorted(gaps[k])
    print(f"{k[:40]:40s} n={len(g)} gap median {g[len(g)//2]:.2f} us mean {sum(g)/len(g):.2f} us, "
          f"dur {sum(durs[k])/len(durs[k]):.2f} us")
