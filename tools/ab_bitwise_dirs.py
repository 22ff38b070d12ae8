#!/usr/bin/env python3
"""Compare the output files (.bin, .csv) of two run directories byte for byte.
  python tools/ab_bitwise_dirs.py DIR_A DIR_B   (exit 1 on any difference)"""
import os
import sys

a, b = sys.argv[1], sys.argv[2]
fa = sorted(f for f in os.listdir(a) if f.endswith((".bin", ".csv")))
fb = sorted(f for f in os.listdir(b) if f.endswith((".bin", ".csv")))
if fa != fb or not fa:
    sys.exit("file sets differ: %s vs %s" % (fa[:5], fb[:5]))
diff = [f for f in fa if open(os.path.join(a, f), "rb").read() != open(os.path.join(b, f), "rb").read()]
print("%d files, %d differ%s" % (len(fa), len(diff), (": " + ", ".join(diff[:8])) if diff else ""))
sys.exit(1 if diff else 0)
