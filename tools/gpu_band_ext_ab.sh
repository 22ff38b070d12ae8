#!/bin/bash
# Band extent A/B (round 3): band and packed parity of the in-tree build, then
# the band passes and the north-star pass alternating the in-tree library and
# tools/diaglib/libsgvamp_prev.so (SHA-256 of the products per run).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q \
    -k "band or ld_matvec_vs_numpy or mfma_strips" --timeout 120 --timeout-method thread \
    > gpurun_out/bext_parity.log 2>&1 || { echo "parity FAILED"; tail -30 gpurun_out/bext_parity.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/bext_parity.log)"
NEW=sgvamp-py_amd/libsgvamp_hip.so; OLD=tools/diaglib/libsgvamp_prev.so
for rep in 1 2; do
  for l in $OLD $NEW; do
    for cfg in "1000000 1000" "200000 2000"; do
      set -- $cfg
      timeout -k 10 200 python -u tools/ldpass_band.py --lib $l --tag $(basename $l) --M $1 --bw $2 \
          --ncols 1,2,8,16 --reps 10 >> gpurun_out/bext_ab.jsonl 2>> gpurun_out/bext_ab.err || exit 1
    done
    timeout -k 10 300 python -u tools/ldpass_ab.py --lib $l --tag $(basename $l) \
        --shapes 64x15625,8x15625 --ncols 2,8,16 >> gpurun_out/bext_ns.jsonl 2>> gpurun_out/bext_ab.err || exit 1
  done
done
python3 - <<'PY'
import json
for f in ("gpurun_out/bext_ab.jsonl", "gpurun_out/bext_ns.jsonl"):
    for l in open(f):
        d = json.loads(l)
        print(d["tag"], d.get("M", d.get("shape")), d.get("bw", ""), d["ncol"],
              "%.4f ms" % d["ms_per_pass"], d["sha"])
PY
