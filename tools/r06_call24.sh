set -o pipefail
cd $GRAFT_REPO_ROOT
export SGV_AB=1
for rep in 1 2 3; do
  for v in 0 1; do
    SGV_MF_PAIR=$v timeout -k 10 300 python -u tools/ldpass_ab.py --tag "SGV_MF_PAIR=$v" --shapes 2x25000,4x25000,8x15625,12x15625 --ncols 8 >> gpurun_out/pairsz_ab.jsonl 2>> gpurun_out/pairsz_ab.err || exit 1
  done
done
python3 tools/ab_table.py gpurun_out/pairsz_ab.jsonl
