set -o pipefail
cd $GRAFT_REPO_ROOT
export SGV_AB=1
for rep in 1 2; do
  for v in 0 1 2 3; do
    SGV_MF_ABL=$v timeout -k 10 300 python -u tools/ldpass_ab.py --tag "ABL=$v" --shapes 64x15625,16x15625 --ncols 4,8 >> gpurun_out/abl_ab.jsonl 2>> gpurun_out/abl_ab.err || exit 1
  done
done
python3 tools/ab_table.py gpurun_out/abl_ab.jsonl
