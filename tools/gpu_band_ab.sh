set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "SGV_X=0" "SGV_MF_SKIP=0" "SGV_PK16=1" "SGV_FIN_LPT=0"; do
    echo "== $v" >> gpurun_out/band_ab.log
    env SGV_AB=1 $v timeout -k 10 200 python -u tools/ldpass_band.py --M 1000000 --bw 1000 --ncols 8,16 --reps 10 2>/dev/null | grep ncol >> gpurun_out/band_ab.log || exit 1
  done
done
cat gpurun_out/band_ab.log | cut -c1-120
