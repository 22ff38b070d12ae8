set -o pipefail
timeout -k 10 60 ./tools/permlane_probe > gpurun_out/r04_permlane_probe.txt 2>&1 || exit 1
cat gpurun_out/r04_permlane_probe.txt
export SGV_AB=1
for rep in 1 2; do
  for v in "SGV_MF_PAIR=0" "SGV_MF_PAIR=1 SGV_MF_PAIR_MAP=0" "SGV_MF_PAIR=1 SGV_MF_PAIR_MAP=1"; do
    env $v timeout -k 10 300 python -u tools/ldpass_ab.py --tag "$v" --shapes 64x15625,8x15625,8x25000 --ncols 4,8 >> gpurun_out/r04_pairmap_ab.jsonl 2>> gpurun_out/r04_pairmap_ab.err || exit 1
  done
done
cat gpurun_out/r04_pairmap_ab.jsonl
unset SGV_AB
timeout -k 10 700 bash tools/gpu_r04_band.sh gpurun_out/r04_band
