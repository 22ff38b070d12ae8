#!/bin/bash
# One driver for the GPU-box measurements (per-step limits: tools/gpu_steps.sh;
# logs and profiler output under gpurun_out/).  Run through gpurun:
#   /usr/local/graft/bin/gpurun -- 'bash tools/gpu_recipes.sh <recipe> <tag> [args]'
# Recipes:
#   suite   TAG [pytest paths]   the driver's GPU suite, smoke(), the default bench line
#   trace   TAG [bench args]     kernel trace + --stats of a bench workload (trace_pass_summary.py)
#   pmc     TAG [bench args]     FETCH_SIZE and WRITE_SIZE in separate --pmc passes (pmc_summary.py)
#   clock   TAG [bench args]     effective clock, MFMA busy, SQ stall mix per dispatch (clock_summary.py)
#   configs TAG                  one bench line per BASELINE.json configuration, the band line,
#                                the N = 8 share and the 8-rank rehearsal
#   ab      TAG VAR "v0 v1 .." SHAPES NCOLS [bench args]   an SGV_AB switch (gpu_ab_multi.sh)
#   stall   TAG [bench args]     VMEM latency (INST_LEVEL / INSTS), active-instruction mix, LDS and
#                                TA back-pressure counters, two --pmc passes (kernel_pmc_table.py)
#   walkpmc TAG                  band walks vs strips (SGV_BAND_WALK 8 / 0) at M = 1e6, bw = 1,000,
#                                4 and 8 columns: clock/stall, LDS and HBM-byte --pmc passes
#   gate50  TAG [K]              the north star's own 50-iteration gate (SGV_FULL_GATE=1)
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
recipe=$1; T=${2:-x}; shift 2
B="--steps 5 --warmup 2 --cpu-baseline off --read-bw 0"
case $recipe in
  suite)
    SEL=${*:-tests}
    exec_steps=("gputests_$T:${SUITE_LIMIT:-1000}:SGV_TEST_TIMES=gpurun_out/testtimes_$T.txt SGV_GATE_LOG=gpurun_out/gates_$T.log python -u -m pytest $SEL -m gpu -x -q -p no:cacheprovider --timeout 900 --timeout-method thread -rs --durations=40"
                "smoke_$T:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
                "bench_$T:300:python bench.py")
    [ -n "$NO_BENCH" ] && unset 'exec_steps[2]' 
    tools/gpu_steps.sh "${exec_steps[@]}" ;;
  trace)
    tools/gpu_steps.sh "trace_$T:400:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o bench --output-format csv -- python3 $R/bench.py $B $*" ;;
  pmc)
    tools/gpu_steps.sh \
      "pmc_fetch_$T:300:cd /tmp && timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$T -o pmc --output-format csv -- python3 $R/bench.py $B --no-files $*" \
      "pmc_write_$T:300:cd /tmp && timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$T -o pmc --output-format csv -- python3 $R/bench.py $B --no-files $*" ;;
  clock)
    P="GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
    tools/gpu_steps.sh "clock_$T:300:cd /tmp && timeout -s KILL 280 rocprofv3 --pmc $P -d $R/gpurun_out/clock_$T -o pmc --output-format csv -- python3 $R/bench.py $B --no-files $*" ;;
  stall)
    P1="GRBM_GUI_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
    P2="GRBM_GUI_ACTIVE GRBM_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES"
    tools/gpu_steps.sh \
      "stall1_$T:120:cd /tmp && timeout -s KILL 100 rocprofv3 --pmc $P1 -d $R/gpurun_out/stall1_$T -o pmc --output-format csv -- python3 $R/bench.py $B --no-files $*" \
      "stall2_$T:120:cd /tmp && timeout -s KILL 100 rocprofv3 --pmc $P2 -d $R/gpurun_out/stall2_$T -o pmc --output-format csv -- python3 $R/bench.py $B --no-files $*" ;;
  walkpmc)
    P1="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"
    P2="GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU"
    L="python3 $R/tools/ldpass_band.py --M 1000000 --bw 1000 --ncols 4,8 --reps 3"
    steps=()
    for v in 8 0; do
      i=0
      for p in "$P1" "$P2" FETCH_SIZE WRITE_SIZE; do
        i=$((i + 1))
        steps+=("wpmc_${T}_w${v}_$i:200:cd /tmp && SGV_AB=1 SGV_BAND_WALK=$v timeout -s KILL 180 rocprofv3 --pmc $p -d $R/gpurun_out/wpmc_${T}_w${v}_$i -o pmc --output-format csv -- $L --tag walk=$v")
      done
    done
    tools/gpu_steps.sh "${steps[@]}" ;;
  configs)
    o=gpurun_out/cfg_$T
    run() {   # name, timeout, args...
      local name=$1 to=$2; shift 2
      timeout -k 10 $to python -u bench.py "$@" > ${o}_$name.json 2> ${o}_$name.err || {
        echo "$name FAILED"; tail -20 ${o}_$name.err; exit 1; }
      python -c "import json; d=json.load(open('${o}_$name.json')); r=d['roofline']; c=d.get('compute_roofline'); print(json.dumps(dict(config='$name', value=round(d['value'],3), ms_per_step=round(d['ms_per_step'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4), passes=round(d['ld_passes_per_step'],2), stream=r.get('box_stream_GBs'), mfma_frac=(round(c['frac'],4) if c else None), xchg=d['exchange']['allgathers_per_step'])))" | tee -a ${o}.jsonl
    }
    Q="--cpu-baseline off --read-bw 0"
    run ns 600 --cpu-baseline off
    run c2 400 --blocks 8 --block-size 25000 --K 1 $Q
    run c3 400 --blocks 8 --block-size 25000 --K 4 $Q
    run c4 400 --K 1 $Q
    run c5 400 --K 8 --ridge 0.1 --lmmse-damp 1 --steps 3 --warmup 1 $Q
    run c5conv 500 --K 8 --ridge 0.1 --lmmse-damp 1 --nsamp 20000 --steps 5 --warmup 2 $Q
    run band 400 --band 1000000,1000 --steps 10 --warmup 2 --no-files $Q
    run ns8blk 400 --blocks 8 --block-size 15625 --K 4 $Q
    run share8 600 --gpus 8 --share-device --steps 3 --warmup 1 $Q ;;
  ab)
    bash tools/gpu_ab_multi.sh gpurun_out/ab_$T "$@" ;;
  gate50)
    tools/gpu_steps.sh "gate50_$T:1100:SGV_FULL_GATE=1 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -s -p no:cacheprovider -k 'north_star_50 and ${1:-4}' --timeout 1050" ;;
  *)
    echo "unknown recipe $recipe"; exit 2 ;;
esac
