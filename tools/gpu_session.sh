#!/bin/bash
# One GPU session: each GPU step under its own time limit; stop at the first fault/abort/timeout.
# Test failures (pytest exit 1) do not stop the session; crashes (>=124, 134, 139) do.
# usage: tools/gpu_session.sh [steps...]   steps: smoke pytest bench prof pmc
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name: $*" | tee -a gpurun_out/session.log
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -lt 0 ]; then
        echo "STOP: $name crashed or timed out (rc=$rc)"; exit $rc
    fi
    return 0
}
for s in "${@:-smoke pytest bench}"; do
  for step in $s; do
    case $step in
      smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
      pytest) run pytest_gpu 1200 python -m pytest tests -m gpu -x -q ;;
      pytestall) run pytest_gpu 1200 python -m pytest tests -m gpu -q ;;
      bench)  run bench 600 python bench.py --steps 20 --warmup 5 ;;
      benchq) run bench 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
      prof)   run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
      ab)     run ab 600 python tools/ab.py --rounds 4 --frames 5 fast wavefront wavefront:PRT_REFILL_BELOW=16 wavefront:PRT_REFILL_BELOW=32 wavefront:PRT_REFILL_BELOW=56 wavefront:PRT_REFILL_BELOW=0 ;;
      abcar)  run abcar 600 python tools/ab.py --scene car_boxed --rounds 3 --frames 5 fast wavefront ;;
      profwf) run profwf 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profwf -o run --output-format csv -- python3 tools/ab.py --rounds 1 --frames 3 wavefront ;;
      abwf)   run abwf 600 python tools/ab.py --rounds 3 --frames 3 fast wavefront wavefront:PRT_WF_CHUNK_MAX=64 wavefront:PRT_WF_CHUNK_MAX=128 wavefront:PRT_WF_BPC=2 wavefront:PRT_WF_BPC=4 wavefront:PRT_WF_BPC=4,PRT_WF_CHUNK_MAX=64 wavefront:PRT_REFILL_BELOW=32,PRT_WF_CHUNK_MAX=64 ;;
      ctrs)   run ctrs 600 python tools/counters.py dragon fast wavefront strict ;;
      pmcwf)  run pmcwf 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d gpurun_out/pmcwf -o run --output-format csv -- python3 tools/ab.py --rounds 1  --frames 2 wavefront fast ;;
      pmcl2)  run pmcl2 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/pmcl2 -o run --output-format csv -- python3 tools/ab.py --rounds 1  --frames 2 wavefront fast ;;
      pmcfetch) run pmcfetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcfetch -o run --output-format csv -- python3 tools/ab.py --rounds 1  --frames 2 wavefront fast ;;
      pmclat) run pmclat 600 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum -d gpurun_out/pmclat -o run --output-format csv -- python3 tools/ab.py --rounds 1  --frames 2 wavefront fast ;;
      abreg)  run abreg 600 python tools/ab.py --rounds 4 --frames 5 fast fast:PRT_PERSIST_REG=0 ;;
      abregcar) run abregcar 600 python tools/ab.py --scene car_boxed --rounds 4 --frames 5 fast fast:PRT_PERSIST_REG=0 ;;
      abold)  for i in 1 2; do
                  run abnew$i 300 python tools/ab.py --rounds 3 --frames 5 fast fast:PRT_WIDE=0
                  PRT_LIB_DIR=build/old/lib run abold$i 300 python tools/ab.py --rounds 3 --frames 5 wavefront
              done ;;
      abwide) run abwide 300 python tools/ab.py --rounds 4 --frames 5 fast fast:PRT_WIDE=0
              run abwidecar 300 python tools/ab.py --scene car_boxed --rounds 4 --frames 5 fast fast:PRT_WIDE=0 ;;
      ctrswide) run ctrswide 300 python tools/counters.py dragon fast ;;
      abocc)  run abocc 300 python tools/ab.py --rounds 4 --frames 5 fast fast:PRT_PERSIST_OCC=4
              run abocccar 300 python tools/ab.py --scene car_boxed --rounds 4 --frames 5 fast fast:PRT_PERSIST_OCC=4 ;;
      abhead) for i in 1 2 3; do
                  run abnew$i 300 python tools/ab.py --rounds 3 --frames 5 fast
                  PRT_LIB_DIR=build/old/lib run abold$i 300 python tools/ab.py --rounds 3 --frames 5 fast
              done ;;
      abheadcar) for i in 1 2; do
                  run abnewcar$i 300 python tools/ab.py --scene car_boxed --rounds 3 --frames 5 fast
                  PRT_LIB_DIR=build/old/lib run aboldcar$i 300 python tools/ab.py --scene car_boxed --rounds 3 --frames 5 fast
              done ;;
      tiles)  run tiles 300 python tools/tile_trace.py
              run tilescar 300 python tools/tile_trace.py --scene car_boxed ;;
      tilesc) run tilesc 300 python tools/tile_trace.py --counters ;;
      abregen) run abregen 300 python tools/ab.py --rounds 4 --frames 5 fast fast:PRT_REGEN=1
              run abregencar 300 python tools/ab.py --scene car_boxed --rounds 4 --frames 5 fast fast:PRT_REGEN=1
              run abregensc 300 python tools/ab.py --scene sportscar --rounds 2 --frames 5 fast fast:PRT_REGEN=1 ;;
      aborder) run aborder 300 python tools/ab.py --rounds 4 --frames 5 fast fast:PRT_TILE_ORDER=center
              run abordercar 300 python tools/ab.py --scene car_boxed --rounds 4 --frames 5 fast fast:PRT_TILE_ORDER=center
              run aborderrand 300 python tools/ab.py --scene sportscar --rounds 3 --frames 5 fast fast:PRT_TILE_ORDER=center ;;
      ab3)    for i in 1 2; do
                  run ab3new$i 300 python tools/ab.py --rounds 3 --frames 5 fast fast:PRT_TILE_ORDER=rows
                  PRT_LIB_DIR=build/old/lib run ab3old$i 300 python tools/ab.py --rounds 3 --frames 5 fast
                  run ab3newcar$i 300 python tools/ab.py --scene car_boxed --rounds 3 --frames 5 fast fast:PRT_TILE_ORDER=rows
                  PRT_LIB_DIR=build/old/lib run ab3oldcar$i 300 python tools/ab.py --scene car_boxed --rounds 3 --frames 5 fast
              done ;;
      abbatch) run abbatch 300 python tools/ab.py --rounds 4 --frames 5 fast fast:PRT_SHADOW_BATCH=0
              run abbatchcar 300 python tools/ab.py --scene car_boxed --rounds 4 --frames 5 fast fast:PRT_SHADOW_BATCH=0
              run abbatchsc 300 python tools/ab.py --scene sportscar --rounds 3 --frames 5 fast fast:PRT_SHADOW_BATCH=0 ;;
      abpf)   for i in 1 2; do
                  run abpfnew$i 300 python tools/ab.py --rounds 3 --frames 5 fast
                  PRT_LIB_DIR=build/old/lib run abpfold$i 300 python tools/ab.py --rounds 3 --frames 5 fast:PRT_SHADOW_BATCH=0
                  run abpfnewcar$i 300 python tools/ab.py --scene car_boxed --rounds 3 --frames 5 fast
                  PRT_LIB_DIR=build/old/lib run abpfoldcar$i 300 python tools/ab.py --scene car_boxed --rounds 3 --frames 5 fast:PRT_SHADOW_BATCH=0
              done ;;
      abprio) run abprio 300 python tools/ab.py --rounds 4 --frames 5 fast fast:PRT_PRIO=1
              run abpriocar 300 python tools/ab.py --scene car_boxed --rounds 4 --frames 5 fast fast:PRT_PRIO=1
              run abpriosc 300 python tools/ab.py --scene sportscar --rounds 3 --frames 5 fast fast:PRT_PRIO=1 ;;
      pytestsplit) PRT_SPLIT=1 run pytest_split 1200 python -m pytest tests -m gpu -q ;;
      absplit) run absplit 300 python tools/ab.py --rounds 4 --frames 5 fast fast:PRT_SPLIT=1
              run absplitcar 300 python tools/ab.py --scene car_boxed --rounds 4 --frames 5 fast fast:PRT_SPLIT=1
              run absplitsc 300 python tools/ab.py --scene sportscar --rounds 3 --frames 5 fast fast:PRT_SPLIT=1 ;;
      profsplit) PRT_SPLIT=1 run profsplit 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profsplit -o run --output-format csv -- python3 tools/ab.py --rounds 1 --frames 5 fast
              PRT_SPLIT=1 run profsplitcar 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profsplitcar -o run --output-format csv -- python3 tools/ab.py --scene car_boxed --rounds 1 --frames 5 fast ;;
      abtri)  for sc in dragon car_boxed sportscar; do
                  run abtri_$sc 300 python tools/ab.py --scene $sc --rounds 3 --frames 5 fast fast:PRT_SPLIT=1
                  PRT_LIB_DIR=build/old/lib run abtriold_$sc 300 python tools/ab.py --scene $sc --rounds 3 --frames 5 fast
              done ;;
      abwc)   for sc in dragon car_boxed sportscar; do
                  run abwc_$sc 300 python tools/ab.py --scene $sc --rounds 3 --frames 5 fast fast:PRT_WCACHE=0 fast:PRT_WCACHE=9
                  PRT_LIB_DIR=build/old/lib run abwcold_$sc 300 python tools/ab.py --scene $sc --rounds 3 --frames 5 fast
              done ;;
      abcol)  for sc in dragon car_boxed sportscar; do
                  run abcol_$sc 300 python tools/ab.py --scene $sc --reupload --rounds 3 --frames 5 fast fast:PRT_WIDE_COLLAPSE=greedy fast:PRT_WIDE_CNODE=2 fast:PRT_WIDE_CNODE=8
              done
              run ctrscol 300 python tools/counters.py dragon fast ;;
      abcn)   for sc in dragon car_boxed; do
                  run abcn_$sc 300 python tools/ab.py --scene $sc --reupload --rounds 6 --frames 5 fast:PRT_WIDE_CNODE=2 fast:PRT_WIDE_CNODE=3 fast fast:PRT_WIDE_COLLAPSE=greedy
              done ;;
      abbits) for i in 1 2; do for sc in dragon car_boxed sportscar; do
                  run abbits_${sc}_$i 300 python tools/ab.py --scene $sc --rounds 3 --frames 5 fast
                  PRT_LIB_DIR=build/old/lib run abbitsold_${sc}_$i 300 python tools/ab.py --scene $sc --rounds 3 --frames 5 fast
              done; done ;;
      abbits3) for i in 1 2; do for sc in dragon car_boxed sportscar; do
                  run ab3u_${sc}_$i 300 python tools/ab.py --scene $sc --rounds 3 --frames 5 fast
                  PRT_LIB_DIR=build/loop/lib run ab3l_${sc}_$i 300 python tools/ab.py --scene $sc --rounds 3 --frames 5 fast
                  PRT_LIB_DIR=build/old/lib run ab3o_${sc}_$i 300 python tools/ab.py --scene $sc --rounds 3 --frames 5 fast
              done; done ;;
      absc)   for L in parallel-ray-tracer_amd/lib build/old/lib; do
                  t=$(basename $(dirname $L))
                  PRT_LIB_DIR=$L run absc_$t 300 python tools/ab.py --scene sportscar --rounds 3 --frames 5 fast fast:PRT_SPLIT=0
                  PRT_LIB_DIR=$L run profsc_$t 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profsc_$t -o run --output-format csv -- python3 tools/ab.py --scene sportscar --rounds 1 --frames 5 fast
              done ;;
      absocc) run abocc_sportscar 300 python tools/ab.py --scene sportscar --rounds 4 --frames 5 fast fast:PRT_SPLIT_OCC_A=3 fast:PRT_SPLIT_OCC_A=2 fast:PRT_SPLIT_OCC_B=3 fast:PRT_SPLIT_OCC_B=2 fast:PRT_SPLIT_OCC_A=3,PRT_SPLIT_OCC_B=3
              run abocc_car 300 python tools/ab.py --scene car_boxed --rounds 3 --frames 5 fast:PRT_SPLIT=1 fast:PRT_SPLIT=1,PRT_SPLIT_OCC_A=3 fast:PRT_SPLIT=1,PRT_SPLIT_OCC_A=2
              PRT_LIB_DIR=build/old/lib run abocc_old 300 python tools/ab.py --scene sportscar --rounds 4 --frames 5 fast ;;
      abcap)  run abcap_sportscar 300 python tools/ab.py --scene sportscar --rounds 4 --frames 5 fast:PRT_SPLIT_OCC_A=2 fast:PRT_SPLIT_OCC_A=1 fast:PRT_SPLIT_OCC_A=2,PRT_SPLIT_OCC_B=3 fast:PRT_SPLIT_OCC_A=1,PRT_SPLIT_OCC_B=2
              for sc in dragon car_boxed; do
                  run abcap_$sc 300 python tools/ab.py --scene $sc --rounds 4 --frames 5 fast fast:PRT_PERSIST_CAP=2 fast:PRT_PERSIST_CAP=1 fast:PRT_SPLIT=1,PRT_SPLIT_OCC_A=2 fast:PRT_SPLIT=1,PRT_SPLIT_OCC_A=1
              done ;;
      abtune) for sc in dragon car_boxed sportscar; do
                  PRT_TUNE_LOG=1 run abtune_$sc 300 python tools/ab.py --scene $sc --rounds 4 --frames 5 fast fast:PRT_TUNE=0
              done ;;
      ranks)  run ranks 300 python tools/rank_rows.py
              run ranks_car 300 python tools/rank_rows.py --scene car_boxed ;;
      *) echo "unknown step $step"; exit 2 ;;
    esac
  done
done
