#!/bin/bash
# BASELINE.json's configurations on one GPU: one bench line each (the driver's 20 steps: one 20-frame launch; no CPU baseline),
# with the autotuner's decision logged (PRT_TUNE_LOG). Output: gpurun_out/cfg_<name>.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name args...
    local n=$1; shift
    PRT_TUNE_LOG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" > gpurun_out/cfg_$n.log 2>&1
    local rc=$?
    echo "$n rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
run dragon
run sportscar --scene sportscar
run car_boxed --scene car_boxed
run dragon871k --scene dragon871k
run two_cars_4k --scene two_cars --width 3840 --height 2160
run car_boxed_4k_64spp --scene car_boxed --width 3840 --height 2160 --spp 64 --steps 2 --warmup 1 --frames 1
