#!/bin/bash
# Round-6 GPU sessions: named steps, each under its own time limit; a crash, abort or timeout ends the session.
# usage: tools/r6.sh step...   (steps below; AB_LIBS / AB_CASES / AB_ROUNDS for the ab step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name: $*" | tee -a gpurun_out/r6.log
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a gpurun_out/r6.log
    tail -3 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -lt 0 ]; then
        echo "STOP: $name crashed or timed out (rc=$rc)"; exit $rc
    fi
    return 0
}
PT="python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread"
for step in "$@"; do
  case $step in
    parq)  run parq 900 $PT tests/test_gpu_parity.py -k "small_frames or 1080p or row_subset or ragged or counts" ;;
    parity) run parity 1200 $PT tests/test_gpu_parity.py tests/test_gpu_build.py tests/test_gpu_stress.py ;;
    new)   run new 900 $PT tests/test_gpu_unpacked.py tests/test_gpu_comm.py tests/test_gpu_configs.py -k "unpacked or rccl or dragon-1920" ;;
    suite) run suite 1500 $PT tests ;;
    seam)  run seam 900 $PT tests/test_gpu_seam.py tests/test_gpu_parity.py -k "seam or hybrid or walkthrough or settles" ;;
    lat)   run lat_dragon 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
           run lat_car 300 python bench.py --scene car_boxed --steps 20 --warmup 5 --no-cpu-baseline
           run lat_871k 300 python bench.py --scene dragon871k --steps 20 --warmup 5 --no-cpu-baseline ;;
    ab)    run ab 1200 bash tools/ab3.sh "${AB_LIBS:-ab_base tree}" "${AB_CASES:-dragon:shdefer car_boxed:persist4}" ${AB_ROUNDS:-2} ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5 ;;
    benchq) run bench 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo R6DONE
