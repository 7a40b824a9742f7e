#!/bin/bash
# One GPU session: each GPU step under its own time limit; stop at the first fault/abort/timeout.
# Test failures (pytest exit 1) do not stop the session; crashes (>=124, 134, 139) do.
# usage: tools/gpu_session.sh [steps...]   steps: smoke pytest pytestall bench benchq prof ab abcar ranks
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
      pytest) run pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread ;;
      pytestall) run pytest_gpu 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ;;
      bench)  run bench 600 python bench.py --steps 20 --warmup 5 ;;
      benchq) run bench 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
      prof)   run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
      ab)     run ab 600 python tools/ab_variants.py persist persist4 shpool coop4 fan ;;
      abcar)  run abcar 600 python tools/ab_variants.py --scene car_boxed persist persist4 shpool coop4 fan ;;
      ranks)  run ranks 300 python tools/rank_rows.py
              run ranks_car 300 python tools/rank_rows.py --scene car_boxed ;;
      *) echo "unknown step $step"; exit 2 ;;
    esac
  done
done
