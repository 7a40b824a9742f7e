#!/bin/bash
# One GPU session: each GPU step under its own time limit; stop at the first fault/abort/timeout.
# Test failures (pytest exit 1) do not stop the session; crashes (>=124, 134, 139) do.
# usage: tools/gpu_session.sh [steps...]   steps: smoke pytest pytestall bench benchq prof ab abcar ranks final
#   final (a round's last session on the final build): the GPU suite, the driver's bench line, the dragon profile
#   (trace + PMC passes, tools/profile.sh -> profiles/ via tools/pmc_traffic.py) and every BASELINE configuration
#   (tools/configs.sh); TAG names the profile (default r5)
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
      ab)     run ab 600 python tools/ab_variants.py persist persist4 shpool shdefer coop4 ;;
      abcar)  run abcar 600 python tools/ab_variants.py --scene car_boxed persist persist4 shpool shdefer coop4 ;;
      ranks)  run ranks 300 python tools/rank_rows.py
              run ranks_car 300 python tools/rank_rows.py --scene car_boxed ;;
      final)  run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
              run bench 600 python bench.py --steps 20 --warmup 5
              bash tools/profile.sh ${TAG:-r5}_dragon && python3 tools/trim_prof.py gpurun_out/prof_${TAG:-r5}_dragon || exit $?
              timeout -k 10 900 bash tools/configs.sh || exit $? ;;
      *) echo "unknown step $step"; exit 2 ;;
    esac
  done
done
