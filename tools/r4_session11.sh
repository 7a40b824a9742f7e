#!/bin/bash
# round 4: 5-byte wide stack entries (the all-levels pool fits deeper trees) -- GPU suite, then A/B per scene
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name" | tee -a gpurun_out/session.log
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
    tail -3 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP: $name (rc=$rc)"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
for sc in dragon sportscar car_boxed; do
  run ab_$sc 300 python tools/ab_variants.py --scene $sc --frames 20 --rounds 3 persist4 shpool shdefer
done
run ab_two_cars 400 python tools/ab_variants.py --scene two_cars --width 3840 --height 2160 --frames 20 --rounds 2 persist4 shpool shdefer
echo ALLDONE
