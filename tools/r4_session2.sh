#!/bin/bash
# Round 4 session 2: the GPU suite, then same-box A/Bs of the batch kernels (persist4 / shpool / stream) on the
# BASELINE scenes, then the bench line. Each GPU step time-limited; stop at a crash.
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
run ab_dragon 300 python tools/ab_variants.py --frames 20 --rounds 2 persist4 shpool stream
run ab_car 300 python tools/ab_variants.py --scene car_boxed --frames 20 --rounds 2 persist4 shpool stream
run ab_sports 300 python tools/ab_variants.py --scene sportscar --frames 20 --rounds 2 persist4 shpool stream
run ab_two 400 python tools/ab_variants.py --scene two_cars --width 3840 --height 2160 --frames 20 --rounds 2 persist4 shpool stream
run bench 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
