#!/bin/bash
# round 4 (final build): GPU suite, bench line, dragon profile (trace + PMC passes), BASELINE configs
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
run bench 600 python bench.py --steps 20 --warmup 5
bash tools/profile.sh ${TAG:-r4g}_dragon && python3 tools/trim_prof.py gpurun_out/prof_${TAG:-r4g}_dragon || exit $?
timeout -k 10 900 bash tools/configs.sh || exit $?
echo ALLDONE
