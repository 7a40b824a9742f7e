#!/bin/bash
# round 4: packed triangle tests -- GPU suite, then same-box A/B (dragon: the pool kernel at TQ_MIN 2 / 3 / 4 against
# the previous commit; the other scenes: PERSIST4 with and without the packed build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
tools/ab_multi.sh "ab_base tree ab_min2 ab_min4" dragon && mv gpurun_out/par.log gpurun_out/par1.log || exit $?
V=persist4 tools/ab_multi.sh "ab_base tree" sportscar car_boxed || exit $?
echo ALLDONE
