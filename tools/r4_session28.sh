#!/bin/bash
# round 4: deferred packed closest tests (PRT_TQ_DEFER 16 / 32 / 48) against the tree, same box; parity of df32
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
V=shdefer tools/ab_multi.sh "tree ab_df16 ab_df32 ab_df48" dragon || exit $?
V=persist4 tools/ab_multi.sh "tree ab_df32" sportscar || exit $?
PRT_LIB_DIR=$PWD/ab_df32 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/par_df32.log 2>&1; echo "par df32 rc=$?"
echo ALLDONE
