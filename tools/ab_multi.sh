#!/bin/bash
# Same-box A/B of several library builds, interleaved: tools/ab_multi.sh "<dir|tree> ..." [scenes...] (V = variants;
# "tree" = the in-tree library). Logs gpurun_out/abm_<scene>_<dir>_<round>.log; then the parity suite on the tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
libs=$1; shift
for sc in ${@:-dragon}; do
  for r in 1 2; do
    for L in $libs; do
      if [ "$L" = tree ]; then unset PRT_LIB_DIR; else export PRT_LIB_DIR="$PWD/$L"; fi
      timeout -k 10 300 python tools/ab_variants.py --scene $sc --rounds 3 ${V:-shdefer} > gpurun_out/abm_${sc}_${L}_$r.log 2>&1 || exit $?
    done
  done
done
unset PRT_LIB_DIR
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_build.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/par.log 2>&1
