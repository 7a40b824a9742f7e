#!/bin/bash
# Same-box A/B of two library builds: PRT_LIB_DIR=<dir> (e.g. a saved ab_base/) vs the in-tree lib, per scene,
# interleaved (base, new, base, new); then the parity suite on the in-tree lib. Each GPU step time-limited.
# usage: tools/ab_libs.sh <base_dir> [scenes...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
base=$1; shift
for sc in ${@:-dragon car_boxed}; do
  for r in 1 2; do
    timeout -k 10 300 env PRT_LIB_DIR="$PWD/$base" python tools/ab_variants.py --scene $sc --rounds 3 ${V:-persist4} \
        > gpurun_out/ab_${sc}_base$r.log 2>&1 || exit $?
    timeout -k 10 300 python tools/ab_variants.py --scene $sc --rounds 3 ${V:-persist4} > gpurun_out/ab_${sc}_new$r.log 2>&1 || exit $?
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_build.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/par.log 2>&1
