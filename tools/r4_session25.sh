#!/bin/bash
# round 4: A/B of the packed PERSIST4 build at 64 spp, and of the 3-wave k_persist's spp = 1 / packed builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "exact_ties" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/ties.log 2>&1; echo "ties rc=$?"
bash tools/ab_spp.sh || exit $?
V=persist tools/ab_multi.sh "tree ab_p3_1 ab_p3_2" sportscar car_boxed dragon || exit $?
for L in tree ab_p3_1 ab_p3_2; do
  for sc in sportscar car_boxed; do
    if [ "$L" = tree ]; then unset PRT_LIB_DIR; else export PRT_LIB_DIR="$PWD/$L"; fi
    timeout -k 10 300 python tools/latency.py --scene $sc --iters 60 default > gpurun_out/lat_${sc}_$L.log 2>&1 || exit $?
  done
done
echo ALLDONE
