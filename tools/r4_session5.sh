#!/bin/bash
# packed-FMA node test and LDS-staged roots: same-box A/B/C (ab_base = scalar FMAs, ab_pk = packed, tree = packed +
# LDS roots) on the batch kernels, then the single-frame rule's latency (tree build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/ab3.sh "ab_base ab_pk tree" "dragon:shpool car_boxed:persist4 sportscar:persist4 two_cars:persist4" 2 || exit $?
export PRT_TUNE_LOG=1
for sc in dragon car_boxed sportscar; do
  timeout -k 10 300 python tools/latency.py --scene $sc --iters 60 default shpool > gpurun_out/lat_$sc.log 2>&1 || exit $?
done
