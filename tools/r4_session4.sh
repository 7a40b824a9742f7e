#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
export PRT_TUNE_LOG=1
for sc in dragon car_boxed sportscar two_cars; do
  timeout -k 10 300 python tools/latency.py --scene $sc --iters 60 default default shpool > gpurun_out/lat_$sc.log 2>&1 || exit $?
done
