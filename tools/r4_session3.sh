#!/bin/bash
# Round 4 session 3: single-frame rule investigation (trial log) on dragon / car_boxed / sportscar, forced configurations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
export PRT_TUNE_LOG=1
for sc in dragon car_boxed sportscar; do
  timeout -k 10 300 python tools/latency.py --scene $sc --iters 45 default persist shpool persist4 \
      hybrid:hot_pct=75,hot_kernel=coop2 hybrid:hot_pct=45 hybrid:hot_pct=60 > gpurun_out/lat_$sc.log 2>&1 || exit $?
done
