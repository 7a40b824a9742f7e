#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
export PRT_TUNE_LOG=1
timeout -k 10 300 python tools/latency.py --scene dragon --iters 120 --walk 0.02 default shpool > gpurun_out/lat_walk_dragon.log 2>&1 || exit $?
timeout -k 10 300 python tools/latency.py --scene dragon --iters 120 --walk 0.005 default shpool > gpurun_out/lat_walk2_dragon.log 2>&1 || exit $?
timeout -k 10 900 bash tools/configs.sh || exit $?
