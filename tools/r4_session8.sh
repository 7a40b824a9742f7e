#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_seam.py tests/test_gpu_parity.py -k "seam or hybrid or walkthrough or rule" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pyt.log 2>&1; echo "pytest rc=$?"
export PRT_TUNE_LOG=1
for w in 0 0.02 0.005; do
  for sc in dragon car_boxed sportscar; do
    timeout -k 10 300 python tools/latency.py --scene $sc --iters 80 --walk $w default shpool > gpurun_out/lat_${sc}_w$w.log 2>&1 || exit $?
  done
done
timeout -k 10 400 python tools/ab_variants.py --frames 20 --rounds 2 shpool shpool:regroup=8 shpool:regroup=24 shpool:regroup=32 shpool:dealing=rows shpool:dealing=columns > gpurun_out/ab_knobs.log 2>&1 || exit $?
