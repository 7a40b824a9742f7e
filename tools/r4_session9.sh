#!/bin/bash
# round 4: the all-levels shadow pool (shdefer) -- parity, then A/B against shpool / persist4 in frame batches,
# plus the pending seam / single-frame-rule checks of session 8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stress.py -k "shdefer" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pyt_shd.log 2>&1; rc=$?; echo "pytest shdefer rc=$rc"; [ $rc -le 1 ] || exit $rc
for sc in dragon sportscar car_boxed; do
  timeout -k 10 300 python tools/ab_variants.py --scene $sc --frames 20 --rounds 3 persist4 shpool shdefer > gpurun_out/ab_shd_$sc.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_seam.py tests/test_gpu_parity.py -k "seam or hybrid or walkthrough or rule" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pyt.log 2>&1; echo "pytest seam rc=$?"
export PRT_TUNE_LOG=1
for w in 0 0.02; do
  for sc in dragon sportscar; do
    timeout -k 10 300 python tools/latency.py --scene $sc --iters 80 --walk $w default shpool > gpurun_out/lat_${sc}_w$w.log 2>&1 || exit $?
  done
done
echo ALLDONE
