#!/bin/bash
# tie re-walk cut: parity of the tie tests, then same-box latency / batch of car_boxed with and without it
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_seam.py -k "ties or strict or car_boxed or small_frames or seam or hybrid or walkthrough or settles" > gpurun_out/tc_par.log 2>&1 || exit $?
for r in 1 2; do for L in ab_nocut tree; do
  if [ $L = tree ]; then E=""; else E="PRT_LIB_DIR=$PWD/$L"; fi
  echo "== $L r$r" >> gpurun_out/tc_lat.log
  timeout -k 10 120 env $E python3 tools/latency.py --scene car_boxed --iters 40 default persist >> gpurun_out/tc_lat.log 2>&1 || exit 1
  timeout -k 10 200 env $E python tools/ab_variants.py --scene car_boxed --frames 20 --rounds 2 persist4 >> gpurun_out/tc_lat.log 2>&1 || exit 1
done; done
