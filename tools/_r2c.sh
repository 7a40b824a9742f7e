cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "batch or bgra or rotated or persist4 or placements or xcd" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r2c_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r2c_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab_variants.py --rounds 3 persist4 persist > gpurun_out/r2c_ab.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab_variants.py --rounds 3 --scene car_boxed persist4 >> gpurun_out/r2c_ab.log 2>&1 || exit $?
cat gpurun_out/r2c_ab.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-single-thread > gpurun_out/r2c_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/r2c_bench.log
bash tools/profile.sh r2c
