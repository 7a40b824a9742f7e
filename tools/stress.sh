#!/bin/bash
# Stress workloads on the GPU box: parity tests, then one bench line per workload (profiles/r2*_stress.jsonl).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_stress.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/stress_tests.log 2>&1 || { tail -30 gpurun_out/stress_tests.log; exit 1; }
tail -3 gpurun_out/stress_tests.log
for sc in sportscar dragon871k random1m; do
    timeout -k 10 300 python bench.py --steps 32 --warmup 8 --scene $sc --no-single-thread \
        > gpurun_out/bench_$sc.log 2>&1 || { tail -20 gpurun_out/bench_$sc.log; exit 1; }
    grep '^{' gpurun_out/bench_$sc.log >> gpurun_out/stress_bench.jsonl
done
echo STRESSDONE
