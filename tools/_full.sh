cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_session.sh smoke pytestall bench || exit $?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
grep '^{' gpurun_out/bench.log | cut -c1-200
timeout -k 10 300 python tools/tile_trace.py 2>&1 | grep -v amdgpu.ids | tail -25
