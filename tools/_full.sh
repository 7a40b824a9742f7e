cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_session.sh smoke pytestall bench || exit $?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
grep '^{' gpurun_out/bench.log
bash tools/profile.sh r2d
