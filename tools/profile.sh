#!/bin/bash
# rocprofv3 passes for one bench configuration (run on the GPU box): kernel trace + stats, then PMC counters
# in separate passes (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950; no trace domains
# are combined with --pmc). Output under gpurun_out/prof_<tag>/ (+ the command and the library's md5, which
# tools/pmc_traffic.py stamps into profiles/pmc_traffic.json).
# usage: tools/profile.sh <tag> [bench args...]   (default: the driver's command, --steps 20 --warmup 5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
args="$@"
out=gpurun_out/prof_$tag
mkdir -p $out
step() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name" | tee -a $out/session.log
    timeout -k 10 $to "$@" > $out/$name.log 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a $out/session.log
    if [ $rc -ne 0 ]; then tail -20 $out/$name.log; exit $rc; fi
}
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency $args"
echo "$B" > $out/cmd.txt
md5sum parallel-ray-tracer_amd/lib/librt_hip.so > $out/lib_md5.txt
step trace 600 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- $B
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- $B
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- $B
step pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $out/pmc_sq -o run --output-format csv -- $B
step pmc_l2 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d $out/pmc_l2 -o run --output-format csv -- $B
step pmc_valu 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $out/pmc_valu -o run --output-format csv -- $B
echo ALLDONE | tee -a $out/session.log
