#!/bin/bash
# PMC passes (separate runs, no trace domains) over tools/ab_variants.py variants on one frame shape, for
# the per-kernel medians of tools/pmc_summary.py. usage: tools/pmc_ab.sh <tag> <ab_variants.py args...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/pmc_$tag
mkdir -p $out
pass() {  # name counters...
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d $out/$name -o run --output-format csv -- python3 tools/ab_variants.py --rounds 1 --frames 3 "${ARGS[@]}" > $out/$name.log 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    [ $rc -eq 0 ] || { tail -5 $out/$name.log; exit $rc; }
}
ARGS=("$@")
pass sq SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD
pass lat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
pass lds SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
echo ALLDONE
