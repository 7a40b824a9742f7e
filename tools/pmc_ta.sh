#!/bin/bash
# Texture-addresser / L1 PMC passes (separate runs, no trace domains) over tools/ab_variants.py variants: is the walk
# bound by the L1's address / data throughput? usage: tools/pmc_ta.sh <tag> <ab_variants.py args...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/pmc_$tag
mkdir -p $out
pass() {  # name counters...
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d $out/$name -o run --output-format csv -- python3 tools/ab_variants.py --rounds 1 --frames 8 "${ARGS[@]}" > $out/$name.log 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    [ $rc -eq 0 ] || { tail -5 $out/$name.log; exit $rc; }
}
ARGS=("$@")
pass ta TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_WAVES
pass tastall TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
pass tawf TA_FLAT_READ_WAVEFRONTS_sum TA_TOTAL_WAVEFRONTS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE
echo ALLDONE
