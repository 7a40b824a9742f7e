#!/bin/bash
# Same-box A/B of library builds on BASELINE config 5 (car_boxed 3840x2160, 64 spp): the bench line per build and
# kernel, interleaved, two rounds. usage: tools/ab_spp.sh "<dir|tree> ..." [variants] (dir: a saved build's lib
# directory, PRT_LIB_DIR; tree: the in-tree build). Logs gpurun_out/spp_<lib>_<variant>_<round>.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
libs=${1:-tree}; variants=${2:-persist4 shdefer}
B="python bench.py --scene car_boxed --width 3840 --height 2160 --spp 64 --steps 3 --warmup 1 --frames 1 --no-cpu-baseline --no-latency"
for r in 1 2; do
  for L in $libs; do
    for v in $variants; do
      if [ "$L" = tree ]; then unset PRT_LIB_DIR; else export PRT_LIB_DIR="$PWD/$L"; fi
      timeout -k 10 300 $B --variant $v > gpurun_out/spp_${L}_${v}_$r.log 2>&1 || exit $?
    done
  done
done
echo ALLDONE
