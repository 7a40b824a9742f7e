#!/bin/bash
# Same-box A/B/C of library builds, interleaved: tools/ab3.sh "<dir|tree> ..." "<scene:variant> ..." [rounds]
# (dir: a saved build's lib directory, PRT_LIB_DIR; tree: the in-tree build). Output gpurun_out/ab3_<scene>.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
libs=$1; cases=$2; rounds=${3:-2}
for c in $cases; do
  sc=${c%%:*}; v=${c#*:}; extra=""
  [ "$sc" = two_cars ] && extra="--width 3840 --height 2160"
  for r in $(seq $rounds); do
    for L in $libs; do
      if [ "$L" = tree ]; then env_lib=""; else env_lib="PRT_LIB_DIR=$PWD/$L"; fi
      echo -n "$L r$r: " >> gpurun_out/ab3_$sc.log
      timeout -k 10 300 env $env_lib python tools/ab_variants.py --scene $sc $extra --frames 20 --rounds 2 $v \
          >> gpurun_out/ab3_$sc.log 2>&1 || exit $?
    done
  done
done
