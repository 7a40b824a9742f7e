cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
B="python bench.py --scene car_boxed --width 3840 --height 2160 --spp 64 --steps 3 --warmup 1 --frames 1 --no-cpu-baseline --no-latency"
for r in 1 2; do
  for L in tree ab_spp; do
    for v in persist4 shdefer; do
      if [ "$L" = tree ]; then unset PRT_LIB_DIR; else export PRT_LIB_DIR="$PWD/$L"; fi
      timeout -k 10 300 $B --variant $v > gpurun_out/spp_${L}_${v}_$r.log 2>&1 || exit $?
    done
  done
done
echo ALLDONE
