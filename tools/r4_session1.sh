#!/bin/bash
# Round 4 session: super-tile dealing A/B (ab_base = before) on dragon (shadow pool) and car_boxed (persist4),
# the two_cars 4K batch kernels, then a profile of the dragon bench (no latency frames: batches only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
V=shpool bash tools/ab_libs.sh ab_base dragon || exit $?
V=persist4 timeout -k 10 300 env PRT_LIB_DIR="$PWD/ab_base" python tools/ab_variants.py --scene car_boxed --rounds 3 persist4 > gpurun_out/ab_car_base.log 2>&1 || exit $?
V=persist4 timeout -k 10 300 python tools/ab_variants.py --scene car_boxed --rounds 3 persist4 > gpurun_out/ab_car_new.log 2>&1 || exit $?
timeout -k 10 400 python tools/ab_variants.py --scene two_cars --width 3840 --height 2160 --frames 20 --rounds 2 persist4 shpool > gpurun_out/ab_two_cars.log 2>&1 || exit $?
bash tools/profile.sh r4b_dragon || exit $?
python3 tools/trim_prof.py gpurun_out/prof_r4b_dragon
