#!/bin/bash
# rocprofv3 kernel trace + PMC passes (tools/profile.sh) of every BASELINE.json configuration, with the same bench
# arguments as tools/configs.sh (so that the pmc_traffic.json keys match the configuration lines).
# usage: tools/profile_configs.sh <round-tag>     output: gpurun_out/prof_<tag>_<config>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
t=$1
prof() {  # tag args...: the passes, then the per-dispatch CSVs trimmed to the path kernels (tools/trim_prof.py)
    local tag=$1; shift
    bash tools/profile.sh $tag "$@" || exit $?
    python3 tools/trim_prof.py gpurun_out/prof_$tag
}
prof ${t}_dragon
prof ${t}_sportscar --scene sportscar
prof ${t}_car_boxed --scene car_boxed
prof ${t}_two_cars_4k --scene two_cars --width 3840 --height 2160
prof ${t}_car_boxed_4k_64spp --scene car_boxed --width 3840 --height 2160 --spp 64 --steps 2 --warmup 1 --frames 1
