#!/bin/bash
# rocprofv3 kernel trace + PMC passes (tools/profile.sh) of every BASELINE.json configuration, with the same bench
# arguments as tools/configs.sh (so that the pmc_traffic.json keys match the configuration lines).
# usage: tools/profile_configs.sh <round-tag> [configs...]   output: gpurun_out/prof_<tag>_<config>/
# (configs: dragon sportscar car_boxed dragon871k two_cars_4k car_boxed_4k_64spp; default all)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
t=$1
shift
want() { [ ${#SEL[@]} -eq 0 ] && return 0; for c in "${SEL[@]}"; do [ "$c" = "$1" ] && return 0; done; return 1; }
SEL=("$@")
prof() {  # tag args...: the passes, then the per-dispatch CSVs trimmed to the path kernels (tools/trim_prof.py)
    local tag=$1; shift
    bash tools/profile.sh $tag "$@" || exit $?
    python3 tools/trim_prof.py gpurun_out/prof_$tag
}
want dragon && prof ${t}_dragon
want sportscar && prof ${t}_sportscar --scene sportscar
want car_boxed && prof ${t}_car_boxed --scene car_boxed
want dragon871k && prof ${t}_dragon871k --scene dragon871k
want two_cars_4k && prof ${t}_two_cars_4k --scene two_cars --width 3840 --height 2160
want car_boxed_4k_64spp && prof ${t}_car_boxed_4k_64spp --scene car_boxed --width 3840 --height 2160 --spp 64 --steps 2 --warmup 1 --frames 1
