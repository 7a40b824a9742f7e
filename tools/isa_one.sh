#!/bin/bash
# VGPR / scratch of single k_persist instantiations, fast: a device-only compile of a translation unit that
# instantiates only the kernels named on the command line (template argument lists of rtd::k_persist), e.g.
#   tools/isa_one.sh "4,false,false,true,4,false,true,2,true,true,true"
# (an argument of the form name:args instantiates rtd::name<args> instead, e.g. k_stream:4,false)
# Prints vgpr / scratch / lds / sgpr per kernel and leaves the assembly in /tmp/isa/one.s (no GPU needed).
cd "$(dirname "$0")/.."
mkdir -p /tmp/isa
{
  echo '#include "rt_kernels.hpp"'
  echo '#include "rt_shpool.hpp"'
  for a in "$@"; do
    case $a in
      *:*) echo "template __global__ void rtd::${a%%:*}<${a#*:}>(rtd::KArgs);" ;;
      *) echo "template __global__ void rtd::k_persist<$a>(rtd::KArgs);" ;;
    esac
  done
} > /tmp/isa/one.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
    -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Iparallel-ray-tracer_amd/csrc/hip \
    $ISA_FLAGS --cuda-device-only -S -o /tmp/isa/one.s /tmp/isa/one.hip || exit 1
python3 - <<'PY'
import re
s = open('/tmp/isa/one.s').read()
# the code of each kernel (between its label and its descriptor) for the spill instructions it really executes
code = {}
for m in re.finditer(r'^(_Z\S+):[^\n]*$(.*?)^\s*\.section\s+\.rodata', s, re.S | re.M):
    code[m.group(1)] = m.group(2)
for b in s.split('.amdhsa_kernel ')[1:]:
    name = b.split('\n')[0]
    g = lambda k: re.search(k + r'\s+(\d+)', b).group(1)
    c = code.get(name, '')
    st, ld = len(re.findall(r'scratch_store', c)), len(re.findall(r'scratch_load', c))
    wl = len(re.findall(r'v_writelane_b32', c))
    print(f"{name[:80]:80s} vgpr {g(r'.amdhsa_next_free_vgpr'):>4} sgpr {g(r'.amdhsa_next_free_sgpr'):>4} "
          f"scratch {g(r'.amdhsa_private_segment_fixed_size'):>4} (spill st/ld {st}/{ld}, sgpr->vgpr-lane {wl}) "
          f"lds {g(r'.amdhsa_group_segment_fixed_size'):>6}")
PY
