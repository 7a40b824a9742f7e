#!/bin/bash
# VGPR / scratch / LDS per kernel of librt_hip (device-only compile to assembly; no GPU needed)
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
    -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Iparallel-ray-tracer_amd/csrc \
    -Iparallel-ray-tracer_amd/csrc/hip --cuda-device-only -S -o /tmp/rt_isa.s \
    parallel-ray-tracer_amd/csrc/hip/rt_hip.hip 2>/dev/null || exit 1
python3 - "$@" <<'PY'
import re, sys
s = open('/tmp/rt_isa.s').read()
pat = sys.argv[1] if len(sys.argv) > 1 else ''
# the code of each kernel (its label to the descriptor) for the spill instructions it really executes: a private
# segment can stay reserved for SGPR spills that were lowered to VGPR lanes (sgpr->lane) and never touch memory
code = {m.group(1): m.group(2) for m in re.finditer(r'^(_Z\S+):[^\n]*$(.*?)^\s*\.section\s+\.rodata', s, re.S | re.M)}
for b in s.split('.amdhsa_kernel ')[1:]:
    name = b.split('\n')[0]
    if pat not in name:
        continue
    g = lambda k: re.search(k + r'\s+(\d+)', b).group(1)
    c = code.get(name, '')
    st, ld = len(re.findall(r'scratch_store', c)), len(re.findall(r'scratch_load', c))
    print(f"{name[:72]:72s} vgpr {g(r'.amdhsa_next_free_vgpr'):>4} agpr-split {g(r'.amdhsa_accum_offset'):>4} "
          f"scratch {g(r'.amdhsa_private_segment_fixed_size'):>4} spill-st/ld {st:>3}/{ld:<3} "
          f"lds {g(r'.amdhsa_group_segment_fixed_size'):>6}")
PY
