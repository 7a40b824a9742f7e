#!/usr/bin/env python3
"""Static instruction counts per basic block of one kernel in an assembly file (tools/isa_one.sh leaves
/tmp/isa/one.s): VALU / SALU / VMEM / LDS instructions per block, and the loop back edges, so that the blocks of the
walks' step loops (wide_node, the leaf-mask loop, the stack, the triangle tests, the pool's refill) can be priced.
usage: tools/isa_blocks.py [asm] [kernel-substring]"""
import re
import sys


def blocks_of(asm, want):
    s = open(asm).read()
    starts = [m.start() for m in re.finditer(r'^_ZN[^\s:]*:', s, re.M)]
    for st in starts:
        name = s[st:s.index(':', st)]
        if want and want not in name:
            continue
        body = s[st:s.index('.Lfunc_end', st)]
        out, cur = [], None
        for raw in body.split('\n'):
            l = raw.strip()
            m = re.match(r'^(\.LBB\d+_\d+):', l)
            if m or l.startswith('_ZN'):
                cur = [m.group(1) if m else 'entry', []]
                out.append(cur)
                continue
            if cur is None or not l or l.startswith((';', '.')):
                continue
            cur[1].append(l.split(';')[0].strip())
        return name, out
    raise SystemExit(f"no kernel matching {want!r} in {asm}")


def main():
    asm = sys.argv[1] if len(sys.argv) > 1 else '/tmp/isa/one.s'
    want = sys.argv[2] if len(sys.argv) > 2 else ''
    name, blocks = blocks_of(asm, want)
    idx = {b[0]: i for i, b in enumerate(blocks)}
    tot = dict(v=0, s=0, vm=0, ds=0)
    print(f"kernel {name}")
    print(f"{'#':>3} {'block':14s} {'VALU':>5} {'SALU':>5} {'VMEM':>5} {'LDS':>4}  back edges")
    for i, (lab, ins) in enumerate(blocks):
        v = sum(1 for x in ins if x.startswith('v_'))
        sa = sum(1 for x in ins if x.startswith('s_'))
        vm = sum(1 for x in ins if x.startswith(('global_', 'buffer_', 'flat_', 'scratch_')))
        ds = sum(1 for x in ins if x.startswith('ds_'))
        for k, x in zip(('v', 's', 'vm', 'ds'), (v, sa, vm, ds)):
            tot[k] += x
        back = [x.split()[-1] for x in ins if x.startswith(('s_cbranch', 's_branch'))
                and x.split()[-1] in idx and idx[x.split()[-1]] <= i]
        print(f"{i:3d} {lab:14s} {v:5d} {sa:5d} {vm:5d} {ds:4d}  {'-> ' + ','.join(back) if back else ''}")
    print(f"total: {tot['v']} VALU, {tot['s']} SALU, {tot['vm']} VMEM, {tot['ds']} LDS instructions in {len(blocks)} blocks")


if __name__ == '__main__':
    main()
