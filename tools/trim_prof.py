#!/usr/bin/env python3
"""Shrink a tools/profile.sh output directory in place (the box's gpurun_out/ comes back only under 64 MiB):
per-dispatch CSVs (kernel trace, counter collection) keep their header and the rows of the persistent path
kernels (k_persist / k_coop / k_fan / k_split / k_pool), which tools/pmc_traffic.py reads; the stats files stay.
usage: tools/trim_prof.py gpurun_out/prof_<tag>"""
import os
import sys

KEEP = ("k_persist", "k_coop", "k_fan", "k_split", "k_pool")
for root, _, files in os.walk(sys.argv[1]):
    for f in files:
        if not (f.endswith("_kernel_trace.csv") or f.endswith("_counter_collection.csv")):
            continue
        p = os.path.join(root, f)
        with open(p) as fh:
            lines = fh.readlines()
        keep = lines[:1] + [l for l in lines[1:] if any(k in l for k in KEEP)]
        with open(p, "w") as fh:
            fh.writelines(keep)
