#!/usr/bin/env python3
"""Median per-dispatch PMC values per kernel from a tools/pmc_ab.sh run.
usage: python tools/pmc_summary.py gpurun_out/pmc_<tag>"""
import csv
import glob
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    vals = {}
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0][:110]
                vals.setdefault(k, {}).setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
                vals[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, cs in sorted(vals.items()):
        if not any(x in k for x in ("k_persist", "k_coop", "k_split")):
            continue
        print(k)
        med = {c: statistics.median(v.values()) for c, v in cs.items()}
        for c, v in sorted(med.items()):
            print(f"   {c:32s} {v:.4g}")
        if "SQ_WAIT_ANY" in med and "SQ_WAVE_CYCLES" in med:
            print(f"   wait_any/wave_cycles            {med['SQ_WAIT_ANY'] / med['SQ_WAVE_CYCLES']:.3f}")
        if "TCP_TCC_READ_REQ_LATENCY_sum" in med:
            print(f"   mean L2 read latency (cycles)   {med['TCP_TCC_READ_REQ_LATENCY_sum'] / med['TCP_TCC_READ_REQ_sum']:.1f}")
        if "SQ_INSTS_VALU" in med and "SQ_WAVES" in med:
            print(f"   VALU insts per wave             {med['SQ_INSTS_VALU'] / med['SQ_WAVES']:.4g}")


if __name__ == "__main__":
    main()
