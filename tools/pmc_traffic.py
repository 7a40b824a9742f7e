#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/: kernel-trace stats (markdown) and the PMC counters of the
bench's production kernel (profiles/pmc_traffic.json, read by bench.py for its roofline fields).

The production kernel is the one with the largest total time in the trace. The entry is keyed by the bench
line's own pmc_key (scene, size, spp, output, frames per launch, ranks: read from the trace pass's JSON line,
so nothing is rescaled to another launch size) and records the md5 of the librt_hip.so the box ran
(profile.sh writes lib_md5.txt): bench.py reports the counters as measured only for that build.

traffic per launch = 2 x FETCH_SIZE + WRITE_SIZE (kB -> bytes): MI355X_MICROARCH.md §HBM — on gfx950
FETCH_SIZE reports half the bytes of 16-B-per-lane reads (the kernel's node/triangle loads are float4
per lane); WRITE_SIZE reads exactly for 16-B stores. Counters come from separate --pmc passes.
usage: tools/pmc_traffic.py gpurun_out/prof_<tag> <round-tag>
"""
import csv
import re
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_SIMD, N_XCD = 1024, 8  # MI355X: 256 CUs x 4 SIMDs, 8 XCDs (GRBM_GUI_ACTIVE counts every XCD)


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def per_kernel(path, counter):
    out = {}
    for r in rows(path):
        if r["Counter_Name"] == counter:
            out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return out


def find(d, sub):
    for k, v in d.items():
        if sub in k:
            return k, v
    return None, None


def bench_line(prof):
    """the bench's JSON line of the trace pass (profile.sh keeps its stdout in trace.log)"""
    for l in open(os.path.join(prof, "trace.log")):
        if l.startswith("{"):
            return json.loads(l)
    raise SystemExit(f"{prof}/trace.log has no bench line")


def main():
    prof, tag = sys.argv[1], sys.argv[2]
    line = bench_line(prof)
    rf = line["roofline"]
    key, frames = rf["pmc_key"], rf["frames_per_launch"]
    cmd = open(os.path.join(prof, "cmd.txt")).read().strip() if os.path.exists(os.path.join(prof, "cmd.txt")) else "bench.py"
    lib_md5 = open(os.path.join(prof, "lib_md5.txt")).read().split()[0]
    pdir = os.path.join(ROOT, "profiles")
    os.makedirs(pdir, exist_ok=True)
    # kernel trace stats
    stats = rows(os.path.join(prof, "trace", "run_kernel_stats.csv"))
    # (the counting launch, RT_FLAG_COUNTERS, is a k_persist<MAXB, false, true, ...> instantiation: never the product)
    PROD = max((r for r in stats if not re.search(r"k_persist<\d+, false, true,", r["Name"])),
               key=lambda r: float(r["TotalDurationNs"]))["Name"]
    lines = [f"# rocprofv3 --kernel-trace --stats ({tag}, {key})", "",
             f"command: `rocprofv3 --kernel-trace --stats -- {cmd}` ({frames} frames per launch; librt_hip.so md5 "
             f"{lib_md5}); bench line: {line['value']:.0f} Mrays/s, HIP-event kernel {rf['kernel_ms']:.3f} ms per launch",
             "", "| kernel | calls | total ms | avg ms | min ms | max ms | % |", "|---|---|---|---|---|---|---|"]
    for r in stats:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                     f"{float(r['AverageNs']) / 1e6:.4f} | {float(r['MinNs']) / 1e6:.4f} | "
                     f"{float(r['MaxNs']) / 1e6:.4f} | {float(r['Percentage']):.2f} |")
    # per-dispatch durations of the production kernel, grouped by grid size: the first frame of a scene
    # is rt_render's autotuning frame (each candidate grid 3 times), the frames after it use one grid
    tr = os.path.join(prof, "trace", "run_kernel_trace.csv")
    groups = {}
    if os.path.exists(tr):
        for r in rows(tr):
            if PROD in r["Kernel_Name"]:
                groups.setdefault(int(r["Grid_Size_X"]) // 256, []).append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    prod_grid = max(groups, key=lambda g: len(groups[g])) if groups else None
    if groups:
        lines += ["", f"## `{PROD}` per dispatch (kernel trace), by grid", "",
                  "| workgroups | launches | median ms | mean ms |", "|---|---|---|---|"]
        for g in sorted(groups):
            v = groups[g]
            lines.append(f"| {g}{' (frames after tuning)' if g == prod_grid else ''} | {len(v)} | "
                         f"{statistics.median(v):.4f} | {statistics.mean(v):.4f} |")
    fetch = per_kernel(os.path.join(prof, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(prof, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    kf, vf = find(fetch, PROD)
    kw, vw = find(write, PROD)
    res = None
    if vf and vw:
        f_kb, w_kb = statistics.median(vf), statistics.median(vw)
        hbm = 2 * f_kb * 1024 + w_kb * 1024
        _, avg = find({r["Name"]: float(r["AverageNs"]) for r in stats}, PROD)
        res = {"kernel": kf, "launches": len(vf), "fetch_size_kb_median": f_kb, "write_size_kb_median": w_kb,
               "fetch_bytes_per_launch": 2 * f_kb * 1024, "write_bytes_per_launch": w_kb * 1024,
               "hbm_bytes_per_launch": hbm, "frames_per_launch": frames, "lib_md5": lib_md5, "command": cmd,
               "bench_kernel_ms": rf["kernel_ms"], "trace_avg_ms": avg / 1e6 if avg else None,
               "trace_median_ms_production_grid": statistics.median(groups[prod_grid]) if groups else None,
               "production_grid_workgroups": prod_grid,
               "hbm_gbs_at_trace_avg": hbm / (avg / 1e9) / 1e9 if avg else None,
               "rule": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md §HBM, gfx950 FETCH_SIZE halving)",
               "source": f"profiles/{tag}_kernel_stats.md, profiles/{tag}/*_summary.csv", "round": tag}
        lines += ["", f"## HBM traffic of `{PROD}` (PMC, separate passes)", "",
                  f"- FETCH_SIZE median {f_kb:.0f} kB/launch, WRITE_SIZE median {w_kb:.0f} kB/launch",
                  f"- traffic = 2 x FETCH + WRITE = {hbm / 1e6:.1f} MB/launch"
                  + (f" = {res['hbm_gbs_at_trace_avg']:.1f} GB/s at the trace average" if avg else "")]
    # other PMC passes, if present: per-kernel medians
    for sub in ("pmc_sq", "pmc_l2", "pmc_valu"):
        p = os.path.join(prof, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        agg = {}
        for r in rows(p):
            if PROD in r["Kernel_Name"]:
                agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        if agg:
            lines += ["", f"### {sub} (`{PROD}`, median per launch)", ""]
            lines += [f"- {k}: {statistics.median(v):.4g}" for k, v in sorted(agg.items())]
            med = {k: statistics.median(v) for k, v in agg.items()}
            if res is not None and "SQ_ACTIVE_INST_VALU" in med and "GRBM_GUI_ACTIVE" in med:
                # SQ_ACTIVE_INST_VALU counts quad-cycles per SIMD; GRBM_GUI_ACTIVE the cycles of every XCD
                cyc = med["GRBM_GUI_ACTIVE"] / N_XCD
                # a wave64 fp32 VALU instruction issues in 2 cycles on a CDNA4 SIMD (32 lanes per clock: 157 TF fp32
                # vector = 256 CUs x 4 SIMDs x 32 lanes x 2 flops x 2.4 GHz)
                res["valu_issue_frac"] = med["SQ_INSTS_VALU"] * 2 / (N_SIMD * cyc)
                res["valu_issue_rule"] = "SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)"
                res["sq_insts_valu_per_launch"] = med.get("SQ_INSTS_VALU")
            if res is not None and "TCP_TCC_READ_REQ_sum" in med:
                res["l2_read_requests_per_launch"] = med["TCP_TCC_READ_REQ_sum"]
                res["l2_read_bytes_per_launch"] = 64 * med["TCP_TCC_READ_REQ_sum"]
                res["l2_read_rule"] = "TCP_TCC_READ_REQ_sum x 64 B (L1 -> L2 read requests)"
                if "TCC_HIT_sum" in med and "TCC_MISS_sum" in med:
                    res["l2_hit_rate"] = med["TCC_HIT_sum"] / max(1.0, med["TCC_HIT_sum"] + med["TCC_MISS_sum"])
            if res is not None and "SQ_WAIT_ANY" in med and "SQ_WAVE_CYCLES" in med:
                res["wave_wait_frac"] = med["SQ_WAIT_ANY"] / max(1.0, med["SQ_WAVE_CYCLES"])
    # CSV copies under profiles/<tag>/: the trace stats as rocprofv3 wrote them, the PMC passes as
    # per-kernel medians (kernel, counter, launches, median, min, max)
    cdir = os.path.join(pdir, tag)
    os.makedirs(cdir, exist_ok=True)
    with open(os.path.join(cdir, "bench_line.json"), "w") as f:  # the trace pass's own bench line
        f.write(json.dumps(line) + "\n")
    os.makedirs(cdir, exist_ok=True)
    shutil.copyfile(os.path.join(prof, "trace", "run_kernel_stats.csv"), os.path.join(cdir, "kernel_stats.csv"))
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_l2", "pmc_valu"):
        p = os.path.join(prof, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        agg = {}
        for r in rows(p):
            agg.setdefault((r["Kernel_Name"], r["Counter_Name"]), []).append(float(r["Counter_Value"]))
        with open(os.path.join(cdir, f"{sub}_summary.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "counter", "launches", "median", "min", "max"])
            for (k, c), v in sorted(agg.items()):
                w.writerow([k, c, len(v), statistics.median(v), min(v), max(v)])
    if res:
        tj_path = os.path.join(pdir, "pmc_traffic.json")
        tj = json.load(open(tj_path)) if os.path.exists(tj_path) else {}
        tj[key] = res
        json.dump(tj, open(tj_path, "w"), indent=1)
    with open(os.path.join(pdir, f"{tag}_kernel_stats.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))
    if res:
        print(json.dumps(res))


if __name__ == "__main__":
    main()
