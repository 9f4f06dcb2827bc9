"""Summarise a rocprofv3 collection (profiles/run_profile.sh) into committed profile files.

    python profiles/summarize.py gpurun_out/prof_<tag> <tag>

Writes profiles/<tag>_kernel_stats.csv (the kernel-trace stats), profiles/<tag>_summary.txt and
profiles/pmc_<tag>.json (per kernel: average duration, counters per launch, derived figures). The JSON
records the library's CN_SRC_HASH (cn_version() on the box): bench.py takes `roofline.traffic` from
the newest pmc_*.json whose hash equals the hash of the sources it runs, and reports null otherwise.

HBM bytes follow MI355X_MICROARCH.md § HBM: FETCH_SIZE / WRITE_SIZE are KiB, and on gfx950 FETCH_SIZE
reports 1/2 of the bytes of wide 16-B-per-lane streaming reads; other access widths "are uncalibrated:
calibrate on a known byte count in your own access pattern". The step kernel's accesses are 8 B per lane,
so run_profile.sh also profiles tools/calib_pmc.py (cn_debug_copy64: a known byte count moved with that
shape, as full 64-lane segments and as 48-B per-env segments); the counters are divided by the
calibration's bytes-per-counted-byte of the full-segment shape (`calibration` in the JSON) and both the
guide's 16-B correction (x2 on FETCH) and the calibrated figure are recorded; `hbm_bytes_per_launch` is
the calibrated one when a calibration is present. Infinity-Cache hits count as fabric traffic here.
Windows: the bench line printed by the profiled run names its timed launch windows (config.launches and
steady_state.launches = [first launch after cn_reset, count]); every figure is also computed over exactly
those dispatches of the kernel (`windows` in the JSON: the kernel-trace average duration of those launches
and their counters), which is what bench.py reports next to the window it timed.
VALU-issue fraction = SQ_INSTS_VALU x 2 cycles (one wave64 VALU instruction occupies a SIMD's issue for
2 cycles; f64 FMA/MUL/ADD take 4, transcendentals 8 on f64 per the microarchitecture guide's
issue-cost table) / (1024 SIMDs x kernel cycles at 2.4 GHz).
"""
import csv
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CLOCK_HZ = 2.4e9
SIMDS = 1024


def find(d, pat):
    f = sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))
    return f[0] if f else None


def counters(path):
    """{kernel: {counter: [per-dispatch values]}} from a counter_collection.csv"""
    out = {}
    if not path:
        return out
    for row in csv.DictReader(open(path)):
        k = row.get("Kernel_Name", "")
        out.setdefault(k, {}).setdefault(row["Counter_Name"], {})
        d = out[k][row["Counter_Name"]]
        disp = row.get("Dispatch_Id", str(len(d)))
        d[disp] = d.get(disp, 0.0) + float(row["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in out.items()}


def dispatch_series(path):
    """{kernel: {counter: [value per dispatch in dispatch order]}} from a counter_collection.csv"""
    out = {}
    if not path:
        return out
    for row in csv.DictReader(open(path)):
        k = row.get("Kernel_Name", "")
        d = out.setdefault(k, {}).setdefault(row["Counter_Name"], {})
        disp = int(row.get("Dispatch_Id", len(d)))
        d[disp] = d.get(disp, 0.0) + float(row["Counter_Value"])
    return {k: {c: [v[i] for i in sorted(v)] for c, v in cs.items()} for k, cs in out.items()}


def trace_durations(path):
    """{kernel: [duration ns per dispatch in dispatch order]} from a kernel_trace.csv"""
    out = {}
    if not path:
        return out
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    for r in rows:
        out.setdefault(r["Kernel_Name"], []).append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return out


def bench_windows(out):
    """[(name, first, count)] of the launch windows the profiled bench line reports (bench_kt.log)."""
    p = os.path.join(out, "bench_kt.log")
    if not os.path.exists(p):
        return []
    for ln in open(p):
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            doc = json.loads(ln)
            w = []
            if "launches" in doc.get("config", {}):
                w.append(("main",) + tuple(doc["config"]["launches"]))
            if "launches" in doc.get("steady_state", {}):
                w.append(("steady",) + tuple(doc["steady_state"]["launches"]))
            return w
    return []


def derive(d, c, dur, cal):
    """HBM bytes, VALU issue and wave figures of counter means `c` over launches of mean duration `dur`."""
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        d["hbm_bytes_guide_16B"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
        d["hbm_bytes_per_launch"] = d["hbm_bytes_guide_16B"]
        if "FETCH_SIZE" in cal and "WRITE_SIZE" in cal:
            d["hbm_read_bytes"] = c["FETCH_SIZE"] * 1024.0 / cal["FETCH_SIZE"]["seg64"]
            d["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024.0 / cal["WRITE_SIZE"]["seg64"]
            d["hbm_bytes_per_launch"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
    if dur and "SQ_INSTS_VALU" in c:
        d["valu_issue_frac"] = c["SQ_INSTS_VALU"] * 2.0 / (SIMDS * dur * 1e-9 * CLOCK_HZ)
    if "SQ_WAVE_CYCLES" in c and "SQ_ACTIVE_INST_ANY" in c:
        d["active_inst_frac"] = c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"]
        d["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
    return d


def short(name):
    return name.split("(")[0].replace("void ", "")[:48]


def main():
    out, tag = sys.argv[1], sys.argv[2]
    ver = open(os.path.join(out, "lib_version.txt")).read().strip() if os.path.exists(
        os.path.join(out, "lib_version.txt")) else ""
    src_hash = ver.split("CN_SRC_HASH=", 1)[1][:64] if "CN_SRC_HASH=" in ver else None
    args = open(os.path.join(out, "bench_args.txt")).read().strip() if os.path.exists(
        os.path.join(out, "bench_args.txt")) else ""
    stats = find(os.path.join(out, "kt"), "*kernel_stats.csv")
    lines = ["rocprofv3 collection %s: bench.py %s" % (tag, args), "library: %s" % ver, ""]
    res = {}
    if stats:
        rows = list(csv.DictReader(open(stats)))
        with open(os.path.join(HERE, "%s_kernel_stats.csv" % tag), "w") as f:
            w = csv.DictWriter(f, fieldnames=rows[0].keys())
            w.writeheader()
            w.writerows(rows)
        lines.append("--kernel-trace --stats")
        for r in rows:
            res.setdefault(r["Name"], {})["avg_duration_ns"] = float(r["AverageNs"])
            res[r["Name"]]["calls"] = int(r["Calls"])
            lines.append("  %-48s calls=%-6s avg=%10.1f ns  min=%10.1f  max=%10.1f  total%%=%s" % (
                short(r["Name"]), r["Calls"], float(r["AverageNs"]), float(r["MinNs"]), float(r["MaxNs"]),
                r.get("Percentage", "")))
    merged = {}
    for p in ("fetch", "write", "sq1", "sq2", "tcc"):
        for k, cs in counters(find(os.path.join(out, p), "*counter_collection.csv")).items():
            for c, v in cs.items():
                merged.setdefault(k, {})[c] = sum(v) / len(v)
    cal = {}
    for p, cname in (("calfetch", "FETCH_SIZE"), ("calwrite", "WRITE_SIZE")):
        for k, cs in counters(find(os.path.join(out, p), "*counter_collection.csv")).items():
            if "copy64" in k and cname in cs:
                v = cs[cname]
                h = len(v) // 2
                nbytes = float(8 << 23)   # tools/calib_pmc.py: 8 M doubles each way
                cal[cname] = {"seg64": sum(v[:h]) / h * 1024.0 / nbytes, "seg6": sum(v[h:]) / (len(v) - h) * 1024.0 / nbytes}
    if cal:
        lines.append("calibration (counted bytes / moved bytes, cn_debug_copy64, 8 B per lane): %s" % json.dumps(cal))
        lines.append("")
    lines.append("")
    lines.append("counters per launch (mean over dispatches)")
    for k in sorted(merged):
        d = res.setdefault(k, {})
        d["counters"] = merged[k]
        c = merged[k]
        lines.append("  %s" % short(k))
        for n in sorted(c):
            lines.append("    %-28s %.6g" % (n, c[n]))
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            d["hbm_bytes_guide_16B"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
            d["hbm_bytes_per_launch"] = d["hbm_bytes_guide_16B"]
            lines.append("    => HBM bytes/launch, guide's 16-B correction (2*FETCH_SIZE + WRITE_SIZE) = %.0f"
                         % d["hbm_bytes_guide_16B"])
            if "FETCH_SIZE" in cal and "WRITE_SIZE" in cal:
                rd = c["FETCH_SIZE"] * 1024.0 / cal["FETCH_SIZE"]["seg64"]
                wr = c["WRITE_SIZE"] * 1024.0 / cal["WRITE_SIZE"]["seg64"]
                d["hbm_read_bytes"], d["hbm_write_bytes"] = rd, wr
                d["hbm_bytes_per_launch"] = rd + wr
                lines.append("    => HBM bytes/launch, calibrated on the 8-B shape: read %.0f + write %.0f = %.0f"
                             % (rd, wr, rd + wr))
        dur = d.get("avg_duration_ns")
        if dur and "SQ_INSTS_VALU" in c:
            cyc = dur * 1e-9 * CLOCK_HZ
            d["valu_issue_frac"] = c["SQ_INSTS_VALU"] * 2.0 / (SIMDS * cyc)
            lines.append("    => VALU-issue fraction (INSTS_VALU x 2 cyc / (1024 SIMD x %.0f cyc)) = %.4f" % (
                cyc, d["valu_issue_frac"]))
        if "SQ_WAVE_CYCLES" in c and "SQ_ACTIVE_INST_ANY" in c:
            d["active_inst_frac"] = c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"]
            d["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
            lines.append("    => per-wave: issuing %.3f, parked on waitcnt/barrier %.3f of wave cycles" % (
                d["active_inst_frac"], d["wait_any_frac"]))
    wins = bench_windows(out)
    durs = trace_durations(find(os.path.join(out, "kt"), "*kernel_trace.csv"))
    series = {}
    for p in ("fetch", "write", "sq1", "sq2", "tcc"):
        for k, cs in dispatch_series(find(os.path.join(out, p), "*counter_collection.csv")).items():
            series.setdefault(k, {}).update(cs)
    if wins:
        lines.append("")
        lines.append("timed windows of the profiled bench line (launches after cn_reset)")
    for k in sorted(durs):
        if "cn_step_kernel" not in k or not wins:
            continue
        dd = durs[k]
        for name, first, count in wins:
            # launches per env step (c5: one per group) from the total dispatch count of the run
            steps_total = max(f + n for _, f, n in wins)
            m = max(1, len(dd) // steps_total) if len(dd) % steps_total == 0 else 1
            sl = slice(first * m, (first + count) * m)
            if len(dd[sl]) != count * m:
                continue
            w = {"name": name, "first": first, "count": count, "launches_per_step": m,
                 "avg_duration_ns": sum(dd[sl]) / len(dd[sl])}
            cm = {}
            for cname, vals in series.get(k, {}).items():
                if len(vals) == len(dd):
                    cm[cname] = sum(vals[sl]) / len(vals[sl])
            w["counters"] = cm
            derive(w, cm, w["avg_duration_ns"], cal)
            res.setdefault(k, {}).setdefault("windows", []).append(w)
            lines.append("  %s %-6s launches %d..%d: avg %.1f ns, HBM %s B/launch, VALU issue %s" % (
                short(k), name, first + 1, first + count, w["avg_duration_ns"],
                "%.0f" % w["hbm_bytes_per_launch"] if "hbm_bytes_per_launch" in w else "-",
                "%.4f" % w["valu_issue_frac"] if "valu_issue_frac" in w else "-"))
    doc = {"tag": tag, "bench_args": args, "lib_version": ver, "lib_src_hash": src_hash, "calibration": cal,
           "kernels": res}
    json.dump(doc, open(os.path.join(HERE, "pmc_%s.json" % tag), "w"), indent=1)
    open(os.path.join(HERE, "%s_summary.txt" % tag), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
