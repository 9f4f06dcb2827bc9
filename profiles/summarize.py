"""Summarise rocprofv3 CSV output into committed profile files.

    python profiles/summarize.py <rocprof out dir> <tag>

Writes profiles/<tag>_kernel_stats.csv (copy of the kernel stats), profiles/<tag>_summary.txt and
profiles/pmc_step_kernel.json (HBM bytes per cn_step_kernel launch, read by bench.py as
roofline.traffic). HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reads 1/2 of the bytes of wide coalesced streaming reads, so the read side is
doubled (that correction is calibrated for 16-B-per-lane streaming loads; this kernel mixes 8-B
loads, so the absolute figure carries that caveat — ratios are unaffected).
"""
import csv
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def find(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return f[0] if f else None


def per_kernel_counter(path, counter):
    vals = {}
    if not path:
        return vals
    for row in csv.DictReader(open(path)):
        if row.get("Counter_Name") != counter:
            continue
        k = row.get("Kernel_Name", "")
        vals.setdefault(k, []).append(float(row["Counter_Value"]))
    return vals


def main():
    out, tag = sys.argv[1], sys.argv[2]
    stats = find(os.path.join(out, "kt"), "*kernel_stats.csv")
    lines = ["rocprofv3 --kernel-trace --stats  (bench.py --steps 400 --warmup 40, 4096 envs x 10 humans, C2)", ""]
    avg = {}
    if stats:
        rows = list(csv.DictReader(open(stats)))
        with open(os.path.join(HERE, "%s_kernel_stats.csv" % tag), "w") as f:
            w = csv.DictWriter(f, fieldnames=rows[0].keys())
            w.writeheader()
            w.writerows(rows)
        for r in rows:
            name = r["Name"]
            avg[name] = float(r["AverageNs"])
            lines.append("%-40s calls=%-6s avg=%10.1f ns  min=%10.1f  max=%10.1f  total%%=%s" % (
                name[:40], r["Calls"], float(r["AverageNs"]), float(r["MinNs"]), float(r["MaxNs"]),
                r.get("Percentage", "")))
    fetch = per_kernel_counter(find(os.path.join(out, "fetch"), "*counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel_counter(find(os.path.join(out, "write"), "*counter_collection.csv"), "WRITE_SIZE")
    lines.append("")
    pmc = {}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(k, [0])) / max(len(fetch.get(k, [1])), 1)
        w = sum(write.get(k, [0])) / max(len(write.get(k, [1])), 1)
        hbm = (2.0 * f + w) * 1024.0
        pmc[k] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w, "hbm_bytes_per_launch": hbm}
        lines.append("%-40s FETCH_SIZE=%10.1f KiB  WRITE_SIZE=%10.1f KiB  HBM(2*fetch+write)=%12.0f B/launch" % (
            k[:40], f, w, hbm))
    step = [k for k in pmc if "cn_step_kernel" in k]
    if step:
        d = dict(pmc[step[0]])
        d["kernel"] = step[0]
        d["avg_duration_ns"] = next((v for n, v in avg.items() if "cn_step_kernel" in n), None)
        d["source"] = "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes (%s)" % tag
        json.dump(d, open(os.path.join(HERE, "pmc_step_kernel.json"), "w"), indent=1)
    open(os.path.join(HERE, "%s_summary.txt" % tag), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
