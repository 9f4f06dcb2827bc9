"""Per-kernel averages of the counter passes of tools/pmc_gru.sh (GRU sequence kernels)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    print("==", d)
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            if "gru" not in k:
                continue
            mm = re.search(r"cn_gru_\w+(<[^>]*>)?", k)
            name = mm.group(0) if mm else k[:60]
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "gru" in row["Name"]:
                mm = re.search(r"cn_gru_\w+(<[^>]*>)?", row["Name"])
                print("  kt %-60s calls %6s avg %8.1f us" % (mm.group(0) if mm else row["Name"][:60], row["Calls"],
                                                            float(row["AverageNs"]) / 1e3))
    for name, cs in acc.items():
        print("  %s" % name)
        for c, v in sorted(cs.items()):
            print("     %-28s %14.4g (mean over %d dispatches)" % (c, sum(v) / len(v), len(v)))
