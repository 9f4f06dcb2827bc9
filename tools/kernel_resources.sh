#!/bin/bash
# Per-kernel register / spill / LDS / occupancy report of the HIP sources (compile-only, no GPU):
#   bash tools/kernel_resources.sh [extra hipcc flags]
R=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result \
  -c --offload-device-only -Rpass-analysis=kernel-resource-usage "$@" "$R/crowdnav_dsrnn_amd/csrc/cn_engine.hip" \
  -o /tmp/cn_res.o 2>&1 | sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass.*//' | python3 -c '
import sys
rows, cur = [], None
for l in sys.stdin:
    l = l.strip()
    if l.startswith("Function Name:"):
        cur = {"name": l.split(":", 1)[1].strip()}; rows.append(cur)
    elif cur is not None and ":" in l:
        k, v = l.split(":", 1); cur[k.strip()] = v.strip()
keys = ["VGPRs", "AGPRs", "SGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]", "LDS Size [bytes/block]", "Occupancy [waves/SIMD]"]
print("%-48s" % "kernel" + "".join("%10s" % k.split()[0][:9] + ("sp" if "Spill" in k else "") for k in keys))
for r in rows:
    print("%-48s" % r["name"][:48] + "".join("%10s" % r.get(k, "-") for k in keys))
'
