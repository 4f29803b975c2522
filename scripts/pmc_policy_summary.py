"""Summarise scripts/pmc_policy.sh: per policy kernel, the matrix-core busy fraction
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), averaged over dispatches."""

import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
path = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)[0]
per = defaultdict(lambda: defaultdict(float))
seen = defaultdict(set)
for row in csv.DictReader(open(path)):
    name = row.get("Kernel_Name", "")
    if "policy_kernel" not in name:
        continue
    key = "actor" if "<50, 300, true>" in name else "critic"
    d = row.get("Dispatch_Id", row.get("Correlation_Id", ""))
    per[key][row["Counter_Name"]] += float(row["Counter_Value"])
    seen[key].add(d)
out = {}
for key, c in per.items():
    nd = max(1, len(seen[key]))
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0 / nd
    busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / nd
    out[key] = {"dispatches": nd, "gpu_cycles_per_dispatch": cyc, "mfma_busy_cycles_per_dispatch": busy,
                "mfma_busy_frac": busy / (cyc * 1024) if cyc else None,
                "raw_totals": dict(c)}
print(json.dumps(out, indent=1))
