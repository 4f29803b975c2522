#!/bin/bash
# HBM traffic of the policy kernels (run on the GPU box): two separate rocprofv3 passes
# (FETCH_SIZE and WRITE_SIZE cannot share a TCC pass) over scripts/policy_driver.py, summarised
# per kernel as bytes per dispatch with the gfx950 FETCH x2 correction (MI355X_MICROARCH.md).
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for pass in fetch:FETCH_SIZE write:WRITE_SIZE; do
  name=${pass%%:*}; ctr=${pass#*:}
  rm -rf gpurun_out/pmcp_$name
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmcp_$name -o run -- \
    python3 scripts/policy_driver.py 8192 10 > gpurun_out/pmcp_$name.log 2>&1
done
python3 - <<'PY' > gpurun_out/pmc_policy_traffic.json
import csv, glob, json
from collections import defaultdict
out = defaultdict(dict)
for name, ctr, scale in (("fetch", "FETCH_SIZE", 2.0), ("write", "WRITE_SIZE", 1.0)):
    path = glob.glob(f"gpurun_out/pmcp_{name}/**/*counter_collection.csv", recursive=True)[0]
    tot, disp = defaultdict(float), defaultdict(set)
    for row in csv.DictReader(open(path)):
        k = row.get("Kernel_Name", "")
        if "policy_kernel" not in k or row["Counter_Name"] != ctr:
            continue
        key = "actor" if "<50, 300, true>" in k else "critic"
        tot[key] += float(row["Counter_Value"]) * 1024.0 * scale  # KiB -> bytes (x2 for FETCH on gfx950)
        disp[key].add(row.get("Dispatch_Id", ""))
    for key in tot:
        out[key][name + "_bytes_per_dispatch"] = tot[key] / max(1, len(disp[key]))
for key, d in out.items():
    n = 8192
    nin = 50 if key == "actor" else 484
    nout = 20 + 20 if key == "actor" else 1
    d["algorithmic_bytes_per_dispatch"] = n * 4 * (nin + nout + 2 * 5 * 128)  # obs, outputs, carry in + out
print(json.dumps(out, indent=1))
PY
cat gpurun_out/pmc_policy_traffic.json
