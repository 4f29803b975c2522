"""Per-kernel registers / spills / LDS of zb_engine.hip as hipcc reports them
(-Rpass-analysis=kernel-resource-usage), one line per kernel. CPU only (cross-compiles).

    python scripts/kernel_resources.py [extra hipcc flags]
"""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ksim-gym-zbot_amd", "csrc")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(ROOT, "include"),
       "-fno-signed-zeros", "-freciprocal-math", "-fno-math-errno", "-fapprox-func", "-fno-slp-vectorize",
       "-Rpass-analysis=kernel-resource-usage", "-c", "-o", "/tmp/zb_engine_res.o", os.path.join(CSRC, "zb_engine.hip"),
       *sys.argv[1:]]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, {}
for line in err.splitlines():
    m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, r in rows.items():
    short = re.sub(r"_ZN2zb\d+", "", name).replace("EEEvNS_8StepArgsE", "").replace("ILi", "<").replace("ELi", ",")
    print(f"{short:34s} VGPR {r.get('VGPRs', '?'):>4} AGPR {r.get('AGPRs', '?'):>3} vspill {r.get('VGPRs Spill', '?'):>3} "
          f"sspill {r.get('SGPRs Spill', '?'):>4} scratch {r.get('ScratchSize [bytes/lane]', '?'):>4} "
          f"occ {r.get('Occupancy [waves/SIMD]', '?')} lds {r.get('LDS Size [bytes/block]', '?')}")
