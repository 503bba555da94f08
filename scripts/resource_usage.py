#!/usr/bin/env python3
"""Per-kernel VGPR/AGPR/spill/occupancy of a HIP source for gfx950.
usage: python scripts/resource_usage.py <file.hip> [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
       "-ffp-contract=off", "-I/root/repo/include", "-c", src, "-o", "/tmp/ru.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, d = None, {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = cur.split("(")[0]
        d[cur] = {}
        continue
    m = re.search(r"remark: +([A-Za-z /\[\]]+?): (\d+)", line)
    if m and cur:
        d[cur][m.group(1).strip()] = m.group(2)
for k, v in d.items():
    if flt in k:
        keys = ["VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill", "Occupancy [waves/SIMD]",
                "LDS Size [bytes/block]"]
        print(f"{k[:70]:70s} " + " ".join(f"{x.split()[0]}{'_sp' if 'Spill' in x else ''}={v.get(x)}" for x in keys))
