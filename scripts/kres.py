#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (read from stdin).
usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python scripts/kres.py [substring]"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark: \s*(Function Name|VGPRs|AGPRs|SGPRs|Occupancy \[waves/SIMD\]|SGPRs Spill|VGPRs Spill|"
                  r"LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                     text=True).stdout.splitlines()
for r, d in zip(rows, dem):
    d = d.replace("(anonymous namespace)::", "").replace("thrs_dev::", "").replace("unsigned int", "u32")
    d = d.split("(")[0]
    if flt and flt not in d:
        continue
    print(f"{d[:60]:60s} V={r.get('VGPRs', '?'):>4} occ={r.get('Occupancy [waves/SIMD]', '?'):>2} "
          f"Sspill={r.get('SGPRs Spill', '?'):>4} Vspill={r.get('VGPRs Spill', '?'):>3}")
