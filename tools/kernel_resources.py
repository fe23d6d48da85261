#!/usr/bin/env python3
"""Per-kernel VGPR / scratch / occupancy table of one HIP source file, from
hipcc -Rpass-analysis=kernel-resource-usage (gfx950).  A non-zero scratch
size means private memory traffic (spills or dynamically indexed arrays).

usage: python tools/kernel_resources.py csrc/ace_pairs_mm.hip [name-filter]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def table(src, filt=""):
    src = os.path.join(ROOT, "additivecausalexpansion_amd", src) if not os.path.isabs(src) else src
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-c", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = subprocess.run(["c++filt", m.group(1)], capture_output=True,
                                  text=True).stdout.strip()
            cur = {"name": re.sub(r"\(.*", "", name)}
            rows.append(cur)
            continue
        m = re.search(r"(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"VGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).split(" [")[0]] = int(m.group(2))
    return [x for x in rows if filt in x["name"]]


if __name__ == "__main__":
    for x in table(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""):
        print(f"{x['name']:55s} vgpr {x.get('VGPRs', 0):4d} scratch {x.get('ScratchSize', 0):4d} "
              f"spill {x.get('VGPRs Spill', 0):3d} occ {x.get('Occupancy', 0)}")
