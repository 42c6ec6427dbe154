#!/usr/bin/env python3
"""Kernel resource table of one HIP source (gfx950): VGPRs, spills, scratch,
occupancy per kernel, from hipcc's kernel-resource-usage remarks.

  python tools/kres.py gsky_amd/csrc/band_f32.hip [name-substring]
"""
import re
import subprocess
import sys

src = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-x", "hip",
       "-c", src, "-o", "/tmp/kres.o", "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|VGPRs Spill|SGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k.split(" [")[0]] = v
for name, r in rows.items():
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    if sub and sub not in dem:
        continue
    short = re.sub(r"\(.*", "", dem).replace("gsky::", "").replace("(anonymous namespace)::", "")
    print("%-70s vgpr %4s spill %4s sspill %4s scratch %4s occ %s lds %s" % (
        short[:70], r.get("VGPRs"), r.get("VGPRs Spill"), r.get("SGPRs Spill"), r.get("ScratchSize"),
        r.get("Occupancy"), r.get("LDS Size")))
