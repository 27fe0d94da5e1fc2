#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy report of kc_kernels.hip for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage). Usage: kres.py [name-filter]"""
import re, subprocess, sys
src = "/root/repo/kmer-counter_amd/csrc/kc_kernels.hip"
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src, "-o", "/tmp/kres.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, cwd="/tmp").stderr
cur = None; rows = {}
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m: continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip(); rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1); rows[cur][k.strip()] = v.strip()
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for name, d in rows.items():
    if flt in name:
        print(f"{name[:60]:60s} vgpr={d.get('VGPRs')} agpr={d.get('AGPRs')} sgpr={d.get('TotalSGPRs')} occ={d.get('Occupancy [waves/SIMD]')} lds={d.get('LDS Size [bytes/block]')} vspill={d.get('VGPRs Spill')} sspill={d.get('SGPRs Spill')}")
