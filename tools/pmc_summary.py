#!/usr/bin/env python3
"""Summarise the PMC passes of tools/gpu_pmc.sh per kernel (per launch) and
write profiles/<name> (default pmc_count_kmers.json, which bench.py's
roofline.traffic reads) — args: out_dir reads k [name].

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (FETCH_SIZE is in KiB and
reports half the bytes of wide streaming reads on gfx950, MI355X_MICROARCH.md
"HBM"; WRITE_SIZE is exact for wide streaming stores)."""
import collections
import csv
import glob
import json
import os
import sys

out, reads = sys.argv[1], int(sys.argv[2])
tot = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(set)
for f in glob.glob(os.path.join(out, "g*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[(name, r["Counter_Name"])].add(r["Dispatch_Id"])
rows = []
for name, d in tot.items():
    n = max(len(launches[(name, c)]) for c in d)
    per = {c: v / max(1, len(launches[(name, c)])) for c, v in d.items()}
    rows.append((name, n, per))
rows.sort(key=lambda x: -x[2].get("SQ_WAVE_CYCLES", 0) * x[1])
for name, n, per in rows:
    if per.get("SQ_WAVE_CYCLES", 0) * n < 1e8 and per.get("WRITE_SIZE", 0) < 1e5:
        continue
    fetch = 2 * per.get("FETCH_SIZE", 0) * 1024
    write = per.get("WRITE_SIZE", 0) * 1024
    wc = per.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{name[:70]:70s} launches={n}")
    print(f"   HBM read {fetch/1e9:.2f} GB  write {write/1e9:.2f} GB  per launch")
    print("   wave-cycle split: " + " ".join(f"{k[3:]}={per.get(k,0)/wc:.2f}" for k in
                                            ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                             "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM",
                                             "SQ_ACTIVE_INST_SCA")))
    print("   insts: " + " ".join(f"{k[3:]}={per.get(k,0):.3g}" for k in
                                 ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
                                  "SQ_INSTS_VMEM_WR", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
                                  "SQ_WAIT_INST_LDS", "GRBM_GUI_ACTIVE")))
k = int(sys.argv[3]) if len(sys.argv) > 3 else 31
name_out = sys.argv[4] if len(sys.argv) > 4 else "pmc_count_kmers.json"
W = (k + 31) // 32
rec = {"reads_per_gpu": reads, "k": k, "kernels": {},
       "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, --kernel-trace only "
                 "(tools/gpu_pmc.sh); HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024), "
                 "per the gfx950 FETCH_SIZE correction in MI355X_MICROARCH.md; keyed by the kernel's "
                 "short name (template arguments, no spaces)"}


def short(name):
    n = name.split("(")[0]
    n = n.replace("void ", "").replace("kc::", "")
    return n.replace(" ", "")


for name, n, per in rows:
    rd = 2 * per.get("FETCH_SIZE", 0) * 1024
    wr = per.get("WRITE_SIZE", 0) * 1024
    if rd + wr == 0:
        continue
    rec["kernels"][short(name)] = {"kernel": name, "bytes_per_launch": rd + wr, "read_bytes": rd,
                                   "write_bytes": wr, "launches": n}
os.makedirs("profiles", exist_ok=True)
json.dump(rec, open(os.path.join("profiles", name_out), "w"), indent=1)
json.dump(rec, open(os.path.join(out, name_out), "w"), indent=1)  # travels back from the box
print("wrote profiles/" + name_out, {t: round(v["bytes_per_launch"] / 1e9, 2) for t, v in rec["kernels"].items()
                                             if v["bytes_per_launch"] > 1e8})
