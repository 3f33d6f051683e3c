"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/*/run_counter_collection.csv) per kernel:
average counter value per dispatch, plus derived ratios."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
pat = sys.argv[2] if len(sys.argv) > 2 else "dec_mfma_kernel"
vals = defaultdict(list)
for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
avg = {c: sum(v) / len(v) for c, v in vals.items()}
for c in sorted(avg):
    print(f"{c:28s} {avg[c]:.4e}  (n={len(vals[c])})")
d = {}
if "SQ_WAVE_CYCLES" in avg:
    wc = avg["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in avg:
            d[k + "/WAVE_CYCLES"] = avg[k] / wc
if "GRBM_GUI_ACTIVE" in avg:
    d["GRBM_GUI_ACTIVE_per_xcd"] = avg["GRBM_GUI_ACTIVE"] / 8
if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
    # MFMA busy cycles summed over SIMDs vs available SIMD-cycles (1024 SIMDs x XCD-avg clocks)
    d["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * avg["GRBM_GUI_ACTIVE"] / 8)
if "FETCH_SIZE" in avg:
    d["hbm_read_bytes_x2_corrected"] = avg["FETCH_SIZE"] * 1024 * 2
if "WRITE_SIZE" in avg:
    d["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
if "TCC_EA0_RDREQ_sum" in avg:
    d["ea_rd_bytes_64B"] = avg["TCC_EA0_RDREQ_sum"] * 64
    d["ea_wr_bytes_64B"] = avg.get("TCC_EA0_WRREQ_sum", 0) * 64
if "TCC_HIT_sum" in avg:
    d["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
print(json.dumps(d, indent=1))
