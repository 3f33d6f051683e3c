"""rocprofv3 kernel trace -> per (kernel, grid) launch statistics.

``--stats`` averages every launch of one kernel symbol together; the bench launches the same
decoder instantiation at two sizes (config 4's B=64 x 256^3 step and config 3's 8 x 128^3
decode), so its average mixes them.  This splits the trace by grid size as well.
Usage: python scripts/prof_by_grid.py <run_kernel_trace.csv> [name-substring] [top-N]"""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
groups = defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if pat not in name:
        continue
    wg = int(r["Workgroup_Size_X"]) * int(r.get("Workgroup_Size_Y", 1) or 1)
    grid = (int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1)
            * int(r.get("Grid_Size_Z", 1) or 1)) // max(1, wg)
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    short = name.replace("(anonymous namespace)::", "").replace("void ", "")
    short = re.sub(r"\(.*", "", short)[:70]
    groups[(short, grid)].append(d)
# one symbol launched at very different sizes on the same grid (a persistent kernel): split
# each (kernel, grid) group where consecutive sorted durations jump by more than 1.5x
split = {}
for (k, g), v in groups.items():
    v = sorted(v)
    start = 0
    for i in range(1, len(v) + 1):
        if i == len(v) or v[i] > 1.5 * v[i - 1]:
            split[(k, g, len(split))] = v[start:i]
            start = i
groups = split
rows = sorted(groups.items(), key=lambda kv: -sum(kv[1]))
tot = sum(sum(v) for v in groups.values())
print(f"{'kernel':70s} {'WGs':>8s} {'calls':>6s} {'avg_ms':>12s} {'min_ms':>12s} {'max_ms':>12s} {'share':>6s}")
for (k, g, _), v in rows[:top]:
    print(f"{k:70s} {g:8d} {len(v):6d} {sum(v)/len(v):12.5f} {min(v):12.5f} {max(v):12.5f} "
          f"{100*sum(v)/tot:5.1f}%")
