"""Per-launch durations of the last N kernels matching a pattern in a rocprofv3 kernel trace."""
import csv
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
n = int(sys.argv[3]) if len(sys.argv) > 3 else 18
rows = [r for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
w = rows[-n:]
tot = 0
for r in w:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    tot += d
    print(f"{d:7.2f} us  grid {int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}x"
          f"{r['Grid_Size_Y']}x{r['Grid_Size_Z']} lds {r['LDS_Block_Size']} vgpr {r['VGPR_Count']}"
          f" {r['Kernel_Name'][:60]}")
span = (int(w[-1]["End_Timestamp"]) - int(w[0]["Start_Timestamp"])) / 1000
print(f"sum {tot:.1f} us, span {span:.1f} us over {len(w)} launches")
