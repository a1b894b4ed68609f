"""Print the kernel timeline of one fit from a rocprofv3 --kernel-trace csv (the last complete
fit: from one grid_kernel dispatch to the next)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if re.search(r"\bgrid_kernel\(", r["Kernel_Name"])]
seg = rows[starts[-2]:starts[-1]]
t0 = int(seg[0]["Start_Timestamp"])
prev = t0
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = re.sub(r"^void |\(anonymous namespace\)::|dbscan::", "", r["Kernel_Name"]).split("(")[0]
    print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:5.1f} dur {(e - s) / 1e3:7.1f}  {name}"
          f"  grid={r['Grid_Size_X']}")
    prev = e
print(f"span {(prev - t0) / 1e3:.1f} us")
