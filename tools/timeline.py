"""Print the kernel timeline of one bench step from a rocprofv3 kernel trace CSV:
kernel name, grid, start offset and duration (us), gap to the previous kernel (us)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
count = int(sys.argv[3]) if len(sys.argv) > 3 else 80
rows = rows[skip:skip + count]
t0 = int(rows[0]["Start_Timestamp"])
prev_end = t0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{r['Kernel_Name'][:28]:28s} grid={r['Grid_Size_X']:>7s} start={(s - t0) / 1e3:9.1f} "
          f"dur={(e - s) / 1e3:8.1f} gap={(s - prev_end) / 1e3:7.1f}")
    prev_end = e
