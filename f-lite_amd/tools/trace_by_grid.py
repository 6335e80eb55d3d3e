"""Kernel times grouped by (kernel, grid size) from rocprofv3 --kernel-trace CSVs (diagnostic): separates launches
of one kernel that differ in shape (self- vs cross-attention, whose grids differ, proj vs cross-proj), without the
launch-order assumptions of trace_split.py. Usage: python tools/trace_by_grid.py run_kernel_trace.csv [SUBSTR ...]"""
import csv
import statistics as st
import sys
from collections import defaultdict

f, subs = sys.argv[1], sys.argv[2:]
groups = defaultdict(list)
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"]
    if subs and not any(s in name for s in subs):
        continue
    grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
    groups[(name.split("(")[0][-60:], grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (name, grid), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
    print(f"{name:62s} grid {grid:>8s}  n {len(d):5d}  mean {st.mean(d):9.1f} us  median {st.median(d):9.1f}  "
          f"total {sum(d) / 1e3:8.1f} ms")
