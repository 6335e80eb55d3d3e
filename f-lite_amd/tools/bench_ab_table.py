"""Table of a tools/bench_ab.sh log: images/s, ms per image and the probe's average kernel time per spec and round,
plus the median per spec. Usage: python tools/bench_ab_table.py LOG"""
import json
import statistics
import sys

rows = {}
tag = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        tag = line.split()[1]
    elif line.startswith("{") and tag:
        d = json.loads(line)
        probe = (d.get("roofline") or {}).get("avg_ms")
        rows.setdefault(tag, []).append((d["value"], d["ms_per_step"], probe))
        print(f"{tag:40s} {d['value']:.5f} img/s {d['ms_per_step']:8.1f} ms  probe {probe}")
print("== median")
for tag, v in rows.items():
    probes = [p for _, _, p in v if p is not None]
    print(f"{tag:40s} {statistics.median(x[0] for x in v):.5f} img/s  probe "
          f"{statistics.median(probes) if probes else None}  (n={len(v)})")
