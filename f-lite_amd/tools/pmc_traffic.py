"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes to HBM bytes per launch of the probed kernels.

Usage (after two separate counter passes over the same bench command, see DESIGN.md "Measurement"):
    python f-lite_amd/tools/pmc_traffic.py <fetch_pass_dir> <write_pass_dir> profiles/pmc_traffic.json

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE is reported in KiB and, on
gfx950, counts exactly half of the bytes of a wide (16 B/lane) coalesced streaming read such as the GEMM's
`buffer_load ... lds` staging -> doubled; WRITE_SIZE (KiB) is exact for 16-B-per-lane stores. Both count
Infinity-Cache hits as well (memory-side L2 requests), so "traffic" is L2->fabric bytes, an upper bound on HBM.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# probe name -> substring of the mangled kernel name that identifies it uniquely
KERNELS = {
    "gateup": "gemm_bf16_kernelILi3ELb0E",  # EPI_SWIGLU_BF16, dense operands
}


def read_pass(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under %s" % d)
    vals = defaultdict(list)
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    fetch = read_pass(fetch_dir, "FETCH_SIZE")
    write = read_pass(write_dir, "WRITE_SIZE")
    res = {}
    for probe, key in KERNELS.items():
        fv = [v for k, vs in fetch.items() if key in k for v in vs]
        wv = [v for k, vs in write.items() if key in k for v in vs]
        if not fv or not wv:
            continue
        fetch_b = 2.0 * 1024.0 * sum(fv) / len(fv)
        write_b = 1024.0 * sum(wv) / len(wv)
        res[probe] = {"kernel_match": key, "launches": len(fv), "fetch_bytes_per_launch": fetch_b,
                      "write_bytes_per_launch": write_b, "hbm_bytes_per_launch": fetch_b + write_b,
                      "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 wide-read half count); WRITE_SIZE KiB x1024"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
