"""Reduce rocprofv3 --pmc passes to HBM bytes and MFMA utilisation per launch of the probed kernel.

Usage (three separate counter passes over the same command, see DESIGN.md "Measurement"):
    python f-lite_amd/tools/pmc_traffic.py <fetch_dir> <write_dir> <mfma_dir> profiles/pmc_traffic.json
      fetch_dir: --pmc FETCH_SIZE
      write_dir: --pmc WRITE_SIZE
      mfma_dir:  --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE is reported in KiB and, on
gfx950, counts exactly half of the bytes of a wide (16 B/lane) coalesced streaming read such as the GEMM's
`buffer_load ... lds` staging -> doubled; WRITE_SIZE (KiB) is exact for 16-B-per-lane stores. Both count
Infinity-Cache hits as well (memory-side L2 requests), so "traffic" is L2->fabric bytes, an upper bound on HBM.

MFMA: SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 = hardware-counted bf16 MFMA FLOPs; SQ_VALU_MFMA_BUSY_CYCLES is summed
over all SIMDs (measured: = number of v_mfma_f32_16x16x32_bf16 x 16 cycles), GRBM_GUI_ACTIVE over the 8 XCDs.
  busy fraction = BUSY / SIMDs / (GUI_ACTIVE / 8) (kernels run slower under counter collection, so the
  wall-clock rate is taken from the kernel-trace pass, not from these timestamps).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# probe name -> substring of the (demangled) kernel name that identifies it uniquely
KERNELS = {
    "gateup": "gemm_bf16_kernel<3, false,",  # EPI_SWIGLU_BF16, dense operands (any tile height)
}
N_SIMD = 256 * 4
N_XCD = 8


def read_pass(d, counters):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under %s" % d)
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values (one per launch)
    durs = defaultdict(list)
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") not in counters:
                    continue
                vals[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
                durs[row["Kernel_Name"]].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return vals, durs


def pick(vals, key, counter):
    return [v for k, cs in vals.items() if key in k for v in cs.get(counter, [])]


def main():
    fetch_dir, write_dir, mfma_dir, out = sys.argv[1:5]
    fetch, _ = read_pass(fetch_dir, {"FETCH_SIZE"})
    write, _ = read_pass(write_dir, {"WRITE_SIZE"})
    mf, mdur = read_pass(mfma_dir, {"SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"})
    res = {}
    for probe, key in KERNELS.items():
        fv = pick(fetch, key, "FETCH_SIZE")
        wv = pick(write, key, "WRITE_SIZE")
        if not fv or not wv:
            continue
        # the first launch of a fresh process runs cold (TLB, clocks): report the steady launches
        fv_s, wv_s = (fv[1:], wv[1:]) if len(fv) > 2 else (fv, wv)
        fetch_b = 2.0 * 1024.0 * sum(fv_s) / len(fv_s)
        write_b = 1024.0 * sum(wv_s) / len(wv_s)
        r = {"kernel_match": key, "launches": len(fv_s), "fetch_bytes_per_launch": fetch_b,
             "write_bytes_per_launch": write_b, "hbm_bytes_per_launch": fetch_b + write_b,
             "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 wide-read half count); WRITE_SIZE KiB x1024; "
                           "first (cold) launch dropped"}
        mops = pick(mf, key, "SQ_INSTS_VALU_MFMA_MOPS_BF16")
        busy = pick(mf, key, "SQ_VALU_MFMA_BUSY_CYCLES")
        gui = pick(mf, key, "GRBM_GUI_ACTIVE")
        if mops and busy and gui:
            n = len(gui)
            lo = 1 if n > 2 else 0
            m = sum(mops[lo:]) / len(mops[lo:])
            b = sum(busy[lo:]) / len(busy[lo:])
            g = sum(gui[lo:]) / len(gui[lo:]) / N_XCD
            r["hw_mfma_flops_per_launch"] = m * 512.0
            r["mfma_busy_frac"] = b / N_SIMD / g
            r["gui_active_cycles_per_xcd"] = g
        res[probe] = r
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
