"""Reduce rocprofv3 passes over tools/pmc_kernels.py to per-kernel-class numbers (one JSON).

    python f-lite_amd/tools/pmc_reduce.py OUT.json trace=<dir> fetch=<dir> write=<dir> mfma=<dir> stall=<dir>
        [residual=bf16|fp32]

Each <dir> holds one rocprofv3 run (--output-format csv) of pmc_kernels.py; `trace` is a --kernel-trace run
(durations at the un-profiled clock), the others one --pmc pass each:
  fetch  FETCH_SIZE
  write  WRITE_SIZE
  mfma   SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
  stall  SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
         SQ_WAIT_INST_LDS
Corrections (MI355X_MICROARCH.md, HBM / rocprofv3 sections): FETCH_SIZE (KiB) doubled on gfx950 for wide
coalesced reads; WRITE_SIZE (KiB) exact for 16-B stores; both are L2->fabric requests, Infinity-Cache hits
included. SQ_VALU_MFMA_BUSY_CYCLES is summed over the 1024 SIMDs, GRBM_GUI_ACTIVE over the 8 XCDs; SQ_WAVE_CYCLES
and the SQ_WAIT_* counters are in quad-cycles (ratios only are used). Clock under collection = GRBM_GUI_ACTIVE /
8 / dispatch duration (meaningful for dispatches >= 0.3 ms). The first (cold) launch of each class is dropped.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

T, B, D, F, H, HD, LC = 4112, 2, 3072, 12288, 12, 256, 512
M = B * T
PEAK_TF = 2516.6
PEAK_GBS = 8000.0
WORK = {  # class -> (kind, algorithmic amount per launch: FLOP or bytes)
    "qkv": ("flop", 2.0 * M * 3 * D * D),
    "proj": ("flop", 2.0 * M * D * D),
    "cross_q": ("flop", 2.0 * M * D * D),
    "gateup": ("flop", 2.0 * M * 2 * F * D),
    "down": ("flop", 2.0 * M * F * D),
    "attn_self": ("flop", 4.0 * B * H * T * T * HD),
    "attn_cross": ("flop", 4.0 * B * H * T * LC * HD),
    "attn_cross_c": ("flop", 4.0 * 1 * H * T * LC * HD),  # uniform-context collapse: the cond sequence only
    "rope_qknorm": ("bytes", 2.0 * (M * 2 * D * 2)),       # q and k read + written, bf16
    "rmsnorm_mod": ("bytes", M * D * 4.0 + M * D * 2.0),   # fp32 residual in, bf16 out (main: residual=bf16)
}


def load_rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    files += glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no rocprofv3 csv under {d}")
    rows = []
    for f in files:
        with open(f, newline="") as fh:
            rows += list(csv.DictReader(fh))
    return rows


def segment(rows, classes):
    """dispatch -> class by the fill_ markers; returns {class: {dispatch_id: {counter: value, '_dur': s}}}."""
    by_disp = {}
    for r in rows:
        did = int(r.get("Dispatch_Id") or r.get("Dispatch_ID") or 0)
        e = by_disp.setdefault(did, {"name": r["Kernel_Name"], "c": {}})
        if "Counter_Name" in r:
            e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        e["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = defaultdict(dict)
    k = -1
    for did in sorted(by_disp):
        e = by_disp[did]
        if "FillFunctor<int>" in e["name"]:
            k += 1
            continue
        if k < 0 or k >= len(classes) or "Functor" in e["name"]:
            continue
        out[classes[k]][did] = dict(e["c"], _dur=e["dur"], _name=e["name"])
    return out


def steady(d, key):
    vals = [v[key] for _, v in sorted(d.items()) if key in v]
    return vals[1:] if len(vals) > 2 else vals


def mean(v):
    return sum(v) / len(v) if v else None


def main():
    out_path = sys.argv[1]
    passes = dict(a.split("=", 1) for a in sys.argv[2:])
    # residual=bf16 (round 6 default, pmc_kernels.py --residual bf16): the norm reads 2 B per element, not 4
    if passes.pop("residual", "bf16") == "bf16":
        WORK["rmsnorm_mod"] = ("bytes", M * D * 2.0 + M * D * 2.0)
    classes = json.loads(os.environ.get("PMC_CLASSES", "null"))
    if classes is None:  # the launch order of tools/pmc_kernels.py (marker k = classes[k])
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from pmc_kernels import CLASSES as classes
    seg = {p: segment(load_rows(d), classes) for p, d in passes.items()}
    res = {}
    for c in classes:
        r = {}
        if "trace" in seg and c in seg["trace"]:
            dur = mean(steady(seg["trace"][c], "_dur"))
            r["kernel"] = next(iter(seg["trace"][c].values()))["_name"][:120]
            r["avg_us"] = dur * 1e6
            kind, amount = WORK[c]
            if kind == "flop":
                r["achieved_tflops"] = amount / dur / 1e12
                r["frac_of_peak"] = r["achieved_tflops"] / PEAK_TF
                r["algorithmic_flop"] = amount
            else:
                r["achieved_gbs"] = amount / dur / 1e9
                r["frac_of_peak"] = r["achieved_gbs"] / PEAK_GBS
                r["algorithmic_bytes"] = amount
        if "fetch" in seg and c in seg["fetch"]:
            r["fetch_bytes"] = 2.0 * 1024.0 * mean(steady(seg["fetch"][c], "FETCH_SIZE"))
        if "write" in seg and c in seg["write"]:
            r["write_bytes"] = 1024.0 * mean(steady(seg["write"][c], "WRITE_SIZE"))
        if "fetch_bytes" in r and "write_bytes" in r:
            r["traffic_bytes"] = r["fetch_bytes"] + r["write_bytes"]
        if "mfma" in seg and c in seg["mfma"]:
            s = seg["mfma"][c]
            busy = mean(steady(s, "SQ_VALU_MFMA_BUSY_CYCLES"))
            gui = mean(steady(s, "GRBM_GUI_ACTIVE"))
            mops = mean(steady(s, "SQ_INSTS_VALU_MFMA_MOPS_BF16"))
            dur = mean(steady(s, "_dur"))
            if gui:
                r["mfma_busy_frac"] = busy / 1024.0 / (gui / 8.0) if busy is not None else None
                r["clock_ghz_under_pmc"] = gui / 8.0 / dur / 1e9
            if mops is not None:
                r["hw_mfma_flop"] = mops * 512.0
        if "stall" in seg and c in seg["stall"]:
            s = seg["stall"][c]
            wc = mean(steady(s, "SQ_WAVE_CYCLES"))
            if wc:
                for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                    v = mean(steady(s, k))
                    if v is not None:
                        r[k.lower() + "_frac"] = v / wc
            bc = mean(steady(s, "SQ_LDS_BANK_CONFLICT"))
            act = mean(steady(s, "SQ_LDS_IDX_ACTIVE"))
            if bc is not None and act:
                r["lds_bank_conflict_frac"] = bc / act
        res[c] = r
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)
    for c, r in res.items():
        print(c, json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items() if k != "kernel"}))


if __name__ == "__main__":
    main()
