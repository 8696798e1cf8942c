#!/usr/bin/env python3
"""Roofline fields of the bench line, recomputed from tracked rocprofv3 outputs.

The binding resource of the traversal kernels is vector issue, not HBM: the scenes are
cache-resident (TEAPOT-F ~0.1 MB, mig29 x16 ~15 MB) and the per-launch HBM bytes the PMC
counters see are the accumulator / frame traffic.  So `frac` is the VALU
issue fraction of the dominant kernel:

    frac = SQ_INSTS_VALU x 2 cycles / (1,024 SIMDs x launch cycles)

(a wave64 VALU instruction occupies its SIMD for 2 cycles, MI355X_MICROARCH.md; 256 CUs x 4
SIMDs), with the launch cycles MEASURED: GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs) per
dispatch, so the clock the chip held under this kernel is in the denominator, not the
2.4 GHz maximum.  achieved / peak carry the same ratio in G wave-instructions per second:
achieved = VALU instructions per launch / the kernel's duration, peak = 1,024 x clock / 2.
Beside it: HBM bytes per launch (FETCH_SIZE x 2 -- gfx950 counts half of a wide read --
+ WRITE_SIZE, KB x 1024) and their fraction of the 8 TB/s peak, the L2 hit rate
(TCC_HIT / (TCC_HIT + TCC_MISS)), wave wait share, and the SURVEY 8(d) algorithmic bytes
(renamed algorithmic_gbs: node / triangle bytes mostly served by L1/L2, never a fraction).

usage:
  roofline.py summarize KEY KERNEL_SUBSTR DIR [DIR ...] [--out profiles/pmc_summary.json] [--tail 0.5 | --last N]
      parse a workload's rocprofv3 runs (kernel-trace stats + PMC passes) under DIRs
  roofline.py show [--summary profiles/pmc_summary.json]
      print every workload's roofline fields, recomputed from the summary
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary.json")
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8 TB/s
SIMDS = 1024               # 256 CUs x 4 SIMDs
VALU_CYCLES = 2            # cycles per wave64 VALU instruction
XCDS = 8
MAX_CLOCK_GHZ = 2.4
COUNTERS = ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
            "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE", "TCC_HIT_sum", "TCC_MISS_sum", "TCC_HIT",
            "TCC_MISS")


def _rows(dirs, pattern):
    for d in dirs:
        for f in sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True)):
            with open(f) as fh:
                yield from csv.DictReader(fh)


def summarize(key, kernel, dirs, tail=None, last=None):
    """Per-launch means of every counter found for kernels whose name contains `kernel`,
    and the kernel-trace average duration (rocprofv3 --stats).  tail (0 < tail <= 1): average
    only the last `tail` fraction of each counter's dispatches (by Dispatch_Id) and, when the
    per-launch kernel trace (*kernel_trace.csv) is there, of the launches -- the steady state
    after the renderer's untimed ramp and tuning frames (the bench's timed region).  last (N):
    the last N dispatches / launches instead -- exactly the bench's timed steps when the kernel
    name matches nothing after them (round 5: the clock ramp queues up to 200 frames without a
    host sync, and under the kernel trace those ramp launches recorded ~2x their duration)."""
    per = {}
    for row in _rows(dirs, "*counter_collection.csv"):
        if kernel not in row.get("Kernel_Name", ""):
            continue
        name = row["Counter_Name"]
        if name in COUNTERS:
            per.setdefault(name, []).append((int(row.get("Dispatch_Id") or 0), float(row["Counter_Value"])))

    def keep(vals):
        if last:
            return sorted(vals)[-last:]
        if not tail:
            return vals
        vals = sorted(vals)
        return vals[len(vals) - max(1, int(round(len(vals) * tail))):]

    kept = {k: keep(v) for k, v in per.items()}
    rec = {"kernel": kernel, "counters": {k: sum(x for _, x in v) / len(v) for k, v in kept.items()},
           "dispatches": {k: len(v) for k, v in kept.items()}}
    for row in _rows(dirs, "*kernel_stats.csv"):
        if kernel in row.get("Name", ""):
            rec["trace_avg_ns"] = float(row["AverageNs"])
            rec["trace_calls"] = int(row["Calls"])
            rec["trace_total_ns"] = float(row["TotalDurationNs"])
            rec["trace_kernel_name"] = row["Name"]
            break
    if tail or last:
        if last:
            rec["last"] = last
        else:
            rec["tail"] = tail
        launches = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                    for r in _rows(dirs, "*kernel_trace.csv") if kernel in r.get("Kernel_Name", "")]
        if launches:
            d = [x for _, x in keep(launches)]
            rec["trace_all_avg_ns"] = rec.get("trace_avg_ns")
            rec["trace_avg_ns"] = sum(d) / len(d)
            rec["trace_steady_launches"] = len(d)
    # share of the kernel in the frame: every kernel's total time in the same trace
    tot = sum(float(r["TotalDurationNs"]) for r in _rows(dirs, "*kernel_stats.csv")
              if not r["Name"].startswith("__amd") and "Functor" not in r["Name"])
    if tot and "trace_total_ns" in rec:
        rec["share_of_gpu_time"] = rec["trace_total_ns"] / tot
    rec["sources"] = sorted(os.path.relpath(d, ROOT) for d in dirs)
    return rec


def roofline(rec, kernel_ms=None, algorithmic_bytes=None):
    """The bench line's roofline object for one summary record.  kernel_ms: the live
    (HIP-event) duration per launch if the caller measured it, else the kernel trace's."""
    c = rec["counters"]
    trace_ms = rec.get("trace_avg_ns", 0.0) / 1e6
    ms = kernel_ms if kernel_ms else trace_ms
    out = {"bound": "valu", "unit": "G wave64-VALU-instr/s", "kernel": rec["kernel"], "kernel_ms": round(ms, 5),
           "kernel_ms_source": "HIP events (live)" if kernel_ms else "rocprofv3 kernel trace"}
    valu = c.get("SQ_INSTS_VALU")
    grbm = c.get("GRBM_GUI_ACTIVE")
    if valu and grbm and trace_ms:
        cycles = grbm / XCDS                      # launch cycles at the clock held
        # GRBM_GUI_ACTIVE / 8 / duration reads high on dispatches shorter than ~0.3 ms
        # (MI355X_MICROARCH.md, DVFS give-back): never above the 2.4 GHz maximum
        clock_ghz = min(MAX_CLOCK_GHZ, cycles / (trace_ms * 1e-3) / 1e9)
        peak = SIMDS * clock_ghz / VALU_CYCLES    # G wave-instructions / s
        achieved = valu / (ms * 1e-3) / 1e9
        out.update(achieved=round(achieved, 2), peak=round(peak, 2), frac=round(achieved / peak, 4),
                   clock_ghz=round(clock_ghz, 3), valu_insts_per_launch=round(valu))
    else:
        out.update(achieved=None, peak=None, frac=None)
    fetch, write = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
    if fetch is not None and write is not None:
        hbm = 2 * fetch * 1024 + write * 1024
        out["traffic"] = round(hbm)
        out["hbm_gbs"] = round(hbm / (ms * 1e-3) / 1e9, 2)
        out["hbm_frac"] = round(hbm / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
    else:
        out["traffic"] = None
    hit, miss = c.get("TCC_HIT_sum", c.get("TCC_HIT")), c.get("TCC_MISS_sum", c.get("TCC_MISS"))
    if hit is not None and miss is not None and hit + miss > 0:
        out["l2_hit"] = round(hit / (hit + miss), 4)
    if c.get("SQ_WAIT_ANY") and c.get("SQ_WAVE_CYCLES"):
        out["wave_wait_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
    if algorithmic_bytes:
        out["algorithmic_gbs"] = round(algorithmic_bytes / (ms * 1e-3) / 1e9, 1)
    if "share_of_gpu_time" in rec:
        out["share_of_frame"] = round(rec["share_of_gpu_time"], 4)
    return out


def load(path=SUMMARY):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("summarize")
    a.add_argument("key")
    a.add_argument("kernel")
    a.add_argument("dirs", nargs="+")
    a.add_argument("--out", default=SUMMARY)
    a.add_argument("--tail", type=float, default=None, help="average the last fraction of the dispatches only")
    a.add_argument("--last", type=int, default=None, help="average the last N dispatches only (the bench's timed steps)")
    b = sub.add_parser("show")
    b.add_argument("--summary", default=SUMMARY)
    args = ap.parse_args()
    if args.cmd == "summarize":
        data = load(args.out)
        data[args.key] = summarize(args.key, args.kernel, args.dirs, tail=args.tail, last=args.last)
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
        print(json.dumps({args.key: roofline(data[args.key])}))
    else:
        for k, rec in sorted(load(args.summary).items()):
            print(k, json.dumps(roofline(rec)))


if __name__ == "__main__":
    sys.exit(main())
