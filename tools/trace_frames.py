#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (run_kernel_trace.csv) of overlapped frames: per kernel
name the launch count, mean / median duration, the mean period between consecutive launches,
and over the whole (or the last --tail fraction of the) trace the GPU busy fraction (union of
kernel intervals over the span) and the mean concurrency (summed durations over the union) --
whether frames in flight keep the GPU busy, and how many frames share it at a time.

usage: trace_frames.py TRACE.csv [--match REGEX] [--tail 0.5] [--json out.json]"""
import argparse
import csv
import json
import re
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="k_render|k_pt_|k_assemble|k_acc_tiles|rccl|nccl|Kernel")
    ap.add_argument("--tail", type=float, default=0.5, help="summarise the last fraction of the launches")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if not re.search(a.match, name):
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    rows = rows[int(len(rows) * (1.0 - a.tail)):] if rows else rows
    if not rows:
        raise SystemExit("no matching kernels")
    span = rows[-1][1] - rows[0][0]
    union, cur_s, cur_e = 0, rows[0][0], rows[0][1]
    for s, e, _ in rows[1:]:
        if s > cur_e:
            union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += cur_e - cur_s
    # idle gaps of the GPU between busy intervals (all matching kernels merged)
    gaps, end = [], rows[0][1]
    for s, e, _ in rows[1:]:
        if s > end:
            gaps.append((s - end) / 1e3)
        end = max(end, e)
    total = sum(e - s for s, e, _ in rows)
    by = {}
    for s, e, n in rows:
        short = re.sub(r"\(.*", "", n)[:80]
        by.setdefault(short, []).append((s, e))
    out = {"launches": len(rows), "span_ms": span / 1e6, "busy_frac": union / span if span else 0.0,
           "mean_concurrency": total / union if union else 0.0,
           "idle_gaps_us": {"count": len(gaps), "total": round(sum(gaps), 1),
                            "mean": round(statistics.mean(gaps), 2) if gaps else 0.0,
                            "max": round(max(gaps), 2) if gaps else 0.0,
                            "over_10us": sum(1 for g in gaps if g > 10.0)},
           "kernels": {}}
    for n, iv in sorted(by.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
        d = [(e - s) / 1e6 for s, e in iv]
        starts = [s for s, _ in iv]
        per = (starts[-1] - starts[0]) / 1e6 / (len(starts) - 1) if len(starts) > 1 else 0.0
        out["kernels"][n] = {"count": len(iv), "mean_ms": statistics.mean(d), "median_ms": statistics.median(d),
                             "max_ms": max(d), "period_ms": per}
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
