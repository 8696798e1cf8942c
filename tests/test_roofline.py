"""The bench line's roofline is reproducible from the tracked rocprofv3 outputs: re-parsing
profiles/r0N/cfgN (kernel-trace stats or per-launch trace + PMC passes) gives the committed summary, and every
config's binding-resource fraction is a fraction (<= 1)."""
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import roofline as rl  # noqa: E402

# the summary's kernel-name filter: "k_render" takes the single-sample build (k_render_w8) and
# the plain one (k_render<0, 1, false>) of the primary+shadow frame
KERNELS = {"cfg2": "k_render", "cfg3": "k_pt_lanes", "cfg4": "k_render", "cfg5": "k_pt_lanes"}


@pytest.mark.parametrize("key", sorted(KERNELS))
def test_summary_recomputes_from_tracked_csvs(key):
    summary = rl.load()
    assert key in summary, f"profiles/pmc_summary.json lacks {key}"
    rec = summary[key]
    dirs = [os.path.join(ROOT, d) for d in rec["sources"]]
    assert all(os.path.isdir(d) for d in dirs), rec["sources"]
    again = rl.summarize(key, KERNELS[key], dirs, tail=rec.get("tail"))
    assert again["counters"] == pytest.approx(rec["counters"])
    assert again["trace_avg_ns"] == pytest.approx(rec["trace_avg_ns"])
    r = rl.roofline(again)
    assert r["bound"] == "valu" and 0 < r["frac"] <= 1
    assert 0 < r["hbm_frac"] < 1 and 0 < r["l2_hit"] < 1
    assert r["clock_ghz"] <= rl.MAX_CLOCK_GHZ
    # a live kernel time replaces the trace's in achieved, not in the measured clock
    live = rl.roofline(again, kernel_ms=r["kernel_ms"] * 2)
    assert live["achieved"] == pytest.approx(r["achieved"] / 2, rel=1e-3) and live["peak"] == r["peak"]
