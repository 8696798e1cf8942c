"""The bench line's roofline is reproducible from the tracked rocprofv3 outputs: re-parsing
profiles/r0N/cfgN (kernel-trace stats or per-launch trace + PMC passes) gives the committed summary, and every
config's binding-resource fraction is a fraction (<= 1)."""
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import roofline as rl  # noqa: E402

# the summary's kernel-name filter, as recorded in it ("k_render_w8": the single-sample build of
# the primary+shadow frame, whose last 60 launches are the bench's timed steps)


@pytest.mark.parametrize("key", ["cfg2", "cfg3", "cfg4", "cfg5"])
def test_summary_recomputes_from_tracked_csvs(key):
    summary = rl.load()
    assert key in summary, f"profiles/pmc_summary.json lacks {key}"
    rec = summary[key]
    dirs = [os.path.join(ROOT, d) for d in rec["sources"]]
    assert all(os.path.isdir(d) for d in dirs), rec["sources"]
    again = rl.summarize(key, rec["kernel"], dirs, tail=rec.get("tail"), last=rec.get("last"))
    assert again["counters"] == pytest.approx(rec["counters"])
    assert again["trace_avg_ns"] == pytest.approx(rec["trace_avg_ns"])
    r = rl.roofline(again)
    assert r["bound"] == "valu" and 0 < r["frac"] <= 1
    assert 0 < r["hbm_frac"] < 1 and 0 < r["l2_hit"] < 1
    assert r["clock_ghz"] <= rl.MAX_CLOCK_GHZ
    # a live kernel time replaces the trace's in achieved, not in the measured clock
    live = rl.roofline(again, kernel_ms=r["kernel_ms"] * 2)
    assert live["achieved"] == pytest.approx(r["achieved"] / 2, rel=1e-3) and live["peak"] == r["peak"]
