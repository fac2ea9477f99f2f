#!/usr/bin/env python3
"""Cross-check bench.py's event-timed roofline against a rocprofv3 kernel trace
of the same bench command, and record the result in profiles/rocprof_kernels.json.

    python tools/frac_check.py <kernel_trace.csv> <bench.json (un-profiled run)> [--source NAME] [--write]

For the dominant GS kernels of the bench configuration (col_main =
col_kernel<col_plan, cw, GS_MAIN, ...>, row_main = row_kernel<row_plan,
GS_MAIN, ...>) it prints the trace's mean duration over every launch (graph
replays of the timed steps, warm-up and the event-timed run), over the launches
of the event-timed run (the last `launches` of that kernel: the bench's last
run of the plan), the bench's own event mean from its un-profiled line, and the
roofline fraction each gives. --write stores them under the bench's config key.
"""
import argparse
import csv
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--source", default=None)
    ap.add_argument("--write", action="store_true")
    a = ap.parse_args()
    line = [ln for ln in open(a.bench) if ln.startswith("{")][-1]
    b = json.loads(line)
    info = b["config"]["col_tile"]
    n, bper, iters = b["config"]["height"], b["config"]["batch_per_gpu"], b["config"]["iters"]
    key = f"gs_{n}x{n}_b{bper}_it{iters}_{b['dtype']}"
    names = {"col_main": f"void slm::col_kernel<{info['col_plan']}, {info['col_cw']}, 0,",
             "row_main": f"void slm::row_kernel<{info['row_plan']}, 0,"}
    rows = list(csv.DictReader(open(a.trace)))
    out = {}
    for cls, prefix in names.items():
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
             if r["Kernel_Name"].startswith(prefix)]
        kb = b["roofline"]["kernels"].get(cls)
        if not d or kb is None:
            continue
        timed = d[-kb["launches"]:]
        model = kb["model_bytes_per_launch"]
        rec = {"launches_all": len(d), "avg_us_all": round(statistics.mean(d), 4),
               "avg_us_timed_run": round(statistics.mean(timed), 4), "median_us_timed_run": round(statistics.median(timed), 4),
               "event_avg_us_same_run": round(kb.get("event_avg_us", kb["avg_us"]), 4),
               "bench_avg_us": round(kb["avg_us"], 4)}
        for k, v in (("all", rec["avg_us_all"]), ("timed_run", rec["avg_us_timed_run"]),
                     ("events", rec["event_avg_us_same_run"]), ("bench", rec["bench_avg_us"])):
            rec[f"frac_{k}"] = round(model / (v * 1e-6) / 1e9 / PEAK, 4)
        out[cls] = rec
        print(f"{cls}: trace all launches {rec['avg_us_all']:.3f} us (frac {rec['frac_all']}), trace of the "
              f"event-timed run {rec['avg_us_timed_run']:.3f} us (frac {rec['frac_timed_run']}), bench per-launch "
              f"events {rec['event_avg_us_same_run']:.3f} us (frac {rec['frac_events']}), bench in-graph "
              f"{rec['bench_avg_us']:.3f} us (frac {rec['frac_bench']}); bench in-graph vs trace all launches "
              f"{100 * (rec['bench_avg_us'] / rec['avg_us_all'] - 1):+.1f} %")
    it = b["roofline"].get("iteration", {}).get("us")
    if it:
        ksum = sum(v["avg_us_all"] for v in out.values())
        print(f"bench wall per iteration {it:.3f} us; trace kernels per iteration {ksum:.3f} us")
    if a.write:
        path = os.path.join(ROOT, "profiles", "rocprof_kernels.json")
        db = json.load(open(path)) if os.path.exists(path) else {}
        db[key] = {"source": a.source or os.path.relpath(a.trace, ROOT), "kernels": out}
        json.dump(db, open(path, "w"), indent=1)
        print(f"wrote {key} to {path}")


if __name__ == "__main__":
    main()
