#!/usr/bin/env python3
"""Summarise a tools/profile.sh output directory: kernel durations and, per
kernel, HBM bytes from FETCH_SIZE / WRITE_SIZE (KB units; FETCH_SIZE doubled for
the gfx950 half-count of wide streaming reads, MI355X_MICROARCH.md HBM)."""
import collections
import csv
import sys


def main(d, markdown=False):
    rows = list(csv.DictReader(open(f"{d}/trace/trace_kernel_stats.csv")))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(int)
    for sub in ("fetch", "write", "sq", "tcc"):
        try:
            for r in csv.DictReader(open(f"{d}/{sub}/{sub}_counter_collection.csv")):
                k = r["Kernel_Name"]
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                if sub == "fetch":
                    cnt[k] += 1
        except FileNotFoundError:
            pass
    out = []
    for r in rows:
        k = r["Name"]
        n = max(cnt[k], 1)
        a = agg.get(k, {})
        fetch = 2 * a.get("FETCH_SIZE", 0) * 1024 / n
        write = a.get("WRITE_SIZE", 0) * 1024 / n
        avg = float(r["AverageNs"]) / 1e3
        out.append((k, int(r["Calls"]), avg, float(r["Percentage"]), fetch, write,
                    (fetch + write) / (avg * 1e3) if avg > 0 else 0.0,
                    a.get("SQ_LDS_BANK_CONFLICT", 0) / n, a.get("SQ_INSTS_LDS", 0) / n))
    if markdown:
        print("| kernel | calls | avg us | % | HBM read MB/launch | HBM write MB/launch | PMC GB/s |")
        print("|---|---|---|---|---|---|---|")
        for k, c, avg, pct, f, w, gbs, _, _ in out:
            print(f"| `{k[:70]}` | {c} | {avg:.2f} | {pct:.1f} | {f/1e6:.1f} | {w/1e6:.1f} | {gbs:.0f} |")
    else:
        for k, c, avg, pct, f, w, gbs, bc, li in out:
            print(f"{k[:58]:58s} n={c:5d} avg={avg:9.2f}us {pct:5.1f}% rd={f/1e6:8.1f}MB wr={w/1e6:8.1f}MB "
                  f"pmc={gbs:7.0f}GB/s ldsconf/inst={bc/max(li,1):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], markdown="--md" in sys.argv)
