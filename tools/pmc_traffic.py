#!/usr/bin/env python3
"""Per-launch HBM traffic of the GS main kernels from rocprofv3 PMC passes.

usage: tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <key> [out.json]

FETCH_SIZE / WRITE_SIZE are in KB per dispatch. FETCH_SIZE is doubled: on
gfx950 it reports half the bytes of wide coalesced streaming reads
(MI355X_MICROARCH.md, HBM / rocprofv3 section); WRITE_SIZE is exact. The
counters sit on the memory side of L2, so Infinity-Cache hits are included.
Writes {key: {"col_main": bytes, "row_main": bytes, ...}} into
profiles/pmc_traffic.json (merged), which bench.py reports as roofline.traffic.
"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_class(name):
    """col_kernel<K, CW, MODE, TT, P> / row_kernel<K, MODE, P>; MODE 0 = GS main pass."""
    m = re.search(r"(col|row)_kernel<([^>]*)>", name)
    if not m:
        return None
    args = [a.strip() for a in m.group(2).split(",")]
    mode = args[2] if m.group(1) == "col" else args[1]
    return f"{m.group(1)}_main" if mode == "0" else None


def per_launch(path, counter):
    tot, cnt = collections.defaultdict(float), collections.defaultdict(int)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        cls = kernel_class(r["Kernel_Name"])
        if cls:
            tot[cls] += float(r["Counter_Value"]) * 1024
            cnt[cls] += 1
    return {k: tot[k] / cnt[k] for k in tot}, cnt


def main():
    fetch_csv, write_csv, key = sys.argv[1:4]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "profiles", "pmc_traffic.json")
    rd, n_rd = per_launch(fetch_csv, "FETCH_SIZE")
    wr, _ = per_launch(write_csv, "WRITE_SIZE")
    entry = {k: round(2 * rd[k] + wr.get(k, 0.0)) for k in rd}
    entry["detail"] = {k: {"read_bytes": round(2 * rd[k]), "write_bytes": round(wr.get(k, 0.0)),
                           "launches_counted": n_rd[k]} for k in rd}
    data = {}
    if os.path.exists(out):
        data = json.load(open(out))
    data[key] = entry
    json.dump(data, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({key: entry}))


if __name__ == "__main__":
    main()
