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
    """Iteration kernel class of a trace name, or None:
    float32 engine col_kernel<K, CW, MODE, TT, P, LID> / row_kernel<K, MODE, P, LID>
    (col MODE 0 GS, 4 / 7 GD gradient / fused -> col_main, 3 -> gd_stats; row MODE 0 GS,
    5 GD -> row_main); complex128 radix plans rz_col_kernel<K, CW, OP> /
    rz_row_kernel<K, OP> and mixed radix mr_col_kernel<OP, BIG> / mr_row_kernel<OP, BIG>
    (col OP 3 GS, 5 / 6 GD gradient -> col_main, 4 -> gd_stats; row OP 4 / 8 GS, 7 GD -> row_main).
    The word boundary keeps mr_/rz_ names out of the float32 branch."""
    m = re.search(r"\b(rz_|mr_)?(col|row)_kernel<([^>]*)>", name)
    if not m:
        return None
    prefix, side = m.group(1) or "", m.group(2)
    args = [a.strip() for a in m.group(3).split(",")]
    try:
        if prefix == "":
            mode = int(args[2] if side == "col" else args[1])
            if side == "col":
                return {0: "col_main", 4: "col_main", 7: "col_main", 3: "gd_stats"}.get(mode)
            return {0: "row_main", 5: "row_main"}.get(mode)
        op = int(args[0] if prefix == "mr_" else (args[2] if side == "col" else args[1]))
    except (IndexError, ValueError):
        return None
    if side == "col":
        return {3: "col_main", 5: "col_main", 6: "col_main", 4: "gd_stats"}.get(op)
    return {4: "row_main", 7: "row_main", 8: "row_main"}.get(op)


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


def plan_of_log(path):
    """[row_plan, col_plan, col_cw, precision, [col engine, row engine]] from the
    `plan {...}` line tools/prof_gs.py prints (the plan the counters observed)."""
    import ast

    for line in open(path):
        if line.startswith("plan {"):
            info = ast.literal_eval(line[5:].strip())
            return [info.get("row_plan"), info.get("col_plan"), info.get("col_cw"), info.get("precision"),
                    list(info.get("engine", ()))]
    return None


def main():
    """usage: pmc_traffic.py FETCH.csv WRITE.csv KEY [OUT.json] [RUN.log]; RUN.log
    (prof_gs.py's stdout) stamps the entry with the plan it measured, which
    bench.py checks against the plan it times (a mismatch reports null)."""
    fetch_csv, write_csv, key = sys.argv[1:4]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "profiles", "pmc_traffic.json")
    log = sys.argv[5] if len(sys.argv) > 5 else None
    rd, n_rd = per_launch(fetch_csv, "FETCH_SIZE")
    wr, _ = per_launch(write_csv, "WRITE_SIZE")
    entry = {k: round(2 * rd[k] + wr.get(k, 0.0)) for k in rd}
    entry["detail"] = {k: {"read_bytes": round(2 * rd[k]), "write_bytes": round(wr.get(k, 0.0)),
                           "launches_counted": n_rd[k]} for k in rd}
    if log:
        entry["plan"] = plan_of_log(log)
    data = {}
    if os.path.exists(out):
        data = json.load(open(out))
    data[key] = entry
    json.dump(data, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({key: entry}))


if __name__ == "__main__":
    main()
