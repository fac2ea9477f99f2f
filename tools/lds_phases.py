#!/usr/bin/env python3
"""Static check of the LDS exchange protocol in a kernel's assembly: between
two s_barrier instructions a wave may write the exchange buffer or read it,
never both (write -> barrier -> read -> barrier -> write ...). A segment that
holds both is a race candidate (reads sunk below the barrier that releases
the next writes). Prints per-segment (writes, reads).

Double-buffered kernels (kernels.hpp, kLdsDouble) read exchange k and write
exchange k + 1 -- the other buffer -- in one segment by design: there a read
that follows a write of the same segment is the race candidate (--double).

    python tools/lds_phases.py /tmp/k5.s col_kernelILi5ELi16ELi0ELi1ELi0E
"""
import re
import sys


def main():
    args = [a for a in sys.argv[1:] if a != "--double"]
    double = "--double" in sys.argv
    text = open(args[0]).read()
    for pat in args[1:]:
        m = re.search(r"^(_Z\S*" + pat + r"\S*?):", text, re.M)
        body = text[m.end():text.find(".Lfunc_end", m.end())]
        segs, w, r, late = [], 0, 0, []
        for ln in body.splitlines():
            op = ln.strip().split(" ")[0]
            if op == "s_barrier":
                segs.append((w, r))
                w = r = 0
            elif op.startswith("ds_write") or op.startswith("ds_store"):
                w += 1
            elif op.startswith("ds_read") or op.startswith("ds_load"):
                r += 1
                if w:
                    late.append(len(segs))
        segs.append((w, r))
        bad = sorted(set(late)) if double else [i for i, (a, b) in enumerate(segs) if a and b]
        print(m.group(1)[:60], "segments", segs, "MIXED at", bad)


if __name__ == "__main__":
    main()
