#!/usr/bin/env python3
"""Register / LDS / occupancy summary of kernels in a hipcc -S device assembly.

    python tools/kinfo.py /tmp/k13.s [substring ...]
"""
import re
import sys


def main():
    text = open(sys.argv[1]).read()
    pats = sys.argv[2:] or [""]
    for m in re.finditer(r"^(_Z\S+?):", text, re.M):
        name = m.group(1)
        if not any(p in name for p in pats):
            continue
        i = text.find("; Kernel info:", m.end())
        blk = text[i:i + 1200]
        g = lambda k: (re.search(r"; " + k + r": (\d+)", blk) or [None, "?"])[1]
        print(f"{name[:70]:70s} vgpr {g('NumVgprs'):>4s} agpr {g('NumAgprs'):>3s} sgpr {g('TotalNumSgprs'):>3s} "
              f"lds {g('LDSByteSize'):>6s} scratch {g('ScratchSize'):>4s} occ {g('Occupancy')}")


if __name__ == "__main__":
    main()
