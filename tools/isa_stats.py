#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc -S device assembly file.

    python tools/isa_stats.py /tmp/k11.s 'col_kernelILi11ELi2ELi0ELi1ELi0E' ...

The hot kernels are fully unrolled (no loops), so the static counts are the
per-wave dynamic counts of one tile.
"""
import collections
import re
import sys


def kernel_body(text, pat):
    m = re.search(r"^(_Z\S*" + pat + r"\S*?):", text, re.M)
    if not m:
        raise SystemExit(f"no kernel matching {pat}")
    start = m.end()
    end = text.find(".Lfunc_end", start)
    meta = {}
    name = m.group(1)
    # the kernel's own descriptor block (.amdhsa_kernel <name> ... .end_amdhsa_kernel):
    # next_free_vgpr counts arch VGPRs + AGPRs (unified file; > 256 = one wave per SIMD)
    i = text.find(".amdhsa_kernel " + name)
    blk = text[i:text.find(".end_amdhsa_kernel", i)] if i >= 0 else ""
    for key, out in (("next_free_vgpr", "vgpr_count"), ("next_free_sgpr", "sgpr_count"),
                     ("group_segment_fixed_size", "group_segment_fixed_size"),
                     ("private_segment_fixed_size", "scratch_bytes"), ("accum_offset", "accum_offset")):
        mm = re.search(r"\.amdhsa_" + key + r"\s+(\d+)", blk)
        if mm:
            meta[out] = int(mm.group(1))
    return name, text[start:end], meta


def classify(line):
    op = line.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_rd"
    if op.startswith(("global_store", "buffer_store", "flat_store", "global_atomic")):
        return "vmem_wr"
    if op == "s_barrier":
        return "barrier"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    text = open(sys.argv[1]).read()
    for pat in sys.argv[2:]:
        name, body, meta = kernel_body(text, pat)
        c = collections.Counter()
        ops = collections.Counter()
        for ln in body.splitlines():
            ln = ln.strip()
            if not ln or ln.startswith((";", ".", "_")) or ln.endswith(":"):
                continue
            c[classify(ln)] += 1
            ops[ln.split()[0]] += 1
        print(name, meta)
        print("  ", dict(c))
        print("   top:", ops.most_common(14))


if __name__ == "__main__":
    main()
