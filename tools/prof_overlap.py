"""Communication / compute overlap from a rocprofv3 trace.

    python tools/prof_overlap.py gpurun_out/prof8b_sharded [--pattern nccl|rccl|Copy]

Reads every `*kernel_trace.csv` (and `*memory_copy_trace.csv`, if the run had --memory-copy-trace) under the directory.
"Comm" intervals are kernels whose name matches --pattern (RCCL's collective kernels are `ncclDevKernel_*` /
`ncclKernel_*`) plus all memory copies; "compute" intervals are all other kernels. Prints, per comm kind, the busy time
and how much of it ran while at least one compute kernel was executing (union of intervals, so concurrent compute
kernels are not double counted), plus the compute-stream idle time that comm did not cover.
"""

import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def _rows(pattern, d):
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def _union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def _overlap(a_list, union_b):
    """total length of intervals a_list intersected with the (sorted, disjoint) union_b."""
    import bisect

    starts = [u[0] for u in union_b]
    tot = 0
    for a, b in a_list:
        i = max(0, bisect.bisect_right(starts, a) - 1)
        while i < len(union_b) and union_b[i][0] < b:
            lo, hi = max(a, union_b[i][0]), min(b, union_b[i][1])
            if hi > lo:
                tot += hi - lo
            i += 1
    return tot


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--pattern", default=r"nccl|rccl")
    args = p.parse_args()
    rx = re.compile(args.pattern, re.I)
    comm = defaultdict(list)
    compute = []
    for r in _rows("*kernel_trace.csv", args.dir):
        name = r.get("Kernel_Name") or r.get("Name", "")
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if rx.search(name):
            kind = re.sub(r"[<(].*", "", name)[:60]
            comm[kind].append((a, b))
        else:
            compute.append((a, b))
    for r in _rows("*memory_copy_trace.csv", args.dir):
        kind = "memcpy " + r.get("Direction", "")
        comm[kind].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if not compute:
        print("no kernel trace found")
        return
    cu = _union(compute)
    span = cu[-1][1] - cu[0][0]
    busy = sum(b - a for a, b in cu)
    print(f"# comm/compute overlap: {args.dir}\n")
    print(f"trace span {span / 1e6:.1f} ms, compute busy (union) {busy / 1e6:.1f} ms, compute idle {(span - busy) / 1e6:.1f} ms\n")
    print("| comm kind | calls | busy ms | overlapped with compute ms | % overlapped |")
    print("|---|---:|---:|---:|---:|")
    for kind, iv in sorted(comm.items(), key=lambda kv: -sum(b - a for a, b in kv[1])):
        u = _union(iv)
        t = sum(b - a for a, b in u)
        ov = _overlap(u, cu)
        print(f"| `{kind}` | {len(iv)} | {t / 1e6:.2f} | {ov / 1e6:.2f} | {100 * ov / max(t, 1):.1f} |")


if __name__ == "__main__":
    main()
