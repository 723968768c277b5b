"""Summarise a `rocprofv3 --kernel-trace --stats --output-format csv -d DIR` run as a markdown table.

    python tools/prof_summary.py gpurun_out/prof8b [--top 40]

Finds every `*kernel_stats.csv` under DIR (one per profiled process) and merges them by kernel name.
"""

import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--top", type=int, default=40)
    args = p.parse_args()
    files = glob.glob(os.path.join(args.dir, "**", "*kernel_stats.csv"), recursive=True)
    tot = defaultdict(float)
    calls = defaultdict(int)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                tot[row["Name"]] += float(row["TotalDurationNs"])
                calls[row["Name"]] += int(row["Calls"])
    grand = sum(tot.values()) or 1.0
    print(f"# rocprofv3 kernel stats: {args.dir} ({len(files)} file(s)), total GPU kernel time {grand / 1e6:.1f} ms\n")
    print("| total ms | calls | avg us | % | kernel |")
    print("|---:|---:|---:|---:|---|")
    for name, ns in sorted(tot.items(), key=lambda kv: -kv[1])[: args.top]:
        short = name.replace("|", "/")[:110]
        print(f"| {ns / 1e6:.1f} | {calls[name]} | {ns / 1e3 / max(calls[name], 1):.1f} | {100 * ns / grand:.1f} | `{short}` |")


if __name__ == "__main__":
    main()
