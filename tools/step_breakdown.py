"""Per-step GPU time by kernel from a rocprofv3 kernel trace: the step is the span between two consecutive fused AdamW
launches (adam_mt), so warm-up / init kernels outside it do not pollute the table.

    python tools/step_breakdown.py gpurun_out/prof8b [--step -1] [--top 30]"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--step", type=int, default=-1, help="which adam-to-adam interval (python index)")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "adam_mt" in r["Kernel_Name"]]
    lo, hi = marks[a.step - 1], marks[a.step]
    seg = rows[lo + 1 : hi + 1]
    t0, t1 = int(rows[lo]["End_Timestamp"]), int(rows[hi]["End_Timestamp"])
    tot, cnt = defaultdict(float), defaultdict(int)
    for r in seg:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:110]
        tot[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        cnt[n] += 1
    busy = sum(tot.values())
    print(f"step span {(t1 - t0) / 1e6:.1f} ms, kernel time {busy:.1f} ms, {len(seg)} kernels\n")
    print("| ms | calls | us/call | kernel |\n|---:|---:|---:|---|")
    for n, v in sorted(tot.items(), key=lambda kv: -kv[1])[: a.top]:
        print(f"| {v:.2f} | {cnt[n]} | {v / cnt[n] * 1e3:.1f} | `{n}` |")


if __name__ == "__main__":
    main()
