"""Summarise `rocprofv3 --pmc ... --output-format csv` runs (tools/pmc_steps.sh) as a markdown table per kernel.

    python tools/pmc_summary.py gpurun_out/pmc/attn gpurun_out/pmc/gemm

Derived columns (MI355X: 256 CUs x 4 SIMDs, counters summed over the 8 XCDs):
  * clock GHz      = GRBM_GUI_ACTIVE / 8 / kernel wall time
  * MFMA busy %    = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs) - share of SIMD-cycles the matrix
                     cores were busy
  * LDS conflict % = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE - extra LDS-array cycles caused by bank conflicts
"""

import csv
import glob
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    cut = name.find("(")
    if cut > 0 and not name.startswith("Cijk") and not name.startswith("Custom"):
        name = name[:cut]
    return name[:72].replace("|", "/")


def stall(dirs):
    """Wave-cycle anatomy (SQ_* counters count quad-cycles except SQ_VALU_MFMA_BUSY_CYCLES): share of wave cycles
    parked on s_waitcnt / barrier (WAIT_ANY), issue-stalled (WAIT_INST_ANY) and issuing (ACTIVE_INST_ANY), plus VALU
    and LDS instruction-issue shares and MFMA busy per SIMD-cycle of the kernel's busy time."""
    for d in dirs:
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        ctr = defaultdict(lambda: defaultdict(float))
        wall = defaultdict(dict)
        for f in files:
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
                wall[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print(f"### {d}\n")
        print("| kernel | dispatches | wall ms | wait (waitcnt/barrier) % | issue-stall % | issuing % | VALU issue % | LDS issue % | MFMA busy % of SQ busy |")
        print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
        for k, c in sorted(ctr.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
            wc = c.get("SQ_WAVE_CYCLES", 0)
            if not wc:
                continue
            busy = c.get("SQ_BUSY_CYCLES", 0)
            pct = lambda n: 100 * c.get(n, 0) / wc  # noqa: E731
            mf = 100 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (busy * 4 * 4) if busy else 0
            print(f"| `{k}` | {len(wall[k])} | {sum(wall[k].values()) / 1e6:.2f} | {pct('SQ_WAIT_ANY'):.1f} | {pct('SQ_WAIT_INST_ANY'):.1f} | "
                  f"{pct('SQ_ACTIVE_INST_ANY'):.1f} | {pct('SQ_ACTIVE_INST_VALU'):.1f} | {pct('SQ_ACTIVE_INST_LDS'):.1f} | {mf:.1f} |")
        print()


def cache(dirs):
    """L2 (TCC) hit rate and the L2 -> fabric read requests (Infinity Cache / HBM) per kernel, with clock and MFMA busy."""
    for d in dirs:
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        ctr = defaultdict(lambda: defaultdict(float))
        wall = defaultdict(dict)
        for f in files:
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
                wall[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print(f"### {d}\n")
        print("| kernel | dispatches | wall ms | clock GHz | MFMA busy % | L2 hit % | L2 misses (M) | fabric read req (M) | fabric GB/s (x64 B) |")
        print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
        for k, c in sorted(ctr.items(), key=lambda kv: -kv[1].get("SQ_VALU_MFMA_BUSY_CYCLES", 0)):
            grbm = c.get("GRBM_GUI_ACTIVE", 0) / 8
            ns = sum(wall[k].values())
            mfma = 100 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (grbm * 1024) if grbm else 0
            hit, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
            rd = c.get("TCC_EA0_RDREQ_sum", 0)
            print(f"| `{k}` | {len(wall[k])} | {ns / 1e6:.2f} | {grbm / ns if ns else 0:.2f} | {mfma:.1f} | "
                  f"{100 * hit / (hit + miss) if hit + miss else 0:.1f} | {miss / 1e6:.1f} | {rd / 1e6:.1f} | {rd * 64 / ns if ns else 0:.0f} |")
        print()


def main(dirs):
    if dirs and dirs[0] == "--stall":
        return stall(dirs[1:])
    if dirs and dirs[0] == "--cache":
        return cache(dirs[1:])
    for d in dirs:
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        ctr = defaultdict(lambda: defaultdict(float))
        wall = defaultdict(dict)
        for f in files:
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
                wall[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print(f"### {d}\n")
        print("| kernel | dispatches | wall ms | clock GHz | MFMA busy % | LDS instr (M) | LDS conflict % |")
        print("|---|---:|---:|---:|---:|---:|---:|")
        for k, c in sorted(ctr.items(), key=lambda kv: -kv[1].get("SQ_VALU_MFMA_BUSY_CYCLES", 0)):
            grbm = c.get("GRBM_GUI_ACTIVE", 0) / 8
            ns = sum(wall[k].values())
            mfma = 100 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (grbm * 1024) if grbm else 0
            lds = c.get("SQ_LDS_IDX_ACTIVE", 0)
            confl = 100 * c.get("SQ_LDS_BANK_CONFLICT", 0) / lds if lds else 0
            clk = grbm / ns if ns else 0
            print(f"| `{k}` | {len(wall[k])} | {ns / 1e6:.2f} | {clk:.2f} | {mfma:.1f} | {c.get('SQ_INSTS_LDS', 0) / 1e6:.1f} | {confl:.1f} |")
        print()


if __name__ == "__main__":
    main(sys.argv[1:])
