"""After a few fp8 training steps, list which per-tensor fp8 GEMM problems hipBLASLt took (ms > 0) or declined (-1)."""
import json
import sys

sys.path.insert(0, ".")
from accelerate_hpc_test_amd.ops._ext import ext  # noqa: E402


def dump(path):
    with open(path, "w") as f:
        json.dump([{"M": m, "N": n, "K": k, "candidates": c, "ms": ms} for m, n, k, c, ms in ext().blaslt_fp8_plans()], f)
