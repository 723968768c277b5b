"""Per-shape hipBLASLt algorithm selection for the plain library GEMMs (linear fwd / dgrad / wgrad).

hipBLASLt's default heuristic picks a solution from a shape→kernel table; on gfx950 it frequently lands on a
MI16x16 / depth-32 tile for our Llama shapes (measured: forward x·Wᵀ GEMMs at ≈1.0 PF/s vs ≈1.5 PF/s for the same
FLOPs in wgrad). PyTorch's TunableOp benchmarks every hipBLASLt/rocBLAS solution per (op, layout, M, N, K) once and
records the winner. We run that search offline on an MI355X (`bench.py --gemm-tuning tune`), commit the result
table under `ops/tuned/`, and load it read-only at start-up (`--gemm-tuning auto`, the default) — no tuning happens
inside a timed run.
"""

from __future__ import annotations

import os
from typing import Optional

TUNED_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned")
DEFAULT_TABLE = os.path.join(TUNED_DIR, "tunableop_gfx950.csv")


def load_tuned_gemms(path: Optional[str] = None) -> bool:
    """Enable TunableOp in lookup-only mode with the committed result table. Returns True if a table was loaded."""
    import torch

    path = path or DEFAULT_TABLE
    if not torch.cuda.is_available() or not os.path.isfile(path):
        return False
    import torch.cuda.tunable as tunable

    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.record_untuned_enable(False)
    ok = tunable.read_file(path)
    return bool(ok)


def start_gemm_tuning(out_path: str, max_duration_ms: int = 30, max_iterations: int = 100) -> None:
    """Enable TunableOp search: every new GEMM shape is benchmarked over all solutions on first use; the table is
    written to `out_path` at exit (or with `finish_gemm_tuning`)."""
    import torch.cuda.tunable as tunable

    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_filename(out_path, insert_device_ordinal=False)
    tunable.set_max_tuning_duration(max_duration_ms)
    tunable.set_max_tuning_iterations(max_iterations)


def finish_gemm_tuning() -> None:
    import torch.cuda.tunable as tunable

    # results are persisted by TunableOp itself (as they are found and at exit); stop searching new shapes
    tunable.tuning_enable(False)
