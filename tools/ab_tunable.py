"""A/B: F.linear fwd+bwd at the Llama-3-8B shapes with the committed TunableOp table on vs off (same process)."""
import json, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from accelerate_hpc_test_amd.ops import gemm_tuning
import torch.cuda.tunable as tunable

def run(lin, x, g, iters=10):
    for _ in range(2):
        y = lin(x); y.backward(g)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(iters):
        y = lin(x); y.backward(g)
    torch.cuda.synchronize(); return (time.perf_counter() - t) / iters * 1000

ok = gemm_tuning.load_tuned_gemms()
print("table loaded:", ok, "entries:", len(tunable.get_results()), flush=True)
for out_f, in_f in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]:
    lin = torch.nn.Linear(in_f, out_f, bias=False, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(8192, in_f, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(8192, out_f, device="cuda", dtype=torch.bfloat16)
    tunable.enable(True); on = run(lin, x, g)
    tunable.enable(False); off = run(lin, x, g)
    fl = 6 * 8192 * in_f * out_f
    print(json.dumps({"out": out_f, "in": in_f, "tuned_ms": round(on, 3), "default_ms": round(off, 3),
                      "tuned_tflops": round(fl / on / 1e9, 1), "default_tflops": round(fl / off / 1e9, 1)}), flush=True)
