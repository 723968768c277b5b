"""Where the bf16 asm GEMM loop's cycles go: the same kernel with the LDS-DMA removed from the loop, the fragment reads
removed, or both (ext().bf16_gemm_asm_probe; timing only, results invalid), at one large shape and at the Llama shapes.

    python tools/bench_gemm_probe.py"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    from accelerate_hpc_test_amd.ops._ext import ext

    names = {0: "full", 1: "no_dma", 2: "no_reads", 3: "mfma_only", 4: "regload", 5: "regstage", 6: "spread", 7: "khalf", 8: "eight_waves"}
    ai = torch.randint(-3, 4, (512, 1024), device="cuda").to(torch.bfloat16)
    bi = torch.randint(-3, 4, (768, 1024), device="cuda").to(torch.bfloat16)
    oi = torch.empty(512, 768, device="cuda", dtype=torch.bfloat16)
    ref = (ai.float() @ bi.float().t()).to(torch.bfloat16)
    for v in (8, 6, 7):
        assert ext().bf16_gemm_asm_probe(ai, bi, oi, v)
        print(json.dumps({"variant": v, "exact": bool(torch.equal(oi, ref)), "max_err": float((oi.float() - ref.float()).abs().max())}),
              flush=True)
    for (m, n, k) in ((8192, 8192, 8192), (8192, 28672, 4096), (8192, 4096, 14336)):
        a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
        o = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        res = {"M": m, "N": n, "K": k}
        ts = {v: [] for v in names}
        for _ in range(3):
            ts["blaslt"] = ts.get("blaslt", []) + [timeit(lambda: torch.mm(a, b.t(), out=o))]
            for v in names:
                ts[v].append(timeit(lambda: ext().bf16_gemm_asm_probe(a, b, o, v)))
        f = 2.0 * m * n * k
        for v, xs in ts.items():
            res[names.get(v, v) + "_tflops"] = round(f / statistics.median(xs) / 1e9, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
