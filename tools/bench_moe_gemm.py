"""MoE expert GEMMs at Mixtral-8x7B shapes (8 experts, top-2, 8192 tokens -> 16384 routed rows): the HIP grouped GEMM
(one launch over the device segment table, no host sync) vs one hipBLASLt GEMM per expert (torch.mm on the segment
slices, which needs the segment table on the host: one device->host copy per layer, timed in). bf16, median ms.

    python tools/bench_moe_gemm.py [--tokens 8192] [--skew 0]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def tm(fn, iters=10, rounds=3):
    out = []
    for _ in range(rounds):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t) / iters * 1e3)
    return statistics.median(out)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tokens", type=int, default=8192)
    p.add_argument("--skew", type=float, default=0.0, help="routing skew: 0 = uniform experts")
    a = p.parse_args()
    from accelerate_hpc_test_amd.models.moe import expert_layout, grouped_mm
    from accelerate_hpc_test_amd.ops import gemm_tuning

    gemm_tuning.load_tuned_gemms()
    E, H, I = 8, 4096, 14336
    g = torch.Generator(device="cuda").manual_seed(0)
    w_logits = torch.linspace(a.skew, -a.skew, E, device="cuda")
    probs = torch.softmax(torch.randn(a.tokens, E, device="cuda", generator=g) + w_logits, -1)
    flat_e = torch.topk(probs, 2, -1)[1].reshape(-1)
    _, _, seg, R = expert_layout(flat_e, E)
    bounds = seg.tolist()
    for name, (N, K) in {"gate_up": (2 * I, H), "down": (H, I)}.items():
        x = torch.randn(R, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(E, N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        out = torch.empty(R, N, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * bounds[-1] * N * K

        def per_expert_fwd():
            b = seg.tolist()  # the host sync a host-driven per-expert loop needs
            for e in range(E):
                lo, hi = b[e], b[e + 1]
                if hi > lo:
                    torch.mm(x[lo:hi], w[e].t(), out=out[lo:hi])

        t_grp = tm(lambda: grouped_mm(x, w, seg, 1, out))
        t_pe = tm(per_expert_fwd)
        # weight gradient: dW_e = dy_e^T x_e over each expert's rows (K-segmented)
        dy = torch.randn(R, N, device="cuda", dtype=torch.bfloat16)
        dyT, xT = dy.t().contiguous(), x.t().contiguous()
        dw = torch.empty(E, N, K, device="cuda", dtype=torch.bfloat16)

        def per_expert_wgrad():
            b = seg.tolist()
            for e in range(E):
                lo, hi = b[e], b[e + 1]
                torch.mm(dyT[:, lo:hi], xT[:, lo:hi].t(), out=dw[e])

        t_grp_w = tm(lambda: grouped_mm(dyT, xT, seg, 2, dw))
        t_pe_w = tm(per_expert_wgrad)
        print(json.dumps({"gemm": name, "rows": bounds[-1], "R": R, "grouped_ms": round(t_grp, 3),
                          "grouped_tflops": round(flops / t_grp / 1e9), "per_expert_ms": round(t_pe, 3),
                          "per_expert_tflops": round(flops / t_pe / 1e9), "grouped_wgrad_ms": round(t_grp_w, 3),
                          "per_expert_wgrad_ms": round(t_pe_w, 3), "wgrad_per_expert_tflops": round(flops / t_pe_w / 1e9),
                          "wgrad_grouped_tflops": round(flops / t_grp_w / 1e9)}), flush=True)


if __name__ == "__main__":
    main()
