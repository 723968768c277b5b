"""A Linear's two backward GEMMs at the Llama-3-8B shapes, each in the layout the training step has its operands in:
the MN-major-A asm kernel (ext().bf16_gemm_asm_amn: dy and W read as stored, transposed in the LDS read) against
the path the step takes today (hipBLASLt after a transposed copy / in the both-token-major class).

  dgrad  dx [T, K] = dy [T, N] . W [N, K]
         today: Wt = transpose(W) (HIP) + hipBLASLt linear(dy, Wt) (TN); also torch dy @ W (NN) for reference
         asm:   dx^T = W^T . dy^T -> bf16_gemm_asm_amn(W, dy, dx, trans_out=True)
  wgrad  dW [N, K] (fp32) = dy^T [N, T] . x [T, K], x saved token-contiguous as x^T [K, T]
         today: blaslt_wgrad_f32(dy, x^T, dW, x_t=True) (searched hipBLASLt algorithm)
         asm:   bf16_gemm_asm_amn(dy, x^T, dW)

    python tools/bench_gemm_amn.py [--tokens 8192] [--iters 20] [--rounds 3]"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
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
    p = argparse.ArgumentParser()
    p.add_argument("--tokens", type=int, default=8192)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--shapes", default="qkv,o,gate_up,down,lm_head")
    args = p.parse_args()
    from accelerate_hpc_test_amd.ops._ext import ext

    T = args.tokens
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336), "lm_head": (128256, 4096)}
    tot = {"dgrad_today": 0.0, "dgrad_asm": 0.0, "wgrad_today": 0.0, "wgrad_asm": 0.0}
    for name in args.shapes.split(","):
        N, K = shapes[name]
        torch.manual_seed(0)
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        xt = torch.randn(K, T, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * T * N * K
        # dgrad
        dx = torch.empty(T, K, device="cuda", dtype=torch.bfloat16)
        ref = (dy.float() @ w.float())
        assert ext().bf16_gemm_asm_amn(w, dy, dx, False, True)
        err_d = ((dx.float() - ref).norm() / ref.norm()).item()
        del ref
        td, tt, tn, ta = [], [], [], []
        wt = ext().transpose_bf16(w)
        for _ in range(args.rounds):
            td.append(timeit(lambda: torch.nn.functional.linear(dy, wt), args.iters))
            tt.append(timeit(lambda: ext().transpose_bf16(w), args.iters))
            tn.append(timeit(lambda: torch.mm(dy, w, out=dx), args.iters))
            ta.append(timeit(lambda: ext().bf16_gemm_asm_amn(w, dy, dx, False, True), args.iters))
        m_tn, m_t, m_nn, m_a = (statistics.median(x) for x in (td, tt, tn, ta))
        today = m_tn + m_t
        tot["dgrad_today"] += today
        tot["dgrad_asm"] += m_a
        print(json.dumps({"gemm": f"{name}.dgrad", "M": T, "N": K, "K": N,
                          "blaslt_tn_tflops": round(flops / m_tn / 1e9, 1), "transpose_ms": round(m_t, 3),
                          "blaslt_nn_tflops": round(flops / m_nn / 1e9, 1), "asm_amn_tflops": round(flops / m_a / 1e9, 1),
                          "today_ms": round(today, 3), "asm_ms": round(m_a, 3), "asm_vs_today": round(today / m_a, 3),
                          "asm_vs_blaslt_tn": round(m_tn / m_a, 3), "asm_rel_err": float(f"{err_d:.3g}")}), flush=True)
        del dx, wt
        # wgrad (fp32 out)
        dw = torch.empty(N, K, device="cuda", dtype=torch.float32)
        dw2 = torch.empty(N, K, device="cuda", dtype=torch.float32)
        ok_bl = ext().blaslt_wgrad_f32(dy, xt, dw2, False, True)
        assert ext().bf16_gemm_asm_amn(dy, xt, dw, False, False)
        ref = dy.float().t() @ xt.float().t()
        err_w = ((dw - ref).norm() / ref.norm()).item()
        del ref
        x = xt.t().contiguous()  # [T, K]: the layer input as the forward has it (no saved transposed copy)
        dw3 = torch.empty(N, K, device="cuda", dtype=torch.float32)
        assert ext().bf16_gemm_asm_amn(x, dy, dw3, False, True, True)
        err_w2 = ((dw3 - dw).norm() / dw.norm()).item()
        tb, ta, tab, tx = [], [], [], []
        for _ in range(args.rounds):
            if ok_bl:
                tb.append(timeit(lambda: ext().blaslt_wgrad_f32(dy, xt, dw2, False, True), args.iters))
            else:
                tb.append(timeit(lambda: torch.mm(dy.t(), xt.t(), out_dtype=torch.float32, out=dw2), args.iters))
            ta.append(timeit(lambda: ext().bf16_gemm_asm_amn(dy, xt, dw, False, False), args.iters))
            tab.append(timeit(lambda: ext().bf16_gemm_asm_amn(x, dy, dw3, False, True, True), args.iters))
            tx.append(timeit(lambda: ext().transpose_bf16(x), args.iters))
        m_b, m_a, m_ab, m_x = statistics.median(tb), statistics.median(ta), statistics.median(tab), statistics.median(tx)
        tot["wgrad_today"] += m_b
        tot["wgrad_asm"] += m_a
        tot["wgrad_asm_abmn"] = tot.get("wgrad_asm_abmn", 0.0) + m_ab
        tot["x_transpose"] = tot.get("x_transpose", 0.0) + m_x
        print(json.dumps({"gemm": f"{name}.wgrad", "M": N, "N": K, "K": T, "blaslt_runner": bool(ok_bl),
                          "blaslt_tflops": round(flops / m_b / 1e9, 1), "asm_amn_tflops": round(flops / m_a / 1e9, 1),
                          "asm_abmn_tflops": round(flops / m_ab / 1e9, 1), "x_transpose_ms": round(m_x, 3),
                          "asm_vs_blaslt": round(m_b / m_a, 3), "abmn_plus_no_transpose_vs_amn": round((m_a + m_x) / m_ab, 3),
                          "asm_rel_err": float(f"{err_w:.3g}"), "abmn_vs_amn_rel": float(f"{err_w2:.3g}")}), flush=True)
        del x, dw3
        del dy, w, xt, dw, dw2
        torch.cuda.empty_cache()
    print(json.dumps({"totals_ms_one_layer_each": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
