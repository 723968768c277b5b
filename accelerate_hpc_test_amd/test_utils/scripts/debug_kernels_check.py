"""Run one kernel of every family on the debug build of the extension (`_C_debug`, device bounds checks compiled in,
SURVEY §5.2) and report, as one JSON line, whether any check fired on valid inputs, whether the deliberate violations
(the check self-test's overshooting grid, an out-of-vocabulary cross-entropy label) were caught, and the largest
difference against the release kernels' results. Run with ACCELERATE_DEBUG_KERNELS=1 (tests/test_debug_kernels_gpu.py)."""

import importlib
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))


def main():
    assert os.environ.get("ACCELERATE_DEBUG_KERNELS") == "1"
    from accelerate_hpc_test_amd.ops import _ext, fp8, fused
    from accelerate_hpc_test_amd.ops.multi_tensor import FusedAdamStep

    dbg = _ext.ext()
    rel = importlib.import_module("accelerate_hpc_test_amd._C")
    assert dbg.debug_build and not rel.debug_build
    dev = "cuda"
    torch.manual_seed(0)
    out = {"families": {}}

    def fam(name, diff):
        out["families"][name] = {"status": int(dbg.debug_status()), "max_diff": float(diff)}

    # attention (fwd + bwd, causal, GQA, K/V prefix)
    q = torch.randn(1, 512, 8, 128, device=dev, dtype=torch.bfloat16)
    k = torch.randn(1, 1024, 2, 128, device=dev, dtype=torch.bfloat16)
    v = torch.randn_like(k)
    s = 1 / math.sqrt(128)
    o1, l1 = dbg.flash_attn_fwd(q, k, v, s, True)
    o2, l2 = rel.flash_attn_fwd(q, k, v, s, True)
    do = torch.randn_like(o1)
    g1 = [torch.empty_like(t) for t in (q, k, v)]
    g2 = [torch.empty_like(t) for t in (q, k, v)]
    dbg.flash_attn_bwd(do, q, k, v, o1, l1, *g1, s, True)
    rel.flash_attn_bwd(do, q, k, v, o2, l2, *g2, s, True)
    fam("attention", max((o1 - o2).abs().max(), *[(a - b).abs().max() for a, b in zip(g1, g2)]))
    # fp8 GEMM (the hand-written MX-MFMA kernel) and MXFP8
    a = torch.randn(512, 512, device=dev, dtype=torch.bfloat16)
    b = torch.randn(256, 512, device=dev, dtype=torch.bfloat16)
    one = torch.ones(1, device=dev)
    a8, b8 = fp8.cast(a, one), fp8.cast(b, one)
    c1 = dbg.fp8_gemm(a8, b8, one, one, 1.0, False, False, None, False)
    c2 = rel.fp8_gemm(a8, b8, one, one, 1.0, False, False, None, False)
    fam("fp8_gemm", (c1.float() - c2.float()).abs().max())
    # grouped GEMM (MoE experts)
    from accelerate_hpc_test_amd.models.moe import expert_layout

    E, H, N = 4, 256, 256
    e = torch.randint(0, E, (300,), device=dev)
    _, _, seg, R = expert_layout(e, E)
    x = torch.randn(R, H, device=dev, dtype=torch.bfloat16)
    w = torch.randn(E, N, H, device=dev, dtype=torch.bfloat16)
    y1, y2 = torch.empty(R, N, device=dev, dtype=torch.bfloat16), torch.empty(R, N, device=dev, dtype=torch.bfloat16)
    dbg.grouped_gemm(x, w, y1, seg, 1, one, torch.ones(E, device=dev), 1.0, False)
    rel.grouped_gemm(x, w, y2, seg, 1, one, torch.ones(E, device=dev), 1.0, False)
    fam("grouped_gemm", (y1.float() - y2.float()).abs().max())
    # RMSNorm + RoPE
    xn = torch.randn(64, 4096, device=dev, dtype=torch.bfloat16)
    wn = torch.randn(4096, device=dev, dtype=torch.bfloat16)
    r1 = dbg.rmsnorm_fwd(xn, None, wn, 1e-5, None)[0]
    r2 = rel.rmsnorm_fwd(xn, None, wn, 1e-5, None)[0]
    qkv = torch.randn(1, 64, 12, 128, device=dev, dtype=torch.bfloat16)
    cos, sin = torch.randn(64, 64, device=dev), torch.randn(64, 64, device=dev)
    p1 = dbg.rope_out(qkv, cos, sin, None, 8, 12, 128, 1.0)
    p2 = rel.rope_out(qkv, cos, sin, None, 8, 12, 128, 1.0)
    fam("norm_rope", max((r1 - r2).abs().max(), (p1 - p2).abs().max()))
    # cross entropy with valid labels, then multi-tensor AdamW
    logits = torch.randn(64, 1000, device=dev, dtype=torch.bfloat16)
    lab = torch.randint(0, 1000, (64,), device=dev)
    x1 = dbg.xent_fwd(logits, lab, -100)[0]
    x2 = rel.xent_fwd(logits, lab, -100)[0]
    fam("xent", (x1 - x2).abs().max())
    ps = [torch.randn(1000, device=dev, requires_grad=True), torch.randn(77, 33, device=dev, requires_grad=True)]
    ref = [p.detach().clone() for p in ps]
    opt = torch.optim.AdamW(ps, lr=1e-2)
    for p in ps:
        p.grad = torch.randn_like(p)
    ref_opt = torch.optim.AdamW([r.requires_grad_() for r in ref], lr=1e-2)
    for r_, p in zip(ref, ps):
        r_.grad = p.grad.clone()
    FusedAdamStep(opt).step()
    ref_opt.step()
    fam("adamw", max((p - r_).abs().max() for p, r_ in zip(ps, ref)))
    # deliberate violations: the check must fire and the access must not happen
    guard = torch.zeros(1024 + 256, device=dev)
    assert dbg.debug_selftest(guard[:1024], 256)
    torch.cuda.synchronize()
    out["selftest_status"] = int(dbg.debug_status())
    out["selftest_guard_untouched"] = bool((guard[1024:] == 0).all()) and bool((guard[:1024] == 1).all())
    bad = lab.clone()
    bad[5] = 5000
    dbg.xent_fwd(logits, bad, -100)
    out["bad_label_status"] = int(dbg.debug_status())
    out["after_clear"] = int(dbg.debug_status())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
