"""Microbenchmark of the HIP flash-attention kernels (fwd / bwd) at Llama-3-8B shapes: TFLOP/s on random data, next
to `torch.nn.functional.scaled_dot_product_attention` (the reference's attention: SDPA inside the user model) with each
ROCm backend torch ships (flash = AOTriton/CK flash kernels, efficient = memory-efficient kernels), GQA via
`enable_gqa`, same shapes and causal masks. `--no-sdpa` skips the library rows."""
import argparse, json, math, time
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from accelerate_hpc_test_amd.ops import _ext

p = argparse.ArgumentParser()
p.add_argument("--S", type=int, default=8192)
p.add_argument("--Hq", type=int, default=32)
p.add_argument("--Hkv", type=int, default=8)
p.add_argument("--B", type=int, default=1)
p.add_argument("--iters", type=int, default=10)
p.add_argument("--no-sdpa", action="store_true")
p.add_argument("--isolated", action="store_true", help="also time single launches after a 50 ms idle gap")
p.add_argument("--dbg", action="store_true", help="also time the causal backward's kernels separately and the dK/dV "
               "diagnostic variants (cache-hot fetch / no LDS commit); timing only")
p.add_argument("--dkdv-variants", default="", help="comma list of dq_waves:dkdv_waves:sched backward kernel choices "
               "(e.g. 8:8:0,4:4:2) timed in interleaved rounds in this process: causal / full backward and the causal "
               "dK/dV and dQ kernels alone")
p.add_argument("--fwd-variants", default="", help="comma list of forward kernels (0 = 8-wave, 1 = one wave per SIMD, "
               "attn_fwd_config) timed in interleaved rounds in this process, causal and full")
p.add_argument("--rounds", type=int, default=3)
a = p.parse_args()
e = _ext.ext()
D = 128
qkv = torch.randn(a.B, a.S, a.Hq + 2 * a.Hkv, D, device="cuda", dtype=torch.bfloat16)
q, k, v = qkv[:, :, :a.Hq], qkv[:, :, a.Hq:a.Hq + a.Hkv], qkv[:, :, a.Hq + a.Hkv:]
dqkv = torch.empty_like(qkv)
dq, dk, dv = dqkv[:, :, :a.Hq], dqkv[:, :, a.Hq:a.Hq + a.Hkv], dqkv[:, :, a.Hq + a.Hkv:]
scale = 1 / math.sqrt(D)
res = {}
for causal in (True, False):
    o, lse = e.flash_attn_fwd(q, k, v, scale, causal)
    do = torch.randn_like(o)
    f = 0.5 if causal else 1.0
    fl_fwd = 4 * a.B * a.Hq * a.S * a.S * D * f
    def tm(fn):
        fn(); torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters): fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / a.iters
    tf = tm(lambda: e.flash_attn_fwd(q, k, v, scale, causal))
    tb = tm(lambda: e.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, scale, causal))
    res["causal" if causal else "full"] = {"fwd_ms": round(tf * 1e3, 3), "fwd_tflops": round(fl_fwd / tf / 1e12, 1),
        "bwd_ms": round(tb * 1e3, 3), "bwd_tflops": round(2.5 * fl_fwd / tb / 1e12, 1)}
if a.dbg:
    o, lse = e.flash_attn_fwd(q, k, v, scale, True)
    do = torch.randn_like(o)
    dbg = {}
    for name, mode in (("dq_only", 8), ("dkdv", 4), ("dkdv_hot_fetch", 1), ("dkdv_no_commit", 2), ("dkdv_hot_no_commit", 3)):
        e.attn_debug_mode(mode)
        for _ in range(2):
            e.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, scale, True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            e.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, scale, True)
        torch.cuda.synchronize()
        dbg[name + "_ms"] = round((time.perf_counter() - t) / a.iters * 1e3, 3)
    e.attn_debug_mode(0)
    res["causal_bwd_parts"] = dbg
if a.dkdv_variants:
    variants = [tuple(int(x) for x in v.split(":")) for v in a.dkdv_variants.split(",")]
    e.attn_debug_mode(0)
    data = {}
    for causal in (True, False):
        o, lse = e.flash_attn_fwd(q, k, v, scale, causal)
        do = torch.randn_like(o)
        data[causal] = (o, lse, do)

    def timed(fn, n):
        fn(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n): fn()
        e1.record(); e1.synchronize()
        return e0.elapsed_time(e1) / n
    best = {}
    for _ in range(a.rounds):
        for qw, w, sch in variants:
            e.attn_dkdv_config(w, sch, qw)
            row = best.setdefault(f"{qw}:{w}:{sch}", {})
            for causal in (True, False):
                o, lse, do = data[causal]
                t = timed(lambda: e.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, scale, causal), a.iters)
                key = "causal_bwd_ms" if causal else "full_bwd_ms"
                row[key] = round(min(row.get(key, 1e9), t), 4)
            o, lse, do = data[True]
            for name, mode in (("causal_dkdv_only_ms", 4), ("causal_dq_only_ms", 8)):  # + the delta pass
                e.attn_debug_mode(mode)
                t = timed(lambda: e.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, scale, True), a.iters)
                e.attn_debug_mode(0)
                row[name] = round(min(row.get(name, 1e9), t), 4)
    e.attn_dkdv_config(4, 6, 8)
    res["dkdv_variants"] = best
if a.fwd_variants:
    fv = {}
    for _ in range(a.rounds):
        for w in (int(x) for x in a.fwd_variants.split(",")):
            e.attn_fwd_config(w)
            for causal in (True, False):
                f = 0.5 if causal else 1.0
                fn = lambda: e.flash_attn_fwd(q, k, v, scale, causal)
                fn(); torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters): fn()
                e1.record(); e1.synchronize()
                ms = e0.elapsed_time(e1) / a.iters
                row = fv.setdefault(f"w4={w}", {})
                key = "causal_fwd_ms" if causal else "full_fwd_ms"
                row[key] = round(min(row.get(key, 1e9), ms), 4)
                row[key.replace("ms", "tflops")] = round(4 * a.B * a.Hq * a.S * a.S * D * f / (row[key] * 1e-3) / 1e12, 1)
    e.attn_fwd_config(0)
    res["fwd_variants"] = fv
if a.isolated:
    # one kernel at a time after an idle gap (clock recovered), timed by events around the single launch: against the
    # back-to-back loop above this separates sustained-power clock effects from the kernels' own cost
    iso = {}
    for causal in (True, False):
        o, lse = e.flash_attn_fwd(q, k, v, scale, causal)
        do = torch.randn_like(o)
        for name, fn in (("fwd", lambda: e.flash_attn_fwd(q, k, v, scale, causal)),
                         ("bwd", lambda: e.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, scale, causal))):
            ts = []
            for _ in range(5):
                torch.cuda.synchronize()
                time.sleep(0.05)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            iso[f"{'causal' if causal else 'full'}_{name}_ms"] = round(sorted(ts)[2], 3)
    res["isolated_median"] = iso
if not a.no_sdpa:
    import torch.nn.functional as F
    from torch.nn.attention import SDPBackend, sdpa_kernel

    def tm2(fn):
        fn(); torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters): fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / a.iters

    qt = q.transpose(1, 2).contiguous().requires_grad_()
    kt = k.transpose(1, 2).contiguous().requires_grad_()
    vt = v.transpose(1, 2).contiguous().requires_grad_()
    for bname, backend in (("sdpa_flash", SDPBackend.FLASH_ATTENTION), ("sdpa_efficient", SDPBackend.EFFICIENT_ATTENTION)):
        for causal in (True, False):
            key = f"{bname}_{'causal' if causal else 'full'}"
            f = 0.5 if causal else 1.0
            fl_fwd = 4 * a.B * a.Hq * a.S * a.S * D * f
            try:
                with sdpa_kernel(backend):
                    with torch.no_grad():
                        tf = tm2(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal, enable_gqa=True))
                    out = F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal, enable_gqa=True)
                    go = torch.randn_like(out)

                    def fb():
                        o2 = F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal, enable_gqa=True)
                        torch.autograd.grad(o2, (qt, kt, vt), go)
                    tfb = tm2(fb)
                tb = max(tfb - tf, 1e-9)
                res[key] = {"fwd_ms": round(tf * 1e3, 3), "fwd_tflops": round(fl_fwd / tf / 1e12, 1),
                            "bwd_ms": round(tb * 1e3, 3), "bwd_tflops": round(2.5 * fl_fwd / tb / 1e12, 1)}
            except Exception as exc:  # noqa: BLE001 - a backend that rejects the shape is reported, not fatal
                res[key] = {"error": repr(exc)[:200]}
print(json.dumps({"shape": vars(a), **res}))
