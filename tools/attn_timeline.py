"""Per-wave timeline of the HIP attention kernels (ext().attn_trace): where the causal kernels lose time against the
MFMA-bound ideal — per-workgroup fixed cost (prologue / epilogue), tail (CUs idle after their last workgroup), or the
per-tile rate itself.

    python tools/attn_timeline.py [--seq 8192] [--mask causal|full] [--pass fwd|bwd]

For each kernel: wall time (first wave start -> last wave end), the busy fraction of the 256 CUs' 2 workgroup slots,
a least-squares fit of workgroup duration = a + b x (64-key tiles it streams), i.e. a = fixed cost per workgroup and
b = time per tile, and the time after the median CU's last workgroup ended. One JSON line per kernel."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch


def analyse(name, tr, tiles_of, slots_per_cu, rate_hz):
    tr = tr.reshape(-1, 8, 4)  # [block, wave, (t0, t1, smid, tag)]
    live = tr[:, :, 1] > 0
    t0 = np.where(live, tr[:, :, 0], np.iinfo(np.int64).max).min(1)
    t1 = np.where(live, tr[:, :, 1], 0).max(1)
    ok = t1 > 0
    t0, t1, smid, tag = t0[ok], t1[ok], tr[ok, 0, 2], tr[ok, 0, 3]
    base = t0.min()
    s = (t0 - base) / rate_hz * 1e6
    e = (t1 - base) / rate_hz * 1e6
    dur = e - s
    tiles = np.array([tiles_of(int(t)) for t in tag], dtype=np.float64)
    A = np.stack([np.ones_like(tiles), tiles], 1)
    (a, b), *_ = np.linalg.lstsq(A, dur, rcond=None)
    wall = e.max()
    ncu = len(np.unique(smid))
    busy = dur.sum() / (wall * ncu * slots_per_cu)
    last = {}
    for cu, end in zip(smid, e):
        last[cu] = max(last.get(cu, 0.0), end)
    ends = np.array(sorted(last.values()))
    by_tag = {}
    for t, d in zip(tag, dur):
        by_tag.setdefault(int(t) & 0xFFFF, []).append(float(d))
    keys = sorted(by_tag)
    pick = sorted({keys[0], keys[len(keys) // 4], keys[len(keys) // 2], keys[3 * len(keys) // 4], keys[-1]})
    tile_us = {int(k): [round(float(np.median(by_tag[k])), 1), tiles_of(k)] for k in pick}  # tile index -> [median us, tiles]
    return {"kernel": name, "median_us_by_tile_index": tile_us, "workgroups": int(len(dur)), "cus_seen": ncu, "wall_us": round(float(wall), 1),
            "slot_busy_frac": round(float(busy), 3), "fixed_us_per_wg": round(float(a), 2),
            "us_per_tile": round(float(b), 3), "tiles_total": int(tiles.sum()),
            "ideal_us_at_fit_rate": round(float(tiles.sum() * b / (ncu * slots_per_cu)), 1),
            "tail_us_after_median_cu_end": round(float(wall - np.median(ends)), 1),
            "first_cu_idle_us": round(float(wall - ends.min()), 1),
            "mean_start_gap_us": round(float(np.diff(np.sort(s)).mean()), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mask", default="causal", choices=["causal", "full"])
    ap.add_argument("--pass", dest="which", default="both", choices=["fwd", "bwd", "both"])
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    a = ap.parse_args()
    from accelerate_hpc_test_amd.ops._ext import ext

    E = ext()
    S, Hq, Hkv, D = a.seq, a.hq, a.hkv, 128
    causal = a.mask == "causal"
    qkv = torch.randn(1, S, Hq + 2 * Hkv, D, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv[:, :, :Hq], qkv[:, :, Hq:Hq + Hkv], qkv[:, :, Hq + Hkv:]
    scale = D ** -0.5
    rate_hz = 100e6  # the constant-rate wall clock (s_memrealtime) runs at 100 MHz on MI355X
    # query heads per forward / dQ workgroup, as flash_attn.hip picks them (1 or 2; 2 -> one 8-wave workgroup per CU)
    two = (Hq // Hkv) % 2 == 0
    nh_f = 2 if two and os.environ.get("ACCELERATE_ATTN_FWD_HEADS", "2") == "2" else 1
    nh_q = 2 if two and os.environ.get("ACCELERATE_ATTN_DQ_HEADS", "2") == "2" else 1
    nq_f, nq = Hq // nh_f * (S // 128), Hq // nh_q * (S // 128)
    nkv = Hkv * (S // 128)
    buf = torch.zeros((nq + nkv) * 32, dtype=torch.int64, device="cuda")
    o, lse = E.flash_attn_fwd(q, k, v, scale, causal)  # warm
    dout = torch.randn_like(o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    E.flash_attn_bwd(dout, q, k, v, o, lse, dq, dk, dv, scale, causal)
    torch.cuda.synchronize()
    fwd_tiles = (lambda t: 2 * ((t & 0xFFFF) + 1)) if causal else (lambda t: S // 64)
    dkdv_tiles = (lambda t: (S - (t & 0xFFFF) * 128) // 64 * (Hq // Hkv)) if causal else (lambda t: S // 64 * (Hq // Hkv))
    if a.which in ("fwd", "both"):
        E.attn_trace(buf)
        E.flash_attn_fwd(q, k, v, scale, causal)
        torch.cuda.synchronize()
        E.attn_trace(torch.empty(0, dtype=torch.int64, device="cuda"))
        tr = buf[: nq_f * 32].cpu().numpy()
        print(json.dumps(dict(analyse("attn_fwd", tr, fwd_tiles, 2 // nh_f, rate_hz), seq=S, mask=a.mask, heads_per_wg=nh_f)),
              flush=True)
    if a.which in ("bwd", "both"):
        buf.zero_()
        E.attn_trace(buf)
        E.flash_attn_bwd(dout, q, k, v, o, lse, dq, dk, dv, scale, causal)
        torch.cuda.synchronize()
        E.attn_trace(torch.empty(0, dtype=torch.int64, device="cuda"))
        tr = buf.cpu().numpy()
        print(json.dumps(dict(analyse("attn_bwd_dq", tr[: nq * 32], fwd_tiles, 2 // nh_q, rate_hz), seq=S, mask=a.mask,
                              heads_per_wg=nh_q)), flush=True)
        print(json.dumps(dict(analyse("attn_bwd_dkdv", tr[nq * 32:], dkdv_tiles, 1, rate_hz), seq=S, mask=a.mask)), flush=True)


if __name__ == "__main__":
    main()
