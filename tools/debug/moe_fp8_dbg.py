import torch, torch.nn.functional as F
import sys; sys.path.insert(0, '.')
from tests.test_kernels_gpu import _routed, _rel
from accelerate_hpc_test_amd.models import moe
from accelerate_hpc_test_amd.ops import fp8
from accelerate_hpc_test_amd.ops.fp8 import E4M3_MAX, Fp8Recipe
torch.manual_seed(0)
counts = [200, 0, 77, 300]; E, H, I = 4, 256, 384
ex = moe.MoEExperts(E, H, I).to('cuda', torch.bfloat16)
with torch.no_grad():
    ex.w_gate_up.normal_(0, 0.05); ex.w_down.normal_(0, 0.05)
x, seg, dest = _routed(counts, H, seed=1)
b = seg.tolist()
def q(t):
    s = E4M3_MAX / t.float().abs().max().clamp_min(1e-12)
    return (t.float() * s).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).float() / s
rec = Fp8Recipe()
y, st = moe._fp8_fwd(x, ex.w_gate_up.data, ex.w_down.data, seg, rec)
h = st[0]
hs = torch.zeros(x.shape[0], 2 * I, device='cuda')
for e in range(E):
    lo, hi = b[e], b[e+1]
    if hi > lo: hs[lo:hi] = q(x)[lo:hi] @ q(ex.w_gate_up[e]).t()
print('h rel', _rel(h, hs), 'h nan', h.isnan().any().item())
w8, w8t, am = moe._expert_weight_fp8(ex.w_gate_up.data, rec, 'k')
print('amax', am.tolist(), [ex.w_gate_up[e].float().abs().max().item() for e in range(E)])
for e in range(E):
    print('w8 eq', e, torch.equal(w8[e].float(), (q(ex.w_gate_up[e]) * (E4M3_MAX/ex.w_gate_up[e].float().abs().max())).to(torch.float8_e4m3fn).float()))
x8 = fp8.cast(x, fp8.Scale(fp8.amax(x), E4M3_MAX))
print('x8 vs q', _rel(x8.float() * fp8.amax(x) / E4M3_MAX, q(x)))
# direct grouped
out = torch.empty_like(h)
moe.grouped_mm(x8, w8, seg, 1, out, fp8.amax(x), am, 1.0 / (E4M3_MAX * E4M3_MAX))
print('direct h rel', _rel(out, hs))
for e in range(E):
    lo, hi = b[e], b[e+1]
    if hi > lo: print(e, _rel(out[lo:hi], hs[lo:hi]), _rel(h[lo:hi], hs[lo:hi]))
