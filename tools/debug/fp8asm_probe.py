"""Compare the asm GEMM's LDS image after the first-tile DMA (FP8ASM_ISSUE) with the intended layout."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from accelerate_hpc_test_amd.ops._ext import ext

K = 512
g = torch.Generator().manual_seed(0)
a = torch.randint(0, 250, (256, K), generator=g, dtype=torch.uint8).cuda()
b = torch.randint(0, 250, (256, K), generator=g, dtype=torch.uint8).cuda()
img = ext().fp8asm_dma_probe(a, b).cpu()
a, b = a.cpu(), b.cpu()
exp = torch.full((135168,), 0x5A, dtype=torch.uint8)
for kt in range(2):
    for op, src in ((0, a), (1, b)):
        base = kt * 67584 + op * 33792
        for c in range(32):
            for rr in range(8):
                row = 8 * c + rr
                o = base + c * 1056 + rr * 128
                exp[o : o + 128] = src[row, kt * 128 : kt * 128 + 128]
bad = (img != exp)
print("mismatching bytes", int(bad.sum()), "of", bad.numel(), flush=True)
for kt in range(2):
    for op in range(2):
        base = kt * 67584 + op * 33792
        chunks = [c for c in range(32) if bad[base + c * 1056 : base + c * 1056 + 1024].any()]
        print(f"kt {kt} op {'AB'[op]}: bad chunks {chunks}", flush=True)
# where did chunk 1's data go? search the image for A row 8's first 16 bytes
for row in (8, 16, 24):
    pat = a[row, 0:16]
    hits = [i for i in range(0, 135168 - 16, 16) if torch.equal(img[i : i + 16], pat)]
    print(f"A row {row} k 0..15 found at {hits} (expected {(row // 8) * 1056 + (row % 8) * 128})", flush=True)
