#!/usr/bin/env python3
"""BASELINE.json platform check: the MFMA hello kernel (k_mfma_hello, one
v_mfma_f32_32x32x16_bf16 per wave) on a batch of tiles, checked against fp32 torch.bmm.
Run under rocprofv3 --pmc for the MFMA counters (scripts/mfma_pmc.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shellac_amd.ops.smoke import mfma_hello  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
tiles = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
a = torch.randn(tiles, 32, 16, generator=g, device=dev).to(torch.bfloat16)
b = torch.randn(tiles, 16, 32, generator=g, device=dev).to(torch.bfloat16)
for _ in range(3):
    c = mfma_hello(a, b)
torch.cuda.synchronize()
err = (c - torch.bmm(a.float(), b.float())).abs().max().item()
print(f"mfma_hello: {tiles} tiles of 32x32x16 bf16, max abs err vs fp32 bmm {err:.2e}")
assert err < 1e-3
