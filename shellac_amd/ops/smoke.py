"""Platform smoke ops named by BASELINE.json: the MFMA "hello" tile kernel."""
from __future__ import annotations

import torch

from .._native import core


def mfma_hello(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Batched 32x16 @ 16x32 bf16 -> fp32 on one ``v_mfma_f32_32x32x16_bf16`` per tile.

    a: [T, 32, 16] bf16, b: [T, 16, 32] bf16 (cuda) -> [T, 32, 32] fp32.
    """
    if not a.is_cuda:
        raise RuntimeError("mfma_hello needs a gfx950 device")
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise TypeError("bf16 inputs required")
    if a.dim() != 3 or tuple(a.shape[1:]) != (32, 16) or tuple(b.shape[1:]) != (16, 32) \
            or a.shape[0] != b.shape[0]:
        raise ValueError(f"bad shapes {tuple(a.shape)} {tuple(b.shape)}")
    a = a.contiguous()
    b = b.contiguous()
    t = a.shape[0]
    c = torch.empty((t, 32, 32), dtype=torch.float32, device=a.device)
    core().mfma_hello(a.data_ptr(), b.data_ptr(), c.data_ptr(), t,
                      torch.cuda.current_stream(a.device).cuda_stream)
    return c
