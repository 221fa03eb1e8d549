"""Device batch helpers for the sharded serving path: routing, permutation, scans,
load-balanced segmented copies. Each op runs the HIP kernel for ``cuda`` tensors
and the C++ host implementation for ``cpu`` tensors (same contract)."""
from __future__ import annotations

import torch

from .._native import core


def _s(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


class ScanWorkspace:
    """Reusable temp storage for device exclusive scans (hipcub)."""

    def __init__(self):
        self._buf: dict[torch.device, torch.Tensor] = {}

    def get(self, n: int, device: torch.device) -> torch.Tensor:
        need = core().scan_tmp_bytes(max(n, 1))
        buf = self._buf.get(device)
        if buf is None or buf.numel() < need:
            buf = torch.empty(max(need, 1 << 16) * 2, dtype=torch.uint8, device=device)
            self._buf[device] = buf
        return buf


_WS = ScanWorkspace()


def exclusive_scan(x: torch.Tensor) -> torch.Tensor:
    """int64 [n] -> int64 [n+1] exclusive prefix sums (out[n] = total)."""
    n = x.numel()
    src = torch.empty(n + 1, dtype=torch.int64, device=x.device)
    src[:n] = x
    src[n] = 0
    out = torch.empty(n + 1, dtype=torch.int64, device=x.device)
    if x.is_cuda:
        tmp = _WS.get(n, x.device)
        core().exclusive_scan(src.data_ptr(), out.data_ptr(), n, tmp.data_ptr(), tmp.numel(), _s(x))
    else:
        core().host_exclusive_scan(src.data_ptr(), out.data_ptr(), n)
    return out


def segcopy(src: torch.Tensor, src_off: torch.Tensor, dst_off: torch.Tensor,
            dst: torch.Tensor) -> torch.Tensor:
    """Copy segment i (dst_off[i+1]-dst_off[i] bytes) from src[src_off[i]:] to dst[dst_off[i]:].
    Offsets and lengths must be multiples of 16."""
    n = src_off.numel()
    assert dst_off.numel() == n + 1
    if src.is_cuda:
        core().segcopy(src.data_ptr(), src_off.data_ptr(), dst_off.data_ptr(), n, dst.data_ptr(),
                       _s(src))
    else:
        core().host_segcopy(src.data_ptr(), src_off.data_ptr(), dst_off.data_ptr(), n, dst.data_ptr())
    return dst


def gather_segments(addrs: torch.Tensor, dst_off: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """Like ``segcopy`` but segment i comes from the absolute address ``addrs[i]``
    (e.g. ``t.data_ptr() + k``) so one launch can assemble a buffer out of several
    tensors. All addresses must be on dst's device; offsets/lengths multiples of 16."""
    n = addrs.numel()
    assert dst_off.numel() == n + 1 and addrs.dtype == torch.int64
    if dst.is_cuda:
        core().segcopy(0, addrs.data_ptr(), dst_off.data_ptr(), n, dst.data_ptr(), _s(dst))
    else:
        core().host_segcopy(0, addrs.data_ptr(), dst_off.data_ptr(), n, dst.data_ptr())
    return dst


def route(keys: torch.Tensor, ring_pts: torch.Tensor, ring_owner: torch.Tensor,
          nranks: int) -> tuple[torch.Tensor, torch.Tensor]:
    """Owner rank of every digest on a consistent-hash ring -> (dest int32 [n], counts int64 [R])."""
    n = keys.shape[0]
    dest = torch.empty(n, dtype=torch.int32, device=keys.device)
    counts = torch.zeros(nranks, dtype=torch.int64, device=keys.device)
    npts = ring_pts.numel()
    if keys.is_cuda:
        core().route_keys(keys.data_ptr(), n, ring_pts.data_ptr(), ring_owner.data_ptr(), npts,
                          dest.data_ptr(), counts.data_ptr(), nranks, _s(keys))
    else:
        core().host_route_keys(keys.data_ptr(), n, ring_pts.data_ptr(), ring_owner.data_ptr(), npts,
                               dest.data_ptr(), counts.data_ptr(), nranks)
    return dest, counts


def scatter_positions(dest: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """Destination-grouped position of every element: perm[i] in [base[d], base[d]+counts[d])."""
    n = dest.numel()
    nranks = counts.numel()
    base = torch.zeros(nranks, dtype=torch.int64, device=dest.device)
    if nranks > 1:
        base[1:] = torch.cumsum(counts, 0)[:-1]
    cursor = torch.zeros(nranks, dtype=torch.int64, device=dest.device)
    perm = torch.empty(n, dtype=torch.int64, device=dest.device)
    if dest.is_cuda:
        core().scatter_by_dest(dest.data_ptr(), base.data_ptr(), n, nranks, cursor.data_ptr(),
                               perm.data_ptr(), _s(dest))
    else:
        core().host_scatter_by_dest(dest.data_ptr(), base.data_ptr(), n, nranks, cursor.data_ptr(),
                                    perm.data_ptr())
    return perm


def permute(x: torch.Tensor, perm: torch.Tensor) -> torch.Tensor:
    """out[perm[i]] = x[i] for rows of x (row bytes multiple of 4)."""
    x = x.contiguous()
    n = x.shape[0]
    out = torch.empty_like(x)
    rec = x.element_size() * (x.numel() // max(n, 1))
    if n == 0:
        return out
    if x.is_cuda:
        core().permute_records(x.data_ptr(), perm.data_ptr(), n, rec, out.data_ptr(), _s(x))
    else:
        core().host_permute_records(x.data_ptr(), perm.data_ptr(), n, rec, out.data_ptr())
    return out
