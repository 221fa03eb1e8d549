"""CPU placement for the serving processes.

A two-socket host runs the proxy's reactors, the load generator and the origin wherever
the scheduler puts them; a request then crosses sockets on every loopback hop. Pinning
each event-loop thread to its own core, all on one socket, keeps a request's socket
buffers and connection state in one L3 (nginx's ``worker_cpu_affinity``)."""
from __future__ import annotations

import os
from typing import List, Sequence


def parse_cpus(spec: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11] ('' -> [])."""
    out: List[int] = []
    for part in (spec or "").split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def format_cpus(cpus: Sequence[int]) -> str:
    return ",".join(str(c) for c in cpus)


def allowed_cpus() -> List[int]:
    try:
        return sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return list(range(os.cpu_count() or 1))


def plan(groups: Sequence[int], cpus: Sequence[int] = ()) -> List[List[int]]:
    """Split the lowest allowed CPUs (on a Linux two-socket host: socket 0's cores
    first) into consecutive groups of the given sizes. Returns [] for every group when
    fewer CPUs are allowed than asked for (no pinning then)."""
    cpus = list(cpus) or allowed_cpus()
    need = sum(groups)
    if need <= 0 or len(cpus) < need:
        return [[] for _ in groups]
    out, k = [], 0
    for g in groups:
        out.append(cpus[k:k + g])
        k += g
    return out


def pin_process(cpus: Sequence[int]) -> None:
    """Restrict this process (and the threads it creates afterwards) to `cpus`."""
    if cpus:
        os.sched_setaffinity(0, set(int(c) for c in cpus))
