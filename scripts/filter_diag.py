#!/usr/bin/env python3
"""Diagnose the HBM backend presence filter after rebuilds: for every stored key that
misses, report whether the filter answered (skip counter moved) or the GPU did.
Scenario of tests/test_hbm_backend_gpu.py::test_hbm_presence_filter_*: 3000 keys
into a 1024-slot index (evictions + filter rebuilds)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from shellac_amd import core  # noqa: E402


def main():
    for filt in (True, False):
        be = core().hbm_backend([0], 64 << 20, 256, 1 << 16, 0, sweep_interval_s=1,
                                presence_filter=filt)
        keys = [b"/pf/%d" % i for i in range(3000)]
        for i, k in enumerate(keys):
            be.set(k, b"v%d" % i, 0, 0)
        deadline = time.time() + 3
        while be.get(keys[-1]) is None and time.time() < deadline:
            time.sleep(0.01)
        time.sleep(2.5)
        st = be.stats()
        live = st["hbm_live_objects"]
        miss_filter, miss_gpu, wrong, hits = [], [], [], 0
        for i, k in enumerate(keys):
            s0 = be.stats().get("hbm_filter_skips", 0)
            r = be.get(k)
            s1 = be.stats().get("hbm_filter_skips", 0)
            if r == (b"v%d" % i, 0):
                hits += 1
            elif r is not None:
                wrong.append(i)
            elif s1 > s0:
                miss_filter.append(i)
            else:
                miss_gpu.append(i)
        print(f"[diag] filter={filt} live={live} hits={hits} rebuilds="
              f"{st.get('hbm_filter_rebuilds')} adds={st.get('hbm_filter_adds')} "
              f"wrong={wrong[:10]} gpu_misses={len(miss_gpu)} filter_misses={len(miss_filter)}",
              flush=True)
        # a key the GPU has but the filter refused would be a false negative: with the
        # filter on, every filter miss whose key is live is a bug; list the newest ones
        print(f"[diag] filter misses (newest 10): {miss_filter[-10:]}", flush=True)


if __name__ == "__main__":
    main()
