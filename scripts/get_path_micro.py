"""The GET half of the N=1 step in isolation (no SET beside it): a 16 GiB shard holding the
bench's 4M objects, 1M-request Zipf(0.99) batches, GPU-event time per batch (median of 20)
of (a) the coalescing lookup alone, (b) lookup + the gather with its expand tail, (e) the
coalescing claims alone (no probe), (f) k_probe of the batch's distinct keys, (g) k_probe
of all 1M requests. (Round 6 also timed a fused lookup + gather here: rejected, see
profiles/archive/r6_fused_gather_rejected.) `python scripts/get_path_micro.py`"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shellac_amd import core  # noqa: E402
from shellac_amd.bench.workload import Workload  # noqa: E402
from shellac_amd.ops.cache import CacheShard, coalesce  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    nkeys, n = 4 << 20, 1 << 20
    wl = Workload(nkeys, dev)
    sh = CacheShard(16 << 30, 1 << 22, 1 << 16, dev)
    for s0 in range(0, nkeys, 1 << 18):
        b = wl.set_batch(torch.arange(s0, s0 + (1 << 18), device=dev))
        sh.store(b.keys, b.values, b.val_off, b.vlen, b.flags, b.expire)
    torch.cuda.synchronize()
    batches = [wl.digests.index_select(0, wl.sample_ids(n, 100 + i)).contiguous()
               for i in range(8)]
    table = torch.zeros(int(core().coalesce_table_slots(n)), dtype=torch.int32, device=dev)
    out = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    osz = torch.empty(n, dtype=torch.int64, device=dev)
    oof = torch.empty(n, dtype=torch.int64, device=dev)

    def timed(fn, reps=20):
        ts = []
        for i in range(reps + 3):
            keys = batches[i % len(batches)]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn(keys)
            b.record()
            b.synchronize()
            if i >= 3:
                ts.append(a.elapsed_time(b) * 1000)
        return statistics.median(ts)

    def look(keys):
        sh.lookup_coalesced(keys, table=table, blocked=True)
        # (the table is left dirty: clean it outside the timed region is not possible
        # here, so this variant re-zeros it)
        table.zero_()

    def look_gather(keys):
        lk, first, cslot = sh.lookup_coalesced(keys, table=table, blocked=True)
        sh.gather(lk, out, out_cap=out.numel(), expand=(first, osz, oof, table, cslot))

    zero = timed(lambda k: table.zero_())
    print(f"table.zero_ {zero:.1f} us")
    print(f"(a) lookup_coalesced alone {timed(look) - zero:.1f} us")
    print(f"(b) lookup + gather(expand) {timed(look_gather):.1f} us")
    lk, _, _ = sh.lookup_coalesced(batches[0], table=table, blocked=True)
    table.zero_()
    print(f"response bytes per batch {int(lk.total().item())}")
    cs = torch.zeros_like(table)

    def co_only(keys):  # k_coalesce<false>: LDS + global claims, no probe
        coalesce(keys, cs)
        cs.zero_()

    uniq = [torch.unique(k, dim=0) for k in batches]
    print(f"distinct keys per batch {uniq[0].shape[0]}")
    print(f"(e) coalesce only (claims, no probe) {timed(co_only) - zero:.1f} us")
    k_u = iter(range(10 ** 9))
    print(f"(f) k_probe of the distinct keys {timed(lambda k: sh.lookup(uniq[next(k_u) % 8])):.1f} us")
    print(f"(g) k_probe of all 1M requests {timed(lambda k: sh.lookup(k)):.1f} us")


if __name__ == "__main__":
    main()
