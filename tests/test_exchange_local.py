"""parallel.exchange.LocalComm: the group of a rank that serves only its own keys (a
host-routed process of an N-GPU job). World 1 and every collective an identity, also when
a default process group exists (then ``group=None`` would mean that world group)."""
import torch

from shellac_amd.parallel.exchange import (LocalComm, all_gather, all_gather_rows, all_reduce,
                                           all_to_all_rows, allreduce_stats, barrier, dist_info,
                                           exchange_counts)


def test_local_comm_is_world_one_identity():
    g = LocalComm()
    assert dist_info(g) == (0, 1)
    x = torch.arange(12, dtype=torch.int64).view(6, 2)
    assert torch.equal(all_to_all_rows(x, [6], [6], g), x)
    assert torch.equal(exchange_counts(torch.tensor([5]), g), torch.tensor([5]))
    out = torch.empty(4, dtype=torch.int64)
    all_gather_rows(out, torch.tensor([1, 2, 3, 4]), g)
    assert out.tolist() == [1, 2, 3, 4]
    outs = [torch.zeros(3)]
    all_gather(outs, torch.ones(3), g)
    assert outs[0].tolist() == [1.0, 1.0, 1.0]
    t = torch.tensor([7])
    all_reduce(t, group=g)
    assert t.item() == 7
    barrier(g)  # no process group needed
    assert allreduce_stats({"a": 3, "b": 4}, "cpu", g) == {"a": 3, "b": 4}
