"""The SPMD harness rendezvous (tests/spmd.py): the parent hosts the TCPStore on a kernel-assigned
port and the ranks connect as clients, so back-to-back and concurrent groups never race for a
port (GPUTEST_r03 lost a bind-then-close race with EADDRINUSE). Stands in for the reference's
multi-task MiniCluster runs (``AllReduceImplTest.java:80-171``)."""
import threading

from tests.spmd import run_spmd


def _sum_ranks(rank, world):
    import torch

    from flink_ml_amd.parallel import comm

    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    comm.all_reduce_sum(t)
    return float(t.item())


def test_back_to_back_groups():
    for _ in range(4):
        assert run_spmd(_sum_ranks, 2) == [3.0, 3.0]


def test_concurrent_groups():
    out, errs = {}, []

    def go(i):
        try:
            out[i] = run_spmd(_sum_ranks, 2)
        except Exception as e:  # pragma: no cover - surfaced below
            errs.append(e)

    th = [threading.Thread(target=go, args=(i,)) for i in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    assert all(out[i] == [3.0, 3.0] for i in range(3))
