"""Multi-process (world_size 2, gloo on CPU) coverage of the data-parallel path:
the gradient all-reduce hook the learner calls between backward and clip+Adam,
and the global env-id sharding that makes per-env trajectories invariant to the
number of GPUs."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from evacx.trainer import make_allreduce_hook
    hook = make_allreduce_hook(dist, world)
    g = torch.arange(10, dtype=torch.float32) * (rank + 1)
    hook(g)
    out[rank] = g.tolist()
    # sharding: rank r owns global env ids [r*E, (r+1)*E) -> seeds 1234 + global id
    E = 5
    seeds = [1234 + rank * E + i for i in range(E)]
    lst = [None] * world
    dist.all_gather_object(lst, seeds)
    if rank == 0:
        out["seeds"] = sum(lst, [])
    dist.barrier()
    dist.destroy_process_group()


def test_grad_allreduce_and_sharding_world2():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "dqn-marl_amd"))
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    expect = [(i * 1 + i * 2) / 2 for i in range(10)]
    assert out[0] == pytest.approx(expect) and out[1] == pytest.approx(expect)
    assert out["seeds"] == [1234 + i for i in range(10)]  # == the single-GPU run's seeds
