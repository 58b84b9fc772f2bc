"""How a stripe batch is split over devices (cfsec_batch_partition, the split
cfsec_rs_*_stripes / cfsec_ec_reconstruct_batch use for host memory) -- host only, no GPU.

Properties: every stripe goes to exactly one device; the devices take contiguous, non-decreasing
runs in stripe order; each device's byte load is within one stripe's bytes of the even share.  A
gloo world-2 run then splits one blobnode tasklet between two ranks with the same function, as a
node-level caller would hand each GPU process its part: together the ranks cover the tasklet
exactly once.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from chubaofs_amd import _lib


def check(nbytes, ndev):
    dev = _lib.batch_partition(nbytes, ndev)
    assert len(dev) == len(nbytes)
    assert all(0 <= d < ndev for d in dev)
    assert all(a <= b for a, b in zip(dev, dev[1:])), "runs must be contiguous and ordered"
    total = sum(nbytes)
    if total:
        load = [0] * ndev
        for b, d in zip(nbytes, dev):
            load[d] += b
        big = max(nbytes)
        for d in range(ndev):
            assert abs(load[d] - total / ndev) <= big, (load, total / ndev, big)
    return dev


@pytest.mark.parametrize("ndev", [1, 2, 3, 4, 8])
def test_partition_properties(ndev):
    rng = np.random.default_rng(ndev)
    for n in (0, 1, 2, 7, 8, 64, 1000):
        check([int(x) for x in rng.integers(1, 1 << 30, n)], ndev)
        check([16 * 349526] * n, ndev)  # a uniform put batch
        # a blobnode tasklet: 64 bids of mixed sizes (work_shard_getter.go BidsSplit, <= 16 MiB/vunit)
        check([int(x) * 36 for x in rng.integers(0, 1 << 18, n)], ndev)


def test_partition_uniform_is_even():
    assert _lib.batch_partition([10] * 8, 4) == [0, 0, 1, 1, 2, 2, 3, 3]
    assert _lib.batch_partition([10] * 64, 8) == [d for d in range(8) for _ in range(8)]
    assert _lib.batch_partition([0, 0, 0], 2) == [0, 0, 1]
    with pytest.raises(_lib.ErrInvalidArg):
        _lib.batch_partition([1, 2], 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, nbytes):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = _lib.batch_partition(nbytes, world)
        mine = torch.tensor([i for i, d in enumerate(dev) if d == rank] or [-1], dtype=torch.int64)
        load = torch.tensor([sum(nbytes[i] for i, d in enumerate(dev) if d == rank)], dtype=torch.int64)
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([len(mine)], dtype=torch.int64))
        width = int(max(s.item() for s in sizes))
        padded = torch.full((width,), -1, dtype=torch.int64)
        padded[:len(mine)] = mine
        got = [torch.zeros(width, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(got, padded)
        loads = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(loads, load)
        covered = sorted(int(i) for g in got for i in g.tolist() if i >= 0)
        assert covered == list(range(len(nbytes))), covered
        assert sum(int(x.item()) for x in loads) == sum(nbytes)
    finally:
        dist.destroy_process_group()


def test_partition_splits_a_tasklet_across_ranks_gloo():
    rng = np.random.default_rng(7)
    nbytes = [int(x) * 36 for x in rng.integers(1, 1 << 18, 64)]  # EC16P20L2: 36 global shards per bid
    mp.spawn(_worker, args=(2, _free_port(), nbytes), nprocs=2, join=True)
