"""CPU, world_size 2 over gloo: pair sharding + the result all-gather reproduce the
single-process result (the N > 1 path of bench.py / fgreg.dist)."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO


def _worker(rank, world, port, out_path, costs):
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from fgreg import dist as fd
    import model_oracle as mo
    # equal-size sharding: each rank solves the Procrustes problems of its pairs
    n_pairs = 5
    rng = np.random.default_rng(0)
    a = torch.from_numpy(rng.normal(size=(6, n_pairs, 40, 3)).astype(np.float32))
    b = a + 0.01 * torch.from_numpy(rng.normal(size=a.shape).astype(np.float32))
    w = torch.from_numpy(rng.uniform(0.8, 1.0, (6, n_pairs, 40)).astype(np.float32))
    s, e = fd.shard_range(n_pairs, world, rank)
    local = mo.weighted_procrustes(a[:, s:e], b[:, s:e], w[:, s:e])          # (6, P_r, 3, 4)
    counts = [fd.shard_range(n_pairs, world, r)[1] - fd.shard_range(n_pairs, world, r)[0]
              for r in range(world)]
    full = fd.gather_pair_results(local, counts, pair_dim=1)
    # balanced shards for variable-size pairs
    shards = fd.balanced_shards(costs, world)
    mine = torch.tensor(shards[rank], dtype=torch.float32).view(1, -1, 1, 1)
    got = fd.gather_pair_results(mine, [len(x) for x in shards], pair_dim=1)
    if rank == 0:
        torch.save({'full': full, 'ref': mo.weighted_procrustes(a, b, w), 'got': got,
                    'shards': shards}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2])
def test_pair_sharding_gather_gloo(tmp_path, world):
    out = str(tmp_path / 'res.pt')
    costs = [20000, 12000, 30000, 8000, 15000, 22000, 9000]
    port = 29500 + os.getpid() % 1000
    mp.start_processes(_worker, args=(world, port, out, costs), nprocs=world, join=True,
                       start_method='spawn')
    res = torch.load(out, weights_only=True)
    assert torch.equal(res['full'], res['ref'])
    order = [i for s in res['shards'] for i in s]
    assert sorted(order) == list(range(len(costs)))
    assert res['got'].view(-1).tolist() == [float(i) for i in order]
    loads = [sum(costs[i] for i in s) for s in res['shards']]
    assert max(loads) - min(loads) <= max(costs)
