"""Multi-rank forward check (run under torch.distributed.run; used by tests/test_gpu_dist.py):
every rank runs fgreg.RegTR.forward on its shard of a ModelNet batch (fgreg.dist.shard_range),
the per-pair poses are all-gathered (fgreg.dist.gather_pair_results, the bench's exchange),
and rank 0 compares them with a single forward over the whole batch on the same weights.
FGREG_DIST_BACKEND=gloo lets the ranks share one GPU (the 1-GPU box); nccl (RCCL) needs one GPU
per rank (tests/test_gpu_dist.py runs it at world size 1 on the 1-GPU box). Exit status 0 = match."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))


def main():
    import fgreg
    from fgreg import dist as fdist
    from fgreg.synthetic import make_batch
    backend = os.environ.get('FGREG_DIST_BACKEND', 'nccl')
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    local = int(os.environ.get('LOCAL_RANK', rank))
    ndev = torch.cuda.device_count()
    dev = torch.device('cuda', local % ndev if backend == 'gloo' else local)
    torch.cuda.set_device(dev)
    dist.init_process_group(backend)
    B = 2 * world + 1                                  # ragged shards
    torch.manual_seed(0)
    model = fgreg.RegTR(fgreg.config.get('modelnet')).to(dev).eval()
    src, tgt, _ = make_batch('modelnet', B)
    b0, b1 = fdist.shard_range(B, world, rank)
    counts = [fdist.shard_range(B, world, r)[1] - fdist.shard_range(B, world, r)[0]
              for r in range(world)]
    T = lambda cl: [torch.from_numpy(c).to(dev) for c in cl]
    out = model({'src_xyz': T(src[b0:b1]), 'tgt_xyz': T(tgt[b0:b1])})
    poses = fdist.gather_pair_results(out['pose'], counts, pair_dim=1)
    # the bench's other collective: max-over-ranks of the elapsed time (device tensor on RCCL)
    el = torch.tensor([float(rank)], dtype=torch.float64, device=dev if backend == 'nccl' else 'cpu')
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    assert float(el.item()) == world - 1
    ok = torch.ones(1, device=dev if backend == 'nccl' else 'cpu')
    if rank == 0:
        full = model({'src_xyz': T(src), 'tgt_xyz': T(tgt)})['pose']
        err = float((poses.cpu() - full.cpu()).abs().max())
        print(f'world {world} backend {dist.get_backend()}: {B} pairs, shards {counts}, '
              f'gathered on {poses.device}, max |pose diff| {err:.3e}', flush=True)
        ok[0] = 1.0 if err < 1e-5 and poses.shape == full.shape else 0.0
    dist.broadcast(ok, 0)
    dist.destroy_process_group()
    sys.exit(0 if ok.item() == 1.0 else 1)


if __name__ == '__main__':
    main()
