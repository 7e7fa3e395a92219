"""Multi-rank forward check (run under torch.distributed.run; used by tests/test_gpu_dist.py):
every rank runs fgreg.RegTR.forward on its shard of a batch, the per-pair poses are
all-gathered (fgreg.dist.gather_pair_results, the bench's exchange), and rank 0 compares them
with a single forward over the whole batch on the same weights.

  default                 ModelNet, 2 * world + 1 pairs (ragged contiguous shards, shard_range)
  --pairs-per-rank P      ModelNet, P pairs per rank (BASELINE configs[3]: P = 8 at world 8 is
                          the global batch of 64 sharded 8 pairs per GPU)
  --workload 3dmatch      variable-size indoor fragment pairs (3DMatch model) sharded by
                          fgreg.dist.balanced_shards on the per-pair point counts, as bench.py
                          shards 3DMatch / 3DLoMatch at world > 1
FGREG_DIST_BACKEND=gloo lets the ranks share one GPU (the 1-GPU box); nccl (RCCL) needs one GPU
per rank (tests/test_gpu_dist.py runs it at world size 1 on the 1-GPU box). Exit status 0 = the
gathered (L, B, 3, 4) poses equal the full-batch forward's."""
import argparse
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))


def _indoor_batch(n_pairs, sizes):
    from fgreg.synthetic import indoor_like_pair
    src, tgt = [], []
    for i in range(n_pairs):
        s, t, _ = indoor_like_pair(i, n_points=sizes[i])
        src.append(s)
        tgt.append(t)
    return src, tgt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--pairs-per-rank', type=int, default=0)
    ap.add_argument('--workload', default='modelnet', choices=['modelnet', '3dmatch'])
    ap.add_argument('--pairs', type=int, default=0, help='3dmatch: total pairs')
    args = ap.parse_args()
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
    torch.manual_seed(0)
    if args.workload == 'modelnet':
        B = args.pairs_per_rank * world if args.pairs_per_rank else 2 * world + 1
        model = fgreg.RegTR(fgreg.config.get('modelnet')).to(dev).eval()
        src, tgt, _ = make_batch('modelnet', B)
        shards = [list(range(*fdist.shard_range(B, world, r))) for r in range(world)]
        how = 'shard_range'
    else:
        B = args.pairs or 2 * world + 1
        sizes = [3000 + (1777 * i) % 6000 for i in range(B)]          # ragged fragments
        model = fgreg.RegTR(fgreg.config.get('3dmatch')).to(dev).eval()
        src, tgt = _indoor_batch(B, sizes)
        shards = fdist.balanced_shards([len(s) + len(t) for s, t in zip(src, tgt)], world)
        how = 'balanced_shards'
    mine = shards[rank]
    counts = [len(s) for s in shards]
    T = lambda cl: [torch.from_numpy(np.ascontiguousarray(c)).to(dev) for c in cl]
    out = model({'src_xyz': T([src[i] for i in mine]), 'tgt_xyz': T([tgt[i] for i in mine])})
    poses = fdist.gather_pair_results(out['pose'], counts, pair_dim=1)
    # the bench's other collective: max-over-ranks of the elapsed time (device tensor on RCCL)
    el = torch.tensor([float(rank)], dtype=torch.float64, device=dev if backend == 'nccl' else 'cpu')
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    assert float(el.item()) == world - 1
    ok = torch.ones(1, device=dev if backend == 'nccl' else 'cpu')
    if rank == 0:
        order = [i for s in shards for i in s]                        # gathered pair order
        full = model({'src_xyz': T(src), 'tgt_xyz': T(tgt)})['pose'][:, order]
        err = float((poses.cpu() - full.cpu()).abs().max())
        print(f'world {world} backend {dist.get_backend()} workload {args.workload}: {B} pairs, '
              f'{how} {counts}, gathered {tuple(poses.shape)} on {poses.device}, '
              f'max |pose diff| {err:.3e}', flush=True)
        # ModelNet pairs are equal-sized: a shard's rows run the same GEMM dispatch as the full
        # batch's, 1e-5. Ragged 3DMatch shards change the row counts M of every GEMM, hence the
        # dispatched tile family and its summation order: rounding-level pose differences, 1e-4.
        tol = 1e-5 if args.workload == 'modelnet' else 1e-4
        ok[0] = 1.0 if err < tol and poses.shape == full.shape else 0.0
    dist.broadcast(ok, 0)
    dist.destroy_process_group()
    sys.exit(0 if ok.item() == 1.0 else 1)


if __name__ == '__main__':
    main()
