#!/usr/bin/env python3
"""Benchmark: point-cloud pairs/s of the registration forward on MI355X.

Workload (BASELINE.json configs[1] / configs[3]): ModelNet40-shaped 2048-pt pairs through
the reference's exact crop test transforms (717 + 717 points per pair,
fgreg.synthetic.modelnet_reference_pair -> fgreg.transforms), 8 pairs
per GPU, full RegTR forward (preprocessing, KPConv/Res2Net encoder, 6-layer cross
encoder, correspondence head, pose) in fp32 with random-init weights of the reference
ModelNet architecture. One step = one forward over one batch already resident in HBM.
N GPUs = N processes (torchrun), pairs sharded 8 per rank with no data-path collective
(weak scaling); each step ends with an RCCL all-gather of the per-pair poses.

Prints ONE JSON line on rank 0 (contract in the task statement), with
  roofline:     the KPConv gather kernel (HBM-bound): algorithmic bytes per launch /
                average launch time from HIP events over the timed region (recorded by
                libfgreg itself around its kernels, fgr_time_next_call, event pairs created
                before the region);
  cpu_baseline: the CPU restatement (oracle/model_oracle.py, kind "port") timed on the
                host cores on a bounded sample of the same workload (rank 0, N = 1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
FP32_MFMA_PEAK_TFLOPS = 157.3
F16_MFMA_PEAK_TFLOPS = 2500.0    # fp16 / bf16 dense (MI355X_MICROARCH.md)
# matrix-core products issued per fp32-equivalent product, by precision mode
PIPE = {'f16x3': 3, 'bf16x6': 6, 'bf16x3': 3, 'fp32': 1}
PRECISION = {'f16x3': 'fp32-accurate scaled split fp16 (3 fp16 MFMA products per fp32 '
                      'product, <= ~3 * 2^-22 relative each)',
             'bf16x6': 'fp32-accurate split bf16 (6 bf16 MFMA products per fp32 product)',
             'bf16x3': 'split bf16, 3 products (~2^-17 relative)',
             'fp32': 'fp32 MFMA / hipBLASLt fp32'}


DATA = {
    'modelnet': 'synthetic ModelNet40-shaped pairs: 2048-pt box-surface raw clouds through the '
                'reference crop test transforms (crop 0.7, euler SE3 45deg/0.5, resample '
                '717+717, jitter, shuffle; fgreg/transforms.py), random-init weights of the '
                'reference ModelNet architecture',
    '3dmatch': 'synthetic 3DMatch-like fragment pairs: 20k pts on the floor and walls of a room, '
               '5 mm noise, second fragment rotated <= 15 deg / moved <= 0.3 m '
               '(fgreg/synthetic.py), random-init weights of the reference 3DMatch architecture',
}
METRIC = {
    'modelnet': 'point-cloud pairs/sec (forward) on ModelNet 2048-pt pairs',
    '3dmatch': 'point-cloud pairs/sec (forward) on 3DMatch ~20k-pt fragment pairs',
}
WORKLOAD = {
    'modelnet': 'ModelNet40 2048-pt pairs, {P} pairs per GPU (BASELINE configs[1] at N=1, '
                'configs[3] at N=8)',
    '3dmatch': '3DMatch ~20k-pt fragment pairs, {P} pair(s) per GPU (BASELINE configs[2])',
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=5)
    p.add_argument('--pairs-per-gpu', type=int, default=None,
                   help='default 8 (modelnet) / 1 (3dmatch)')
    p.add_argument('--workload', choices=('modelnet', '3dmatch'), default='modelnet',
                   help='modelnet: BASELINE configs[1]/[3] (the headline line); 3dmatch: '
                        'configs[2], 20k-pt fragment pairs, a parity / stress line')
    p.add_argument('--cpu-seconds', type=float, default=10.0,
                   help='budget of the CPU baseline sample (0 disables it)')
    p.add_argument('--no-cpu-baseline', action='store_true')
    return p.parse_args()


def _pmc_traffic():
    """Per-launch HBM bytes of the gather kernel from the committed PMC summary, if any."""
    path = os.path.join(REPO, 'profiles', 'pmc_kpconv_gather.json')
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get('hbm_bytes_per_launch')


def main():
    args = parse()
    import fgreg
    from fgreg import linear as lin
    from fgreg import ops
    from fgreg.synthetic import make_batch

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit(f'--gpus {args.gpus} but WORLD_SIZE={world}')
    torch.cuda.set_device(local_rank)
    dev = torch.device('cuda', local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('nccl', device_id=dev)

    cfg = fgreg.config.get(args.workload)
    torch.manual_seed(0)
    np.random.seed(0)
    model = fgreg.RegTR(cfg).to(dev).eval()
    P = args.pairs_per_gpu or (8 if args.workload == 'modelnet' else 1)
    src, tgt, pose_gt = make_batch(args.workload, P, start=rank * P)   # this rank's shard of pairs
    batch_src = [torch.from_numpy(s).to(dev) for s in src]
    batch_tgt = [torch.from_numpy(t).to(dev) for t in tgt]
    from fgreg import dist as fdist

    def step():
        out = model({'src_xyz': batch_src, 'tgt_xyz': batch_tgt})
        if dist is not None:   # the one exchange: per-pair poses of every rank (RCCL)
            out['pose_all'] = fdist.gather_pair_results(out['pose'], [P] * world, pair_dim=1)
        return out

    with torch.no_grad():
        for _ in range(max(args.warmup, 1)):
            step()
        # algorithmic work per launch (untimed pass with counting on)
        timer = ops.KernelTimer(['kpconv_gather', 'attention', 'gemm'])
        timer.count = True
        ops.TIMER = timer
        step()
        torch.cuda.synchronize()
        gather_bytes = list(timer.work['kpconv_gather'])
        attn_flops = list(timer.work['attention'])
        gemm_flops = list(timer.work['gemm'])
        timer.count = False
        timer.reset_events()
        timer.names.discard('gemm')       # GEMM events: separate pass below, not in `value`
        timer.prealloc(args.steps * (len(gather_bytes) + len(attn_flops)))

        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        # instrumented pass for the GEMM roofline (every dense layer), outside the timed region
        gtimer = ops.KernelTimer(['gemm'])
        gtimer.prealloc(args.steps * len(gemm_flops))
        ops.TIMER = gtimer
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        ops.TIMER = None
        # test-step tail: compute_loss + _compute_metrics on the
        # outputs of one step, outside the timed region
        tail_ms, tail_inputs = test_tail(model, batch_src, batch_tgt, src, tgt, pose_gt, dev,
                                          args.steps)

    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    g_ms = timer.total_ms('kpconv_gather')
    g_launches = len(timer.events['kpconv_gather'])
    a_ms = timer.total_ms('attention')
    a_launches = len(timer.events['attention'])
    g_bytes_step = float(sum(gather_bytes))
    a_flops_step = float(sum(attn_flops))
    g_avg_s = g_ms / 1e3 / max(g_launches, 1)
    g_bytes_launch = g_bytes_step / max(len(gather_bytes), 1)
    g_achieved = g_bytes_launch / g_avg_s / 1e9 if g_avg_s > 0 else 0.0
    a_achieved = a_flops_step * args.steps / (a_ms / 1e3) / 1e12 if a_ms > 0 else 0.0
    m_ms = gtimer.total_ms('gemm')
    m_flops_step = float(sum(gemm_flops))
    m_achieved = m_flops_step * args.steps / (m_ms / 1e3) / 1e12 if m_ms > 0 else 0.0
    traffic = _pmc_traffic() if args.workload == 'modelnet' else None   # PMC pass: modelnet

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_seconds > 0:
        cpu = cpu_baseline(cfg, model, src, tgt, args.cpu_seconds, tail_inputs)

    if rank == 0:
        pairs = world * P * args.steps
        line = {
            'metric': METRIC[args.workload],
            'value': pairs / elapsed,
            'unit': 'pairs/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': elapsed / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'f32',
            'data': DATA[args.workload],
            'config': {'workload': WORKLOAD[args.workload].format(P=P),
                       'pairs_per_gpu': P, 'global_batch': P * world,
                       'points_per_cloud': int(np.mean([len(c) for c in src])),
                       'parallelism': f'pair-sharded dp{world}'},
            'roofline': {'kernel': 'fgr_kpconv_gather', 'bound': 'hbm',
                         'achieved': g_achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': g_achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'algorithmic_bytes_per_launch': g_bytes_launch,
                         'avg_launch_us': g_avg_s * 1e6, 'launches_per_step': len(gather_bytes),
                         'share_of_step': g_ms / (elapsed * 1e3)},
            'roofline_attention': {'kernel': f'fgr_attention_{ops.ATTN_MODE}', 'bound': 'mfma',
                                   'achieved': a_achieved, 'peak': FP32_MFMA_PEAK_TFLOPS,
                                   'unit': 'TFLOP/s (fp32-equivalent)',
                                   'frac': a_achieved / FP32_MFMA_PEAK_TFLOPS,
                                   'flops_per_step': a_flops_step,
                                   'avg_launch_us': a_ms * 1e3 / max(a_launches, 1),
                                   'share_of_step': a_ms / (elapsed * 1e3),
                                   'precision': PRECISION.get(ops.ATTN_MODE, ops.ATTN_MODE),
                                   'matrix_pipe_tflops': PIPE.get(ops.ATTN_MODE, 1) * a_achieved,
                                   'matrix_pipe_frac': PIPE.get(ops.ATTN_MODE, 1) * a_achieved /
                                   (F16_MFMA_PEAK_TFLOPS if ops.ATTN_MODE != 'fp32'
                                    else FP32_MFMA_PEAK_TFLOPS)},
            'roofline_gemm': {'kernel': f'fgr_gemm_{lin.MODE} (all dense layers)', 'bound': 'mfma',
                              'achieved': m_achieved, 'peak': FP32_MFMA_PEAK_TFLOPS,
                              'unit': 'TFLOP/s (fp32-equivalent)',
                              'frac': m_achieved / FP32_MFMA_PEAK_TFLOPS,
                              'flops_per_step': m_flops_step,
                              'launches_per_step': len(gemm_flops),
                              'share_of_step': m_ms / (elapsed * 1e3),
                              'precision': PRECISION.get(lin.MODE, lin.MODE),
                              'matrix_pipe_frac': PIPE.get(lin.MODE, 1) * m_achieved /
                              (F16_MFMA_PEAK_TFLOPS if lin.MODE != 'fp32'
                               else FP32_MFMA_PEAK_TFLOPS)},
            'test_tail': {'what': f'compute_loss + _compute_metrics of one step ({P} pair(s): '
                                  'overlap pyramid, BCE, 2x InfoNCE, CorrCriterion, se3_compare)',
                          'ms_per_step': tail_ms},
            'cpu_baseline': cpu,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _overlap_flags(a, b, pose, radius=0.05):
    """Per-point ground-truth overlap flags of a pair (nearest point of the other cloud
    under the true pose within radius), the loss input the reference's dataset provides."""
    from scipy.spatial import cKDTree
    aw = a @ pose[:, :3].T + pose[:, 3]
    return ((cKDTree(b).query(aw)[0] < radius).astype(np.float32),
            (cKDTree(aw).query(b)[0] < radius).astype(np.float32))


def test_tail(model, batch_src, batch_tgt, src, tgt, pose_gt, dev, iters):
    """Times fgreg.loss.compute_loss + compute_metrics on the outputs of one forward."""
    from fgreg import loss as floss
    flags = [_overlap_flags(s, t, p) for s, t, p in zip(src, tgt, pose_gt)]
    with torch.no_grad():
        batch = {'src_xyz': batch_src, 'tgt_xyz': batch_tgt}
        out = model(batch)                                  # fills batch['kpconv_meta']
        batch['pose'] = torch.from_numpy(pose_gt).to(dev)
        batch['src_overlap'] = [torch.from_numpy(f[0]).to(dev) for f in flags]
        batch['tgt_overlap'] = [torch.from_numpy(f[1]).to(dev) for f in flags]
        floss.compute_loss(model, out, batch)               # warm (weight splits)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            floss.compute_loss(model, out, batch)
            floss.compute_metrics(out, batch)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / iters * 1e3
    return ms, (out, batch)


def cpu_baseline(cfg, model, src, tgt, budget_s, tail_inputs=None):
    """CPU restatement (oracle/model_oracle.py, "port") on the same pairs, for ~budget_s."""
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    import model_oracle as mo
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    threads = torch.get_num_threads()
    n_pairs, t_tot, it = 0, 0.0, 0
    while t_tot < budget_s and it < 64:
        b = it % len(src)
        t0 = time.perf_counter()
        mo.forward(cfg, sd, [src[b]], [tgt[b]], mode=mo.geom.INDEX)
        t_tot += time.perf_counter() - t0
        n_pairs += 1
        it += 1
    res = {'value': n_pairs / t_tot, 'unit': 'pairs/s', 'cores': threads, 'kind': 'port',
           'sample': f'{n_pairs} pairs (B=1 forwards) of the same workload, '
                     f'{t_tot:.1f} s, torch CPU fp32 with {threads} threads'}
    if tail_inputs is not None:       # the test-step tail on the same outputs (loss_oracle)
        import loss_oracle as lo
        out, batch = tail_inputs
        cpu = lambda v: [t.cpu() for t in v] if isinstance(v, list) else v.cpu()
        pred = {k: cpu(v) for k, v in out.items()}
        meta = {k: cpu(batch['kpconv_meta'][k]) for k in ('points', 'pools', 'stack_lengths')}
        b = {'pose': batch['pose'].cpu(), 'src_overlap': cpu(batch['src_overlap']),
             'tgt_overlap': cpu(batch['tgt_overlap']), 'kpconv_meta': meta}
        W = model.feature_criterion.W.detach().cpu()
        W_un = model.feature_criterion_un.W.detach().cpu()
        t0 = time.perf_counter()
        lo.compute_loss(cfg, W, W_un, pred, b)
        lo.pose_errors(pred['pose'], b['pose'])
        res['test_tail_ms'] = (time.perf_counter() - t0) * 1e3
    return res


if __name__ == '__main__':
    main()
