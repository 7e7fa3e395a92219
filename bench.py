#!/usr/bin/env python3
"""Benchmark: point-cloud pairs/s of the registration forward on MI355X.

Workloads (``--workload``; BASELINE.json configs):
  modelnet  (default, configs[1] at N=1 / configs[3] at N=8) ModelNet40-shaped 2048-pt pairs
            through the reference's exact crop test transforms (717 + 717 points per pair,
            fgreg.synthetic.modelnet_reference_pair -> fgreg.transforms), 8 pairs per GPU;
  3dmatch   (configs[2]) 20k + 20k-pt indoor fragment pairs, 1 pair per GPU;
  raw2048   (SURVEY §8(d) D2 stress) the 2048-pt raw clouds fed directly, 8 pairs per GPU;
  3dlomatch (configs[4]) 20k + 20k-pt low-overlap (10-30%) fragment pairs, 1 pair per GPU, in
            the bf16 compute mode (fgreg.set_precision('bf16'): bf16 MFMA GEMMs + attention).
``--precision fp32|bf16`` overrides the workload's default compute mode (bf16 for 3dlomatch,
fp32-accurate f16x3 otherwise).
Full RegTR forward (preprocessing, KPConv/Res2Net encoder, 6-layer cross encoder,
correspondence head, pose) with random-init weights of the reference architecture. One step =
one forward over one batch already resident in HBM. N GPUs = N processes (torchrun), pairs
sharded per rank with no data-path collective (weak scaling); each step ends with an RCCL
all-gather of the per-pair poses.

Prints ONE JSON line on rank 0 (contract in the task statement), with
  roofline:            the KPConv gather kernel (the north star's HBM target): algorithmic
                       bytes per launch / average launch time from HIP events recorded by
                       libfgreg itself around its kernels inside the timed region;
  roofline_attention,
  roofline_gemm,
  rooflines_other:     every other kernel family (radius search, grid subsampling,
                       InstanceNorm, LayerNorm, pose) from a separate instrumented replay of
                       the same steps AFTER the timed region (so `value` carries no
                       instrumentation but the gather's); MFMA fractions are against the
                       matrix pipe the kernels actually run on (fp16 MFMA, 3 products per
                       fp32-equivalent product for f16x3), the fp32-MFMA figure as a note;
  cpu_baseline:        the CPU restatement (oracle/model_oracle.py, kind "port") timed on the
                       host cores on a bounded sample of the same workload (rank 0, N = 1).
``--profile``: warmup + timed steps only (no counting, instrumented, tail or CPU legs), for
``rocprofv3 --kernel-trace --stats`` runs whose per-step kernel sums must stay within
ms_per_step (tools/kernel_stats.py).
"""
import argparse
import json
import os
import platform
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
PIPE = {'f16x3': 3, 'bf16': 1}
PRECISION = {'f16x3': 'fp32-accurate scaled split fp16 (3 fp16 MFMA products per fp32 '
                      'product, <= ~3 * 2^-22 relative each)',
             'bf16': 'bf16 (one bf16 MFMA product per product, fp32 accumulation, ~2^-9 '
                     'relative per product)'}
DTYPE = {'f16x3': 'f32 (emulated on the fp16 MFMA pipe: f16x3 split products)',
         'bf16': 'bf16 (bf16 MFMA GEMMs + attention; fp32 accumulation, storage, norms, '
                 'geometry and pose)'}

DATA = {
    'modelnet': 'synthetic ModelNet40-shaped pairs: 2048-pt box-surface raw clouds through the '
                'reference crop test transforms (crop 0.7, euler SE3 45deg/0.5, resample '
                '717+717, jitter, shuffle; fgreg/transforms.py), random-init weights of the '
                'reference ModelNet architecture',
    'raw2048': 'synthetic ModelNet40-shaped raw clouds: 2048+2048-pt box-surface clouds fed '
               'directly (no crop / resample; SURVEY D2 stress), random-init weights of the '
               'reference ModelNet architecture',
    '3dmatch': 'synthetic 3DMatch-like fragment pairs: 20k pts on the floor and walls of a room, '
               '5 mm noise, second fragment rotated <= 15 deg / moved <= 0.3 m '
               '(fgreg/synthetic.py), random-init weights of the reference 3DMatch architecture',
    '3dlomatch': 'synthetic 3DLoMatch-like fragment pairs: 20k + 20k pts cut from opposite ends '
                 'of a 6 x 3 x 2.5 m room with 10-30% shared extent, 5 mm noise, rotated <= 15 '
                 'deg / moved <= 0.3 m (fgreg/synthetic.py lowoverlap_pair), random-init '
                 'weights of the reference 3DMatch architecture',
}
METRIC = {
    'modelnet': 'point-cloud pairs/sec (forward) on ModelNet 2048-pt pairs',
    'raw2048': 'point-cloud pairs/sec (forward) on raw 2048+2048-pt pairs',
    '3dmatch': 'point-cloud pairs/sec (forward) on 3DMatch ~20k-pt fragment pairs',
    '3dlomatch': 'point-cloud pairs/sec (forward) on 3DLoMatch low-overlap ~20k-pt fragment pairs',
}
WORKLOAD = {
    'modelnet': 'ModelNet40 2048-pt pairs, {P} pairs per GPU (BASELINE configs[1] at N=1, '
                'configs[3] at N=8)',
    'raw2048': 'raw 2048+2048-pt pairs, {P} pairs per GPU (SURVEY D2 stress input)',
    '3dmatch': '3DMatch ~20k-pt fragment pairs, {P} pair(s) per GPU (BASELINE configs[2])',
    '3dlomatch': '3DLoMatch low-overlap ~20k-pt fragment pairs, bf16 features/attention, {P} '
                 'pair(s) per GPU (BASELINE configs[4])',
}
CFG_NAME = {'modelnet': 'modelnet', 'raw2048': 'modelnet', '3dmatch': '3dmatch',
            '3dlomatch': '3dlomatch'}
PAIRS = {'modelnet': 8, 'raw2048': 8, '3dmatch': 1, '3dlomatch': 1}
PRECISION_DEFAULT = {'3dlomatch': 'bf16'}
# D4 byte / flop definitions per timed family
OTHER = {
    'radius_search': ('hbm', '12 (Nq + Ns) + 8 Nq K bytes (int64 table)'),
    'grid_subsample': ('hbm', '12 (N_in + N_out) bytes (count + fill calls)'),
    'instnorm': ('hbm', '8 N C bytes (+ 4 N C residual, + 4 N row divisor)'),
    'layernorm': ('hbm', '8 N d bytes (+ 4 N d per add / pre-bias)'),
    'pose': ('hbm', '28 B per (layer, point) + 48 B per pose'),
    'max_pool': ('hbm', '8 H + 4 C bytes per query + 4 C per distinct support row'),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=50)
    p.add_argument('--warmup', type=int, default=10)
    p.add_argument('--pairs-per-gpu', type=int, default=None,
                   help='default 8 (modelnet, raw2048) / 1 (3dmatch)')
    p.add_argument('--workload', choices=tuple(METRIC), default='modelnet',
                   help='modelnet: BASELINE configs[1]/[3] (the headline line); 3dmatch: '
                        'configs[2]; 3dlomatch: configs[4] (bf16); raw2048: the uncropped '
                        'stress input')
    p.add_argument('--precision', choices=('fp32', 'bf16'), default=None,
                   help='compute mode (default: bf16 for 3dlomatch, fp32-accurate otherwise)')
    p.add_argument('--cpu-seconds', type=float, default=10.0,
                   help='budget of the CPU baseline B=1 sample (0 disables it)')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--lead-cycles', type=int, default=0,
                   help='spin kernel ahead of every per-launch timed call of the rooflines\' '
                        'eager replay (ops.KernelTimer.lead_cycles; 0 = off)')
    p.add_argument('--no-pipeline', action='store_true',
                   help='time back-to-back model(batch) calls instead of fgreg.pipeline (which '
                        'preprocesses step i + 1 on a side stream while step i\'s core runs)')
    p.add_argument('--profile', action='store_true',
                   help='warmup + timed steps only (for rocprofv3 kernel-trace runs)')
    p.add_argument('--train', action='store_true',
                   help='time training steps instead (SURVEY §8(f) row 4): train() forward + '
                        'backward + clip_grad_norm_ + AdamW step; a side line, not the headline')
    p.add_argument('--gather-table', default=None,
                   help='write the per-launch KPConv gather table (JSON) here')
    p.add_argument('--gemm-table', default=None,
                   help='write the per-shape GEMM table (M, N, K, launches, us, TFLOP/s, '
                        'bytes, fractions) of the instrumented replay to this JSON file')
    return p.parse_args()


def _pmc_traffic(kernel, workload):
    """Per-launch HBM bytes of `kernel` on `workload` from this round's committed PMC summary
    (tools/pmc_traffic.py output, tools/gpu_round.sh), or None when there is none."""
    path = os.path.join(REPO, 'profiles', f'pmc_kpconv_{workload}.json')
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    if d.get('op') != kernel:
        return None, None
    return d.get('hbm_bytes_per_launch'), os.path.relpath(path, REPO)


def _cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or 'unknown'


_TRAIN_STEP_HOOK = None


def train_main(args):
    """ms per training step of the workload's batch on one GPU (trainer.py:110-125: forward,
    compute_loss, loss.backward(), clip_grad_norm_, optimizer.step()). The loss is the
    reference's compute_loss (finegrained_regtr.py:252-309) as a differentiable graph
    (fgreg.loss.compute_loss_train: overlap BCE, InfoNCE on the match logits, correspondence
    MAE, the reference's weights) against the synthetic pairs' ground-truth poses and
    per-point overlap flags."""
    import fgreg
    from fgreg import linear as lin
    from fgreg.loss import compute_loss_train
    from fgreg.synthetic import make_batch
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    wl = args.workload
    fgreg.set_precision(args.precision or PRECISION_DEFAULT.get(wl, 'fp32'))
    cfg = fgreg.config.get(CFG_NAME[wl])
    torch.manual_seed(0)
    np.random.seed(0)
    model = fgreg.RegTR(cfg).to(dev).train()
    P = args.pairs_per_gpu or PAIRS[wl]
    kind = {'raw2048': 'modelnet_raw'}.get(wl, wl)
    src, tgt, pose_gt = make_batch(kind, P)
    flags = [_overlap_flags(a, b, p) for a, b, p in zip(src, tgt, pose_gt)]
    batch = {'src_xyz': [torch.from_numpy(a).to(dev) for a in src],
             'tgt_xyz': [torch.from_numpy(b).to(dev) for b in tgt],
             'pose': torch.from_numpy(np.asarray(pose_gt, np.float32)).to(dev),
             'src_overlap': [torch.from_numpy(f[0]).to(dev) for f in flags],
             'tgt_overlap': [torch.from_numpy(f[1]).to(dev) for f in flags]}
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=1e-4, weight_decay=1e-4, foreach=True)

    def step(split=None):
        opt.zero_grad(set_to_none=True)
        out = model(batch)
        loss = compute_loss_train(model, out, batch)['total']
        if split is not None:
            split[0].record()
        loss.backward()
        if split is not None:
            split[1].record()
        torch.nn.utils.clip_grad_norm_(params, 0.1)
        opt.step()

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize()
    if _TRAIN_STEP_HOOK is not None:          # tools/train_torch_prof.py: the step closure
        _TRAIN_STEP_HOOK(step)
    if args.gemm_table:
        # per-shape device time of the dense products (forward + dX GEMMs) and of the weight
        # gradients (fgr_gemm_f16x3_wgrad), events around each launch, 3 extra steps
        from fgreg import ops
        ops.TIMER = ops.KernelTimer(['gemm', 'wgrad'])
        ops.TIMER.lead_cycles = args.lead_cycles
        t_steps = 3
        t0 = time.perf_counter()
        for _ in range(t_steps):
            step()
        torch.cuda.synchronize()
        step_ms = (time.perf_counter() - t0) / t_steps * 1e3
        write_gemm_table(args.gemm_table, ops.TIMER, t_steps, step_ms, lin.MODE)
        write_gemm_table(args.gemm_table.replace('.json', '') + '_wgrad.json', ops.TIMER, t_steps,
                         step_ms, lin.MODE, name='wgrad')
        ops.TIMER = None
    if args.profile:
        torch.cuda._sleep(1000)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if args.profile:
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    line = {'metric': f'training step ms ({METRIC[wl].split(" on ")[1]})',
            'value': elapsed / args.steps * 1e3, 'unit': 'ms/step', 'n_gpus': 1,
            'steps': args.steps, 'warmup': args.warmup, 'higher_is_better': False,
            'pairs_per_s': P * args.steps / elapsed, 'dtype': DTYPE[lin.MODE],
            'data': DATA[wl], 'config': {'workload': WORKLOAD[wl].format(P=P), 'pairs_per_gpu': P,
                                         'precision': fgreg.precision(), 'mode': 'train()'},
            'what': 'train() forward (Res2Net BatchNorm on batch statistics) + the reference\'s '
                    'compute_loss (fgreg.loss.compute_loss_train) + backward + '
                    'clip_grad_norm_(0.1) + AdamW step (torch foreach); eager launches (no HIP '
                    'graph in training); gradients deterministic (no floating-point atomics)'}
    if not args.profile:
        # forward / backward split of extra steps (events around backward)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        fw, bw = [], []
        for _ in range(min(args.steps, 10)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            step(ev)
            torch.cuda.synchronize()
            tot = (time.perf_counter() - t0) * 1e3
            b = ev[0].elapsed_time(ev[1])
            bw.append(b)
            fw.append(tot - b)
        line['split_ms'] = {'forward_loss_optimizer': float(np.median(fw)),
                            'backward': float(np.median(bw))}
    print(json.dumps(line), flush=True)


def main():
    args = parse()
    if args.train:
        if args.gpus != 1:
            raise SystemExit('--train runs on one GPU')
        return train_main(args)
    import fgreg
    from fgreg import linear as lin
    from fgreg import ops
    from fgreg.synthetic import make_batch

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit(f'--gpus {args.gpus} but WORLD_SIZE={world}')
    # one rank per GPU; FGREG_DIST_BACKEND=gloo runs the multi-rank path on fewer GPUs than
    # ranks (ranks share devices round-robin) for a hardware rehearsal of the N > 1 code
    backend = os.environ.get('FGREG_DIST_BACKEND', 'nccl')
    local_dev = local_rank % max(torch.cuda.device_count(), 1) if backend == 'gloo' else local_rank
    torch.cuda.set_device(local_dev)
    dev = torch.device('cuda', local_dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)      # RCCL over xGMI
        else:
            dist.init_process_group(backend)

    wl = args.workload
    fgreg.set_precision(args.precision or PRECISION_DEFAULT.get(wl, 'fp32'))
    cfg = fgreg.config.get(CFG_NAME[wl])
    torch.manual_seed(0)
    np.random.seed(0)
    model = fgreg.RegTR(cfg).to(dev).eval()
    P = args.pairs_per_gpu or PAIRS[wl]
    kind = {'raw2048': 'modelnet_raw'}.get(wl, wl)
    from fgreg import dist as fdist
    if wl in ('3dmatch', '3dlomatch') and world > 1:
        # variable-size fragments: the global batch of P * world pairs is assigned to ranks by
        # point count (fgreg.dist.balanced_shards); every rank draws the same
        # global batch (seeded per pair index) and keeps its shard
        g_src, g_tgt, g_pose = make_batch(kind, P * world)
        shards = fdist.balanced_shards([len(a) + len(b) for a, b in zip(g_src, g_tgt)], world)
        mine = shards[rank]
        src, tgt, pose_gt = [g_src[i] for i in mine], [g_tgt[i] for i in mine], g_pose[mine]
        counts = [len(sh) for sh in shards]
        sharding = 'balanced_shards (greedy by points per pair)'
    else:
        src, tgt, pose_gt = make_batch(kind, P, start=rank * P)   # this rank's block of pairs
        counts = [P] * world
        sharding = 'contiguous blocks (shard_range)'
    P = len(src)
    batch_src = [torch.from_numpy(s).to(dev) for s in src]
    batch_tgt = [torch.from_numpy(t).to(dev) for t in tgt]

    def finish(out):
        if dist is not None:   # the one exchange: per-pair poses of every rank (RCCL)
            out['pose_all'] = fdist.gather_pair_results(out['pose'], counts, pair_dim=1)
        return out

    def step():
        return finish(model({'src_xyz': batch_src, 'tgt_xyz': batch_tgt}))

    def run(n):
        """n full forwards of the batch: pipelined (fgreg.pipeline: step i + 1's
        preprocessing on a side stream during step i's core) unless --no-pipeline"""
        if args.no_pipeline:
            for _ in range(n):
                step()
            return
        batches = ({'src_xyz': batch_src, 'tgt_xyz': batch_tgt} for _ in range(n))
        for out in fgreg.pipeline(model, batches):
            finish(out)

    def timed(n):
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(n)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        return time.perf_counter() - t0

    from fgreg import regtr as fregtr
    fpipe = sys.modules['fgreg.pipeline']            # the module (fgreg.pipeline is the function)
    with torch.no_grad():
        # >= 2 warmup steps: the second sighting of the batch's shape signature captures the
        # HIP graph of the post-preprocessing forward (fgreg/regtr.py), replayed from then on
        run(max(args.warmup, 2))
        if args.profile:
            # marker kernels around the timed region: tools/kernel_stats.py sums only the
            # dispatches between them (torch's spin kernel, ~1 us)
            torch.cuda._sleep(1000)
            elapsed = timed(args.steps)
            torch.cuda._sleep(1000)
            torch.cuda.synchronize()
        else:
            # algorithmic work per launch (untimed pass with counting on)
            fams = ['kpconv_gather', 'attention', 'gemm', 'res2net'] + list(OTHER)
            timer = ops.KernelTimer(fams)
            timer.count = True
            ops.TIMER = timer
            step()
            torch.cuda.synchronize()
            work = {n: list(timer.work[n]) for n in fams}
            ops.TIMER = None
            # timed region: nothing instrumented (graph replay of the core forward)
            elapsed = timed(args.steps)
            # one forward at a time (back-to-back model(batch), graph replay): the latency of
            # a step, reported beside the pipelined throughput
            elapsed_seq = None
            if not args.no_pipeline:
                no_pipe, args.no_pipeline = args.no_pipeline, True
                try:
                    elapsed_seq = timed(args.steps)
                finally:
                    args.no_pipeline = no_pipe
            # the same steps with the HIP-graph cache off (every launch eager): what inputs
            # whose shape signature never repeats get, reported beside `value`
            fregtr.GRAPHS = False
            try:
                run(2)
                elapsed_eager = timed(args.steps)
            finally:
                fregtr.GRAPHS = True
            # per-launch HIP events for every kernel family: an eager replay of the same
            # steps right after the timed region (a graph replay has no per-launch hook); the
            # rocprofv3 trace of the timed region (profiles/) cross-checks the durations
            rtimer = ops.KernelTimer(fams)
            rtimer.prealloc(args.steps * sum(len(work[n]) + 2 for n in rtimer.names))
            rtimer.lead_cycles = args.lead_cycles
            ops.TIMER = rtimer
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            ops.TIMER = None
            timer = rtimer
            # test-step tail: compute_loss + _compute_metrics on the
            # outputs of one step, outside the timed region
            tail_ms, tail_inputs = test_tail(model, batch_src, batch_tgt, src, tgt, pose_gt, dev,
                                              args.steps)

    el = torch.tensor([elapsed, elapsed_eager if not args.profile else 0.0], dtype=torch.float64,
                      device=dev if backend == 'nccl' else 'cpu')
    if dist is not None:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed, elapsed_eager = float(el[0].item()), float(el[1].item())
    step_ms = elapsed / args.steps * 1e3
    n_total = sum(counts)

    line = {
        'metric': METRIC[wl], 'value': n_total * args.steps / elapsed, 'unit': 'pairs/s',
        'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': step_ms,
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': DTYPE[lin.MODE], 'data': DATA[wl],
        'config': {'workload': WORKLOAD[wl].format(P=P), 'pairs_per_gpu': P,
                   'global_batch': n_total,
                   'points_per_cloud': int(np.mean([len(c) for c in src])),
                   'parallelism': f'pair-sharded dp{world}',
                   'sharding': sharding, 'pairs_per_rank': counts,
                   'precision': fgreg.precision(),
                   'hip_graph': ('post-preprocessing forward replayed from the shape-keyed graph '
                                 'cache; preprocessing eager' if fregtr.GRAPHS else 'off'),
                   'pipeline': ('off: back-to-back model(batch) calls' if args.no_pipeline else
                                'fgreg.pipeline: every step is a full forward; step i + 1\'s '
                                'preprocessing runs on a side stream while step i\'s core runs; '
                                f'consecutive cores alternate over {fpipe.STREAMS} core streams '
                                '(one HIP-graph instance each), so their launches overlap')},
    }
    if not args.profile and elapsed_seq is not None:
        line['sequential'] = {
            'value': n_total * args.steps / elapsed_seq, 'unit': 'pairs/s',
            'ms_per_step': elapsed_seq / args.steps * 1e3,
            'what': 'the same steps one forward at a time (back-to-back model(batch), graph '
                    'replay, no overlap of consecutive forwards): the per-batch latency'}
    if not args.profile:
        line['eager'] = {
            'value': n_total * args.steps / elapsed_eager, 'unit': 'pairs/s',
            'ms_per_step': elapsed_eager / args.steps * 1e3,
            'what': 'the same timed steps with the HIP-graph cache off (FGREG_GRAPHS=0: every '
                    'launch eager), i.e. inputs whose shape signature never repeats'}
    if args.profile:
        line['profile'] = 'warmup + timed steps only (rocprofv3 companion run)'
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    # ---- rooflines ---------------------------------------------------------------------
    def kpconv_roofline(name, kernel):
        b_launch = float(np.mean(work[name])) if work[name] else 0.0
        ms = timer.total_ms(name)
        avg_s = ms / 1e3 / max(len(timer.events[name]), 1)
        ach = b_launch / avg_s / 1e9 if avg_s > 0 else 0.0
        traffic, traffic_src = _pmc_traffic(kernel, wl)
        return {
            'kernel': kernel, 'bound': 'hbm', 'achieved': ach,
            'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': ach / HBM_PEAK_GBS,
            'traffic': traffic, 'traffic_source': traffic_src,
            'algorithmic_bytes_per_launch': b_launch, 'avg_launch_us': avg_s * 1e6,
            'launches_per_step': len(work[name]),
            'share_of_step': ms / args.steps / step_ms,
            'timing': 'HIP events recorded by libfgreg around each launch (fgr_time_next_call), '
                      'eager replay of the timed steps, a spin kernel queued ahead of each timed '
                      f'call (--lead-cycles {args.lead_cycles})'}

    # the KPConv stage's gather-weight kernel (the dominant HBM-bound kernel)
    line['roofline'] = kpconv_roofline('kpconv_gather', 'fgr_kpconv_gather')

    def mfma_family(name, mode, kernel):
        ms = rtimer.total_ms(name)
        flops = float(sum(work[name]))
        ach = flops * args.steps / (ms / 1e3) / 1e12 if ms > 0 else 0.0
        pipe = PIPE[mode]
        peak = F16_MFMA_PEAK_TFLOPS / pipe
        return {'kernel': kernel, 'bound': 'mfma', 'achieved': ach, 'peak': peak,
                'unit': 'TFLOP/s (fp32-equivalent)', 'frac': ach / peak,
                'peak_note': (f'fp16 dense MFMA {F16_MFMA_PEAK_TFLOPS:.0f} TF / {pipe} products '
                              f'per fp32-equivalent product; vs the {FP32_MFMA_PEAK_TFLOPS} TF '
                              f'fp32-MFMA peak this would read {ach / FP32_MFMA_PEAK_TFLOPS:.2f}'),
                'flops_per_step': flops, 'launches_per_step': len(work[name]),
                'avg_launch_us': ms * 1e3 / max(len(rtimer.events[name]), 1),
                'share_of_step': ms / args.steps / step_ms,
                'precision': PRECISION.get(mode, mode)}

    if args.gemm_table and rank == 0:
        write_gemm_table(args.gemm_table, rtimer, args.steps, step_ms, lin.MODE)
    if args.gather_table and rank == 0:
        write_gather_table(args.gather_table, rtimer, work['kpconv_gather'], args.steps, step_ms)
    line['roofline_attention'] = mfma_family('attention', ops.ATTN_MODE,
                                             f'fgr_attention_{ops.ATTN_MODE}')
    line['roofline_gemm'] = mfma_family('gemm', lin.MODE, f'fgr_gemm_{lin.MODE} (all dense layers)')
    if work['res2net']:
        # the Res2Net hierarchy (fgr_res2net_chain_h3: 3 fp16 products per product;
        # fgr_res2net_chain6: 6 bf16 products): work counted in matrix-core products
        ms = rtimer.total_ms('res2net')
        prod = float(sum(work['res2net']))
        ach = prod * args.steps / (ms / 1e3) / 1e12 if ms > 0 else 0.0
        kinds = sorted(set(rtimer.labels['res2net']))
        line['roofline_res2net'] = {
            'kernel': 'fgr_res2net_chain_' + '+'.join('h3' if k == 'h3' else '6' for k in kinds),
            'bound': 'mfma', 'achieved': ach, 'peak': F16_MFMA_PEAK_TFLOPS,
            'unit': 'TFLOP/s (fp16 / bf16 matrix-core products)', 'frac': ach / F16_MFMA_PEAK_TFLOPS,
            'work': '2 N w^2 (scale - 1) per chain x 3 (h3) / 6 (bf16x6) products',
            'products_per_step': prod, 'launches_per_step': len(work['res2net']),
            'avg_launch_us': ms * 1e3 / max(len(rtimer.events['res2net']), 1),
            'us_per_step': ms * 1e3 / args.steps, 'share_of_step': ms / args.steps / step_ms}
    other = {}
    for name, (bound, what) in OTHER.items():
        ms = rtimer.total_ms(name)
        b = float(sum(work[name]))
        if ms <= 0 or b <= 0:
            continue
        ach = b * args.steps / (ms / 1e3) / 1e9
        other[name] = {'bound': bound, 'achieved': ach, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                       'frac': ach / HBM_PEAK_GBS, 'bytes_per_step': b, 'algorithmic': what,
                       'calls_per_step': len(work[name]),
                       'us_per_step': ms * 1e3 / args.steps,
                       'share_of_step': ms / args.steps / step_ms}
    line['rooflines_other'] = other
    line['test_tail'] = {'what': f'compute_loss + _compute_metrics of one step ({P} pair(s): '
                                 'overlap pyramid, BCE, 2x InfoNCE, CorrCriterion, se3_compare)',
                         'ms_per_step': tail_ms}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_seconds > 0:
        cpu = cpu_baseline(cfg, model, src, tgt, args.cpu_seconds, tail_inputs, wl)
    line['cpu_baseline'] = cpu
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def write_gather_table(path, rtimer, work, steps, step_ms):
    """Per-launch table of the KPConv gather: per call of a step (nq
    queries, H table width, Cin, K kernel points), the valid neighbours per query (recovered
    from the algorithmic bytes), the event-timed us averaged over the
    replayed steps, the algorithmic bytes and their fraction of the HBM peak."""
    per = len(work)
    ev, lab = rtimer.events['kpconv_gather'], rtimer.labels['kpconv_gather']
    rows = []
    for i in range(per):
        ts = [ev[j][0].elapsed_time(ev[j][1]) for j in range(i, len(ev), per)]
        us = float(np.mean(ts)) * 1e3
        nq, H, cin, K = lab[i]
        byt = float(work[i])
        valid = (byt - nq * (8 * H + 12 + 4 * K * cin + 4)) / (12 + 4 * cin) / max(nq, 1)
        rows.append({'call': i, 'nq': nq, 'H': H, 'cin': cin, 'K': K,
                     'valid_per_query': valid, 'us': us, 'mbytes': byt / 1e6,
                     'wf_write_mbytes': nq * K * cin * 4 / 1e6,
                     'gbs': byt / (us * 1e-6) / 1e9, 'frac': byt / (us * 1e-6) / 1e9 / HBM_PEAK_GBS})
    tot_b = sum(r['mbytes'] for r in rows) * 1e6
    tot_us = sum(r['us'] for r in rows)
    with open(path, 'w') as f:
        json.dump({'hbm_peak_gbs': HBM_PEAK_GBS, 'ms_per_step': step_ms,
                   'gather_us_per_step': tot_us,
                   'frac_all': tot_b / (tot_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 'calls': rows},
                  f, indent=1)


def write_gemm_table(path, rtimer, steps, step_ms, mode, name='gemm'):
    """Per-shape table of the dense layers (bytes, flops, time and the binding
    roof per shape). bytes = the minimum operand traffic 4 M K (A) + 4 N K (f16x3 image:
    2 terms x 2 B; 2 N K for the single-term bf16 image) + 4 M N (C), assuming every operand
    is read once."""
    pipe = PIPE[mode]
    wb = 2.0 if mode == 'bf16' else 4.0
    mfma_peak = F16_MFMA_PEAK_TFLOPS / pipe
    rows = []
    for lab, (ms, cnt) in sorted(rtimer.per_label(name).items(), key=lambda kv: -kv[1][0]):
        us = ms * 1e3 / cnt
        if lab[0] == 'ffn':
            # the fused feed-forward sub-layer (ops.ffn): M x d in, hidden F, two products;
            # bytes = x read once, both weight images, the output
            _, m, n, k = lab
            flops = 4.0 * m * n * k
            byt = 4.0 * m * n + 2 * wb * n * k + 4.0 * m * n
        else:
            m, n, k = lab
            flops = 2.0 * m * n * k
            byt = 4.0 * m * k + wb * n * k + 4.0 * m * n
        tf = flops / (us * 1e-6) / 1e12
        gbs = byt / (us * 1e-6) / 1e9
        t_mfma = flops / (mfma_peak * 1e12) * 1e6
        t_hbm = byt / (HBM_PEAK_GBS * 1e9) * 1e6
        rows.append({'M': m, 'N': n, 'K': k, 'launches_per_step': cnt / steps, 'us': us,
                     'kind': 'ffn (d = N, hidden = K)' if lab[0] == 'ffn' else 'gemm',
                     'us_per_step': ms * 1e3 / steps, 'gflop': flops / 1e9, 'mbytes': byt / 1e6,
                     'tflops_fp32_equiv': tf, 'gbs': gbs, 'mfma_frac': tf / mfma_peak,
                     'hbm_frac': gbs / HBM_PEAK_GBS,
                     'binding_roof': 'mfma' if t_mfma >= t_hbm else 'hbm',
                     'roof_frac': max(t_mfma, t_hbm) / us})
    tot = sum(r['us_per_step'] for r in rows)
    with open(path, 'w') as f:
        json.dump({'mode': mode, 'mfma_peak_tflops_fp32_equiv': mfma_peak,
                   'hbm_peak_gbs': HBM_PEAK_GBS, 'ms_per_step': step_ms,
                   'gemm_us_per_step': tot, 'shapes': rows}, f, indent=1)


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


def _calibration():
    path = os.path.join(REPO, 'profiles', 'cpu_calibration.json')
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def _physical_cores():
    """Physical cores in this process's affinity mask (SMT siblings counted once), from
    /proc/cpuinfo's (physical id, core id) pairs; the affinity count if that is unreadable."""
    cpus = os.sched_getaffinity(0)
    try:
        cores, cur, phys = set(), None, 0
        with open('/proc/cpuinfo') as f:
            for line in f:
                k, _, v = line.partition(':')
                k = k.strip()
                if k == 'processor':
                    cur = int(v)
                elif k == 'physical id':
                    phys = int(v)
                elif k == 'core id' and cur in cpus:
                    cores.add((phys, int(v)))
        return len(cores) or len(cpus)
    except (OSError, ValueError):
        return len(cpus)


def _cgroup_cpus():
    """The CPU quota of this process's cgroup in CPUs (cgroup v2 cpu.max, else v1
    cfs_quota / cfs_period), or None when unlimited / unreadable: a lease can hand out a
    256-CPU affinity mask with a quota of a few dozen CPUs, and more torch threads than the
    quota only oversubscribe it (128 threads ran 8x slower than 16)."""
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, per = f.read().split()[:2]
        return None if q == 'max' else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as f:
            q = int(f.read())
        with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as f:
            per = int(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def _cpu_leg(mo, cfg, sd, src, tgt, budget_s, threads, max_iter=64):
    """B=1 forwards of the port with `threads` torch threads for ~budget_s -> (pairs, s)."""
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        n_pairs, t_tot, it = 0, 0.0, 0
        while (t_tot < budget_s or it < 1) and it < max_iter:
            b = it % len(src)
            t0 = time.perf_counter()
            mo.forward(cfg, sd, [src[b]], [tgt[b]], mode=mo.geom.INDEX)
            t_tot += time.perf_counter() - t0
            n_pairs += 1
            it += 1
    finally:
        torch.set_num_threads(prev)
    return n_pairs, t_tot


def cpu_baseline(cfg, model, src, tgt, budget_s, tail_inputs=None, workload='modelnet'):
    """CPU restatement (oracle/model_oracle.py, "port") on the same pairs, B=1 forwards (SURVEY
    §8(d) D5). The usable cores are the physical cores of the affinity mask capped by the
    cgroup CPU quota; torch thread counts 8, 16, 32, 64, 128 (and the per-GPU share and the
    usable count) up to the physical cores are swept for ~budget_s / 8 each, the fastest is
    timed for ~budget_s and is `value` (its thread count is `cores`); the all-physical-cores
    and per-GPU-share legs of the sweep are reported beside it. Then one B=len(batch) leg at
    the best count."""
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    import model_oracle as mo
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    share = torch.get_num_threads()
    phys = _physical_cores()
    quota = _cgroup_cpus()
    usable = max(1, min(phys, int(quota))) if quota else phys
    cands = sorted({t for t in (8, 16, 32, 64, 128, share, usable, phys) if 1 <= t <= phys})
    mo.forward(cfg, sd, [src[0]], [tgt[0]], mode=mo.geom.INDEX)       # warm (allocator, pools)
    sweep = {}
    for t in cands:
        n, tt = _cpu_leg(mo, cfg, sd, src, tgt, budget_s / 8, t, max_iter=16)
        sweep[t] = n / tt
    best = max(sweep, key=sweep.get)
    n_pairs, t_tot = _cpu_leg(mo, cfg, sd, src, tgt, budget_s, best)
    res = {'value': n_pairs / t_tot, 'unit': 'pairs/s', 'cores': best, 'kind': 'port',
           'cpu_model': _cpu_model(),
           'cores_note': {'torch_threads': best,
                          'basis': 'the fastest torch thread count of the sweep (pairs/s by '
                                   'thread count in thread_sweep)',
                          'physical_cores': phys, 'cgroup_quota_cpus': quota,
                          'usable_cores': usable,
                          'omp_num_threads': os.environ.get('OMP_NUM_THREADS'),
                          'affinity_cpus': len(os.sched_getaffinity(0)),
                          'machine_cpus': os.cpu_count()},
           'thread_sweep': {str(t): v for t, v in sorted(sweep.items())},
           'all_physical_cores': {'value': sweep.get(phys), 'unit': 'pairs/s', 'cores': phys},
           'per_gpu_share': {'value': sweep.get(share), 'unit': 'pairs/s', 'cores': share,
                             'what': 'the B=1 leg on the per-GPU CPU share of the lease '
                                     '(torch threads = OMP_NUM_THREADS), from the sweep'},
           'sample': f'{n_pairs} pairs (B=1 forwards) of the same workload, '
                     f'{t_tot:.1f} s, torch CPU fp32 with {best} threads'}
    if len(src) > 1:
        prev = torch.get_num_threads()
        torch.set_num_threads(best)
        try:
            t0 = time.perf_counter()
            mo.forward(cfg, sd, list(src), list(tgt), mode=mo.geom.INDEX)
            tb = time.perf_counter() - t0
        finally:
            torch.set_num_threads(prev)
        res['batch_leg'] = {'pairs_per_batch': len(src), 'value': len(src) / tb,
                            'unit': 'pairs/s', 'seconds': tb}
    cal = _calibration()
    if cal is not None:
        # the ratio measured on this workload's architecture / cloud size (3DLoMatch: 3DMatch's)
        key = {'raw2048': 'modelnet', '3dlomatch': '3dmatch'}.get(workload, workload)
        per = cal.get('per_workload', {}).get(key)
        ratio = per['reference_over_port'] if per else cal.get('reference_over_port')
        res['calibration'] = {'reference_over_port': ratio, 'workload': key if per else 'modelnet',
                              'hardware': cal.get('hardware'), 'source': cal.get('source'),
                              'reference_estimate_pairs_per_s': res['value'] * ratio}
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
