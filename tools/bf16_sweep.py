"""bf16 forward (BASELINE configs[4]) against the fp32 CPU oracle over many random models
(VERDICT r2 item 1): for each seed, the 3DLoMatch-config model of tests/test_gpu_bf16.py is run
in bf16 with the correspondence head in bf16 and in f16x3 (fgreg.regtr.HEAD_MODE), and every
per-pair output's normwise error plus the last-layer pose error are printed as one JSON line.

  python tools/bf16_sweep.py --seeds 0-7 --points 6000 [--out gpurun_out/bf16_sweep.jsonl]
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
sys.path.insert(0, os.path.join(REPO, 'oracle'))
sys.path.insert(0, os.path.join(REPO, 'tests'))

KEYS = ['src_feat_un', 'tgt_feat_un', 'src_feat', 'tgt_feat', 'src_kp_warped', 'tgt_kp_warped',
        'src_overlap', 'tgt_overlap']


def _seeds(spec):
    out = []
    for part in spec.split(','):
        if '-' in part:
            a, b = part.split('-')
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--seeds', default='0-7')
    ap.add_argument('--points', type=int, default=6000)
    ap.add_argument('--heads', default='bf16,f16x3')
    ap.add_argument('--out', default=None)
    args = ap.parse_args()
    import fgreg
    import fgreg.config as fc
    from fgreg import regtr
    from fgreg.synthetic import make_batch
    import model_oracle as mo
    from conftest import rel_err
    from test_gpu_bf16 import _random_model, _rot_deg
    dev = torch.device('cuda:0')
    fgreg.set_precision('bf16')
    cfg = fc.get('3dlomatch')
    fout = open(args.out, 'a') if args.out else None
    for seed in _seeds(args.seeds):
        model = _random_model(cfg, seed)
        sd = {k: v.clone() for k, v in model.state_dict().items()}
        model = model.to(dev)
        src, tgt, _ = make_batch('3dlomatch', 1, start=seed, n_points=args.points)
        t0 = time.time()
        ref = mo.forward(cfg, sd, src, tgt, mode=mo.geom.INDEX)
        t_ref = time.time() - t0
        pr = ref['pose'].numpy()[-1, 0]
        for head in args.heads.split(','):
            regtr.HEAD_MODE = None if head == 'bf16' else head
            batch = {'src_xyz': [torch.from_numpy(s).to(dev) for s in src],
                     'tgt_xyz': [torch.from_numpy(t).to(dev) for t in tgt]}
            with torch.no_grad():
                out = model(batch)
            errs = {k: rel_err(out[k][0], ref[k][0]) for k in KEYS}
            p = out['pose'].cpu().numpy()[-1, 0]
            rec = {'seed': seed, 'points': args.points, 'head': head,
                   'max_feat_err': max(errs.values()), 'errs': errs,
                   'rot_deg': _rot_deg(p, pr), 'trans_m': float(np.linalg.norm(p[:, 3] - pr[:, 3])),
                   'oracle_s': t_ref}
            line = json.dumps(rec)
            print(line, flush=True)
            if fout:
                fout.write(line + '\n')
                fout.flush()
    regtr.HEAD_MODE = None


if __name__ == '__main__':
    main()
