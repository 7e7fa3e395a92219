"""Cross-process determinism (development tool, GPU): the bf16 3DLoMatch test batch through
the GPU forward and the CPU oracle, outputs saved per process for a bitwise comparison.
usage: python tools/det_cross.py OUT.pt"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, ROOT)


def main():
    import fgreg
    import fgreg.config as fc
    from fgreg.synthetic import make_batch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import model_oracle as mo
    from test_gpu_bf16 import _random_model
    fgreg.set_precision('bf16')
    dev = torch.device('cuda:0')
    cfg = fc.get('3dlomatch')
    model = _random_model(cfg, 13)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    src, tgt, _ = make_batch('3dlomatch', 1, n_points=6000)
    model = model.to(dev)
    with torch.no_grad():
        out = model({'src_xyz': [torch.from_numpy(s).to(dev) for s in src],
                     'tgt_xyz': [torch.from_numpy(t).to(dev) for t in tgt]})
        ref = mo.forward(cfg, sd, src, tgt, mode=mo.geom.INDEX)
    keep = {}
    for k in ('src_feat_un', 'tgt_feat_un', 'src_kp_warped', 'tgt_kp_warped', 'pose'):
        keep['gpu_' + k] = out[k][0].cpu() if k != 'pose' else out[k].cpu()
        keep['ref_' + k] = ref[k][0] if k != 'pose' else ref[k]
    torch.save(keep, sys.argv[1])
    print('saved', sys.argv[1], flush=True)


if __name__ == '__main__':
    main()
