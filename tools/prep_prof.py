import cProfile, pstats, sys, os, time, torch, numpy as np
sys.path.insert(0, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd')
import fgreg
from fgreg.synthetic import make_batch
wl = sys.argv[1]
dev = torch.device('cuda:0'); torch.manual_seed(0); np.random.seed(0)
model = fgreg.RegTR(fgreg.config.get(wl)).to(dev).eval()
P = 8 if wl == 'modelnet' else 1
src, tgt, _ = make_batch(wl, P)
pts = [torch.from_numpy(a).to(dev) for a in src] + [torch.from_numpy(a).to(dev) for a in tgt]
with torch.no_grad():
    for _ in range(5): model.preprocessor(pts)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20): model.preprocessor(pts)
    torch.cuda.synchronize()
    print('prep alone ms', (time.perf_counter() - t0) / 20 * 1e3)
    pr = cProfile.Profile(); pr.enable()
    for _ in range(20): model.preprocessor(pts)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats('tottime').print_stats(18)
