import sys, time
sys.path.insert(0, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd')
import torch
from fgreg import ops
torch.zeros(1, device='cuda')
assert ops._stream() == torch.cuda.current_stream().cuda_stream
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    assert ops._stream() == s.cuda_stream == torch.cuda.current_stream().cuda_stream
    w = ops._workspace(torch.device('cuda:0'), 100)
    assert (torch.device('cuda:0'), s.cuda_stream) in ops._WS
for f, name in ((ops._stream, 'raw'), (lambda: torch.cuda.current_stream().cuda_stream, 'torch')):
    t = time.perf_counter()
    for _ in range(20000):
        f()
    print(name, round((time.perf_counter() - t) / 20000 * 1e6, 2), 'us per call')
print('stream check ok')
