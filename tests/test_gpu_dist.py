"""The sharded multi-rank forward on the GPU (BASELINE configs[3]'s code path): two ranks run
fgreg.RegTR.forward on their shards and all-gather the poses; they must equal one forward
over the whole batch. On the 1-GPU box the ranks share the device over gloo (RCCL needs one
GPU per rank); the 8-GPU RCCL run is the driver's scaling bench. The RCCL branch itself
(device-tensor all_gather / all_reduce, fgreg/dist.py) runs at world size 1 on the box's GPU."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _run(nproc, *args, backend='gloo', timeout=240):
    env = dict(os.environ, FGREG_DIST_BACKEND=backend, OMP_NUM_THREADS='2')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={nproc}',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
           os.path.join(REPO, 'tools', 'dist_forward_check.py'), *args]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def test_sharded_forward_matches_single_process():
    assert 'max |pose diff|' in _run(2)


def test_configs3_world8_rehearsal():
    """BASELINE configs[3] at its real size: global batch 64, 8 ModelNet pairs per rank on 8
    ranks (gloo, all on the box's one GPU: the 8-GPU RCCL run is the driver's). The gathered
    (6, 64, 3, 4) poses equal one 64-pair forward."""
    out = _run(8, '--pairs-per-rank', '8', timeout=600)
    assert '64 pairs' in out and '(6, 64, 3, 4)' in out and '[8, 8, 8, 8, 8, 8, 8, 8]' in out


def test_balanced_shards_3dmatch_world4():
    """Variable-size indoor fragment pairs (the 3DMatch model), sharded over 4 ranks by
    fgreg.dist.balanced_shards (bench.py's 3DMatch / 3DLoMatch sharding at world > 1): the
    gathered poses equal one forward over all pairs."""
    out = _run(4, '--workload', '3dmatch', '--pairs', '7', timeout=600)
    assert 'balanced_shards' in out and 'max |pose diff|' in out


def test_rccl_branch_world1():
    """fgreg.dist.gather_pair_results and the bench's max-over-ranks all_reduce on DEVICE tensors
    over a real 'nccl' (RCCL) process group: world size 1 (one GPU per rank), in a fresh torchrun
    child. The poses gathered through RCCL must equal the plain forward's."""
    out = _run(1, backend='nccl')
    assert 'backend nccl' in out and 'gathered' in out and 'on cuda' in out
