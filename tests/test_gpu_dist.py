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


def test_sharded_forward_matches_single_process():
    env = dict(os.environ, FGREG_DIST_BACKEND='gloo', OMP_NUM_THREADS='4')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
           os.path.join(REPO, 'tools', 'dist_forward_check.py')]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0, r.stderr[-2000:]
    assert 'max |pose diff|' in r.stdout


def test_rccl_branch_world1():
    """fgreg.dist.gather_pair_results and the bench's max-over-ranks all_reduce on DEVICE tensors
    over a real 'nccl' (RCCL) process group: world size 1 (one GPU per rank), in a fresh torchrun
    child. The poses gathered through RCCL must equal the plain forward's."""
    env = dict(os.environ, FGREG_DIST_BACKEND='nccl', OMP_NUM_THREADS='4')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=1',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
           os.path.join(REPO, 'tools', 'dist_forward_check.py')]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0, r.stderr[-2000:]
    assert 'backend nccl' in r.stdout and 'gathered on cuda' in r.stdout
