"""CPU, build container only: the drop-in models/finegrained_regtr.py (package file
finegrained_regtr.py) constructs inside the reference's own module tree and its
state_dict matches the reference RegTR key for key (so CheckPointManager.load works).
Skipped where the reference is not mounted (the GPU box)."""
import os
import sys

import pytest
import torch

from conftest import PKG, REPO

REF = '/root/reference'
LIBREF = os.path.join(REPO, 'oracle', '_ref', 'libkpconv_ref.so')

pytestmark = pytest.mark.skipif(not (os.path.isdir(REF) and os.path.exists(LIBREF)),
                                reason='reference checkout / oracle/_ref not available')


def test_dropin_state_dict_matches_reference():
    sys.path.insert(0, os.path.join(REPO, 'tests', 'golden'))
    import make_golden as mg
    fr, fk = mg.import_reference()
    import importlib.util
    spec = importlib.util.spec_from_file_location('fgreg_dropin', os.path.join(PKG, 'finegrained_regtr.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for conf in ('modelnet.yaml', '3dmatch.yaml'):
        cfg = mg.load_cfg(conf)
        cwd = os.getcwd()
        os.chdir(REF)
        try:
            ref = fr.RegTR(cfg)
        finally:
            os.chdir(cwd)
        mine = mod.RegTR(cfg)
        a, b = ref.state_dict(), mine.state_dict()
        assert set(a) == set(b)
        for k in a:
            assert a[k].shape == b[k].shape, k
        # a reference checkpoint loads strictly
        mine.load_state_dict(a, strict=True)
        assert torch.equal(mine.kpf_encoder.encoder_blocks[1].KPConv.weights,
                           ref.kpf_encoder.encoder_blocks[1].KPConv.weights)
        assert callable(mine.compute_loss) and mine.forward.__qualname__ == 'RegTR.forward'
