"""Deterministic model weights derived from parameter names (fixture infrastructure).

The forward / loss / training fixtures used to store every weight of the model they were
computed with. Instead, make_golden.py now overwrites the reference model's freshly built
state_dict with values that depend only on (key, shape, seed) -- the same function the tests
call to rebuild the state_dict -- so a fixture stores the key / shape list and the few values
the reference draws itself (its randomly rotated kernel points), not the weights.

Values per key (scales of PyTorch's default initialisers, so activations stay O(1)):
  *.num_batches_tracked     0
  *.running_mean            0.1 N(0, 1)
  *.running_var             0.75 + 0.5 U(0, 1)
  1-D *.weight              1 + 0.1 N(0, 1)      (BatchNorm / LayerNorm affine)
  1-D *.bias                0.1 N(0, 1)          (conf_logits_decoder.bias: the fixture's bias)
  n-D *                     U(-b, b), b = 1 / sqrt(prod(shape[1:])) for (out, in) Linear
                            weights, 1 / sqrt(K * Cin) for (K, Cin, Cout) KPConv weights
"""
import zlib

import numpy as np


def _rng(key, seed):
    return np.random.default_rng([zlib.crc32(key.encode()), seed])


def named_value(key, shape, seed, logit_bias):
    shape = tuple(int(s) for s in shape)
    if key.endswith('num_batches_tracked'):
        return np.zeros(shape, np.int64)
    rng = _rng(key, seed)
    if key.endswith('running_mean'):
        v = 0.1 * rng.standard_normal(shape)
    elif key.endswith('running_var'):
        v = 0.75 + 0.5 * rng.random(shape)
    elif len(shape) == 1 and key.endswith('weight'):
        v = 1.0 + 0.1 * rng.standard_normal(shape)
    elif len(shape) == 1:
        if key == 'correspondence_decoder.conf_logits_decoder.bias':
            return np.full(shape, logit_bias, np.float32)
        v = 0.1 * rng.standard_normal(shape)
    else:
        fan_in = shape[0] * shape[1] if len(shape) == 3 else int(np.prod(shape[1:]))
        b = 1.0 / np.sqrt(max(fan_in, 1))
        v = rng.uniform(-b, b, shape)
    return v.astype(np.float32)


def named_state_dict(keys_shapes, seed, logit_bias, stored=None):
    """{key: np.ndarray} for every (key, shape); keys present in ``stored`` (values the
    reference drew itself, e.g. kernel points) are taken from it."""
    stored = stored or {}
    return {k: (stored[k] if k in stored else named_value(k, s, seed, logit_bias))
            for k, s in keys_shapes}
