"""KPConv + Res2Net backbone on the libfgreg kernels.

Module names and parameter shapes are those of the reference
(models/backbone_kpconv/finegrained_kpconv.py, finegrained_kpconv_blocks.py,
res2net.py), so a reference checkpoint's ``kpf_encoder.*`` keys load unchanged.
The compute path is:

* ``PreprocessorHIP``  -- PreprocessorGPU.forward (finegrained_kpconv.py:431-542) on
  fgr_grid_subsample_* / fgr_radius_search;
* ``KPConv``            -- fgr_kpconv_gather (HBM-bound gather-weight) + one
  (Nq, K*Cin) x (K*Cin, Cout) GEMM; the 1/nnorm normaliser is folded into the
  following instance norm;
* ``BatchNormBlock``    -- fgr_instnorm (per-cloud InstanceNorm1d, fused act/residual);
* ``my_res2Net``        -- BatchNorm folded into the Linear weights (eval) + GEMMs.

This module holds the inference forward; the training forward (Res2Net BatchNorm on batch
statistics, every op differentiable on libfgreg's backward kernels) composes the same modules
in fgreg/training.py.
"""
import math
import os
from typing import List

import numpy as np

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .linear import linear


# ------------------------------------------------------------------------------------------
# Preprocessing
# ------------------------------------------------------------------------------------------
class PreprocessorHIP(nn.Module):
    """KPConv metadata on the GPU (PreprocessorGPU, finegrained_kpconv.py:422-542).

    ``neighbor_mode`` 'ball_query' (default) reproduces the reference's GPU path
    (first K supports in index order, width K); 'nanoflann' reproduces its CPU
    ``Preprocessor`` (K nearest sorted by distance, width min(max, K)).
    """

    def __init__(self, cfg, neighbor_mode='ball_query'):
        super().__init__()
        self.cfg = cfg
        self.mode = {'ball_query': ops.NB_INDEX, 'nanoflann': ops.NB_DIST}[neighbor_mode]

    def _lengths_to_device(self, lens, device):
        if device.type != 'cuda':
            return torch.tensor(lens, dtype=torch.int64, device=device)
        buf = getattr(self, '_pin', None)
        if buf is None or buf.numel() < len(lens):
            buf = torch.empty(max(64, len(lens)), dtype=torch.int64, pin_memory=True)
            self._pin, self._pin_ev = buf, None
        if self._pin_ev is not None:
            self._pin_ev.synchronize()       # the previous copy out of the buffer is done
        buf[:len(lens)].copy_(torch.tensor(lens, dtype=torch.int64))
        out = buf[:len(lens)].to(device, non_blocking=True)
        self._pin_ev = torch.cuda.Event()
        self._pin_ev.record()
        return out

    def forward(self, pts: List[torch.Tensor]):
        cfg = self.cfg
        limits = cfg.neighborhood_limits
        device = pts[0].device
        r_normal = cfg.first_subsampling_dl * cfg.conv_radius
        arch = cfg.architecture
        lens = [int(p.shape[0]) for p in pts]
        points = torch.cat([p.float() for p in pts], 0).contiguous()
        # device lengths / offsets of every level without a synchronising copy: level 0's
        # lengths by an asynchronous copy from a pinned staging buffer (reused: the previous
        # forward's copy completed at its voxel-count readback), offsets by
        # fgr_lengths_to_offsets; deeper levels straight from the voxel counts. So nothing in
        # the forward waits on the GPU before the first count readback, and those launches
        # queue behind the previous step's work.
        len_dev = self._lengths_to_device(lens, device)
        off = ops.lengths_to_offsets(len_dev)
        meta = {'points': [], 'neighbors': [], 'pools': [], 'upsamples': [], 'stack_lengths': []}
        host = {'lengths': [], 'offsets': []}
        layer_blocks, layer = [], 0
        for bi, block in enumerate(arch):
            if 'global' in block or 'upsample' in block:
                break
            if not ('pool' in block or 'strided' in block):
                layer_blocks.append(block)
                if bi < len(arch) - 1 and 'upsample' not in arch[bi + 1]:
                    continue
            if any('deformable' in b for b in layer_blocks[:-1]) or 'deformable' in block:
                raise NotImplementedError('deformable KPConv is not used by the reference configs')
            r = r_normal
            # one cell grid over this level's points serves the conv and the pool tables
            # (same supports, same radius); None for small clouds (brute-force scan)
            grid = ops.radius_grid(points, off, lens, r)
            if layer_blocks:
                conv_i = ops.radius_search(points, off, lens, points, off, lens, r, limits[layer],
                                           self.mode, grid=grid)
            else:
                conv_i = torch.zeros((0, 1), dtype=torch.int64, device=device)
            if 'pool' in block or 'strided' in block:
                dl = 2 * r_normal / cfg.conv_radius
                pool_p, pool_lens, pool_len_dev, pool_off = ops.grid_subsample(points, off, lens, dl,
                                                                               device_layout=True)
                pool_i = ops.radius_search(pool_p, pool_off, pool_lens, points, off, lens, r,
                                           limits[layer], self.mode, grid=grid)
                up_grid = ops.radius_grid(pool_p, pool_off, pool_lens, 2 * r)
                up_i = ops.radius_search(points, off, lens, pool_p, pool_off, pool_lens, 2 * r,
                                         limits[layer], self.mode, grid=up_grid)
            else:
                pool_p = torch.zeros((0, 3), dtype=torch.float32, device=device)
                pool_lens, pool_off, pool_len_dev = [], None, None
                pool_i = torch.zeros((0, 1), dtype=torch.int64, device=device)
                up_i = torch.zeros((0, 1), dtype=torch.int64, device=device)
            meta['points'].append(points)
            meta['neighbors'].append(conv_i)
            meta['pools'].append(pool_i)
            meta['upsamples'].append(up_i)
            meta['stack_lengths'].append(len_dev)
            host['lengths'].append(lens)
            host['offsets'].append(off)
            points, lens, off, len_dev = pool_p, pool_lens, pool_off, pool_len_dev
            r_normal *= 2
            layer += 1
            layer_blocks = []
        meta['_host'] = host  # host-side lengths + device offsets, reused by the encoder
        return meta


class FixedMetaPreprocessor(nn.Module):
    """Returns a precomputed kpconv_meta (used to run the forward on the reference's own
    neighbour tables in the parity tests)."""

    def __init__(self, meta):
        super().__init__()
        self.meta = meta

    def forward(self, pts):
        return dict(self.meta)


def host_layout(meta, level):
    """(lengths list, device offsets) of a pyramid level, computed once per meta."""
    host = meta.get('_host')
    if host is None:
        host = {'lengths': [], 'offsets': []}
        for sl in meta['stack_lengths']:
            lens = [int(v) for v in sl.tolist()]
            host['lengths'].append(lens)
            host['offsets'].append(ops.offsets(lens, sl.device))
        meta['_host'] = host
    return host['lengths'][level], host['offsets'][level]


# ------------------------------------------------------------------------------------------
# Kernel points
# ------------------------------------------------------------------------------------------
def kernel_disposition(n_kp=15, seed=42, iters=400):
    """A rigid KPConv kernel disposition: one point fixed at the centre, the others
    spread by a repulsive potential inside the unit ball and rescaled so that their
    mean radius is 0.66 (the recipe of kernels/kernel_points.py:321-384, re-derived;
    checkpoints carry their own ``kernel_points`` so this only seeds a fresh init)."""
    rng = np.random.default_rng(seed)
    p = rng.normal(size=(n_kp, 3))
    p[0] = 0
    p[1:] *= 0.5 / np.linalg.norm(p[1:], axis=1, keepdims=True)
    for it in range(iters):
        d = p[:, None, :] - p[None, :, :]
        r = np.linalg.norm(d, axis=-1) + np.eye(n_kp)
        grad = -(d / r[..., None] ** 3).sum(1) + 2.0 * p  # repulsion + confinement
        grad[0] = 0
        p -= 0.01 * grad / (np.linalg.norm(grad, axis=1, keepdims=True).max() + 1e-12)
    p[1:] *= 0.66 / np.mean(np.linalg.norm(p[1:], axis=1))
    return p


def init_kernel_points(radius, n_kp, rng=np.random):
    """Random z-rotation + N(0, 0.01) noise + scale, as load_kernels (kernel_points.py:430-469)."""
    kp = kernel_disposition(n_kp)
    theta = rng.rand() * 2 * np.pi
    c, s = np.cos(theta), np.sin(theta)
    R = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]], dtype=np.float32)
    kp = kp + rng.normal(scale=0.01, size=kp.shape)
    return np.matmul(radius * kp, R).astype(np.float32)


# ------------------------------------------------------------------------------------------
# Blocks
# ------------------------------------------------------------------------------------------
class KPConv(nn.Module):
    """Rigid KPConv (finegrained_kpconv_blocks.py:171-401): linear influence, sum mode."""

    def __init__(self, kernel_size, p_dim, in_channels, out_channels, KP_extent, radius,
                 fixed_kernel_points='center', KP_influence='linear', aggregation_mode='sum',
                 deformable=False, modulated=False):
        super().__init__()
        if deformable or KP_influence != 'linear' or aggregation_mode != 'sum' or p_dim != 3:
            raise NotImplementedError('only the rigid/linear/sum KPConv of the reference configs')
        self.K, self.p_dim = kernel_size, p_dim
        self.in_channels, self.out_channels = in_channels, out_channels
        self.radius, self.KP_extent = radius, KP_extent
        self.weights = nn.Parameter(torch.zeros((kernel_size, in_channels, out_channels)))
        nn.init.kaiming_uniform_(self.weights, a=math.sqrt(5))
        self.kernel_points = nn.Parameter(
            torch.tensor(init_kernel_points(radius, kernel_size)), requires_grad=False)

    def forward_unnormalized(self, q_pts, s_pts, neighb_inds, x):
        """-> (sum_k WF_k @ W_k (Nq, Cout), nnorm (Nq,)). The reference divides the first
        by the second (:395-399); callers fuse that division into the next kernel."""
        wf, nnorm = ops.kpconv_gather(q_pts, s_pts, neighb_inds, x, self.kernel_points,
                                      self.KP_extent)
        out = linear(wf.view(wf.shape[0], -1), self.weights, transpose=True)
        return out, nnorm

    def forward(self, q_pts, s_pts, neighb_inds, x):
        out, nnorm = self.forward_unnormalized(q_pts, s_pts, neighb_inds, x)
        return out / nnorm.unsqueeze(1)


class BatchNormBlock(nn.Module):
    """Per-cloud InstanceNorm1d (finegrained_kpconv_blocks.py:462-518); no parameters."""

    def __init__(self, in_dim, use_bn, bn_momentum):
        super().__init__()
        if not use_bn:
            raise NotImplementedError('use_batch_norm=False is not used by the reference configs')
        self.in_dim = in_dim

    def forward(self, x, off, lengths, row_div=None, act=ops.ACT_NONE, residual=None,
                post_act=ops.ACT_NONE):
        return ops.instnorm(x, off, lengths, row_div=row_div, act=act, residual=residual,
                            post_act=post_act)


class UnaryBlock(nn.Module):
    """Linear(no bias) -> InstanceNorm -> LeakyReLU(0.1) (blocks:521-555)."""

    def __init__(self, in_dim, out_dim, use_bn, bn_momentum, no_relu=False):
        super().__init__()
        self.in_dim, self.out_dim, self.no_relu = in_dim, out_dim, no_relu
        self.mlp = nn.Linear(in_dim, out_dim, bias=False)
        self.batch_norm = BatchNormBlock(out_dim, use_bn, bn_momentum)

    def forward(self, x, off, lengths, residual=None, post_act=ops.ACT_NONE):
        y = linear(x, self.mlp.weight)
        act = ops.ACT_NONE if self.no_relu else ops.ACT_LEAKY
        return self.batch_norm(y, off, lengths, act=act, residual=residual, post_act=post_act)


class my_Bottle2neck(nn.Module):  # noqa: N801 -- reference name (res2net.py:84)
    """Res2Net bottleneck on Linear + BatchNorm1d (res2net.py:84-159), stype 'normal'."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, baseWidth=26, scale=4,
                 stype='normal'):
        super().__init__()
        width = int(math.floor(planes * (baseWidth / 64.0)))
        self.conv1 = nn.Linear(inplanes, width * scale, bias=False)
        self.bn1 = nn.BatchNorm1d(width * scale)
        self.nums = 1 if scale == 1 else scale - 1
        self.convs = nn.ModuleList([nn.Linear(width, width, bias=False) for _ in range(self.nums)])
        self.bns = nn.ModuleList([nn.BatchNorm1d(width) for _ in range(self.nums)])
        self.conv3 = nn.Linear(width * scale, planes, bias=False)
        self.bn3 = nn.BatchNorm1d(planes)
        self.downsample = downsample
        self.stype, self.scale, self.width = stype, scale, width
        self._folded = None

    # -- eval: BatchNorm folded into the Linear weights ---------------------------------
    @staticmethod
    def _fold(lin, bn):
        s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
        return (lin.weight * s[:, None]).contiguous(), (bn.bias - bn.running_mean * s).contiguous()

    def _folded_params(self):
        # version AND storage pointer: Module.to() / .cuda() swap .data without a version bump
        key = tuple((p._version, p.data_ptr()) for p in self.parameters()) + tuple(
            (b._version, b.data_ptr()) for b in self.buffers())
        if self._folded is None or self._folded[0] != key:
            with torch.no_grad():
                w1, b1 = self._fold(self.conv1, self.bn1)
                ws = [self._fold(c, b) for c, b in zip(self.convs, self.bns)]
                w3, b3 = self._fold(self.conv3, self.bn3)
                if self.downsample is not None:
                    wd, bd = self._fold(self.downsample[0], self.downsample[1])
                    w3d = torch.cat([w3, wd], 1).contiguous()   # [conv3 | downsample] along K
                    b3d = (b3 + bd).contiguous()
                else:
                    w3d, b3d = w3, b3
                chain = None
                if w1.is_cuda and self.nums > 0 and self.downsample is not None:
                    wst = torch.stack([wi for wi, _ in ws])
                    bst = torch.stack([bi for _, bi in ws]).contiguous()
                    # w = 224: the bf16x6 chain unless FGREG_R2N224=h3 (A/B); else h3
                    if self.width == 224 and os.environ.get('FGREG_R2N224', 'x6') != 'h3':
                        chain = (bst, ops.res2net_fragments3(wst), None)
                    elif ops.res2net_chain_supported(self.width, True):
                        chain = (bst,) + ops.res2net_fragments_h3(wst)
            self._folded = (key, w1, b1, ws, w3d, b3d, chain)
            ops.note_state(w1, b1, w3d, b3d, *[t for wb in ws for t in wb],
                           *(chain if chain is not None else ()))
        return self._folded[1:]

    def forward(self, x, shortcut=None):
        """-> relu(bn3(conv3(cat)) + downsample(x)); with ``shortcut`` (the enclosing
        bottleneck block's identity shortcut) -> LeakyReLU_0.1(that + shortcut), fused into
        the last GEMM's epilogue (finegrained_kpconv_blocks.py:715-725)."""
        if self.training:       # batch statistics, differentiable (fgreg/training.py)
            from .training import bottle2neck_train
            y = bottle2neck_train(self, x)
            return y if shortcut is None else F.leaky_relu(y + shortcut, 0.1)
        w1, b1, ws, w3d, b3d, chain = self._folded_params()
        out = linear(x, w1, b1, act=ops.ACT_RELU)
        w = self.width
        down = self.downsample is not None
        cat_in = torch.empty((x.shape[0], w * self.scale + (x.shape[1] if down else 0)),
                             dtype=x.dtype, device=x.device)
        if chain is not None:
            # one launch for the whole hierarchy + the [.. | x] concat (fgr_res2net_chain*)
            ops.res2net_chain(out, w, self.scale, chain[1], chain[0], x, cat_in, w_scale=chain[2])
        else:
            # widths / layouts without a chain kernel: one GEMM (+ bias + ReLU) per step
            sp = None
            for i in range(self.nums):
                chunk = out[:, i * w:(i + 1) * w]
                sp = chunk if i == 0 else sp + chunk
                sp = linear(sp, ws[i][0], ws[i][1], act=ops.ACT_RELU,
                            out=cat_in[:, i * w:(i + 1) * w])
            if self.scale != 1:
                cat_in[:, self.nums * w:self.scale * w] = out[:, self.nums * w:self.scale * w]
            if down:
                cat_in[:, self.scale * w:] = x
        if down:        # [conv3 | downsample] in one GEMM, the shortcut in its epilogue
            if shortcut is not None:
                return linear(cat_in, w3d, b3d, act=ops.ACT_RELU_RES_LEAKY, residual=shortcut)
            return linear(cat_in, w3d, b3d, act=ops.ACT_RELU)
        y = linear(cat_in, w3d, b3d, act=ops.ACT_RELU, residual=x)    # identity downsample
        return y if shortcut is None else F.leaky_relu(y + shortcut, 0.1)


class my_res2Net(nn.Module):  # noqa: N801 -- reference name (res2net.py:231)
    def __init__(self, block, in_dim, out_dim, baseWidth=26, scale=4):
        super().__init__()
        downsample = None
        if in_dim != out_dim * block.expansion:
            downsample = nn.Sequential(nn.Linear(in_dim, out_dim, bias=False),
                                       nn.BatchNorm1d(out_dim))
        self.layer1 = nn.Sequential(block(in_dim, out_dim, 1, downsample=downsample,
                                          stype='normal', baseWidth=baseWidth, scale=scale))

    def forward(self, x, shortcut=None):
        return self.layer1(x) if shortcut is None else self.layer1[0](x, shortcut)


def _level_inputs(block, layer_ind, batch):
    if 'strided' in block:
        q = batch['points'][layer_ind + 1]
        s = batch['points'][layer_ind]
        idx = batch['pools'][layer_ind]
        post = layer_ind + 1
    else:
        q = s = batch['points'][layer_ind]
        idx = batch['neighbors'][layer_ind]
        post = layer_ind
    return q, s, idx, post


class SimpleBlock(nn.Module):
    """KPConv -> InstanceNorm -> LeakyReLU (blocks:578-634)."""

    def __init__(self, block_name, in_dim, out_dim, radius, layer_ind, config):
        super().__init__()
        extent = radius * config.KP_extent / config.conv_radius
        self.block_name, self.layer_ind = block_name, layer_ind
        self.in_dim, self.out_dim = in_dim, out_dim
        self.KPConv = KPConv(config.num_kernel_points, config.in_points_dim, in_dim, out_dim // 2,
                             extent, radius, fixed_kernel_points=config.fixed_kernel_points,
                             KP_influence=config.KP_influence,
                             aggregation_mode=config.aggregation_mode,
                             deformable='deform' in block_name, modulated=config.modulated)
        self.batch_norm = BatchNormBlock(out_dim // 2, config.use_batch_norm,
                                         config.batch_norm_momentum)

    def forward(self, x, batch):
        q, s, idx, post = _level_inputs(self.block_name, self.layer_ind, batch)
        lens, off = host_layout(batch, post)
        y, nnorm = self.KPConv.forward_unnormalized(q, s, idx, x)
        return self.batch_norm(y, off, lens, row_div=nnorm, act=ops.ACT_LEAKY)


class ResnetBottleneckBlock(nn.Module):
    """unary1 -> KPConv -> IN -> Res2Net -> (+ shortcut) -> LeakyReLU (blocks:637-727)."""

    def __init__(self, block_name, in_dim, out_dim, radius, layer_ind, config, flag=False):
        super().__init__()
        extent = radius * config.KP_extent / config.conv_radius
        self.block_name, self.layer_ind = block_name, layer_ind
        self.in_dim, self.out_dim = in_dim, out_dim
        use_bn, mom = config.use_batch_norm, config.batch_norm_momentum
        self.unary1 = (UnaryBlock(in_dim, out_dim // 4, use_bn, mom) if in_dim != out_dim // 4
                       else nn.Identity())
        self.KPConv = KPConv(config.num_kernel_points, config.in_points_dim, out_dim // 4,
                             out_dim // 4, extent, radius,
                             fixed_kernel_points=config.fixed_kernel_points,
                             KP_influence=config.KP_influence,
                             aggregation_mode=config.aggregation_mode,
                             deformable='deform' in block_name, modulated=config.modulated)
        self.batch_norm_conv = BatchNormBlock(out_dim // 4, use_bn, mom)
        self.res2net = my_res2Net(my_Bottle2neck, out_dim // 4, out_dim, baseWidth=14, scale=8)
        self.unary_shortcut = (UnaryBlock(in_dim, out_dim, use_bn, mom, no_relu=True)
                               if in_dim != out_dim else nn.Identity())

    def forward(self, features, batch):
        q, s, idx, post = _level_inputs(self.block_name, self.layer_ind, batch)
        lens_pre, off_pre = host_layout(batch, self.layer_ind)
        lens_post, off_post = host_layout(batch, post)
        if isinstance(self.unary1, UnaryBlock):
            x = self.unary1(features, off_pre, lens_pre)
        else:
            x = features
        y, nnorm = self.KPConv.forward_unnormalized(q, s, idx, x)
        y = self.batch_norm_conv(y, off_post, lens_post, row_div=nnorm)
        # res2net ends in ReLU, so the reference's LeakyReLU at :715 is the identity here
        shortcut = ops.max_pool(features, idx) if 'strided' in self.block_name else features
        if isinstance(self.unary_shortcut, UnaryBlock):
            y = self.res2net(y)
            # LeakyReLU(y + IN(shortcut @ W^T)) in one kernel (:722-725)
            return self.unary_shortcut(shortcut, off_post, lens_post, residual=y,
                                       post_act=ops.ACT_LEAKY)
        # identity shortcut: LeakyReLU(y + shortcut) in the Res2Net's last GEMM epilogue
        return self.res2net(y, shortcut=shortcut)


def block_decider(block_name, radius, in_dim, out_dim, layer_ind, config, flag=False):
    """finegrained_kpconv_blocks.py:414-460 (the block types of the reference configs)."""
    if block_name == 'simple':
        return SimpleBlock(block_name, in_dim, out_dim, radius, layer_ind, config)
    if block_name in ('resnetb', 'resnetb_strided'):
        return ResnetBottleneckBlock(block_name, in_dim, out_dim, radius, layer_ind, config, flag)
    raise NotImplementedError(f'block {block_name!r} is not used by the reference configs')


class KPFEncoder(nn.Module):
    """finegrained_kpconv.py:22-95."""

    def __init__(self, config, d_bottle, increase_channel_when_downsample=True):
        super().__init__()
        octave = 0
        r = config.first_subsampling_dl * config.conv_radius
        in_dim, out_dim = config.in_feats_dim, config.first_feats_dim
        self.encoder_blocks = nn.ModuleList()
        self.encoder_skip_dims, self.encoder_skips = [], []
        block_i, block = 0, ''
        for block_i, block in enumerate(config.architecture):
            if any(t in block for t in ('pool', 'strided', 'upsample', 'global')):
                self.encoder_skips.append(block_i)
                self.encoder_skip_dims.append(in_dim)
            if 'upsample' in block:
                break
            self.encoder_blocks.append(block_decider(block, r, in_dim, out_dim, octave, config,
                                                     flag=True))
            in_dim = out_dim // 2 if 'simple' in block else out_dim
            if 'pool' in block or 'strided' in block:
                octave += 1
                r *= 2
                if increase_channel_when_downsample:
                    out_dim *= 2
        if 'upsample' not in block:
            self.encoder_skips.append(block_i)
            self.encoder_skip_dims.append(in_dim)

    def forward(self, x, batch):
        skip_x = []
        for block_i, block_op in enumerate(self.encoder_blocks):
            if block_i in self.encoder_skips:
                skip_x.append(x)
            x = block_op(x, batch)
        return x, skip_x
