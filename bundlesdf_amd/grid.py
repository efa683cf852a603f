"""GridEncoder — the torch-module boundary of the reference
(mycuda/torch_ngp_grid_encoder/grid.py:26-171): same constructor, attributes,
parameter/buffer names, init and forward, on top of the libnof kernels.
"""
import numpy as np
import torch
import torch.nn as nn
from torch.autograd import Function

from . import gridencoder

_gridtype_to_id = {"hash": 0, "tiled": 1}


def _autocast_on():
    try:
        return torch.is_autocast_enabled("cuda")
    except TypeError:  # older torch signature
        return torch.is_autocast_enabled()


class _grid_encode(Function):
    """grid.py:31-99."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, inputs, embeddings, offsets, per_level_scale, base_resolution, calc_grad_inputs=False,
                gridtype=0, align_corners=False):
        inputs = inputs.contiguous()
        B, D = inputs.shape
        L = offsets.shape[0] - 1
        C = embeddings.shape[1]
        S = np.log2(per_level_scale)
        H = base_resolution
        # grid.py:50-51: half-precision embeddings under autocast when C is even
        if _autocast_on() and C % 2 == 0:
            embeddings = embeddings.to(torch.half)
        outputs = torch.empty(L, B, C, device=inputs.device, dtype=embeddings.dtype)
        if calc_grad_inputs:
            dy_dx = torch.empty(B, L * D * C, device=inputs.device, dtype=embeddings.dtype)
        else:
            dy_dx = torch.empty(1, device=inputs.device, dtype=embeddings.dtype)
        gridencoder.grid_encode_forward(inputs, embeddings, offsets, outputs, B, D, C, L, S, H, calc_grad_inputs,
                                        dy_dx, gridtype, align_corners)
        outputs = outputs.permute(1, 0, 2).reshape(B, L * C)
        ctx.save_for_backward(inputs, embeddings, offsets, dy_dx)
        ctx.dims = [B, D, C, L, S, H, gridtype]
        ctx.calc_grad_inputs = calc_grad_inputs
        ctx.align_corners = align_corners
        return outputs

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad):
        inputs, embeddings, offsets, dy_dx = ctx.saved_tensors
        B, D, C, L, S, H, gridtype = ctx.dims
        calc_grad_inputs = ctx.calc_grad_inputs
        align_corners = ctx.align_corners
        grad = grad.view(B, L, C).permute(1, 0, 2).contiguous()
        grad_embeddings = torch.zeros_like(embeddings)
        if calc_grad_inputs:
            grad_inputs = torch.zeros_like(inputs, dtype=embeddings.dtype)
        else:
            grad_inputs = torch.zeros(1, device=inputs.device, dtype=embeddings.dtype)
        gridencoder.grid_encode_backward(grad.to(embeddings.dtype), inputs, embeddings, offsets, grad_embeddings, B,
                                         D, C, L, S, H, calc_grad_inputs, dy_dx, grad_inputs, gridtype,
                                         align_corners)
        if calc_grad_inputs:
            return grad_inputs.to(inputs.dtype), grad_embeddings, None, None, None, None, None, None
        return None, grad_embeddings, None, None, None, None, None, None


grid_encode = _grid_encode.apply


def level_layout(input_dim, n_levels, level_dim, base_resolution, log2_hashmap_size, desired_resolution,
                 align_corners=False):
    """Offsets / per-level scale as grid.py:110-135 computes them (float64 on host)."""
    per_level_scale = np.exp2(np.log2(desired_resolution / base_resolution) / (n_levels - 1))
    offsets, offset = [], 0
    max_params = 2 ** log2_hashmap_size
    for i in range(n_levels):
        resolution = int(np.ceil(base_resolution * per_level_scale ** i))
        params_in_level = min(max_params, (resolution if align_corners else resolution + 1) ** input_dim)
        params_in_level = int(np.ceil(params_in_level / 8) * 8)
        offsets.append(offset)
        offset += params_in_level
    offsets.append(offset)
    return per_level_scale, np.array(offsets, dtype=np.int32)


class GridEncoder(nn.Module):
    """grid.py:106-171."""

    def __init__(self, input_dim=3, n_levels=16, level_dim=2, base_resolution=16, log2_hashmap_size=19,
                 desired_resolution=None, gridtype="hash", align_corners=False):
        super().__init__()
        per_level_scale, offsets = level_layout(input_dim, n_levels, level_dim, base_resolution, log2_hashmap_size,
                                                desired_resolution, align_corners)
        self.input_dim = input_dim
        self.n_levels = n_levels
        self.level_dim = level_dim
        self.per_level_scale = per_level_scale
        self.log2_hashmap_size = log2_hashmap_size
        self.base_resolution = base_resolution
        self.out_dim = n_levels * level_dim
        self.gridtype = gridtype
        self.gridtype_id = _gridtype_to_id[gridtype]
        self.align_corners = align_corners
        self.max_params = 2 ** log2_hashmap_size
        self.register_buffer("offsets", torch.from_numpy(offsets))
        self.n_params = self.offsets[-1] * level_dim
        self.embeddings = nn.Parameter(torch.empty(int(offsets[-1]), level_dim))
        self.reset_parameters()

    def reset_parameters(self):
        std = 1e-4
        self.embeddings.data.uniform_(-std, std)

    def __repr__(self):
        return (f"GridEncoder: input_dim={self.input_dim} n_levels={self.n_levels} level_dim={self.level_dim} "
                f"resolution={self.base_resolution} -> "
                f"{int(round(self.base_resolution * self.per_level_scale ** (self.n_levels - 1)))} "
                f"per_level_scale={self.per_level_scale:.4f} params={tuple(self.embeddings.shape)} "
                f"gridtype={self.gridtype} align_corners={self.align_corners}")

    def forward(self, inputs, bound=1):
        inputs = (inputs + bound) / (2 * bound)
        prefix_shape = list(inputs.shape[:-1])
        inputs = inputs.view(-1, self.input_dim)
        outputs = grid_encode(inputs, self.embeddings, self.offsets, self.per_level_scale, self.base_resolution,
                              inputs.requires_grad, self.gridtype_id, self.align_corners)
        return outputs.view(prefix_shape + [self.out_dim])
