"""Module `gridencoder` — drop-in for the reference's pybind extension
(mycuda/torch_ngp_grid_encoder/bindings.cpp:14-17), backed by libnof.

Same function names, positional signatures, in-place output convention and
error behaviour (TORCH_CHECK -> RuntimeError) as gridencoder.cu:447-502.
"""
import torch

from . import _lib

_DTYPES = {torch.float32: 0, torch.float16: 1}


def _check_common(named):
    for name, t in named:
        _lib.require_device(t, name)
    for name, t in named:
        _lib.require_contiguous(t, name)


def _check_floating(t, name):
    if t.dtype not in (torch.float32, torch.float16, torch.float64):
        raise RuntimeError(f"{name} must be a floating tensor")


def _emb_dtype(embeddings):
    if embeddings.dtype not in _DTYPES:
        raise RuntimeError(f"grid_encode: unsupported embeddings dtype {embeddings.dtype} (float32/float16)")
    return _DTYPES[embeddings.dtype]


def grid_encode_forward(inputs, embeddings, offsets, outputs, B, D, C, L, S, H, calc_grad_inputs, dy_dx, gridtype,
                        align_corners):
    """gridencoder.cu:447-470. outputs [L,B,C] and dy_dx [B,L*D*C] written in place."""
    _check_common([("inputs", inputs), ("embeddings", embeddings), ("offsets", offsets), ("outputs", outputs),
                   ("dy_dx", dy_dx)])
    for n, t in (("inputs", inputs), ("embeddings", embeddings), ("outputs", outputs), ("dy_dx", dy_dx)):
        _check_floating(t, n)
    if offsets.dtype != torch.int32:
        raise RuntimeError("offsets must be an int tensor")
    if inputs.dtype != torch.float32:
        raise RuntimeError(f"expected scalar type Float but found {inputs.dtype}")
    dt = _emb_dtype(embeddings)
    for n, t in (("outputs", outputs), ("dy_dx", dy_dx)):
        if t.dtype != embeddings.dtype:
            raise RuntimeError(f"{n}: expected scalar type {embeddings.dtype} but found {t.dtype}")
    rc = _lib.lib().nof_grid_encode_forward(
        _lib.ptr(inputs), _lib.ptr(embeddings), _lib.ptr(offsets), _lib.ptr(outputs), int(B), int(D), int(C), int(L),
        float(S), int(H), int(bool(calc_grad_inputs)), _lib.ptr(dy_dx), int(gridtype), int(bool(align_corners)), dt,
        _lib.stream_of(inputs))
    _lib.check(rc, "grid_encode_forward")


def grid_encode_backward(grad, inputs, embeddings, offsets, grad_embeddings, B, D, C, L, S, H, calc_grad_inputs, dy_dx,
                         grad_inputs, gridtype, align_corners):
    """gridencoder.cu:472-502. grad_embeddings (zeroed by caller) and grad_inputs written in place."""
    _check_common([("grad", grad), ("inputs", inputs), ("embeddings", embeddings), ("offsets", offsets),
                   ("grad_embeddings", grad_embeddings), ("dy_dx", dy_dx), ("grad_inputs", grad_inputs)])
    for n, t in (("grad", grad), ("inputs", inputs), ("embeddings", embeddings), ("grad_embeddings", grad_embeddings),
                 ("dy_dx", dy_dx), ("grad_inputs", grad_inputs)):
        _check_floating(t, n)
    if offsets.dtype != torch.int32:
        raise RuntimeError("offsets must be an int tensor")
    if inputs.dtype != torch.float32:
        raise RuntimeError(f"expected scalar type Float but found {inputs.dtype}")
    if grad.dtype not in _DTYPES:
        raise RuntimeError(f"grid_encode_backward: unsupported grad dtype {grad.dtype}")
    dt = _DTYPES[grad.dtype]
    for n, t in (("grad_embeddings", grad_embeddings), ("dy_dx", dy_dx), ("grad_inputs", grad_inputs)):
        if t.dtype != grad.dtype:
            raise RuntimeError(f"{n}: expected scalar type {grad.dtype} but found {t.dtype}")
    rc = _lib.lib().nof_grid_encode_backward(
        _lib.ptr(grad), _lib.ptr(inputs), _lib.ptr(embeddings), _lib.ptr(offsets), _lib.ptr(grad_embeddings), int(B),
        int(D), int(C), int(L), float(S), int(H), int(bool(calc_grad_inputs)), _lib.ptr(dy_dx), _lib.ptr(grad_inputs),
        int(gridtype), int(bool(align_corners)), dt, _lib.stream_of(inputs))
    _lib.check(rc, "grid_encode_backward")
