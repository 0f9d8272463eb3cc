"""Shared access to libgsr_hip.so for gs_train (no fallback: a missing library raises)."""
from __future__ import annotations

import ctypes

import torch

from diff_gaussian_rasterization import _lib


def lib():
    return _lib.load()


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {_lib.last_error()}")


def ptr(t: torch.Tensor | None):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() > 0 else ctypes.c_void_p(0)


def stream(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_gpu(*tensors: torch.Tensor) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("gs_train kernels require tensors on a ROCm GPU device")
