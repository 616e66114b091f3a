"""Static floor fields on the device (csrc/floor.hip).

``Map.Init_Potential`` (Louvre_Evacuation/envs/map.py:127-148) for a batch of layouts
of one grid size in one launch, bit-identical to the reference's heapq Dijkstra (see
the kernel's header for why a parallel relaxation reaches the same float64 values).
This is the building block for per-env randomised layouts: the host produces each
layout's pre-potential validity mask, exits and fire term (``evacx.layout.potential_inputs``),
the device the fields.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .env import _stream

_inited = False


def flib():
    global _inited
    L = _lib.lib()
    if not _inited:
        L.evx_floor_last_error.restype = C.c_char_p
        L.evx_floor_field.argtypes = [C.c_int32, C.c_int32, C.c_int32] + [C.c_void_p] * 6
        _inited = True
    return L


def floor_fields(valid: torch.Tensor, source: torch.Tensor, pen: Optional[torch.Tensor] = None,
                 out: Optional[torch.Tensor] = None, passes: Optional[torch.Tensor] = None) -> torch.Tensor:
    """valid, source: u8 [n, GX, GY] on the GPU; pen: f64 [n, GX, GY] or None.
    Returns the floor fields f64 [n, GX, GY] (inf where unreachable)."""
    if valid.dim() != 3 or source.shape != valid.shape:
        raise ValueError("valid/source must be [n, GX, GY] of one shape")
    if valid.dtype != torch.uint8 or source.dtype != torch.uint8:
        raise TypeError("valid/source must be uint8")
    if not valid.is_cuda:
        raise _lib.EvacxError("floor_fields: inputs must be on the GPU (no CPU fallback)")
    n, GX, GY = valid.shape
    valid, source = valid.contiguous(), source.contiguous()
    if pen is not None:
        if pen.shape != valid.shape or pen.dtype != torch.float64:
            raise TypeError("pen must be float64 [n, GX, GY]")
        pen = pen.contiguous()
    if out is None:
        out = torch.empty(n, GX, GY, dtype=torch.float64, device=valid.device)
    rc = flib().evx_floor_field(n, GX, GY, valid.data_ptr(), source.data_ptr(),
                                None if pen is None else pen.data_ptr(), out.data_ptr(),
                                None if passes is None else passes.data_ptr(), _stream())
    if rc != 0:
        raise _lib.EvacxError(f"floor_field failed ({rc}): {flib().evx_floor_last_error().decode()}")
    return out


def floor_fields_for(specs: Sequence, danger0: Optional[Sequence[np.ndarray]] = None,
                     device="cuda") -> Tuple[torch.Tensor, torch.Tensor]:
    """Floor fields of several layouts (evacx.layout.LayoutSpec, one grid size) on the
    device; returns (fields f64 [n, GX, GY], relaxation passes i32 [n])."""
    from .layout import potential_inputs
    ins = [potential_inputs(s, None if danger0 is None else danger0[i]) for i, s in enumerate(specs)]
    v = torch.from_numpy(np.stack([a[0] for a in ins])).to(device)
    s = torch.from_numpy(np.stack([a[1] for a in ins])).to(device)
    p = torch.from_numpy(np.stack([a[2] for a in ins])).to(device)
    passes = torch.zeros(len(specs), dtype=torch.int32, device=device)
    return floor_fields(v, s, p, passes=passes), passes
