"""GPU-resident prioritized replay (BASELINE config cfg5).

The reference's replay is a uniform ``deque`` (Louvre_Evacuation/agents/dqn_agent.py:89,
``random.sample`` at :132). ``PrioReplay`` keeps the same compact-observation ring as
``trainer.Replay`` and adds the proportional prioritized variant of Schaul et al.
(2016) on the device (csrc/prio.hip, ``evx_prio_*`` in include/evacx.h):

* sum and min segment trees of the leaf priorities p_i^alpha over the ring's slots;
* new transitions get the largest leaf priority so far (``expose``);
* stratified sampling (one draw per 1/B of the total mass) with importance weights
  w = (p / p_min)^-beta, beta annealed to 1 by the trainer;
* after a learn step the sampled slots get (|TD error| + eps)^alpha (``update``).

Slots a concurrently running push is about to overwrite are *hidden* (priority 0) so
the lagged schedule's learn step never samples them (``expose(n_hide=...)``).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from .env import OBS_WORDS, _stream
from .trainer import Replay


class evx_prio(C.Structure):
    _fields_ = [("capacity", C.c_int64), ("sum", C.c_void_p), ("mn", C.c_void_p), ("max_leaf", C.c_void_p),
                ("owner", C.c_void_p)]


_inited = False


def plib():
    global _inited
    L = _lib.lib()
    if not _inited:
        P = C.POINTER(evx_prio)
        L.evx_prio_last_error.restype = C.c_char_p
        L.evx_prio_init.argtypes = [P, C.c_void_p]
        L.evx_prio_set_range.argtypes = [P, C.c_int64, C.c_int64, C.c_int64, C.c_void_p]
        L.evx_prio_update.argtypes = [P, C.c_void_p, C.c_void_p, C.c_int32, C.c_double, C.c_double, C.c_void_p]
        L.evx_prio_sample.argtypes = [C.c_void_p, P, C.c_int32, C.c_double, C.c_uint64, C.c_uint64] + \
            [C.c_void_p] * 8
        _inited = True
    return L


def pcheck(rc, what):
    if rc != 0:
        raise _lib.EvacxError(f"{what} failed ({rc}): {plib().evx_prio_last_error().decode()}")


class PrioReplay(Replay):
    """Replay ring + device priority trees. capacity must be a power of two."""

    def __init__(self, capacity: int, device, alpha: float = 0.6, eps: float = 1e-6):
        if capacity & (capacity - 1) or capacity < 1024:
            raise ValueError("prioritized replay capacity must be a power of two >= 1024")
        super().__init__(capacity, device)
        self.alpha, self.eps = float(alpha), float(eps)
        f64 = dict(dtype=torch.float64, device=device)
        self.tsum = torch.zeros(2 * capacity, **f64)
        self.tmin = torch.zeros(2 * capacity, **f64)
        self.max_leaf = torch.zeros(1, **f64)
        self.owner = torch.zeros(capacity, dtype=torch.int32, device=device)
        self.t = evx_prio(capacity=capacity, sum=self.tsum.data_ptr(), mn=self.tmin.data_ptr(),
                          max_leaf=self.max_leaf.data_ptr(), owner=self.owner.data_ptr())
        pcheck(plib().evx_prio_init(C.byref(self.t), _stream()), "prio_init")
        self.unexposed = 0  # pushed transitions whose leaves are not set yet

    def push(self, *args, **kw):
        n = args[5] if len(args) > 5 else kw["n"]
        super().push(*args, **kw)
        self.unexposed = min(self.capacity, self.unexposed + n)

    def expose(self, n_hide: int = 0):
        """Give the transitions pushed since the last call the max priority and hide the
        next n_hide slots (those the next push overwrites)."""
        n_new = min(self.unexposed, self.capacity - n_hide)
        start = (self.pos - n_new) % self.capacity
        pcheck(plib().evx_prio_set_range(C.byref(self.t), start, n_new, n_hide, _stream()), "prio_set_range")
        self.unexposed = 0

    def sample_prio(self, B, beta, seed, offset, out, idx, w):
        pcheck(plib().evx_prio_sample(C.byref(self.c), C.byref(self.t), B, beta, seed, offset,
                                      out["s"].data_ptr(), out["s2"].data_ptr(), out["a"].data_ptr(),
                                      out["r"].data_ptr(), out["done"].data_ptr(), idx.data_ptr(), w.data_ptr(),
                                      _stream()), "prio_sample")

    def update(self, idx, td_abs, B):
        pcheck(plib().evx_prio_update(C.byref(self.t), idx.data_ptr(), td_abs.data_ptr(), B, self.eps, self.alpha,
                                      _stream()), "prio_update")


__all__ = ["PrioReplay", "evx_prio", "OBS_WORDS"]
