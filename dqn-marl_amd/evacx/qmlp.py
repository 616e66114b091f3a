"""Host driver of the fused MLP Q-network kernels (csrc/qmlp.hip, include/evacx.h).

The MLP variant of DQNNetwork (agents/dqn_agent.py:15-61; 726 -> 512 -> 256 -> 5)
evaluated straight from compact observations: fc1 expands them on the fly, fc2+fc3
and DQNAgent.act's epsilon-greedy (:101-124) run in one more kernel. bf16 operand
copies of fc1/fc2 weights are re-packed from the fp32 master parameters after every
update. Two arithmetic modes: x3=True (the reference's fp32: every f32 operand as a
bf16 hi + lo pair, products hi*hi + hi*lo + lo*hi on the bf16 MFMA) and x3=False (bf16
operands, f32 accumulation).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .env import _stream

HID, HID2, NACT, K1, K1P = 512, 256, 5, 726, 512
K1X = 640  # x3: compact K + one danger-residual slot per cell
NCELL, CENTRE_COL = 121, 60 * 6 + 5


def compact_ref_cols() -> np.ndarray:
    """Reference column (of the 726 flattened 11x11x6 inputs) of each of fc1's compact
    features k < 484 (k = 4 * cell + f <-> channel f + 1; evx_qmlp_pack)."""
    k = np.arange(4 * NCELL)
    return (k >> 2) * 6 + (k & 3) + 1


class evx_qmlp_params(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ["w1", "b1c", "w2", "w2t", "b2", "w3", "b3", "w1o", "stat"]] + \
        [("stat_fs", C.c_int32), ("x3", C.c_int32)] + [(n, C.c_void_p) for n in ["w1l", "w2l", "w2tl", "w1ol"]] + \
        [("stat_x0", C.c_int32), ("stat_nx", C.c_int32), ("stat_xin", C.c_void_p)]


class evx_qmlp_dropout(C.Structure):
    _fields_ = [("seed", C.c_uint32), ("stream", C.c_uint32), ("p", C.c_float), ("row0", C.c_uint32),
                ("mask", C.c_void_p)]


class evx_qmlp_grads(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ["w1", "b1", "w2", "b2", "w3", "b3", "part"]]


class evx_qmlp_fwd_out(C.Structure):
    _fields_ = [("h1", C.c_void_p), ("x", C.c_void_p), ("h2", C.c_void_p), ("q", C.c_void_p),
                ("actions", C.c_void_p), ("epsilon", C.c_float), ("act_seed", C.c_uint64),
                ("act_offset", C.c_uint64), ("perm", C.c_void_p), ("rows_per_env", C.c_int32),
                ("act_ws", C.c_void_p)]


_inited = False


def mlib():
    global _inited
    L = _lib.lib()
    if not _inited:
        L.evx_qmlp_last_error.restype = C.c_char_p
        L.evx_qmlp_pack.argtypes = [C.c_void_p] * 9
        L.evx_qmlp_pack3.argtypes = [C.c_void_p] * 11
        if hasattr(L, "evx_qmlp_stat_x"):  # (absent from older builds loaded through EVX_LIB for A/Bs)
            L.evx_qmlp_stat_x.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(evx_qmlp_params),
                                          C.c_void_p, C.c_void_p]
            L.evx_qmlp_expand_x3.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
        L.evx_qmlp_stat.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(evx_qmlp_params), C.c_void_p,
                                    C.c_void_p]
        L.evx_qmlp_forward.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(evx_qmlp_params),
                                       C.POINTER(evx_qmlp_dropout), C.POINTER(evx_qmlp_fwd_out), C.c_void_p]
        L.evx_qmlp_act.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(evx_qmlp_params),
                                   C.POINTER(evx_qmlp_dropout), C.POINTER(evx_qmlp_fwd_out), C.c_void_p]
        L.evx_qmlp_act64.argtypes = L.evx_qmlp_act.argtypes
        L.evx_qmlp_forward2.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.POINTER(evx_qmlp_params),
                                        C.POINTER(evx_qmlp_dropout), C.POINTER(evx_qmlp_fwd_out), C.c_void_p,
                                        C.POINTER(evx_qmlp_params), C.POINTER(evx_qmlp_dropout),
                                        C.POINTER(evx_qmlp_fwd_out), C.c_void_p]
        L.evx_qmlp_backward_ss.argtypes = [C.POINTER(evx_qmlp_params), C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_float, C.c_void_p, C.c_void_p, C.POINTER(evx_qmlp_grads),
                                           C.c_int32, C.c_void_p, C.c_void_p]
        L.evx_qmlp_td_backward_ss.argtypes = [C.POINTER(evx_qmlp_params), C.c_int32] + [C.c_void_p] * 5 + \
            [C.c_float] + [C.c_void_p] * 6 + [C.c_float, C.c_void_p, C.c_void_p, C.POINTER(evx_qmlp_grads),
                                              C.c_void_p, C.c_void_p]
        L.evx_qmlp_norm_parts.restype = C.c_int32
        L.evx_qmlp_nparams.restype = C.c_int64
        if hasattr(L, "evx_qmlp_act_ws_ints"):  # (absent from older builds loaded through EVX_LIB for A/Bs)
            L.evx_qmlp_act_ws_ints.restype = C.c_int64
            L.evx_qmlp_act_ws_ints.argtypes = [C.c_int32]
        L.evx_qmlp_sumsq_parts.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.evx_qmlp_adam_pack3.argtypes = [C.c_void_p] * 4 + [C.c_float, C.c_void_p] + [C.c_void_p] * 10 + \
            [C.c_int32, C.c_void_p, C.c_void_p]
        L.evx_qmlp_pack_occ3.argtypes = [C.c_void_p] * 4
        L.evx_qmlp_backward_part_floats.restype = C.c_int64
        L.evx_qmlp_backward_part_floats.argtypes = [C.c_int32]
        L.evx_qmlp_backward.argtypes = [C.POINTER(evx_qmlp_params), C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_float, C.c_void_p, C.c_void_p, C.POINTER(evx_qmlp_grads),
                                        C.c_int32, C.c_void_p]
        # grouped nets (evacx.qgroup)
        L.evx_qmlp_act_g.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.POINTER(evx_qmlp_params),
                                     C.POINTER(evx_qmlp_dropout), C.POINTER(evx_qmlp_fwd_out), C.c_void_p]
        L.evx_qmlp_forward2_g.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.POINTER(evx_qmlp_params),
                                          C.POINTER(evx_qmlp_dropout), C.POINTER(evx_qmlp_fwd_out), C.c_void_p,
                                          C.POINTER(evx_qmlp_params), C.POINTER(evx_qmlp_dropout),
                                          C.POINTER(evx_qmlp_fwd_out), C.c_void_p]
        L.evx_qmlp_backward_ss_g.argtypes = [C.POINTER(evx_qmlp_params), C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                                             C.c_void_p, C.c_void_p, C.c_float, C.c_void_p, C.c_void_p,
                                             C.POINTER(evx_qmlp_grads), C.c_void_p, C.c_void_p]
        L.evx_qmlp_adam_pack3_g.argtypes = [C.c_void_p] * 4 + [C.c_float, C.c_void_p] + [C.c_void_p] * 10 + \
            [C.c_int32, C.c_void_p, C.c_int32, C.c_void_p]
        L.evx_qmix_last_error.restype = C.c_char_p
        L.evx_qmix_nparams.restype = C.c_int32
        L.evx_qmix_part_floats.restype = C.c_int64
        L.evx_qmix_part_floats.argtypes = [C.c_int32, C.c_int32]
        L.evx_qmix_loss.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_float,
                                    C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
        _inited = True
    return L


def act_ws_ints(n: int) -> int:
    """int32 elements of the act's workspace for n rows (evx_qmlp_act_ws_ints)."""
    L = mlib()
    return int(L.evx_qmlp_act_ws_ints(int(n))) if hasattr(L, "evx_qmlp_act_ws_ints") else 0


def mcheck(rc, what):
    if rc != 0:
        raise _lib.EvacxError(f"{what} failed ({rc}): {mlib().evx_qmlp_last_error().decode()}")


def _p(t):
    return None if t is None else t.data_ptr()


def _need(what, t, n, per_row):
    """Host-side bounds check before a launch: a kernel indexing past a caller's buffer faults the GPU."""
    if t is not None and t.numel() < n * per_row:
        raise ValueError(f"qmlp {what}: {t.numel()} elements, needs {n} x {per_row}")


class MLPFast:
    """bf16 operand copies of one MLP parameter set (evacx.qnet.FlatParams) + forward.
    x3=True: the f32-accurate mode (hi + lo operand pairs; evx_qmlp_pack3)."""

    # operand buffers: name -> (elements, dtype); x3 adds the lo copies
    @staticmethod
    def buffer_sizes(x3: bool):
        kx = K1X if x3 else K1P
        d = {"w1b": (HID * kx, torch.int16), "w2b": (HID2 * HID, torch.int16), "w2t": (HID * HID2, torch.int16),
             "b1c": (HID, torch.float32), "w1o": (HID * 128, torch.int16)}
        if x3:
            d.update(w1ol=(HID * 128, torch.int16), w1l=(HID * K1P, torch.int16), w2l=(HID2 * HID, torch.int16),
                     w2tl=(HID * HID2, torch.int16))
        return d

    def __init__(self, params, device, x3: bool = False, store=None):
        """store: optional name -> preallocated tensor of buffer_sizes(x3) (evacx.qgroup: every net's
        operands one slice of a [nets][...] array, as the grouped kernels address them)."""
        self.P = params
        self.device = torch.device(device)
        self.x3 = bool(x3)
        self.kx = K1X if self.x3 else K1P  # width of fc1's expanded input (the learner's saved X)
        sizes = self.buffer_sizes(self.x3)

        def buf(name):
            n, dt = sizes[name]
            if store is not None:
                t = store[name]
                if t.numel() != n or t.dtype != dt or not t.is_contiguous():
                    raise ValueError(f"MLPFast store[{name}]: needs {n} contiguous {dt}")
                return t
            return torch.zeros(n, dtype=dt, device=self.device)
        self.w1b = buf("w1b")
        self.w2b = buf("w2b")
        self.w2t = buf("w2t")
        self.b1c = buf("b1c")
        self.w1o = buf("w1o")  # fc1's occupancy columns (act fast path; x3: hi)
        self.w1ol = buf("w1ol") if self.x3 else None  # x3: their lo part
        self.c = evx_qmlp_params(w1=self.w1b.data_ptr(), b1c=self.b1c.data_ptr(), w2=self.w2b.data_ptr(),
                                 w2t=self.w2t.data_ptr(), b2=params["fc2.bias"].data_ptr(),
                                 w3=params["fc3.weight"].data_ptr(), b3=params["fc3.bias"].data_ptr())
        if self.x3:
            self.w1l = buf("w1l")
            self.w2l = buf("w2l")
            self.w2tl = buf("w2tl")
            self.c.x3 = 1
            self.c.w1l, self.c.w2l, self.c.w2tl = self.w1l.data_ptr(), self.w2l.data_ptr(), self.w2tl.data_ptr()
            self.c.w1ol = self.w1ol.data_ptr()
        self._static = None  # (lay_c, centre obs, table) of attach_static
        self._part = None  # split-K scratch of the weight-gradient GEMMs (backward)
        self.repack()

    @property
    def planes(self) -> int:
        """Planes of a split activation buffer (h1, dz2, dz1): 2 in x3 mode (hi, lo)."""
        return 2 if self.x3 else 1

    def repack(self):
        if self.x3:
            mcheck(mlib().evx_qmlp_pack3(self.P["fc1.weight"].data_ptr(), self.P["fc1.bias"].data_ptr(),
                                         self.P["fc2.weight"].data_ptr(), self.w1b.data_ptr(), self.w1l.data_ptr(),
                                         self.b1c.data_ptr(), self.w2b.data_ptr(), self.w2l.data_ptr(),
                                         self.w2t.data_ptr(), self.w2tl.data_ptr(), _stream()), "qmlp_pack3")
            mcheck(mlib().evx_qmlp_pack_occ3(self.P["fc1.weight"].data_ptr(), self.w1o.data_ptr(),
                                             self.w1ol.data_ptr(), _stream()), "qmlp_pack_occ3")
            if self._static is not None:
                self._rebuild_static()
            return
        mcheck(mlib().evx_qmlp_pack(self.P["fc1.weight"].data_ptr(), self.P["fc1.bias"].data_ptr(),
                                    self.P["fc2.weight"].data_ptr(), self.w1b.data_ptr(), self.b1c.data_ptr(),
                                    self.w2b.data_ptr(), self.w2t.data_ptr(), self.w1o.data_ptr(), _stream()),
               "qmlp_pack")
        if self._static is not None:
            self._rebuild_static()

    def adam_step(self, p, g, m, v, max_norm: float, hyper, ss, norm_out=None):
        """clip_grad_norm_ (from the squared-norm partials ss) + Adam on the flat buffers and this
        network's x3 operand repack, one launch (evx_qmlp_adam_pack3); hyper: evacx.qnet.evx_adam."""
        if not self.x3:
            raise ValueError("adam_step: the fused repack writes the x3 operand layout")
        mcheck(mlib().evx_qmlp_adam_pack3(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), float(max_norm),
                                          C.byref(hyper), self.w1b.data_ptr(), self.w1l.data_ptr(),
                                          self.b1c.data_ptr(), self.w2b.data_ptr(), self.w2l.data_ptr(),
                                          self.w2t.data_ptr(), self.w2tl.data_ptr(), self.w1o.data_ptr(),
                                          self.w1ol.data_ptr(), ss.data_ptr(), int(mlib().evx_qmlp_norm_parts()),
                                          _p(norm_out), _stream()),
               "qmlp_adam_pack3")
        if self._static is not None:  # the act table follows the weights
            self._rebuild_static()

    @staticmethod
    def sumsq_parts(g, ss):
        """The squared-norm partials of a flat gradient buffer (evx_qmlp_sumsq_parts)."""
        mcheck(mlib().evx_qmlp_sumsq_parts(g.data_ptr(), ss.data_ptr(), _stream()), "qmlp_sumsq_parts")

    def attach_static(self, lay_c, L: int, W: int, t_max: int, x_range=None):
        """Enable act()'s fast path for observations at fire step >= t_max (the fire has
        stopped spreading): fc1's pre-activation at zero occupancy for every window centre
        of the layout, [nx (W+2)][512] f32 (x3: f32-accurate), rebuilt with every repack and
        every optimizer step (adam_step). x_range = (x0, x1): only centres with x0 <= x <= x1
        (Map.robot_range, envs/map.py:75: a robot never leaves it), default every x.
        The table (like the operand copies) follows the fp32 parameters only through repack() and
        adam_step(): after any other write of the weights (load_state_dict, a broadcast) call
        repack() (Learner.weights_written) -- the act and, at B >= 32768, the learner's online
        forward read fc1 from this table."""
        x0, x1 = (0, L + 1) if x_range is None else (int(x_range[0]), int(x_range[1]))
        if not 0 <= x0 <= x1 <= L + 1:
            raise ValueError("attach_static: x_range must lie in [0, L + 1]")
        nx = x1 - x0 + 1
        cx, cy = np.meshgrid(np.arange(x0, x1 + 1), np.arange(W + 2), indexing="ij")
        ob = np.zeros((nx * (W + 2), 8), np.int32)
        ob[:, 4], ob[:, 5], ob[:, 6] = cx.ravel(), cy.ravel(), t_max
        self._static = (lay_c, torch.from_numpy(ob).to(self.device),
                        torch.empty(nx * (W + 2), HID, dtype=torch.float32, device=self.device))
        # x3: the table rows' fc1 inputs are fixed (every centre at the last fire step, no occupancy):
        # expanded once here, every rebuild reads them (evx_qmlp_stat_x) instead of regenerating them
        self._static_x = None
        if self.x3 and hasattr(mlib(), "evx_qmlp_stat_x"):
            n = self._static[1].shape[0]
            self._static_x = torch.empty(n * K1X, dtype=torch.int16, device=self.device)
            mcheck(mlib().evx_qmlp_expand_x3(C.byref(lay_c), self._static[1].data_ptr(), n,
                                             self._static_x.data_ptr(), _stream()), "qmlp_expand_x3")
        self._rebuild_static()
        self.c.w1o, self.c.stat, self.c.stat_fs = self.w1o.data_ptr(), self._static[2].data_ptr(), int(t_max)
        self.c.stat_x0, self.c.stat_nx = x0, nx
        self.c.stat_xin = None if self._static_x is None else self._static_x.data_ptr()

    def detach_static(self):
        self._static = None
        self._static_x = None
        self.c.w1o = self.c.stat = self.c.stat_xin = None
        self.c.stat_x0 = self.c.stat_nx = 0

    def _rebuild_static(self):
        lay_c, ob, T = self._static
        if getattr(self, "_static_x", None) is not None:
            mcheck(mlib().evx_qmlp_stat_x(C.byref(lay_c), ob.data_ptr(), self._static_x.data_ptr(), ob.shape[0],
                                          C.byref(self.c), T.data_ptr(), _stream()), "qmlp_stat_x")
            return
        self.stat_table(lay_c, ob, ob.shape[0], T)

    def stat_table(self, lay_c, obs: torch.Tensor, n: int, out: torch.Tensor):
        """evx_qmlp_stat: fc1's pre-activation (f32, bias included) of n observations -> out [n][512]."""
        mcheck(mlib().evx_qmlp_stat(C.byref(lay_c), obs.data_ptr(), n, C.byref(self.c), out.data_ptr(), _stream()),
               "qmlp_stat")

    def forward(self, lay_c, obs: torch.Tensor, n: int, h1: torch.Tensor, drop=None, x=None, h2=None, q=None,
                actions=None, epsilon=0.0, act_seed=0, act_offset=0):
        """obs: compact observations (int32 words, 8 per row). drop: (seed, stream, p) or None."""
        _need("forward obs", obs, n, 8)
        _need("forward q", q, n, NACT)
        d = self._drop(drop) if drop else None
        o = evx_qmlp_fwd_out(h1=_p(h1), x=_p(x), h2=_p(h2), q=_p(q), actions=_p(actions), epsilon=float(epsilon),
                             act_seed=act_seed, act_offset=act_offset)
        mcheck(mlib().evx_qmlp_forward(C.byref(lay_c), obs.data_ptr(), n, C.byref(self.c),
                                       C.byref(d) if d is not None else None, C.byref(o), _stream()),
               "qmlp_forward")


    def act(self, lay_c, obs: torch.Tensor, n: int, drop=None, q=None, actions=None, epsilon=0.0, act_seed=0,
            act_offset=0, perm=None, rows_per_env=0, kernel64: bool = False, ws=None):
        """DQNAgent.act in one launch (evx_qmlp_act): Q values and/or epsilon-greedy actions.
        perm (int32 [n / rows_per_env], device; evacx.env.VecEnv.act_perm): the batch visits the
        envs in this order (results stay at their own rows). kernel64: the 64-row kernel only
        (evx_qmlp_act64; the default may take the persistent 128-row kernel, same bits).
        ws: an int32 workspace of act_ws_ints(n) elements (evx_qmlp_fwd_out.act_ws), zeroed once,
        one per act in flight; every act resets its counters."""
        if ws is not None and (ws.dtype != torch.int32 or ws.numel() < act_ws_ints(n) or not ws.is_cuda):
            raise ValueError("qmlp act: ws must be a device int32 tensor of act_ws_ints(n) elements")
        _need("act obs", obs, n, 8)
        _need("act q", q, n, NACT)
        _need("act actions", actions, n, 1)
        # rows_per_env even: dropout row pairs stay together in a tile
        if perm is not None and (rows_per_env <= 0 or rows_per_env % 2
                                 or n % rows_per_env or perm.numel() < n // rows_per_env):
            raise ValueError("qmlp act: perm needs an even rows_per_env dividing n and n / rows_per_env "
                             "entries")
        d = self._drop(drop) if drop else None
        o = evx_qmlp_fwd_out(q=_p(q), actions=_p(actions), epsilon=float(epsilon), act_seed=act_seed,
                             act_offset=act_offset, perm=_p(perm), rows_per_env=int(rows_per_env), act_ws=_p(ws))
        fn = mlib().evx_qmlp_act64 if kernel64 else mlib().evx_qmlp_act
        mcheck(fn(C.byref(lay_c), obs.data_ptr(), n, C.byref(self.c), C.byref(d) if d is not None else None,
                  C.byref(o), _stream()), "qmlp_act")

    @staticmethod
    def _drop(drop):
        """drop: (seed, stream, p[, keep_mask uint8 [n][512] or None[, row0]]) -- an explicit mask
        (the reference's captured torch masks, tests) replaces the hash; row0 (even) keys the
        hash rows by global agent id."""
        m = drop[3] if len(drop) > 3 else None
        row0 = int(drop[4]) if len(drop) > 4 else 0
        return evx_qmlp_dropout(seed=drop[0] & 0xFFFFFFFF, stream=drop[1] & 0xFFFFFFFF, p=drop[2], row0=row0,
                                mask=None if m is None else m.data_ptr())

    @staticmethod
    def _out(h1, x=None, h2=None, q=None):
        return evx_qmlp_fwd_out(h1=_p(h1), x=_p(x), h2=_p(h2), q=_p(q))

    @staticmethod
    def forward_pair(lay_c, n, net0, obs0, drop0, out0: dict, net1, obs1, drop1, out1: dict):
        """Two forwards (e.g. online and target) in one launch pair; out*: h1, x, h2, q tensors."""
        _need("forward_pair obs0", obs0, n, 8)
        _need("forward_pair obs1", obs1, n, 8)
        for o in (out0, out1):
            _need("forward_pair q", o.get("q"), n, NACT)
        d0, d1 = MLPFast._drop(drop0), MLPFast._drop(drop1)
        o0, o1 = MLPFast._out(**out0), MLPFast._out(**out1)
        mcheck(mlib().evx_qmlp_forward2(C.byref(lay_c), n, obs0.data_ptr(), C.byref(net0.c), C.byref(d0), C.byref(o0),
                                        obs1.data_ptr(), C.byref(net1.c), C.byref(d1), C.byref(o1), _stream()),
               "qmlp_forward2")

    def _grads(self, B, grads):
        g = evx_qmlp_grads(**{k: grads[f"fc{k[1]}.{'weight' if k[0] == 'w' else 'bias'}"].data_ptr()
                              for k in ["w1", "b1", "w2", "b2", "w3", "b3"]})
        # every gradient sum through partials added in a fixed order (the same bits on every run)
        nf = int(mlib().evx_qmlp_backward_part_floats(B))
        if self._part is None or self._part.numel() < nf:
            self._part = torch.empty(nf, dtype=torch.float32, device=self.device)
        g.part = self._part.data_ptr()
        return g

    def td_backward(self, B: int, Q, Qt, act, rew, done, gamma: float, loss, x, h1, h2, drop_p: float, dz2, dz1, grads,
                    weights=None, td_abs=None, ss: Optional[torch.Tensor] = None):
        """DQNAgent.learn's TD step + loss.backward() in one (evx_qmlp_td_backward_ss): loss[0] = the
        mean squared TD error, the gradients overwritten; ss (or None) as backward's."""
        pl = self.planes
        for name, t, n in [("x", x, B * self.kx), ("h1", h1, pl * B * HID), ("dz1", dz1, pl * B * HID),
                           ("dz2", dz2, pl * B * HID2), ("h2", h2, B * HID2), ("Q", Q, B * NACT), ("Qt", Qt, B * NACT),
                           ("act", act, B), ("rew", rew, B), ("done", done, B)]:
            if t.numel() < n:
                raise ValueError(f"qmlp td_backward: {name} has {t.numel()} elements, needs {n}")
        if ss is not None:
            _need("td_backward ss", ss, 1, int(mlib().evx_qmlp_norm_parts()))
        g = self._grads(B, grads)
        mcheck(mlib().evx_qmlp_td_backward_ss(C.byref(self.c), B, Q.data_ptr(), Qt.data_ptr(), act.data_ptr(),
                                              rew.data_ptr(), done.data_ptr(), float(gamma), _p(weights),
                                              loss.data_ptr(), _p(td_abs), x.data_ptr(), h1.data_ptr(), h2.data_ptr(),
                                              float(drop_p), dz2.data_ptr(), dz1.data_ptr(), C.byref(g), _p(ss),
                                              _stream()), "qmlp_td_backward_ss")

    def backward(self, B: int, dq: torch.Tensor, x: torch.Tensor, h1: torch.Tensor, h2: torch.Tensor, drop_p: float,
                 dz2: torch.Tensor, dz1: torch.Tensor, grads, zero=True, ss: Optional[torch.Tensor] = None):
        """d loss / d params of the saved forward into `grads` (evacx.qnet.FlatParams).
        Buffer sizes are checked here, before anything is launched: x [B][kx], h1 / dz1
        [planes][B][512], dz2 [planes][B][256]. ss: f32 [>= evx_qmlp_norm_parts()] receives
        clip_grad_norm_'s squared-norm partials of the final gradients (evx_qmlp_backward_ss)."""
        pl = self.planes
        for name, t, n in [("x", x, B * self.kx), ("h1", h1, pl * B * HID), ("dz1", dz1, pl * B * HID),
                           ("dz2", dz2, pl * B * HID2), ("h2", h2, B * HID2), ("dq", dq, B * NACT)]:
            if t.numel() < n:
                raise ValueError(f"qmlp backward: {name} has {t.numel()} elements, needs {n}")
        g = self._grads(B, grads)
        if ss is not None:
            _need("backward ss", ss, 1, int(mlib().evx_qmlp_norm_parts()))
            mcheck(mlib().evx_qmlp_backward_ss(C.byref(self.c), B, dq.data_ptr(), x.data_ptr(), h1.data_ptr(),
                                               h2.data_ptr(), float(drop_p), dz2.data_ptr(), dz1.data_ptr(), C.byref(g),
                                               int(zero), ss.data_ptr(), _stream()), "qmlp_backward_ss")
            return
        mcheck(mlib().evx_qmlp_backward(C.byref(self.c), B, dq.data_ptr(), x.data_ptr(), h1.data_ptr(), h2.data_ptr(),
                                        float(drop_p), dz2.data_ptr(), dz1.data_ptr(), C.byref(g), int(zero),
                                        _stream()), "qmlp_backward")


# ------------------------------------------------------------ host restatements
def _fmix32(h):
    h = np.asarray(h, np.uint64) & 0xFFFFFFFF
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


def dropout_keep(seed: int, stream: int, p: float, rows: int, cols: int = HID, row0: int = 0) -> np.ndarray:
    """The kernels' dropout keep mask [rows][cols] (bool), restated on the host (tests):
    one hash per (row pair, column), low 16 bits for the even row, high for the odd;
    keep iff the 16-bit value >= floor(p * 65536)."""
    seed, stream = seed & 0xFFFFFFFF, stream & 0xFFFFFFFF
    s = int(_fmix32((stream * 0x632BE5AB + 0x9E3779B9) & 0xFFFFFFFF))
    r = np.arange(row0, row0 + rows, dtype=np.uint64)
    pair = r >> 1
    ph = _fmix32(np.uint64(seed ^ s) ^ ((pair * 0x9E3779B1) & 0xFFFFFFFF))
    c = np.arange(cols, dtype=np.uint64)
    ch = (c * 0x85EBCA77 + 0x27D4EB2F) & 0xFFFFFFFF
    h = _fmix32(ph[:, None] ^ ch[None, :])
    half = np.where((r & 1)[:, None] == 1, h >> 16, h & 0xFFFF)
    thresh = max(1, int(p * 65536.0)) if p > 0 else 0
    return half >= thresh
