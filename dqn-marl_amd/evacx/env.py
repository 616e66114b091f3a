"""Device-resident vectorised evacuation environments (host driver of libevacx).

``DeviceLayout`` uploads the static tables of one layout (evacx.layout) to HBM
once; ``VecEnv`` holds E env instances as one structure-of-arrays state in HBM
and steps all of them with one kernel launch (include/evacx.h). Nothing here
computes the environment: it allocates, packs and launches.
"""
from __future__ import annotations

import ctypes as C
import math
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .layout import LayoutSpec, LayoutTables, build_tables

REWARD_DEFAULTS = dict(evac_reward=50.0, death_penalty=200.0, death_acc_penalty=0.5, alive_bonus=1.0)
OBS_WORDS = 8  # sizeof(evx_obs) / 4


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_dev = getattr(torch._C, "_cuda_getDevice", None)


def _stream() -> int:
    """The current HIP stream handle. Called by every launch: the raw C accessors cost ~1 us, where
    torch.cuda.current_stream() builds a Stream object after device / availability checks (~8 us
    of host time each, ~16 per training step -- tools/host_profile.py)."""
    if _raw_stream is not None and _cur_dev is not None:
        return _raw_stream(_cur_dev())
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def pack_xy(x, y) -> np.ndarray:
    x = np.asarray(x, np.int64) & 0xFFFF
    y = np.asarray(y, np.int64) & 0xFFFF
    return (x | (y << 16)).astype(np.uint32).view(np.int32)


def unpack_xy(v) -> np.ndarray:
    u = np.asarray(v).view(np.uint32).astype(np.int64)
    x = (u & 0xFFFF).astype(np.int16).astype(np.int32)
    y = (u >> 16).astype(np.int16).astype(np.int32)
    return np.stack([x, y], -1)


def repel_threshold(repel_range: float) -> int:
    """Smallest integer n with sqrt(n) >= repel_range (so dist < range <=> d2 < n)."""
    if not repel_range > 0:
        return 0
    n = max(0, int(math.ceil(repel_range * repel_range)) - 2)
    while math.sqrt(n) < repel_range:
        n += 1
    return n


# People.MoveTO order (envs/people.py:8-17): direction d moves by (MOVE_DX[d], MOVE_DY[d])
MOVE_DX = [((0x8246 >> (2 * d)) & 3) - 1 for d in range(8)]
MOVE_DY = [((0xA091 >> (2 * d)) & 3) - 1 for d in range(8)]


def neighbour_valid_mask(valid: np.ndarray, L: int, W: int) -> np.ndarray:
    """[G] uint8, bit d set iff Map.Check_Valid(x + dx_d, y + dy_d) (envs/map.py:85-92)."""
    GX, GY = L + 2, W + 2
    v = np.asarray(valid, bool).reshape(GX, GY)
    inner = np.zeros((GX, GY), bool)
    inner[1:L + 1, 1:W + 1] = v[1:L + 1, 1:W + 1]
    pad = np.zeros((GX + 2, GY + 2), bool)
    pad[1:-1, 1:-1] = inner
    m = np.zeros((GX, GY), np.uint8)
    for d in range(8):
        m |= (pad[1 + MOVE_DX[d]:1 + MOVE_DX[d] + GX, 1 + MOVE_DY[d]:1 + MOVE_DY[d] + GY].astype(np.uint8) << d)
    return m.reshape(-1)


def floor_delta5(floor: np.ndarray, L: int, W: int) -> np.ndarray:
    """[G][8] float64: (floor[c] - floor[c + MoveTO[d]]) * 5.0 -- Map.getDeltaP * 5.0 of
    People.find_best_direction (envs/people.py:268,282), evaluated once in IEEE double
    exactly as the reference does per candidate; 0 where the neighbour is off the grid."""
    GX, GY = L + 2, W + 2
    f = np.asarray(floor, np.float64).reshape(GX, GY)
    out = np.zeros((GX, GY, 8), np.float64)
    with np.errstate(invalid="ignore"):  # inf - inf on invalid cells: never a candidate
        _fill_delta5(f, out, GX, GY)
    return out.reshape(-1)


def _fill_delta5(f, out, GX, GY):
    for d in range(8):
        dx, dy = MOVE_DX[d], MOVE_DY[d]
        xs = slice(max(0, -dx), GX - max(0, dx))
        ys = slice(max(0, -dy), GY - max(0, dy))
        xn = slice(max(0, -dx) + dx, GX - max(0, dx) + dx)
        yn = slice(max(0, -dy) + dy, GY - max(0, dy) + dy)
        out[xs, ys, d] = (f[xs, ys] - f[xn, yn]) * 5.0


def bf16_bits(x: np.ndarray) -> np.ndarray:
    """float32 -> bf16 bit patterns, round to nearest even (no NaNs here)."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint32)


def obs_feature_map(tables: LayoutTables) -> np.ndarray:
    """evx_layout.obs_feat: the observation channels of EvacuationEnv._get_state
    (envs/evacuation_env.py:84-120) that do not depend on the people, for every map cell
    of a grid padded by FEAT_PAD on each side and every fire step -- bf16(danger) in bits
    0-15, barrier (!Check_Valid or barrier_list) in bit 16, exit in bit 17 -- exactly as
    obs_expand_kernel evaluates them cell by cell."""
    spec, pad = tables.spec, _lib.FEAT_PAD
    L, W = spec.L, spec.W
    mx = np.arange(-pad, L + 2 + pad)[:, None]
    my = np.arange(-pad, W + 2 + pad)[None, :]
    inb = (mx >= 0) & (mx <= L + 1) & (my >= 0) & (my <= W + 1)
    cx, cy = np.clip(mx, 0, L + 1), np.clip(my, 0, W + 1)
    valid_t = np.asarray(tables.valid, bool)[cx, cy]
    barrier_t = np.asarray(tables.barrier, bool)[cx, cy]
    valid = (mx >= 1) & (mx <= L) & (my >= 1) & (my <= W) & valid_t
    bar = ~valid | (inb & barrier_t)
    ext = (mx == spec.exit[0]) & (my == spec.exit[1])
    static = (bar.astype(np.uint32) << 16) | (ext.astype(np.uint32) << 17)
    do32 = np.asarray(tables.danger_o, np.float64).astype(np.float32)
    T, OX, OY = do32.shape
    ti, tj = mx - tables.obs_origin[0], my - tables.obs_origin[1]
    inside = (ti >= 0) & (ti < OX) & (tj >= 0) & (tj < OY)
    dg = np.zeros((T,) + inside.shape, np.float32)
    dg[:, inside] = do32[:, np.broadcast_to(ti, inside.shape)[inside], np.broadcast_to(tj, inside.shape)[inside]]
    return (bf16_bits(dg) | static[None]).astype(np.uint32)


def obs_feature_lo(tables: LayoutTables) -> np.ndarray:
    """evx_layout.obs_feat_lo: the bf16 residual of obs_feat's danger feature,
    bf16(d - bf16(d)) of d = float32(danger), same indexing: with it the f32-accurate MLP
    kernels carry the danger input as hi + lo (16 significant bits)."""
    hi_bits = obs_feature_map(tables) & 0xFFFF
    hi = (hi_bits << 16).astype(np.uint32).view(np.float32)
    spec, pad = tables.spec, _lib.FEAT_PAD
    L, W = spec.L, spec.W
    mx = np.arange(-pad, L + 2 + pad)[:, None]
    my = np.arange(-pad, W + 2 + pad)[None, :]
    do32 = np.asarray(tables.danger_o, np.float64).astype(np.float32)
    T, OX, OY = do32.shape
    ti, tj = mx - tables.obs_origin[0], my - tables.obs_origin[1]
    inside = (ti >= 0) & (ti < OX) & (tj >= 0) & (tj < OY)
    dg = np.zeros((T,) + inside.shape, np.float32)
    dg[:, inside] = do32[:, np.broadcast_to(ti, inside.shape)[inside], np.broadcast_to(tj, inside.shape)[inside]]
    return bf16_bits(dg - hi).astype(np.uint16)


class DeviceLayout:
    """Static tables of one layout in HBM + the evx_layout descriptor."""

    def __init__(self, tables: LayoutTables, P: int, device="cuda", repel_k=-20.0, repel_range=5.0,
                 **reward):
        spec = tables.spec
        self.spec, self.tables, self.P, self.R = spec, tables, int(P), spec.R
        self.device = torch.device(device)
        self.GX, self.GY = spec.L + 2, spec.W + 2
        self.G = self.GX * self.GY
        self.RW = (self.G + 31) // 32
        d = self.device
        cell = (tables.valid.astype(np.uint8) | (tables.exit_mask.astype(np.uint8) << 1)
                | (tables.barrier.astype(np.uint8) << 2)).reshape(-1)
        vb = np.zeros(self.RW * 32, np.uint8)
        vb[:self.G] = tables.valid.reshape(-1)
        bits = np.packbits(vb.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").astype(np.uint32).reshape(-1)
        self.t = dict(
            floor=torch.from_numpy(np.ascontiguousarray(tables.floor.reshape(-1))).to(d),
            cellinfo=torch.from_numpy(cell).to(d),
            valid_bits=torch.from_numpy(bits.view(np.int32)).to(d),
            danger_p=torch.from_numpy(np.ascontiguousarray(tables.danger_p.reshape(-1))).to(d),
            danger_o=torch.from_numpy(np.ascontiguousarray(tables.danger_o.reshape(-1))).to(d),
            robot_init=torch.from_numpy(np.asarray(spec.robot_init, np.int32).reshape(-1)).to(d),
        )
        self.t["nbr_valid"] = torch.from_numpy(neighbour_valid_mask(tables.valid, spec.L, spec.W)).to(d)
        self.t["floor_d5"] = torch.from_numpy(floor_delta5(tables.floor, spec.L, spec.W)).to(d)
        self.t["danger_o32"] = self.t["danger_o"].to(torch.float32)
        self.t["obs_feat"] = torch.from_numpy(obs_feature_map(tables).view(np.int32).reshape(-1)).to(d)
        self.t["obs_feat_lo"] = torch.from_numpy(obs_feature_lo(tables).view(np.int16).reshape(-1)).to(d)
        T = tables.danger_p.shape[0] - 1
        OX, OY = tables.danger_o.shape[1:]
        self.c = _lib.evx_layout(
            L=spec.L, W=spec.W, P=self.P, R=self.R, t_max=T, ox0=tables.obs_origin[0], oy0=tables.obs_origin[1],
            OX=OX, OY=OY, exit_x=spec.exit[0], exit_y=spec.exit[1], rx_lo=spec.robot_range[0],
            rx_hi=spec.robot_range[1], reset_view_x=spec.reset_view[0], reset_view_y=spec.reset_view[1],
            reset_robots=int(bool(spec.reset_robots)), flags=0)
        for k, v in self.t.items():
            setattr(self.c, k, v.data_ptr())
        self.set_params(repel_k=repel_k, repel_range=repel_range, **dict(REWARD_DEFAULTS, **reward))

    def set_params(self, **kw):
        """Runtime-mutable coefficients (the reference's class attributes)."""
        for k, v in kw.items():
            if k == "repel_range":
                self.c.repel_range = float(v)
                self.c.repel_d2 = repel_threshold(float(v))
            else:
                setattr(self.c, k, float(v))

    @classmethod
    def from_spec(cls, spec: LayoutSpec, P: int, device="cuda", **kw):
        return cls(build_tables(spec), P, device, **kw)


class LayoutSet:
    """Several layouts of one size for per-env layouts: every env of a
    VecEnv picks one (``VecEnv(..., layout_of=...)``); the env kernels read the env's
    entry of a device array of evx_layout descriptors (evx_layout.layout_set), and the
    observation readers the layout recorded in each evx_obs. Same L, W, P, R, fire steps
    and observation window for all (the LDS and scratch sizes follow from those)."""

    def __init__(self, layouts: Sequence["DeviceLayout"]):
        if not layouts:
            raise ValueError("LayoutSet: no layouts")
        l0 = layouts[0]
        for l in layouts:
            same = (l.spec.L, l.spec.W, l.P, l.R, l.c.t_max, l.c.OX, l.c.OY, l.c.ox0, l.c.oy0) == \
                   (l0.spec.L, l0.spec.W, l0.P, l0.R, l0.c.t_max, l0.c.OX, l0.c.OY, l0.c.ox0, l0.c.oy0)
            if not same:
                raise ValueError("LayoutSet: layouts must share L, W, P, R, fire steps and the observation window")
        self.layouts = list(layouts)
        self.spec, self.tables, self.P, self.R, self.device = l0.spec, l0.tables, l0.P, l0.R, l0.device
        self.GX, self.GY, self.G, self.RW, self.t = l0.GX, l0.GY, l0.G, l0.RW, l0.t
        self.c = _lib.evx_layout.from_buffer_copy(l0.c)
        self._upload()

    def _upload(self):
        raw = torch.frombuffer(bytearray(b"".join(bytes(l.c) for l in self.layouts)), dtype=torch.uint8)
        feats = torch.tensor([l.c.obs_feat for l in self.layouts], dtype=torch.int64)
        feats_lo = torch.tensor([l.c.obs_feat_lo for l in self.layouts], dtype=torch.int64)
        if getattr(self, "_set", None) is None:
            self._set = raw.to(self.device)
            self._feats = feats.to(self.device)
            self._feats_lo = feats_lo.to(self.device)
        else:
            # set_params: new coefficients go into the SAME device buffers. Kernels queued on other
            # streams (a trainer's env / act streams) may still read the old ones, so the device is
            # drained first: no launch ever sees a mix of old and new coefficients (set_params is a
            # rare host call -- the reference's class attributes -- not part of a step)
            torch.cuda.synchronize(self.device)
            self._set.copy_(raw, non_blocking=False)
            self._feats.copy_(feats)
            self._feats_lo.copy_(feats_lo)
        for name, _ in _lib.evx_layout._fields_:  # the set's own descriptor: layout 0's sizes and coefficients
            if name not in ("layout_set", "obs_feats", "obs_feats_lo"):
                setattr(self.c, name, getattr(self.layouts[0].c, name))
        self.c.layout_set = self._set.data_ptr()
        self.c.obs_feats = self._feats.data_ptr()
        self.c.obs_feats_lo = self._feats_lo.data_ptr()

    def set_params(self, **kw):
        """Runtime-mutable coefficients, for every layout of the set."""
        for l in self.layouts:
            l.set_params(**kw)
        self._upload()

    def __len__(self):
        return len(self.layouts)


def _perm_ws(E: int, device) -> torch.Tensor:
    n = int(_lib.lib().evx_perm_ws_bytes(E))
    return torch.zeros(max(n, 1), dtype=torch.uint8, device=device)


class VecEnv:
    """E env instances of one layout (or of a LayoutSet, one layout per env), state
    resident in HBM (SoA, env-major)."""

    def __init__(self, layout, E: int, thmap: bool = False, obs_buffers: int = 1,
                 layout_of: Optional[Sequence[int]] = None):
        """obs_buffers=2: every step writes its observations into the other of two
        buffers, so the previous step's stay readable (``obs_prev``) without a copy.
        layout: a DeviceLayout, or a LayoutSet with ``layout_of`` = each env's layout."""
        self.lay = layout
        self.E = int(E)
        self.layout_idx = None
        if isinstance(layout, LayoutSet):
            if layout_of is None or len(layout_of) != E:
                raise ValueError("VecEnv over a LayoutSet needs layout_of (one layout index per env)")
            li = np.asarray(layout_of, np.int32)
            if li.min() < 0 or li.max() >= len(layout):
                raise ValueError("layout_of: index out of the set")
            self.layout_idx = torch.from_numpy(li).to(layout.device)
        elif layout_of is not None:
            raise ValueError("layout_of needs a LayoutSet")
        P, R, d = layout.P, layout.R, layout.device
        i32 = dict(dtype=torch.int32, device=d)
        f64 = dict(dtype=torch.float64, device=d)
        self.pk = torch.zeros(E * P, **i32)
        self.health = torch.zeros(E * P, **f64)
        self.acc = torch.zeros(E * P, **f64)
        self.rmap = torch.zeros(E * layout.RW, **i32)
        self.thmap = torch.zeros(E * layout.G, **i32) if thmap else None
        specs = [layout.spec] * E if self.layout_idx is None else \
            [layout.layouts[i].spec for i in self.layout_idx.cpu().tolist()]
        self.robots = torch.from_numpy(np.concatenate(
            [pack_xy([p[0] for p in s.robot_init], [p[1] for p in s.robot_init]) for s in specs])).to(d)
        self.view = torch.from_numpy(np.array([pack_xy(*s.reset_view) for s in specs]).astype(np.int32).reshape(E)).to(d)
        self.scal = torch.zeros(E * 4, **i32)
        self.py_mt = torch.zeros(E * 625, **i32)
        self.np_mt = torch.zeros(E * 625, **i32)
        sw = int(_lib.lib().evx_step_scratch_words(C.byref(layout.c)))
        if sw < 0:
            raise _lib.EvacxError(_lib.lib().evx_last_error().decode())
        self.scratch = torch.zeros(E * sw, **i32)
        # dispatch order (evx_env_order), scheduling only; order[E] = envs whose rows
        # phase runs on a whole workgroup (0: none). Two buffers: compute_order(ahead=True)
        # fills the one the step after the next reads while the next step reads the other.
        self._orders = [torch.cat([torch.arange(E, **i32), torch.zeros(1, **i32)]) for _ in range(2)]
        self._ord = 0
        self._order_ahead = False
        # outputs
        self.reward = torch.zeros(E, **f64)
        self.done = torch.zeros(E, dtype=torch.uint8, device=d)
        self.counts = torch.zeros(E * 2, **i32)
        assert obs_buffers in (1, 2)
        self._obs = [torch.zeros(E * R * OBS_WORDS, **i32) for _ in range(obs_buffers)]
        self._ob = 0
        self.err = torch.zeros(1, **i32)
        # every env's class byte for the scheduling permutations (evx_env_orders): written by the step
        # and reset kernels; split parts view their envs' slice of it
        self.perm_ws = _perm_ws(E, d)
        self.c = _lib.evx_state(E=E, pk=_ptr(self.pk), health=_ptr(self.health), acc=_ptr(self.acc),
                                rmap=_ptr(self.rmap), thmap=_ptr(self.thmap), robots=_ptr(self.robots),
                                view=_ptr(self.view), scal=_ptr(self.scal), py_mt=_ptr(self.py_mt),
                                np_mt=_ptr(self.np_mt), scratch=_ptr(self.scratch), order=_ptr(self.order),
                                layout_idx=_ptr(self.layout_idx), perm_ws=_ptr(self.perm_ws))
        self.obs_term: Optional[torch.Tensor] = None
        self._parts: List["VecEnv"] = []
        self.out = _lib.evx_step_out(reward=_ptr(self.reward), done=_ptr(self.done), counts=_ptr(self.counts),
                                     obs=_ptr(self.obs), err=_ptr(self.err))

    def split(self, G: int) -> List["VecEnv"]:
        """G VecEnvs over consecutive E/G envs each, sharing this one's storage: they step
        independently (e.g. on their own streams, so one part's launch tail overlaps the
        next part's work), while this object still reads and resets all E envs (its step
        steps every part). The parts must step together: each flips its observation
        buffers once per step."""
        if G < 2 or self.E % G:
            raise ValueError("split: E must be a multiple of G >= 2")
        if self.obs_term is None:
            self.obs_term = torch.zeros_like(self._obs[0])
        n, lay = self.E // G, self.lay
        P, R, RW, GG = lay.P, lay.R, lay.RW, lay.G
        sw = self.scratch.numel() // self.E
        i32 = dict(dtype=torch.int32, device=lay.device)
        parts = []
        for g in range(G):
            lo = g * n

            def cut(t, k):
                return None if t is None else t[lo * k:(lo + n) * k]
            p = VecEnv.__new__(VecEnv)
            p.lay, p.E, p._parts = lay, n, []
            p.pk, p.health, p.acc = cut(self.pk, P), cut(self.health, P), cut(self.acc, P)
            p.rmap, p.thmap = cut(self.rmap, RW), cut(self.thmap, GG)
            p.robots, p.view, p.scal = cut(self.robots, R), cut(self.view, 1), cut(self.scal, 4)
            p.py_mt, p.np_mt, p.scratch = cut(self.py_mt, 625), cut(self.np_mt, 625), cut(self.scratch, sw)
            p._orders = [torch.cat([torch.arange(n, **i32), torch.zeros(1, **i32)]) for _ in range(2)]
            p._ord, p._order_ahead = 0, False
            p.reward, p.done, p.counts = cut(self.reward, 1), cut(self.done, 1), cut(self.counts, 2)
            p._obs = [cut(b, R * OBS_WORDS) for b in self._obs]
            p._ob = self._ob
            p.err = self.err
            p.obs_term = cut(self.obs_term, R * OBS_WORDS)
            p.perm_ws = self.perm_ws[lo:lo + n]
            p.c = _lib.evx_state(E=n, pk=_ptr(p.pk), health=_ptr(p.health), acc=_ptr(p.acc), rmap=_ptr(p.rmap),
                                 thmap=_ptr(p.thmap), robots=_ptr(p.robots), view=_ptr(p.view), scal=_ptr(p.scal),
                                 py_mt=_ptr(p.py_mt), np_mt=_ptr(p.np_mt), scratch=_ptr(p.scratch),
                                 order=_ptr(p.order), layout_idx=_ptr(cut(self.layout_idx, 1)),
                                 perm_ws=_ptr(p.perm_ws))
            p.layout_idx = cut(self.layout_idx, 1)
            p.out = _lib.evx_step_out(reward=_ptr(p.reward), done=_ptr(p.done), counts=_ptr(p.counts),
                                      obs=_ptr(p.obs), err=_ptr(p.err))
            parts.append(p)
        self._parts = parts
        return parts

    @property
    def obs(self) -> torch.Tensor:
        """Compact observations of the current state (int32 words, OBS_WORDS per robot)."""
        return self._obs[self._parts[0]._ob if self._parts else self._ob]

    @property
    def obs_prev(self) -> torch.Tensor:
        """With obs_buffers=2: the observations before the last step (until the next one)."""
        return self._obs[(self._parts[0]._ob if self._parts else self._ob) ^ 1]

    @property
    def order(self) -> torch.Tensor:
        """The dispatch order the next step reads ([E] env ids + heavy count)."""
        return self._orders[self._ord]

    # -------------------------------------------------------------- seeding
    def seed(self, seeds: Sequence[int]):
        """random.seed(s) / numpy.random.seed(s) per env (host MT19937 init)."""
        s = np.ascontiguousarray(np.asarray(seeds, np.int64) % (1 << 32), np.uint32)
        assert s.shape == (self.E,)
        py = np.zeros((self.E, 625), np.uint32)
        nps = np.zeros((self.E, 625), np.uint32)
        _lib.check(_lib.lib().evx_seed_host(s.ctypes.data, self.E, py.ctypes.data, nps.ctypes.data), "seed")
        self.set_rng(py, nps)

    def set_rng(self, py_states: np.ndarray, np_states: np.ndarray, env_ids=None):
        py = torch.from_numpy(np.ascontiguousarray(py_states, np.uint32).view(np.int32).reshape(-1, 625))
        nps = torch.from_numpy(np.ascontiguousarray(np_states, np.uint32).view(np.int32).reshape(-1, 625))
        if env_ids is None:
            self.py_mt.copy_(py.reshape(-1))
            self.np_mt.copy_(nps.reshape(-1))
        else:
            self.py_mt.view(self.E, 625)[env_ids] = py.to(self.py_mt.device)
            self.np_mt.view(self.E, 625)[env_ids] = nps.to(self.np_mt.device)

    def get_rng(self):
        return (self.py_mt.view(self.E, 625).cpu().numpy().view(np.uint32),
                self.np_mt.view(self.E, 625).cpu().numpy().view(np.uint32))

    # ---------------------------------------------------------------- steps
    def reset(self, mask: Optional[torch.Tensor] = None):
        m = None if mask is None else mask.to(torch.uint8).contiguous()
        _lib.check(_lib.lib().evx_env_reset(C.byref(self.lay.c), C.byref(self.c), _ptr(m), _ptr(self.obs),
                                            _ptr(self.err), _stream()), "evx_env_reset")

    def act_perm(self, out: torch.Tensor) -> torch.Tensor:
        """Env visiting order for the act (evx_act_perm): the envs whose fire has reached the
        layout's last step first (the x3 act's table path), then the rest, each in env order."""
        if out.numel() < self.E or out.dtype != torch.int32:
            raise ValueError("act_perm: out must be int32 with >= E entries")
        _lib.check(_lib.lib().evx_act_perm(C.byref(self.lay.c), C.byref(self.c), out.data_ptr(), _stream()),
                   "evx_act_perm")
        return out

    def compute_orders(self, perm: Optional[torch.Tensor] = None):
        """The next step's dispatch order and (perm, int32 [>= E]) the next act's env order in one
        launch (evx_env_orders) from the class bytes the last step / reset wrote. Scheduling only."""
        if self._parts:
            raise ValueError("compute_orders: order each part")
        if perm is not None and (perm.numel() < self.E or perm.dtype != torch.int32):
            raise ValueError("compute_orders: perm must be int32 with >= E entries")
        _lib.check(_lib.lib().evx_env_orders(C.byref(self.lay.c), C.byref(self.c), _ptr(perm), _stream()),
                   "evx_env_orders")

    def refresh_classes(self):
        """Rewrite the class bytes from the state words (after writing scal from the host)."""
        _lib.check(_lib.lib().evx_env_classes(C.byref(self.lay.c), C.byref(self.c), _stream()), "evx_env_classes")

    def compute_order(self, force: bool = False, ahead: bool = False):
        """Dispatch order of the next step: heavy env-steps first, the heaviest with a
        whole workgroup each (scheduling only; the results do not depend on it). Small
        batches keep the identity order unless forced (tests). ahead=True: fill the other
        order buffer, for the step after the next one, from the state as it is when the
        kernel runs (it may overlap the next step, which reads the current buffer).

        The default form ranks the class bytes the last step / reset wrote (evx_state.perm_ws),
        reading each byte more than once, so it must not overlap a step or reset of these envs.
        ahead=True therefore clears perm_ws in its copy of the state: evx_env_order then takes the
        one-workgroup kernel, which reads every env's counters from the state words ONCE into LDS
        and so yields a permutation even while a step rewrites them. After writing evx_state.scal
        from the host, call refresh_classes() before the next compute_order() / compute_orders()."""
        if self._parts:
            for p in self._parts:
                p.compute_order(force=force, ahead=ahead)
            return
        if self.E < 256 and not force:
            return
        c = self.c
        if ahead:
            c = _lib.evx_state.from_buffer_copy(self.c)
            c.order = _ptr(self._orders[self._ord ^ 1])
            c.perm_ws = None  # one read per env (env_order_kernel's LDS snapshot), see above
            self._order_ahead = True
        _lib.check(_lib.lib().evx_env_order(C.byref(self.lay.c), C.byref(c), _stream()), "evx_env_order")

    def step(self, actions: torch.Tensor, order: bool = True, auto_reset: bool = False, part: int = 0):
        """order=False: the caller already ran compute_order() for this state (see
        evacx.trainer). auto_reset: envs that finish are reset inside the same launch
        (evx_env_reset semantics); their terminal observations land in self.obs_term
        and self.obs holds the post-reset ones (self.done still flags them).
        part: 0 = one launch; 1 then 2 = the heavy envs of the dispatch order, then the
        rest (evx_env_step_part; the two launches may run on different streams, part 1
        issued first: it flips the observation buffer and computes the order)."""
        a = actions.to(torch.int32).contiguous()
        assert a.numel() == self.E * self.lay.R
        if self._parts:  # split: every part steps its envs (same stream here)
            k = self._parts[0].E * self.lay.R
            for i, p in enumerate(self._parts):
                p.step(a[i * k:(i + 1) * k], order=order, auto_reset=auto_reset)
            return
        if part != 2:
            if order:
                self.compute_order()
            if len(self._obs) == 2:  # write into the other buffer: the current one becomes obs_prev
                self._ob ^= 1
                self.out.obs = _ptr(self._obs[self._ob])
            if auto_reset and self.obs_term is None:
                self.obs_term = torch.zeros_like(self.obs)
            self.out.obs_term = self.obs_term.data_ptr() if auto_reset else None
        if part == 0:
            _lib.check(_lib.lib().evx_env_step(C.byref(self.lay.c), C.byref(self.c), a.data_ptr(), C.byref(self.out),
                                               _stream()), "evx_env_step")
        else:
            _lib.check(_lib.lib().evx_env_step_part(C.byref(self.lay.c), C.byref(self.c), a.data_ptr(),
                                                    C.byref(self.out), int(part), _stream()), "evx_env_step_part")
            if part == 1:
                return
        if self._order_ahead:  # the order computed ahead is the one the following step reads
            self._ord ^= 1
            self.c.order = _ptr(self._orders[self._ord])
            self._order_ahead = False

    def expand_obs(self, dtype=torch.float32, obs: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Reference-layout observation tensor [E, R, 11, 11, 6]."""
        ob = self.obs if obs is None else obs
        n = ob.numel() // OBS_WORDS
        out = torch.empty((n, 11, 11, 6), dtype=dtype, device=ob.device)
        fn = _lib.lib().evx_obs_expand_f32 if dtype == torch.float32 else _lib.lib().evx_obs_expand_f64
        assert dtype in (torch.float32, torch.float64)
        _lib.check(fn(C.byref(self.lay.c), ob.data_ptr(), n, out.data_ptr(), _stream()), "evx_obs_expand")
        return out.view(-1, self.lay.R, 11, 11, 6)

    def check_err(self):
        v = int(self.err.item())
        if v:
            raise _lib.EvacxError(f"device error word {v}")

    # ----------------------------------------------------- host inspection
    def host_states(self, ids) -> list:
        """host_state of several envs with one device-to-host copy per field (tests)."""
        lay = self.lay
        P, R = lay.P, lay.R
        idx = torch.as_tensor(list(ids), dtype=torch.long, device=self.pk.device)
        pk = self.pk.view(self.E, P)[idx].cpu().numpy().view(np.uint32)
        health = self.health.view(self.E, P)[idx].cpu().numpy()
        acc = self.acc.view(self.E, P)[idx].cpu().numpy()
        bits = self.rmap.view(self.E, lay.RW)[idx].cpu().numpy().view(np.uint32)
        robots = self.robots.view(self.E, R)[idx].cpu().numpy()
        view = self.view[idx].cpu().numpy()
        scal = self.scal.view(self.E, 4)[idx].cpu().numpy()
        py = self.py_mt.view(self.E, 625)[idx].cpu().numpy().view(np.uint32)
        nps = self.np_mt.view(self.E, 625)[idx].cpu().numpy().view(np.uint32)
        th = None if self.thmap is None else self.thmap.view(self.E, lay.GX, lay.GY)[idx].cpu().numpy()
        out = []
        for j in range(len(idx)):
            rm = ((bits[j][:, None] >> np.arange(32, dtype=np.uint32)[None, :]) & 1).astype(np.uint8).reshape(-1)
            out.append(dict(pos=np.stack([pk[j] & 0xFFF, (pk[j] >> 12) & 0xFFF], -1).astype(np.int32),
                            flags=((pk[j] >> 24) & 3).astype(np.uint8), health=health[j], acc=acc[j],
                            rmap=rm[:lay.G].reshape(lay.GX, lay.GY), robots=unpack_xy(robots[j]),
                            view=unpack_xy(view[j:j + 1])[0], scal=scal[j], py_mt=py[j], np_mt=nps[j],
                            thmap=None if th is None else th[j]))
        return out

    def host_state(self, e: int) -> dict:
        """One env's state in the oracle's representation (tests / drop-in)."""
        lay = self.lay
        P, R = lay.P, lay.R
        pk = self.pk.view(self.E, P)[e].cpu().numpy().view(np.uint32)
        pos = np.stack([pk & 0xFFF, (pk >> 12) & 0xFFF], -1).astype(np.int32)
        flags = ((pk >> 24) & 3).astype(np.uint8)
        bits = self.rmap.view(self.E, lay.RW)[e].cpu().numpy().view(np.uint32)
        rm = ((bits[:, None] >> np.arange(32, dtype=np.uint32)[None, :]) & 1).astype(np.uint8).reshape(-1)
        out = dict(pos=pos, flags=flags,
                   health=self.health.view(self.E, P)[e].cpu().numpy(),
                   acc=self.acc.view(self.E, P)[e].cpu().numpy(),
                   rmap=rm[:lay.G].reshape(lay.GX, lay.GY),
                   robots=unpack_xy(self.robots.view(self.E, R)[e].cpu().numpy()),
                   view=unpack_xy(self.view[e:e + 1].cpu().numpy())[0],
                   scal=self.scal.view(self.E, 4)[e].cpu().numpy(),
                   py_mt=self.py_mt.view(self.E, 625)[e].cpu().numpy().view(np.uint32),
                   np_mt=self.np_mt.view(self.E, 625)[e].cpu().numpy().view(np.uint32))
        out["thmap"] = None if self.thmap is None else self.thmap.view(self.E, lay.GX, lay.GY)[e].cpu().numpy()
        return out
