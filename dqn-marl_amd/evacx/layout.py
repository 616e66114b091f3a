"""Static layout tables for the evacuation cellular automaton (host precompute).

Everything here runs once per layout on the host, with numpy, and the result is
uploaded to HBM where every env instance of that layout shares it read-only:

* ``floor``     -- the static floor field ``Map.space`` after ``Map.Init_Potential``
                   (``envs/map.py:127-148``): 8-neighbour Dijkstra from the exit plus
                   ``200 * danger(t=0)**2``; walls, barriers, unreachable cells = inf.
* ``valid``     -- ``Map.Check_Valid`` per padded cell (``envs/map.py:85-92``).
* ``exit_mask`` -- ``Map.checkSavefy`` at the cell centre (``envs/map.py:93-113``).
* ``barrier``   -- membership in ``Map.barrier_list`` (``envs/map.py:43-73``).
* ``danger_p``  -- ``FireSpreadModel.get_max_danger`` of the map's fire model at
                   person positions ``(x+.5, y+.5)`` for every fire step 0..max_steps
                   (``envs/fire_model.py:69-188``; used by ``People.run``).
* ``danger_o``  -- the same for the env's fire model at integer observation
                   coordinates, over the padded grid widened by the 5-cell
                   observation half-window (``envs/evacuation_env.py:106``).

The fire model is deterministic in (step, position) but runs through
``numpy.exp``, so the tables are produced here by numpy exactly as the
reference does it and never recomputed on the device.
"""
from __future__ import annotations

import dataclasses
import heapq
from typing import List, Optional, Sequence, Tuple

import numpy as np

OBS_HALF = 5

# MoveTO (envs/map.py:11-19)
MOVE_DX = (1, 0, -1, 0, 1, -1, -1, 1)
MOVE_DY = (0, -1, 0, 1, -1, -1, 1, 1)

# ProgressiveFireModel additional sources (envs/fire_model.py:45-51)
REF_ADDITIONAL = (
    {"center": (25, 20), "size": (5, 5), "intensity": 0.8},
    {"center": (13, 18), "size": (5, 5), "intensity": 0.8},
    {"center": (20, 10), "size": (4, 4), "intensity": 0.7},
    {"center": (14, 22), "size": (4, 4), "intensity": 0.6},
    {"center": (26, 14), "size": (3, 3), "intensity": 0.5},
)


@dataclasses.dataclass
class LayoutSpec:
    """Geometry + fire schedule of one evacuation layout.

    Defaults reproduce the reference layout of ``EvacuationEnv.__init__``
    (``envs/evacuation_env.py:21-59``) and ``Map.__init__`` (``envs/map.py:38-79``).
    """
    L: int = 36
    W: int = 30
    exit: Tuple[int, int] = (36, 15)
    barriers: Sequence[Tuple[Tuple[int, int], Tuple[int, int]]] = (((18, 14), (20, 16)),)
    # env.fire_model sources (obs channel 2); None -> the reference's (19,15) 2x2
    obs_fire: Optional[Sequence[dict]] = None
    additional_fire: Sequence[dict] = REF_ADDITIONAL
    fire_max_steps: int = 180
    base_radius: float = 5.0
    max_radius: float = 20.0
    min_danger: float = 0.05
    robot_range: Tuple[int, int] = (15, 30)
    reset_view: Tuple[int, int] = (15, 15)
    robot_init: Sequence[Tuple[int, int]] = ((15, 15),)
    reset_robots: bool = False

    @property
    def R(self) -> int:
        return len(self.robot_init)

    def map_fire(self) -> List[dict]:
        """Map.fire_model sources: one 2x2 FireSource per barrier (envs/map.py:58-65)."""
        return [{"center": ((A[0] + B[0]) / 2, (A[1] + B[1]) / 2), "size": (2, 2), "intensity": 0.4}
                for (A, B) in _norm_barriers(self.barriers)]

    def env_fire(self) -> List[dict]:
        if self.obs_fire is None:
            return [{"center": (19, 15), "size": (2, 2), "intensity": 0.4}]
        return [dict(s) for s in self.obs_fire]


def reference_single() -> LayoutSpec:
    """EvacuationEnv defaults (configs/dqn.yaml env section)."""
    return LayoutSpec()


def reference_multi(robot_init=((10, 15), (20, 15)), **kw) -> LayoutSpec:
    """EvacuationEnvMulti: robots at (10,15),(20,15), re-placed on reset."""
    ri = tuple(tuple(p) for p in robot_init)
    return LayoutSpec(robot_init=ri, reset_view=ri[0], reset_robots=True, **kw)


def reference_scaled_multi(L, W, R) -> LayoutSpec:
    """The reference's hard-coded geometry at a larger grid (used by the g64/g128 fixtures)."""
    init = tuple((15 + (i * 15) // max(R - 1, 1), 4 + (i * (W - 8)) // max(R - 1, 1)) for i in range(R))
    return reference_multi(robot_init=init, L=L, W=W, exit=(L, W // 2))


def synthetic(L: int, W: int, R: int) -> LayoutSpec:
    """Synthetic benchmark layout: the reference geometry scaled by
    (L/36, W/30) -- exit at (L, W/2), one 3x3 barrier, fire centres scaled, robot
    x-range (15/36 L, 30/36 L); R robots spread over their range."""
    sx, sy = L / 36.0, W / 30.0
    bx, by = int(round(18 * sx)), int(round(14 * sy))
    barriers = (((bx, by), (bx + 2, by + 2)),)
    fc = (bx + 1, by + 1)
    add = tuple({"center": (int(round(s["center"][0] * sx)), int(round(s["center"][1] * sy))),
                 "size": s["size"], "intensity": s["intensity"]} for s in REF_ADDITIONAL)
    rlo, rhi = int(round(15 / 36 * L)), int(round(30 / 36 * L))
    init = []
    for i in range(R):
        x = rlo + (i * (rhi - rlo)) // max(R - 1, 1)
        y = 2 + (i * (W - 4)) // max(R - 1, 1)
        if bx <= x <= bx + 2 and by <= y <= by + 2:
            y = by + 3
        init.append((x, y))
    return LayoutSpec(L=L, W=W, exit=(L, W // 2), barriers=barriers,
                      obs_fire=({"center": fc, "size": (2, 2), "intensity": 0.4},),
                      additional_fire=add, robot_range=(rlo, rhi), reset_view=init[0],
                      robot_init=tuple(init), reset_robots=True)


def random_layout(L: int, W: int, R: int, seed: int, n_barriers: int = 4) -> LayoutSpec:
    """A randomised variant of synthetic(L, W, R) for per-env layouts:
    n_barriers rectangles (2..L/12 x 2..W/12 cells) away from the robots' start cells and
    the exit, the exit moved along the far wall (x = L), the additional fire sources
    jittered by up to L/8. Deterministic in seed."""
    base = synthetic(L, W, R)
    rng = np.random.RandomState(seed)
    ex = (L, int(rng.randint(2, W - 1)))
    keep = {tuple(p) for p in base.robot_init} | {ex, (ex[0] - 1, ex[1])}
    bars = []
    while len(bars) < n_barriers:
        w, h = int(rng.randint(2, max(3, L // 12 + 1))), int(rng.randint(2, max(3, W // 12 + 1)))
        x0, y0 = int(rng.randint(2, L - w)), int(rng.randint(2, W - h))
        cells = {(x, y) for x in range(x0 - 1, x0 + w + 1) for y in range(y0 - 1, y0 + h + 1)}
        if cells & keep:
            continue
        bars.append(((x0, y0), (x0 + w - 1, y0 + h - 1)))
    j = max(1, L // 8)
    add = tuple(dict(s, center=(int(np.clip(s["center"][0] + rng.randint(-j, j + 1), 2, L - 1)),
                                int(np.clip(s["center"][1] + rng.randint(-j, j + 1), 2, W - 1))))
                for s in base.additional_fire)
    return dataclasses.replace(base, exit=ex, barriers=tuple(bars), additional_fire=add)


def _norm_barriers(barriers):
    out = []
    for (A, B) in barriers:  # Init_Barrier (envs/map.py:25-33)
        if A[0] > B[0]:
            A, B = B, A
        x1, y1 = A
        x2, y2 = B
        out.append(((x1, y1), (x2, y2)) if y1 < y2 else ((x1, y2), (x2, y1)))
    return out


# ----------------------------------------------------------------------------
# ProgressiveFireModel restatement (envs/fire_model.py:4-199)
# ----------------------------------------------------------------------------
class FireSchedule:
    def __init__(self, initial: Sequence[dict], additional: Sequence[dict], max_steps: int,
                 base_radius=5.0, max_radius=20.0, min_danger=0.05):
        self.max_steps = max_steps
        self.initial = [dict(s) for s in initial]
        self.final = []
        for ini in self.initial:  # :34-42
            self.final.append({"center": ini["center"],
                               "size": (min(8, ini["size"][0] * 4), min(8, ini["size"][1] * 4)),
                               "intensity": min(1.0, ini["intensity"] + 0.4)})
        self.final.extend(dict(s) for s in additional)
        self.base_radius, self.max_radius, self.min_danger = base_radius, max_radius, min_danger

    def sources(self, step: int) -> List[dict]:
        """_interpolate_fire_sources (:69-136)."""
        if step >= self.max_steps:
            return [dict(s) for s in self.final]
        progress = step / self.max_steps
        if progress < 0.2:
            rate = progress * 2
        elif progress < 0.5:
            rate = 0.5 + (progress - 0.2) * 1
        elif progress < 0.8:
            rate = 1.0 + (progress - 0.5) * 0.8
        else:
            rate = 1.3 + (progress - 0.8) * 0.5
        rate = min(rate, 1.0)
        cur = []
        n0 = len(self.initial)
        for ini, fin in zip(self.initial, self.final[:n0]):
            sx = ini["size"][0] + (fin["size"][0] - ini["size"][0]) * rate
            sy = ini["size"][1] + (fin["size"][1] - ini["size"][1]) * rate
            it = ini["intensity"] + (fin["intensity"] - ini["intensity"]) * rate
            cur.append({"center": ini["center"], "size": (int(sx), int(sy)), "intensity": it})
        for i in range(len(self.final) - n0):
            fs = self.final[n0 + i]
            thr = 0.3 + (i * 0.15)
            if progress >= thr:
                npg = min((progress - thr) / (1.0 - thr), 1.0)
                sx = 1 + (fs["size"][0] - 1) * npg
                sy = 1 + (fs["size"][1] - 1) * npg
                it = 0.2 + (fs["intensity"] - 0.2) * npg
                cur.append({"center": fs["center"], "size": (int(sx), int(sy)), "intensity": it})
        return cur

    def radius(self, step: int) -> float:
        """get_current_influence_radius (:138-141)."""
        progress = min(step / self.max_steps, 1.0)
        return self.base_radius + (self.max_radius - self.base_radius) * progress

    def danger_grid(self, step: int, px: np.ndarray, py: np.ndarray) -> np.ndarray:
        """get_max_danger (:143-188), vectorised over positions (px, py float64)."""
        out = np.zeros(np.broadcast(px, py).shape, np.float64)
        R = self.radius(step)
        for s in self.sources(step):
            cx, cy = s["center"]
            dist = np.sqrt((px - cx) ** 2 + (py - cy) ** 2)
            core = max(s["size"][0], s["size"][1]) / 2.0
            inten = s["intensity"]
            base = np.where(dist <= R * 0.3, inten * 1.0,
                            np.where(dist <= R * 0.5, inten * 0.8,
                                     np.where(dist <= R * 0.7, inten * 0.6, inten * 0.4)))
            decay = np.exp(-(dist - core) / 6.0)
            d = np.maximum(base * decay, self.min_danger)
            d = np.where(dist <= R, d, 0.0)
            d = np.where(dist <= core, inten, d)
            out = np.maximum(out, d)
        return out

    def danger_scalar(self, step: int, pos):
        """Scalar get_max_danger keeping the reference's Python/numpy scalar types."""
        md = 0.0
        R = self.radius(step)
        for s in self.sources(step):
            c = s["center"]
            dist = np.sqrt((pos[0] - c[0]) ** 2 + (pos[1] - c[1]) ** 2)
            core = max(s["size"][0], s["size"][1]) / 2.0
            inten = s["intensity"]
            if dist <= core:
                d = inten
            elif dist <= R:
                if dist <= R * 0.3:
                    base = inten * 1.0
                elif dist <= R * 0.5:
                    base = inten * 0.8
                elif dist <= R * 0.7:
                    base = inten * 0.6
                else:
                    base = inten * 0.4
                d = max(base * np.exp(-(dist - core) / 6.0), self.min_danger)
            else:
                d = 0.0
            md = max(md, d)
        return md


@dataclasses.dataclass
class LayoutTables:
    spec: LayoutSpec
    floor: np.ndarray       # [GX, GY] f64
    valid: np.ndarray       # [GX, GY] u8
    exit_mask: np.ndarray   # [GX, GY] u8
    barrier: np.ndarray     # [GX, GY] u8
    danger_p: np.ndarray    # [T+1, GX, GY] f64
    danger_o: np.ndarray    # [T+1, OX, OY] f64
    obs_origin: Tuple[int, int]

    @property
    def GX(self):
        return self.spec.L + 2

    @property
    def GY(self):
        return self.spec.W + 2


def map_space(spec: LayoutSpec):
    """Map.__init__ (envs/map.py:38-79): the pre-potential grid ``space`` (walls and
    barriers inf, exit 1, else 0) and ``barrier_list``."""
    L, W = spec.L, spec.W
    GX, GY = L + 2, W + 2
    inf = float("inf")
    space = np.zeros((GX, GY))
    barrier_list = []
    for j in range(GY):
        space[0][j] = space[L + 1][j] = inf
        barrier_list += [(0, j), (L + 1, j)]
    for i in range(GX):
        space[i][0] = space[i][W + 1] = inf
        barrier_list += [(i, 0), (i, W + 1)]
    for (A, B) in _norm_barriers(spec.barriers):
        for i in range(A[0], B[0] + 1):
            for j in range(A[1], B[1] + 1):
                space[i][j] = inf
                barrier_list.append((i, j))
    ex, ey = spec.exit
    space[ex][ey] = 1
    if ex == L:
        space[ex + 1][ey] = 1
    if ey == W:
        space[ex][ey + 1] = 1
    if (ex, ey) in barrier_list:
        barrier_list.remove((ex, ey))

    return space, barrier_list


def _check_valid(L, W, sp, x, y):
    """Map.Check_Valid (envs/map.py:85-92) on grid ``sp``."""
    x, y = int(x), int(y)
    if x >= L + 1 or x <= 0 or y >= W + 1 or y <= 0:
        return False
    return sp[x][y] != float("inf")


def potential_inputs(spec: LayoutSpec, danger0: Optional[np.ndarray] = None):
    """Inputs of the device floor field (evx_floor_field) for one layout:
    Check_Valid on the pre-potential grid (u8 [GX, GY]), the exit sources (u8), and the
    fire term 200 * danger(0, (i, j)) ** 2 (f64; envs/map.py:143-146) evaluated with
    CPython floats as the reference does -- from ``danger0`` [GX, GY] (danger at integer
    coordinates, t = 0) when given, else from the layout's fire schedule."""
    L, W = spec.L, spec.W
    GX, GY = L + 2, W + 2
    space, _ = map_space(spec)
    valid = np.zeros((GX, GY), np.uint8)
    for x in range(GX):
        for y in range(GY):
            valid[x, y] = _check_valid(L, W, space, x, y)
    src = np.zeros((GX, GY), np.uint8)
    src[spec.exit[0], spec.exit[1]] = 1
    if danger0 is None:
        pf = FireSchedule(spec.map_fire(), spec.additional_fire, spec.fire_max_steps, spec.base_radius,
                          spec.max_radius, spec.min_danger)
        danger0 = np.array([[pf.danger_scalar(0, (i, j)) for j in range(GY)] for i in range(GX)])
    pen = np.array([[200 * (float(d) ** 2) for d in row] for row in np.asarray(danger0, np.float64).tolist()])
    return valid, src, pen


def build_tables(spec: LayoutSpec, t_max: Optional[int] = None, floor: Optional[np.ndarray] = None) -> LayoutTables:
    """The layout's static tables. ``floor``: the floor field computed elsewhere (the device
    kernel, ``build_tables_device``); default: the reference's heapq Init_Potential on the host."""
    L, W = spec.L, spec.W
    GX, GY = L + 2, W + 2
    inf = float("inf")
    ex, ey = spec.exit
    space, barrier_list = map_space(spec)

    def check_valid(sp, x, y):
        return _check_valid(L, W, sp, x, y)

    pfire = FireSchedule(spec.map_fire(), spec.additional_fire, spec.fire_max_steps,
                         spec.base_radius, spec.max_radius, spec.min_danger)
    ofire = FireSchedule(spec.env_fire(), spec.additional_fire, spec.fire_max_steps,
                         spec.base_radius, spec.max_radius, spec.min_danger)
    if floor is None:
        # Init_Potential (envs/map.py:127-148)
        mind = np.full((GX, GY), inf)
        heap = []
        mind[ex][ey] = 1
        heapq.heappush(heap, (1, ex, ey))
        while heap:
            cd, x, y = heapq.heappop(heap)
            for i in range(8):
                nx, ny = x + MOVE_DX[i], y + MOVE_DY[i]
                cost = 1.0 if i < 4 else 1.4
                if check_valid(space, nx, ny):
                    nd = cd + cost
                    if nd < mind[nx][ny]:
                        mind[nx][ny] = nd
                        heapq.heappush(heap, (nd, nx, ny))
        for i in range(GX):
            for j in range(GY):
                if mind[i][j] != inf:
                    danger = pfire.danger_scalar(0, (i, j))
                    mind[i][j] += 200 * (danger ** 2)
        floor = mind
    else:
        floor = np.asarray(floor, np.float64)
        if floor.shape != (GX, GY):
            raise ValueError(f"floor must be [{GX}, {GY}]")
    valid = np.zeros((GX, GY), np.uint8)
    exitm = np.zeros((GX, GY), np.uint8)
    barr = np.zeros((GX, GY), np.uint8)
    for (bx, by) in barrier_list:
        barr[bx, by] = 1
    for x in range(GX):
        for y in range(GY):
            valid[x, y] = check_valid(floor, x, y)
            cx = min(max(x, 0), L + 1)
            cy = min(max(y, 0), W + 1)
            exitm[x, y] = abs(cx - ex) <= 1 and abs(cy - ey) <= 1
    T = spec.fire_max_steps if t_max is None else t_max
    xs = np.arange(GX, dtype=np.float64)[:, None] + 0.5
    ys = np.arange(GY, dtype=np.float64)[None, :] + 0.5
    dp = np.stack([pfire.danger_grid(t, xs, ys) for t in range(T + 1)])
    ox0, oy0 = -OBS_HALF, -OBS_HALF
    oxs = np.arange(ox0, ox0 + GX + 2 * OBS_HALF, dtype=np.float64)[:, None]
    oys = np.arange(oy0, oy0 + GY + 2 * OBS_HALF, dtype=np.float64)[None, :]
    do = np.stack([ofire.danger_grid(t, oxs, oys) for t in range(T + 1)])
    return LayoutTables(spec=spec, floor=floor, valid=valid, exit_mask=exitm, barrier=barr,
                        danger_p=dp, danger_o=do, obs_origin=(ox0, oy0))


def build_tables_device(specs: Sequence[LayoutSpec], t_max: Optional[int] = None, device="cuda") -> List[LayoutTables]:
    """build_tables for several layouts of one grid size with every floor field computed by
    the device kernel in one launch (evacx.floor.floor_fields_for, csrc/floor.hip):
    the same float64 fields as the reference's heapq Init_Potential (tests/test_floor_gpu.py).
    The danger tables stay on the host: they go through numpy's exp (fire_model.py:183)."""
    from .floor import floor_fields_for
    fields, _ = floor_fields_for(list(specs), device=device)
    fl = fields.cpu().numpy()
    return [build_tables(s, t_max, floor=fl[i]) for i, s in enumerate(specs)]
