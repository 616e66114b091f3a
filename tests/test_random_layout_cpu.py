"""evacx.layout.random_layout (per-env layouts): deterministic, the
robots start on valid cells, the exit is reachable from them, layouts of one size."""
import numpy as np

import evacx.layout as lay
from oracle import oracle as orc


def test_random_layouts_are_valid_and_reachable():
    specs = [lay.random_layout(64, 64, 8, 100 + k) for k in range(3)]
    assert specs[0] == lay.random_layout(64, 64, 8, 100)  # deterministic in the seed
    assert len({s.exit for s in specs} | {tuple(s.barriers) for s in specs}) > 1
    for s in specs:
        valid, src, pen = lay.potential_inputs(s)
        f = orc.floor_field(valid, src, pen)
        for (x, y) in s.robot_init:
            assert valid[x, y] == 1, (s.exit, (x, y))
            assert np.isfinite(f[x, y])
        assert (s.L, s.W, s.R) == (64, 64, 8)
