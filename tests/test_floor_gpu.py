"""Device floor field (csrc/floor.hip, evx_floor_field) vs the
reference's Map.Init_Potential: bit for bit on the reference layouts of the golden
fixtures, and on batches of random mazes vs the pinned oracle (oracle.floor_field),
both on the LDS-resident path (<= 18,432 cells) and the global-memory path."""
import numpy as np
import pytest
import torch

from golden_util import load
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("lname,grid", [("cfg1_layout", None), ("g64_layout", 64), ("g128_layout", 128)])
def test_floor_field_matches_reference(lname, grid):
    _need_gpu()
    import evacx.layout as lay
    from evacx.floor import floor_fields_for
    spec = lay.reference_single() if grid is None else lay.reference_scaled_multi(grid, grid, 8)
    g = load(lname)
    f, passes = floor_fields_for([spec], [g["danger_int0"]])
    torch.cuda.synchronize()
    assert np.array_equal(f[0].cpu().numpy(), g["floor"])
    assert int(passes[0]) >= 2


def _mazes(n, GX, GY, seed, block=0.3):
    rng = np.random.default_rng(seed)
    valid = (rng.random((n, GX, GY)) >= block).astype(np.uint8)
    valid[:, 0, :] = valid[:, -1, :] = valid[:, :, 0] = valid[:, :, -1] = 0
    src = np.zeros_like(valid)
    for i in range(n):
        k = 1 + i % 3  # one to three exits
        src[i, rng.integers(1, GX - 1, k), rng.integers(1, GY - 1, k)] = 1
    pen = np.where(rng.random((n, GX, GY)) < 0.2, 200 * rng.random((n, GX, GY)) ** 2, 0.0)
    return valid, src, pen


@pytest.mark.parametrize("GX,GY,n", [(40, 57, 5), (130, 130, 3), (152, 161, 3)])
def test_floor_field_random_mazes_match_oracle(GX, GY, n):
    _need_gpu()
    from evacx.floor import floor_fields
    valid, src, pen = _mazes(n, GX, GY, seed=GX * GY)
    passes = torch.zeros(n, dtype=torch.int32, device="cuda")
    f = floor_fields(torch.from_numpy(valid).cuda(), torch.from_numpy(src).cuda(),
                     torch.from_numpy(pen).cuda(), passes=passes).cpu().numpy()
    for i in range(n):
        want = orc.floor_field(valid[i], src[i], pen[i])
        assert np.array_equal(f[i], want), i
        assert np.isfinite(want).sum() > GX * GY // 4  # a connected maze, not a trivial case
    assert (passes.cpu().numpy() < GX * GY).all()


def test_floor_field_no_exit_and_no_pen():
    _need_gpu()
    from evacx.floor import floor_fields
    valid, src, _ = _mazes(2, 30, 30, seed=3, block=0.0)
    src[0] = 0  # layout 0 has no exit: everything unreachable
    f = floor_fields(torch.from_numpy(valid).cuda(), torch.from_numpy(src).cuda()).cpu().numpy()
    assert np.isinf(f[0]).all()
    assert np.array_equal(f[1], orc.floor_field(valid[1], src[1]))


def test_build_tables_device_equals_host_build():
    """The product path's layout tables (build_tables_device: every floor field from the device
    kernel in one launch) equal the host heapq build, field for field, on the bench's
    synthetic 128x128 layout and on random per-env layouts."""
    _need_gpu()
    import evacx.layout as lay
    specs = [lay.synthetic(128, 128, 16)] + [lay.random_layout(128, 128, 16, 4242 + k) for k in range(3)]
    dev = lay.build_tables_device(specs, t_max=8)
    for s, td in zip(specs, dev):
        th = lay.build_tables(s, t_max=8)
        for f in ("floor", "valid", "exit_mask", "barrier", "danger_p", "danger_o"):
            assert np.array_equal(getattr(td, f), getattr(th, f)), f
