"""The device-resident vectorised training loop (evacx.trainer) on the GPU."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("precision", ["bf16", "f32"])
def test_vec_trainer_runs_and_learns(precision):
    _need_gpu()
    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import VecTrainer
    spec = synthetic(64, 64, 4)
    lay = DeviceLayout(build_tables(spec), 300)
    tr = VecTrainer(lay, 64, precision=precision, batch=256, replay_capacity=4096, epsilon_decay=0.99,
                    target_every=5)
    p0 = tr.learner.online.flat.clone()
    losses = []
    for _ in range(20):
        tr.step()
        if tr.last_loss is not None:
            losses.append(tr.last_loss.item())
    tr.env.check_err()
    assert tr.replay.size == min(4096, 20 * 64 * 4)
    assert len(losses) == 20 and all(np.isfinite(losses))
    assert tr.epsilon < 1.0
    assert not torch.equal(p0, tr.learner.online.flat)
    a = tr.actions.cpu().numpy()
    assert a.min() >= 0 and a.max() <= 4
    # replay holds the transitions: actions in range, compact obs centred inside the grid
    obs = tr.replay.s.view(-1, 8)[:tr.replay.size].cpu().numpy()
    assert (obs[:, 4] >= 0).all() and (obs[:, 4] <= 65).all()


def test_replay_push_sample_roundtrip():
    _need_gpu()
    from evacx.trainer import Replay
    rp = Replay(100, torch.device("cuda"))
    n = 30
    s = torch.arange(n * 8, dtype=torch.int32, device="cuda")
    s2 = s + 1000
    a = torch.arange(n, dtype=torch.int32, device="cuda") % 5
    r_env = torch.arange(n // 3, dtype=torch.float64, device="cuda")
    d_env = (torch.arange(n // 3, device="cuda") % 2).to(torch.uint8)
    for _ in range(4):
        rp.push(s, s2, a, r_env, d_env, n, 3)
    assert rp.size == 100 and rp.pos == 20
    out = dict(s=torch.zeros(64 * 8, dtype=torch.int32, device="cuda"),
               s2=torch.zeros(64 * 8, dtype=torch.int32, device="cuda"),
               a=torch.zeros(64, dtype=torch.int32, device="cuda"),
               r=torch.zeros(64, dtype=torch.float32, device="cuda"),
               done=torch.zeros(64, dtype=torch.uint8, device="cuda"))
    rp.sample(64, 5, 0, out)
    so = out["s"].view(64, 8).cpu().numpy()
    i = so[:, 0] // 8  # which agent row each sample came from
    assert np.array_equal(out["s2"].view(64, 8).cpu().numpy()[:, 0], so[:, 0] + 1000)
    assert np.array_equal(out["a"].cpu().numpy(), i % 5)
    assert np.array_equal(out["r"].cpu().numpy(), (i // 3).astype(np.float32))
    assert np.array_equal(out["done"].cpu().numpy(), (i // 3) % 2)
