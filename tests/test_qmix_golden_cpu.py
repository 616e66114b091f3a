"""The QMIX mixer pinned to the reference's own MixingNetwork (runners/train_qmix.py:39-54) and
learn-step sequence (:78-113): tests/golden/qmix_mixer.npz (tools/capture_golden.py qmix,
captured by executing the reference's class in this container) holds three steps' inputs (the
agents' chosen and target-max Q values, reward, done), loss, d loss / d q, the mixer's raw and
clipped gradients, its norm, and parameters / Adam moments after each step. Here: the build's
evacx.qmix.MixingNetwork (what QMixLearnStep and the drop-in runners/train_qmix.py use) from
the same initial parameters, the same sequence, on the CPU -- the same numbers to f32
rounding. The device mixer kernel (evx_qmix_loss) is held to the same fixture in
tests/test_qmix_golden_gpu.py."""
import numpy as np
import torch

from golden_util import load


def test_mixer_steps_match_reference():
    from evacx.qmix import MixingNetwork
    fx = load("qmix_mixer")
    names = [str(n) for n in fx["names"]]
    mixing = MixingNetwork(2)
    mixing.load_state_dict({k: torch.from_numpy(fx["init_" + k]) for k in names})
    target = MixingNetwork(2)
    target.load_state_dict(mixing.state_dict())
    opt = torch.optim.Adam(mixing.parameters(), lr=1e-3)
    for s in range(3):
        p = f"s{s}_"
        q = torch.from_numpy(fx[p + "q"]).requires_grad_(True)
        with torch.no_grad():
            y = torch.from_numpy(fx[p + "r"]) + 0.99 * target(torch.from_numpy(fx[p + "tq"])) * \
                (~torch.from_numpy(fx[p + "d"]).bool())
        loss = torch.nn.functional.mse_loss(mixing(q), y)
        opt.zero_grad()
        loss.backward()
        for k, prm in mixing.named_parameters():
            np.testing.assert_allclose(prm.grad.numpy(), fx[p + "raw_" + k], rtol=1e-5, atol=1e-6, err_msg=k)
        norm = torch.nn.utils.clip_grad_norm_(mixing.parameters(), 1.0)
        opt.step()
        assert abs(loss.item() - float(fx[p + "loss"])) <= 1e-6 * abs(float(fx[p + "loss"]))
        assert abs(norm.item() - float(fx[p + "norm"])) <= 1e-5 * float(fx[p + "norm"])
        np.testing.assert_allclose(q.grad.numpy(), fx[p + "dq"], rtol=1e-5, atol=1e-6)
        for k, prm in mixing.named_parameters():
            np.testing.assert_allclose(prm.grad.numpy(), fx[p + "grad_" + k], rtol=1e-5, atol=1e-8, err_msg=k)
            np.testing.assert_allclose(prm.detach().numpy(), fx[p + "param_" + k], rtol=1e-6, atol=1e-7, err_msg=k)
            np.testing.assert_allclose(opt.state[prm]["exp_avg_sq"].numpy(), fx[p + "v_" + k], rtol=1e-5, atol=1e-12)


def test_fixture_exercises_the_relu_and_done_branches():
    fx = load("qmix_mixer")
    for s in range(3):
        act = fx[f"s{s}_hidden_active"]
        assert 0.05 < act.mean() < 0.95  # hidden units on both sides of the ReLU
        assert 0 < fx[f"s{s}_d"].sum() < len(fx[f"s{s}_d"])
