"""The fused MLP host driver (evacx/qmlp.py) refuses short caller buffers BEFORE anything is
launched: the C-ABI takes row counts, not buffer lengths, and a kernel reading past a
caller's allocation faults the GPU (round 2, commit f884920). No GPU needed: the checks run
on the host and raise ValueError before the library is called (CPU tensors stand in for the
device buffers; reaching a launch would fail differently)."""
import pytest
import torch

from evacx.qmlp import HID, HID2, NACT, MLPFast


class _NoLaunch(MLPFast):
    """An MLPFast whose construction skips the device repack; every path that gets past the
    guards would have to call the library, which this test must never reach."""

    def __init__(self, x3=True):
        self.x3, self.kx, self._part = x3, 640 if x3 else 512, None


def _obs(rows):
    return torch.zeros(rows * 8, dtype=torch.int32)


@pytest.mark.parametrize("n,rows", [(16, 15), (1024, 1000), (33, 0)])
def test_forward_rejects_short_obs(n, rows):
    f = _NoLaunch()
    with pytest.raises(ValueError, match="forward obs"):
        f.forward(None, _obs(rows), n, torch.zeros(2 * n * HID, dtype=torch.int16))


def test_forward_rejects_short_q():
    f = _NoLaunch()
    with pytest.raises(ValueError, match="forward q"):
        f.forward(None, _obs(64), 64, None, q=torch.zeros(63, NACT))


@pytest.mark.parametrize("what", ["obs", "q", "actions"])
def test_act_rejects_short_buffers(what):
    f = _NoLaunch()
    n = 128
    kw = dict(q=torch.zeros(n, NACT), actions=torch.zeros(n, dtype=torch.int32))
    obs = _obs(n)
    if what == "obs":
        obs = _obs(n - 1)
    else:
        kw[what] = kw[what][:-1]
    with pytest.raises(ValueError, match=f"act {what}"):
        f.act(None, obs, n, **kw)


def test_act_rejects_bad_perm():
    f = _NoLaunch()
    with pytest.raises(ValueError, match="perm"):
        f.act(None, _obs(96), 96, perm=torch.zeros(5, dtype=torch.int32), rows_per_env=16)


@pytest.mark.parametrize("which", ["obs0", "obs1", "q"])
def test_forward_pair_rejects_short_buffers(which):
    n = 256
    o0, o1 = _obs(n), _obs(n)
    out0, out1 = dict(q=torch.zeros(n, NACT)), dict(q=torch.zeros(n, NACT))
    if which == "obs0":
        o0 = _obs(n - 2)
    elif which == "obs1":
        o1 = _obs(n - 2)
    else:
        out1["q"] = torch.zeros(n - 1, NACT)
    with pytest.raises(ValueError, match=f"forward_pair {which}"):
        MLPFast.forward_pair(None, n, _NoLaunch(), o0, (0, 0, 0.2), out0, _NoLaunch(), o1, (0, 0, 0.2), out1)


@pytest.mark.parametrize("short", ["x", "h1", "dz1", "dz2", "h2", "dq"])
def test_backward_rejects_short_saved_buffers(short):
    f = _NoLaunch()
    B = 512
    bufs = dict(dq=torch.zeros(B * NACT), x=torch.zeros(B * f.kx, dtype=torch.int16),
                h1=torch.zeros(2 * B * HID, dtype=torch.int16), h2=torch.zeros(B * HID2),
                dz2=torch.zeros(2 * B * HID2, dtype=torch.int16), dz1=torch.zeros(2 * B * HID, dtype=torch.int16))
    bufs[short] = bufs[short][:-1]
    with pytest.raises(ValueError, match=f"backward: {short}"):
        f.backward(B, bufs["dq"], bufs["x"], bufs["h1"], bufs["h2"], 0.2, bufs["dz2"], bufs["dz1"], grads=None)


@pytest.mark.parametrize("prec", ["fp32", "x3", "exactf32", ""])
def test_trainer_rejects_unknown_precision(prec):
    """VecTrainer takes "f32" (x3 fused kernels / x3 conv), "bf16" or "exact" (dense exact-f32 GEMMs),
    and refuses anything else before touching the device."""
    from evacx.trainer import VecTrainer
    with pytest.raises(ValueError, match="precision"):
        VecTrainer(None, 1, precision=prec)


def test_learner_rejects_unknown_precision():
    from evacx.qnet import Learner
    with pytest.raises(ValueError, match="precision"):
        Learner(kind="mlp", device="cpu", precision="f16")
