"""The C-ABI keeps no hidden state (caller-owned buffers, explicit stream): work
issued on two streams at once must give the bits the same work gives run one after the other.

* two VecEnvs stepping concurrently on two streams, each with its own dispatch order and act
  permutation (evx_env_order / evx_act_perm through evx_state.perm_ws, the caller's workspace)
  -- every state field, reward and observation equal to the serial run's;
* two learners' TD steps (evx_td_loss_w: per-block partials in the caller's workspace, summed
  in block order by a second launch) on two streams -- loss, gradients and parameters equal;
* the conv Q-net's act forward under two scratch tags on two streams (the trainer's env groups:
  Learner.q_values(tag=...)) -- Q equal to the serial calls';
* evx_pix_nchw beyond the LDS tile's 134 channels (element-wise path) equals torch's permute.
Reference boundary: SURVEY §8(b); envs/evacuation_env.py:122-172, agents/dqn_agent.py:101-168."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _envs(n_env, seeds):
    from evacx.env import DeviceLayout, VecEnv
    from evacx.layout import build_tables, synthetic
    lay = DeviceLayout(build_tables(synthetic(24, 20, 4)), 380)
    out = []
    for s in seeds:
        v = VecEnv(lay, n_env)
        v.seed([s + i for i in range(n_env)])
        v.reset()
        out.append(v)
    return lay, out


def test_two_envs_on_two_streams_match_serial():
    _need_gpu()
    E = 1024
    lay, (a0, a1) = _envs(E, [100, 5000])
    _, (b0, b1) = _envs(E, [100, 5000])
    g = torch.Generator(device="cuda").manual_seed(1)
    acts = [torch.randint(0, 5, (E * lay.R,), device="cuda", dtype=torch.int32, generator=g) for _ in range(30)]
    perm = [torch.zeros(E, dtype=torch.int32, device="cuda") for _ in range(4)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    for t in range(30):
        for v, p in ((a0, perm[0]), (a1, perm[1])):  # serial
            v.compute_order()
            v.act_perm(p)
            v.step(acts[t], order=False, auto_reset=True)
        cur = torch.cuda.current_stream()
        for v, p, s in ((b0, perm[2], streams[0]), (b1, perm[3], streams[1])):  # concurrent
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                v.compute_order()
                v.act_perm(p)
                v.step(acts[t], order=False, auto_reset=True)
        for s in streams:
            cur.wait_stream(s)
        torch.cuda.synchronize()
        assert torch.equal(perm[0], perm[2]) and torch.equal(perm[1], perm[3]), t
        for x, y in ((a0, b0), (a1, b1)):
            assert torch.equal(x.order, y.order), t
            assert torch.equal(x.obs, y.obs) and torch.equal(x.reward, y.reward), t
    for x, y in ((a0, b0), (a1, b1)):
        for name in ["pk", "health", "acc", "rmap", "scal", "py_mt", "np_mt", "robots", "view"]:
            assert torch.equal(getattr(x, name), getattr(y, name)), name
        x.check_err()
        y.check_err()


def test_two_learners_td_steps_on_two_streams_match_serial():
    """Learner.learn on the dense path: evx_gemm forwards, evx_td_loss_w, backward, clip + Adam."""
    _need_gpu()
    from evacx.qnet import Learner
    from test_qnet_gpu import make_batch
    batches = [[t.cuda() for t in make_batch(3000, s)] for s in (7, 8)]
    ser = [Learner(kind="mlp", precision="f32", seed=s, lr=1e-3) for s in (1, 2)]
    con = [Learner(kind="mlp", precision="f32", seed=s, lr=1e-3) for s in (1, 2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    for _ in range(3):
        loss_s = []
        for lr, (x, x2, a, r, d, m1, m2) in zip(ser, batches):
            loss_s.append(lr.learn(x, a, r, d, x2, mask_online=m1, mask_target=m2).clone())
        cur = torch.cuda.current_stream()
        loss_c = []
        for lr, (x, x2, a, r, d, m1, m2), s in zip(con, batches, streams):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                loss_c.append(lr.learn(x, a, r, d, x2, mask_online=m1, mask_target=m2).clone())
        for s in streams:
            cur.wait_stream(s)
        torch.cuda.synchronize()
        for ls, lc in zip(loss_s, loss_c):
            assert torch.equal(ls, lc)
    for p, q in zip(ser, con):
        assert torch.equal(p.grads.flat, q.grads.flat)
        assert torch.equal(p.online.flat, q.online.flat)


def test_conv_act_tags_on_two_streams_match_serial():
    _need_gpu()
    from evacx.qnet import Learner
    from test_qnet_gpu import make_batch
    lr = Learner(kind="conv", precision="x3", seed=5)
    xs = [make_batch(96, s)[0].cuda() for s in (1, 2)]
    ms = [make_batch(96, s)[5].cuda() for s in (1, 2)]
    ser = [lr.q_values(x, mask=m, tag=t).clone() for x, m, t in zip(xs, ms, ("act", "act1"))]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    cur = torch.cuda.current_stream()
    torch.cuda.synchronize()
    for _ in range(3):
        out = []
        for x, m, t, s in zip(xs, ms, ("act", "act1"), streams):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                out.append(lr.q_values(x, mask=m, tag=t).clone())
        for s in streams:
            cur.wait_stream(s)
        torch.cuda.synchronize()
        for a, b in zip(ser, out):
            assert torch.equal(a, b)


@pytest.mark.parametrize("C", [64, 150])
def test_pix_nchw_any_channel_count(C):
    _need_gpu()
    import ctypes as Ct
    from evacx.qnet import qcheck, qlib
    B = 5
    pix = torch.randn(B, 121, C, device="cuda")
    out = torch.empty(B, C, 121, device="cuda")
    qcheck(qlib().evx_pix_nchw(pix.data_ptr(), B, C, 1, out.data_ptr(), None), "pix_nchw")
    back = torch.empty_like(pix)
    qcheck(qlib().evx_pix_nchw(out.data_ptr(), B, C, 0, back.data_ptr(), None), "pix_nchw")
    torch.cuda.synchronize()
    assert torch.equal(out, pix.permute(0, 2, 1))
    assert torch.equal(back, pix)
    _ = Ct  # ctypes loaded by qlib


def test_trainer_exact_precision_runs_exact_gemms():
    """precision="exact" on the MLP: no fused kernels (the dense evx_gemm f32 path), reported as f32."""
    _need_gpu()
    from evacx.env import DeviceLayout
    from evacx.layout import build_tables, synthetic
    from evacx.trainer import VecTrainer
    lay = DeviceLayout(build_tables(synthetic(24, 20, 4)), 380)
    tr = VecTrainer(lay, 16, kind="mlp", precision="exact", batch=32, replay_capacity=1024)
    assert tr.learner.fast is None and tr.q_arith == "f32"
    for _ in range(3):
        tr.step()
    tr.sync()
    torch.cuda.synchronize()
    assert tr.learn_steps >= 2 and np.isfinite(float(tr.last_loss.item()))
    tr2 = VecTrainer(lay, 16, kind="mlp", precision="f32", batch=32, replay_capacity=1024)
    assert tr2.learner.fast is not None and tr2.q_arith == "x3"
