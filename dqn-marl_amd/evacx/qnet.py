"""Device Q-networks and the DQN learner step (host driver of libevacx's learner kernels).

Reference: Louvre_Evacuation/agents/dqn_agent.py
  * DQNNetwork (:15-61): conv 6->32->64->128 (3x3, pad 1) on the 11x11x6 patch,
    fc 15488->512 (+ReLU, Dropout 0.2) ->256 (+ReLU) ->5.     -> ``ConvQNet``
  * the build-defined MLP variant for the vectorised configs:
    726->512 (+ReLU, Dropout) ->256 (+ReLU) ->5.              -> ``MLPQNet``
  * DQNAgent.learn (:126-168): Q(s).gather(a), r + gamma max Q_tgt(s') ~done, MSE,
    backward, clip_grad_norm_(1.0), Adam.                      -> ``Learner.learn``

Parameters, gradients and Adam moments each live in ONE flat fp32 buffer (the
reference's state_dict order), so clip+Adam is one fused kernel and a multi-GPU
gradient all-reduce is one collective. Every contraction runs in evx_gemm
(MFMA); torch only allocates.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import torch

from . import _lib
from .env import _stream

PREC = {"f32": 0, "bf16": 1, "x3": 2}
RELU, ACCUM, SPLIT_AB, OUT_SPLIT = 1, 2, 4, 8
DROPOUT_P = 0.2


class evx_gemm_desc(C.Structure):
    _fields_ = [("M", C.c_int32), ("N", C.c_int32), ("K", C.c_int32), ("precision", C.c_int32),
                ("flags", C.c_int32), ("alpha", C.c_float),
                ("A", C.c_void_p), ("sam", C.c_int64), ("sak", C.c_int64),
                ("B", C.c_void_p), ("sbk", C.c_int64), ("sbn", C.c_int64),
                ("C", C.c_void_p), ("ldc", C.c_int64), ("bias", C.c_void_p),
                ("mask", C.c_void_p), ("ldm", C.c_int64), ("mask_scale", C.c_float),
                ("gate", C.c_void_p), ("ldg", C.c_int64), ("ws", C.c_void_p), ("ws_elems", C.c_int64)]


class evx_adam(C.Structure):
    _fields_ = [("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float),
                ("weight_decay", C.c_float), ("step", C.c_int64)]


_q_inited = False


def qlib():
    global _q_inited
    L = _lib.lib()
    if not _q_inited:
        L.evx_q_last_error.restype = C.c_char_p
        L.evx_gemm.argtypes = [C.POINTER(evx_gemm_desc), C.c_void_p]
        L.evx_gemm_ws_elems.argtypes = [C.POINTER(evx_gemm_desc)]
        L.evx_gemm_ws_elems.restype = C.c_int64
        L.evx_conv3x3_ws_elems.argtypes = [C.POINTER(evx_gemm_desc), C.c_int32, C.c_int32]
        L.evx_conv3x3_ws_elems.restype = C.c_int64
        L.evx_colsum.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p,
                                 C.c_int32, C.c_void_p]
        L.evx_td_loss_ws_floats.restype = C.c_int64
        L.evx_td_loss_ws_floats.argtypes = [C.c_int32, C.c_int32]
        L.evx_td_loss.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_float,
                                  C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
        L.evx_td_loss_w.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_float, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_int64, C.c_void_p]
        L.evx_td_loss_zero.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_float, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p]
        L.evx_td_loss_zero_g.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_float, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p]
        L.evx_sumsq_norm.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
        L.evx_clip_adam.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p,
                                    C.c_float, C.POINTER(evx_adam), C.c_void_p]
        L.evx_dropout_mask.argtypes = [C.c_void_p, C.c_int64, C.c_float, C.c_uint64, C.c_uint64, C.c_void_p]
        L.evx_act.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_float, C.c_uint64, C.c_uint64, C.c_void_p,
                              C.c_void_p]
        L.evx_im2col3x3.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        L.evx_col2im3x3.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        L.evx_pix_nchw.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        L.evx_pix_split.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        L.evx_relu_grad.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
        L.evx_conv3x3_gemm.argtypes = [C.POINTER(evx_gemm_desc), C.c_int32, C.c_int32, C.c_void_p]
        _q_inited = True
    return L


def qcheck(rc, what):
    if rc != 0:
        raise _lib.EvacxError(f"{what} failed ({rc}): {qlib().evx_q_last_error().decode()}")


def _p(t):
    return None if t is None else t.data_ptr()


def td_workspace(ws, B: int, nets: int, device, tag: str = "") -> torch.Tensor:
    """The TD loss's partials buffer (evx_td_loss_ws_floats) from a _Workspace pool."""
    n = max(1, int(qlib().evx_td_loss_ws_floats(B, nets)))
    return ws.get(tag + "td_ws", (n,), torch.float32, device)


_WS_NEED: Dict[Tuple, int] = {}


def _attach_ws(d, ws, tag, device, conv=None):
    """Workspace of a descriptor (evx_gemm_ws_elems: split-K partials; conv = (mode, channels):
    evx_conv3x3_ws_elems, which also covers the conv forward's packed weights): ws is a _Workspace
    (a buffer per tag and size, kept for the pool's life, so a stream never sees another stream's
    scratch freed or rewritten under it), a f32 tensor, or None (the GEMM runs in one pass)."""
    if ws is None:
        return
    key = (d.M, d.N, d.K, d.precision, d.flags, bool(d.bias), bool(d.mask), bool(d.gate), d.sbk, d.sbn, conv)
    need = _WS_NEED.get(key)
    if need is None:
        need = _WS_NEED[key] = int(qlib().evx_conv3x3_ws_elems(C.byref(d), conv[0], conv[1]) if conv
                                   else qlib().evx_gemm_ws_elems(C.byref(d)))
    if need <= 0:
        return
    if isinstance(ws, torch.Tensor):
        if ws.dtype != torch.float32:
            raise ValueError("gemm workspace must be float32")
        d.ws, d.ws_elems = ws.data_ptr(), ws.numel()
        return
    buf = ws.get(tag + "splitk", (need,), torch.float32, device)
    d.ws, d.ws_elems = buf.data_ptr(), need


def gemm(M, N, K, A, sam, sak, B, sbk, sbn, Cm, ldc, precision="f32", bias=None, relu=False, mask=None,
         ldm=0, mask_scale=1.0, gate=None, ldg=0, accumulate=False, alpha=1.0, ws=None, tag="", split_ab=False):
    """evx_gemm; split_ab: A and B are bf16 hi / lo planes (int16 tensors, x3, k-contiguous)."""
    d = evx_gemm_desc(M=M, N=N, K=K, precision=PREC[precision],
                      flags=(RELU if relu else 0) | (ACCUM if accumulate else 0) | (SPLIT_AB if split_ab else 0),
                      alpha=alpha, A=_p(A), sam=sam, sak=sak, B=_p(B), sbk=sbk, sbn=sbn, C=_p(Cm), ldc=ldc,
                      bias=_p(bias), mask=_p(mask), ldm=ldm, mask_scale=mask_scale, gate=_p(gate), ldg=ldg)
    _attach_ws(d, ws, tag, Cm.device)
    qcheck(qlib().evx_gemm(C.byref(d), _stream()), "evx_gemm")


CONV_FWD, CONV_DX, CONV_DW = 1, 2, 3


def conv_gemm(mode, M, N, K, A, B, Cm, cs, sam=0, sak=0, sbk=0, sbn=0, bias=None, relu=False, gate=None,
              ldg=0, ws=None, tag="", out_split=False):
    """evx_conv3x3_gemm (x3): implicit-GEMM 3x3 conv forward / dX / dW on pixel-major activations.
    out_split: the output as bf16 hi / lo planes (Cm int16 [2][M][N]; the LDS-staged forward)."""
    d = evx_gemm_desc(M=M, N=N, K=K, precision=PREC["x3"], flags=(RELU if relu else 0) | (OUT_SPLIT if out_split else 0),
                      alpha=1.0, A=_p(A),
                      sam=sam, sak=sak, B=_p(B), sbk=sbk, sbn=sbn, C=_p(Cm), ldc=N, bias=_p(bias), mask=None,
                      ldm=0, mask_scale=1.0, gate=_p(gate), ldg=ldg)
    _attach_ws(d, ws, tag + f"cv{mode}_", Cm.device, conv=(mode, cs))
    qcheck(qlib().evx_conv3x3_gemm(C.byref(d), mode, cs, _stream()), "evx_conv3x3_gemm")


def colsum(X, M, N, out, scratch):
    qcheck(qlib().evx_colsum(_p(X), N, M, N, _p(out), 0, _p(scratch), scratch.numel(), _stream()), "evx_colsum")


# ----------------------------------------------------------------------------
# parameter layout
# ----------------------------------------------------------------------------
def layer_specs(kind: str, hidden: int = 512, actions: int = 5, in_dim: int = 726) -> List[Tuple]:
    """(name, type, fan_in, fan_out[, conv channels]) in the reference state_dict order."""
    if kind == "conv":
        return [("conv1", "conv", 6, 32), ("conv2", "conv", 32, 64), ("conv3", "conv", 64, 128),
                ("fc1", "fc", 11 * 11 * 128, hidden), ("fc2", "fc", hidden, hidden // 2),
                ("fc3", "fc", hidden // 2, actions)]
    if kind == "mlp":
        return [("fc1", "fc", in_dim, hidden), ("fc2", "fc", hidden, hidden // 2),
                ("fc3", "fc", hidden // 2, actions)]
    raise ValueError(kind)


def param_shapes(specs) -> "OrderedDict[str, Tuple[int, ...]]":
    out = OrderedDict()
    for name, typ, fi, fo in specs:
        out[name + ".weight"] = (fo, fi, 3, 3) if typ == "conv" else (fo, fi)
        out[name + ".bias"] = (fo,)
    return out


class FlatParams:
    """All tensors of one network in one flat fp32 device buffer (state_dict order)."""

    def __init__(self, shapes, device, data: Optional[torch.Tensor] = None):
        self.shapes = shapes
        self.numel = sum(int(torch.Size(s).numel()) for s in shapes.values())
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=device) if data is None else data
        self.views: Dict[str, torch.Tensor] = OrderedDict()
        o = 0
        for k, s in shapes.items():
            n = int(torch.Size(s).numel())
            self.views[k] = self.flat[o:o + n].view(s)
            o += n

    def __getitem__(self, k):
        return self.views[k]

    def state_dict(self):
        return OrderedDict((k, v.detach().clone()) for k, v in self.views.items())

    def load_state_dict(self, sd):
        for k, v in self.views.items():
            v.copy_(sd[k].to(v.device, torch.float32).view(v.shape))

    def init_from_global_torch(self):
        """The reference's own initialisation: each layer's nn.Conv2d / nn.Linear
        reset_parameters (kaiming_uniform_(w, a=sqrt(5)), then bias ~ U(+-1/sqrt(fan_in)))
        drawn from torch's global CPU generator in state_dict order, so after
        torch.manual_seed(s) the weights and the generator's position equal a freshly built
        reference DQNNetwork's (agents/dqn_agent.py:22-31)."""
        import math
        for k, v in self.views.items():
            if k.endswith(".weight"):
                w = torch.empty(self.shapes[k])
                torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
                v.copy_(w)
            else:
                ws = self.shapes[k[:-5] + ".weight"]
                fan_in = ws[1] * (ws[2] * ws[3] if len(ws) == 4 else 1)
                bound = 1.0 / math.sqrt(fan_in) if fan_in > 0 else 0.0
                v.copy_(torch.empty(self.shapes[k]).uniform_(-bound, bound))

    def init_like_torch(self, seed: int):
        """nn.Conv2d / nn.Linear default init (kaiming_uniform a=sqrt(5) -> U(+-1/sqrt(fan_in)))."""
        g = torch.Generator().manual_seed(seed)
        for k, v in self.views.items():
            w_name = k[:-5] + ".weight" if k.endswith(".bias") else k
            ws = self.shapes[w_name]
            fan_in = ws[1] * (ws[2] * ws[3] if len(ws) == 4 else 1)
            bound = 1.0 / (fan_in ** 0.5)
            v.copy_((torch.rand(v.shape, generator=g) * 2 - 1) * bound)


# ----------------------------------------------------------------------------
# networks
# ----------------------------------------------------------------------------
class _Workspace:
    def __init__(self):
        self.bufs: Dict[Tuple, torch.Tensor] = {}

    def get(self, name, shape, dtype, device):
        key = (name, tuple(shape), dtype)
        t = self.bufs.get(key)
        if t is None:
            t = torch.empty(shape, dtype=dtype, device=device)
            self.bufs[key] = t
        return t


class QNet:
    """Forward/backward of the reference DQNNetwork (or the MLP variant) on evx_gemm."""

    def __init__(self, kind: str, params: FlatParams, precision="f32", hidden=512, actions=5):
        self.kind, self.P, self.prec = kind, params, precision
        self.hidden, self.actions = hidden, actions
        # x3 conv layers as implicit GEMMs (the exact-f32 path keeps im2col + GEMM)
        self.implicit = kind == "conv" and precision == "x3"
        self.device = params.flat.device
        self.ws = _Workspace()
        self.saved = None

    # ------------------------------------------------------------ fc stack
    def _fc_forward(self, X, B, K0, mask, tag, w1=None, split=False):
        """split: X and w1 are bf16 hi / lo planes (int16 [2][B][K0], [2][H][K0]) -- the act's fc1."""
        P, ws, dev, H, A = self.P, self.ws, self.device, self.hidden, self.actions
        H1 = ws.get(tag + "h1", (B, H), torch.float32, dev)
        gemm(B, H, K0, X, K0, 1, P["fc1.weight"] if w1 is None else w1, 1, K0, H1, H, self.prec, bias=P["fc1.bias"],
             relu=True,
             mask=mask, ldm=H, mask_scale=1.0 / (1.0 - DROPOUT_P), ws=self.ws, tag=tag, split_ab=split)
        H2 = ws.get(tag + "h2", (B, H // 2), torch.float32, dev)
        gemm(B, H // 2, H, H1, H, 1, P["fc2.weight"], 1, H, H2, H // 2, self.prec, bias=P["fc2.bias"], relu=True, ws=self.ws, tag=tag)
        Q = ws.get(tag + "q", (B, A), torch.float32, dev)
        gemm(B, A, H // 2, H2, H // 2, 1, P["fc3.weight"], 1, H // 2, Q, A, self.prec, bias=P["fc3.bias"], ws=self.ws, tag=tag)
        return H1, H2, Q

    def forward(self, x: torch.Tensor, mask: Optional[torch.Tensor], save=True, tag="") -> torch.Tensor:
        """x: [B, 11, 11, 6] (or [B, 726]) fp32; mask: [B, hidden] uint8 dropout keep-mask or None (eval)."""
        B = x.shape[0]
        x = x.reshape(B, -1).contiguous()
        if self.kind == "mlp":
            H1, H2, Q = self._fc_forward(x, B, x.shape[1], mask, tag)
            if save:
                self.saved = dict(B=B, x=x, H1=H1, H2=H2, mask=mask)
            return Q
        ws, dev, P = self.ws, self.device, self.P
        L = qlib()
        Mp = B * 121
        ins, cols, ys = [x], [], []
        cur, C_in = x, 6
        # without saves (the act): conv3's output leaves as bf16 hi / lo planes and fc1 runs on
        # pre-split operands (EVX_GEMM_SPLIT_AB: its K tiles staged as 16-B copies)
        split = self.implicit and not save
        for li, (cname, cout) in enumerate([("conv1", 32), ("conv2", 64), ("conv3", 128)]):
            K9 = C_in * 9
            if self.implicit:  # x3: the taps gathered in the GEMM's tile fetch (no im2col buffer)
                osp = split and li == 2
                Y = ws.get(tag + f"y{li}" + ("s" if osp else ""), (2 * Mp, cout) if osp else (Mp, cout),
                           torch.int16 if osp else torch.float32, dev)
                conv_gemm(CONV_FWD, Mp, cout, K9, cur, P[cname + ".weight"], Y, C_in, sbk=9, sbn=K9,
                          bias=P[cname + ".bias"], relu=True, ws=self.ws, tag=tag, out_split=osp)
                cols.append(cur)  # the layer input, gathered again by the dW GEMM
                ys.append(Y)
                cur, C_in = Y, cout
                continue
            col = ws.get(tag + f"col{li}", (Mp, K9), torch.float32, dev)
            qcheck(L.evx_im2col3x3(_p(cur), B, C_in, 1, _p(col), _stream()), "im2col")
            Y = ws.get(tag + f"y{li}", (Mp, cout), torch.float32, dev)
            gemm(Mp, cout, K9, col, K9, 1, P[cname + ".weight"], 1, K9, Y, cout, self.prec, bias=P[cname + ".bias"],
                 relu=True, ws=self.ws, tag=tag)
            cols.append(col)
            ys.append(Y)
            cur, C_in = Y, cout
        if self.implicit:
            # fc1 reads conv3's pixel-major output as it lies ([B][121 * 128], column p * 128 + c)
            # against a copy of fc1.weight with its columns in that order (the reference flattens
            # NCHW: column c * 121 + p). The copy is made per forward (31.7 MB, ~20 us) instead of
            # transposing the activations (8192 rows: 507 MB, 0.57 ms).
            if split:
                W1s = ws.get(tag + "w1s", (2 * self.hidden, 128 * 121), torch.int16, dev)
                qcheck(L.evx_pix_split(_p(P["fc1.weight"]), self.hidden, 128, _p(W1s), _stream()), "pix_split")
                _, _, Q = self._fc_forward(cur, B, 128 * 121, mask, tag, w1=W1s, split=True)
                return Q
            W1p = ws.get(tag + "w1p", (self.hidden, 128 * 121), torch.float32, dev)
            qcheck(L.evx_pix_nchw(_p(P["fc1.weight"]), self.hidden, 128, 0, _p(W1p), _stream()), "pix_nchw")
            F = cur.view(B, 128 * 121)
            H1, H2, Q = self._fc_forward(F, B, 128 * 121, mask, tag, w1=W1p)
            if save:
                self.saved = dict(B=B, x=F, H1=H1, H2=H2, mask=mask, cols=cols, ys=ys, w1p=W1p)
            return Q
        F = ws.get(tag + "flat", (B, 128 * 121), torch.float32, dev)
        qcheck(L.evx_pix_nchw(_p(cur), B, 128, 1, _p(F), _stream()), "pix_nchw")  # torch reshape of NCHW
        H1, H2, Q = self._fc_forward(F, B, 128 * 121, mask, tag)
        if save:
            self.saved = dict(B=B, x=F, H1=H1, H2=H2, mask=mask, cols=cols, ys=ys)
        return Q

    def backward(self, dQ: torch.Tensor, grads: FlatParams):
        """Writes d loss / d params into `grads` (overwrites) for the saved forward."""
        s = self.saved
        assert s is not None, "forward(save=True) first"
        B, X, H1, H2, mask = s["B"], s["x"], s["H1"], s["H2"], s["mask"]
        P, ws, dev, H, A, pr = self.P, self.ws, self.device, self.hidden, self.actions, self.prec
        K0 = X.shape[1]
        # colsum partials: one per 64 rows and column (evx_colsum)
        scratch = ws.get("colsum", (max(1, (max(B * 121, B) + 63) // 64) * max(H, 128),), torch.float32, dev)
        # fc3
        gemm(A, H // 2, B, dQ, 1, A, H2, H // 2, 1, grads["fc3.weight"], H // 2, pr, ws=self.ws, tag="bw_")
        colsum(dQ, B, A, grads["fc3.bias"], scratch)
        dZ2 = ws.get("dz2", (B, H // 2), torch.float32, dev)
        gemm(B, H // 2, A, dQ, A, 1, P["fc3.weight"], H // 2, 1, dZ2, H // 2, pr, gate=H2, ldg=H // 2, ws=self.ws, tag="bw_")
        # fc2
        gemm(H // 2, H, B, dZ2, 1, H // 2, H1, H, 1, grads["fc2.weight"], H, pr, ws=self.ws, tag="bw_")
        colsum(dZ2, B, H // 2, grads["fc2.bias"], scratch)
        dZ1 = ws.get("dz1", (B, H), torch.float32, dev)
        gemm(B, H, H // 2, dZ2, H // 2, 1, P["fc2.weight"], H, 1, dZ1, H, pr, mask=mask, ldm=H,
             mask_scale=1.0 / (1.0 - DROPOUT_P), gate=H1, ldg=H, ws=self.ws, tag="bw_")
        # fc1
        L = qlib()
        W1p = s.get("w1p")
        if W1p is None:
            gemm(H, K0, B, dZ1, 1, H, X, K0, 1, grads["fc1.weight"], K0, pr, ws=self.ws, tag="bw_")
        else:  # X is pixel-major: dW1 in that column order, then back to the reference's
            dW1p = ws.get("dw1p", (H, K0), torch.float32, dev)
            gemm(H, K0, B, dZ1, 1, H, X, K0, 1, dW1p, K0, pr, ws=self.ws, tag="bw_")
            qcheck(L.evx_pix_nchw(_p(dW1p), H, 128, 1, _p(grads["fc1.weight"]), _stream()), "pix_nchw")
        colsum(dZ1, B, H, grads["fc1.bias"], scratch)
        if self.kind == "mlp":
            return
        Mp = B * 121
        dY = ws.get("dy2", (Mp, 128), torch.float32, dev)
        if W1p is not None:  # dF in pixel order is conv3's dY
            gemm(B, K0, H, dZ1, H, 1, W1p, K0, 1, dY.view(B, K0), K0, pr, gate=X, ldg=K0, ws=self.ws, tag="bw_")
        else:
            dF = ws.get("dflat", (B, K0), torch.float32, dev)
            gemm(B, K0, H, dZ1, H, 1, P["fc1.weight"], K0, 1, dF, K0, pr, gate=X, ldg=K0, ws=self.ws, tag="bw_")  # gate: relu(conv3) > 0
            qcheck(L.evx_pix_nchw(_p(dF), B, 128, 0, _p(dY), _stream()), "pix_nchw")
        cols, ys = s["cols"], s["ys"]
        for li, (cname, cin, cout) in reversed(list(enumerate([("conv1", 6, 32), ("conv2", 32, 64),
                                                                ("conv3", 64, 128)]))):
            K9 = cin * 9
            if self.implicit:  # cols[li] is the layer input [Mp][cin]
                conv_gemm(CONV_DW, cout, K9, Mp, dY, cols[li], grads[cname + ".weight"], cin, sam=1, sak=cout, ws=self.ws, tag="bw_")
                colsum(dY, Mp, cout, grads[cname + ".bias"], scratch)
                if li == 0:
                    break
                dYp = ws.get(f"dyp{li}", (Mp, cin), torch.float32, dev)
                conv_gemm(CONV_DX, Mp, cin, cout * 9, dY, P[cname + ".weight"], dYp, cout, sbk=K9, sbn=9,
                          gate=ys[li - 1], ldg=cin, ws=self.ws, tag="bw_")
                dY = dYp
                continue
            gemm(cout, K9, Mp, dY, 1, cout, cols[li], K9, 1, grads[cname + ".weight"], K9, pr, ws=self.ws, tag="bw_")
            colsum(dY, Mp, cout, grads[cname + ".bias"], scratch)
            if li == 0:
                break
            dcol = ws.get(f"dcol{li}", (Mp, K9), torch.float32, dev)
            gemm(Mp, K9, cout, dY, cout, 1, P[cname + ".weight"], K9, 1, dcol, K9, pr, ws=self.ws, tag="bw_")
            dx = ws.get(f"dx{li}", (B, cin * 121), torch.float32, dev)
            qcheck(L.evx_col2im3x3(_p(dcol), B, cin, _p(dx), _stream()), "col2im")
            dYp = ws.get(f"dyp{li}", (Mp, cin), torch.float32, dev)
            qcheck(L.evx_pix_nchw(_p(dx), B, cin, 0, _p(dYp), _stream()), "pix_nchw")
            qcheck(L.evx_relu_grad(_p(dYp), _p(ys[li - 1]), dYp.numel(), _stream()), "relu_grad")
            dY = dYp


class Learner:
    """Online + target networks, fused clip+Adam, TD loss: DQNAgent.learn on the device."""

    def __init__(self, kind="mlp", device="cuda", lr=1e-4, gamma=0.99, max_norm=1.0, precision="f32",
                 hidden=512, actions=5, seed=0, betas=(0.9, 0.999), eps=1e-8):
        if precision not in ("f32", "bf16", "x3", "exact"):
            raise ValueError(f"precision must be 'f32', 'bf16', 'x3' or 'exact', not {precision!r}")
        # "exact": every product on the exact-f32 MFMA GEMMs (evx_gemm f32), no fused MLP kernels
        fused_ok = precision != "exact"
        precision = "f32" if precision == "exact" else precision
        self.kind, self.device = kind, torch.device(device)
        self.shapes = param_shapes(layer_specs(kind, hidden, actions))
        self.online = FlatParams(self.shapes, self.device)
        self.online.init_like_torch(seed)
        self.target = FlatParams(self.shapes, self.device)
        self.target.flat.copy_(self.online.flat)
        self.grads = FlatParams(self.shapes, self.device)
        self.m = torch.zeros_like(self.online.flat)
        self.v = torch.zeros_like(self.online.flat)
        self.adam_step = 0
        self.lr, self.gamma, self.max_norm, self.betas, self.eps = lr, gamma, max_norm, betas, eps
        self.hidden, self.actions, self.precision = hidden, actions, precision
        self.net = QNet(kind, self.online, precision, hidden, actions)
        self.tnet = QNet(kind, self.target, precision, hidden, actions)
        self.norm = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.loss = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.scratch = torch.zeros(2048, dtype=torch.float32, device=self.device)
        self.seed = seed
        self.rng_offset = 0
        self.grad_hook = None  # e.g. an all-reduce over the flat grad buffer
        # MLP: the fused kernels of csrc/qmlp.hip (forward from compact observations); f32 runs
        # them in the x3 (f32-accurate) mode, bf16 with bf16 operands. The dense-tensor path
        # (forward / learn on expanded observations) keeps evx_gemm at `precision`.
        self.fast = self.fast_t = None
        if fused_ok and kind == "mlp" and hidden == 512 and actions == 5:
            from .qmlp import MLPFast
            self.fast = MLPFast(self.online, self.device, x3=precision != "bf16")
            self.fast_t = MLPFast(self.target, self.device, x3=precision != "bf16")
        self.drop_stream = 0
        # x3 MLP: the TD step inside the backward, the norm partials out of its reductions, clip +
        # Adam + operand repack in one launch (fused_opt = False: the separate td_loss / backward /
        # sumsq / clip_adam / pack3 launches -- tests compare the two)
        self.fused_opt = self.fast is not None and self.fast.x3
        if self.fused_opt:
            from .qmlp import mlib
            assert self.online.numel == int(mlib().evx_qmlp_nparams()), "MLP parameter count"
        self._ss = torch.zeros(1024, dtype=torch.float32, device=self.device)
        self._ss_fresh = False

    # ------------------------------------------------------------ dropout
    def dropout_mask(self, B, tag="m"):
        m = self.net.ws.get("mask_" + tag, (B, self.hidden), torch.uint8, self.device)
        qcheck(qlib().evx_dropout_mask(_p(m), m.numel(), DROPOUT_P, self.seed, self.rng_offset, _stream()),
               "dropout_mask")
        self.rng_offset += (m.numel() + 3) // 4
        return m

    def q_values(self, x, train=True, mask=None, target=False, tag: str = "act"):
        """tag names this call's scratch (activations, split-K partials, packed weights, dropout
        mask): forwards that may run concurrently on different streams need different tags."""
        B = x.shape[0]
        if mask is None and train:
            mask = self.dropout_mask(B, tag)
        net = self.tnet if target else self.net
        return net.forward(x, mask if train else None, save=False, tag=tag + "_")

    def learn(self, s, a, r, done, s2, mask_online=None, mask_target=None, weights=None, td_abs=None):
        """One DQNAgent.learn step on device tensors; returns the loss tensor (no host sync).
        weights / td_abs: prioritized replay's importance weights in, |TD error| out."""
        B = s.shape[0]
        if mask_online is None:
            mask_online = self.dropout_mask(B, "on")
        if mask_target is None:
            mask_target = self.dropout_mask(B, "tg")
        Q = self.net.forward(s, mask_online, save=True)
        Qt = self.tnet.forward(s2, mask_target, save=False, tag="t_")
        dQ = self.net.ws.get("dq", (B, self.actions), torch.float32, self.device)
        L = qlib()
        tw = td_workspace(self.net.ws, B, 1, self.device)
        qcheck(L.evx_td_loss_w(_p(Q), _p(Qt), self.actions, _p(a), _p(r), _p(done), self.gamma, B, _p(weights),
                               _p(dQ), _p(self.loss), _p(td_abs), _p(tw), tw.numel(), _stream()), "td_loss")
        self.net.backward(dQ, self.grads)
        if self.grad_hook is not None:
            self.grad_hook(self.grads.flat)
        self.step_optimizer()
        return self.loss

    def learn_obs(self, lay_c, s_obs, a, r, done, s2_obs, B, update: bool = True, weights=None, td_abs=None,
                  mask_online=None, mask_target=None, drop_row0: int = 0):
        """DQNAgent.learn on compact observations with the fused kernels (x3 = f32-accurate,
        or bf16): online forward (saves X, H1, H2), target forward, TD loss, backward,
        clip+Adam. update=False stops after the gradients (the caller runs step_optimizer
        later). mask_online / mask_target: explicit uint8 [B][512] dropout keep masks (tests:
        the reference's captured torch masks) in place of the hash."""
        from .qmlp import HID, HID2
        for name, t in (("s_obs", s_obs), ("s2_obs", s2_obs)):  # evx_obs rows are 8 words
            if t.numel() < B * 8:
                raise ValueError(f"learn_obs: {name} holds {t.numel() // 8} observations, B = {B}")
        ws, dev = self.net.ws, self.device
        pl, kx = self.fast.planes, self.fast.kx

        def buf(name, per_row, dt):
            return ws.get(name, (B * per_row,), dt, dev)
        X = buf("fx", kx, torch.int16)
        H1 = buf("fh1", pl * HID, torch.int16)
        H2 = buf("fh2", HID2, torch.float32).view(B, HID2)
        Q = buf("fq", self.actions, torch.float32).view(B, self.actions)
        H1t = buf("fh1t", pl * HID, torch.int16)
        Qt = buf("fqt", self.actions, torch.float32).view(B, self.actions)
        dQ = buf("fdq", self.actions, torch.float32).view(B, self.actions)
        dz2 = buf("fdz2", pl * HID2, torch.int16)
        dz1 = buf("fdz1", pl * HID, torch.int16)
        self.drop_stream += 2
        # drop_row0 (even): the dropout hash rows start there (evacx.qgroup keys net g's batch rows g * B + i)
        d_on = (self.seed, self.drop_stream, DROPOUT_P, mask_online, drop_row0)
        d_tg = (self.seed, self.drop_stream + 1, DROPOUT_P, mask_target, drop_row0)
        type(self.fast).forward_pair(lay_c, B, self.fast, s_obs, d_on, dict(h1=H1, x=X, h2=H2, q=Q), self.fast_t,
                                     s2_obs, d_tg, dict(h1=H1t, q=Qt))
        L = qlib()
        if self.fused_opt:
            # the TD step inside the backward's first kernel, the gradients overwritten by its ordered
            # reductions, which also leave the norm partials unless an all-reduce will change the gradients
            self.fast.td_backward(B, Q, Qt, a, r, done, self.gamma, self.loss, X, H1, H2, DROPOUT_P, dz2, dz1,
                                  self.grads, weights=weights, td_abs=td_abs,
                                  ss=self._ss if self.grad_hook is None else None)
            self._ss_fresh = self.grad_hook is None
        else:
            tw = td_workspace(ws, B, 1, dev)
            qcheck(L.evx_td_loss_w(_p(Q), _p(Qt), self.actions, _p(a), _p(r), _p(done), self.gamma, B, _p(weights),
                                   _p(dQ), _p(self.loss), _p(td_abs), _p(tw), tw.numel(), _stream()), "td_loss")
            self.fast.backward(B, dQ, X, H1, H2, DROPOUT_P, dz2, dz1, self.grads)
        if self.grad_hook is not None:
            self.grad_hook(self.grads.flat)
        if update:
            self.step_optimizer()
        return self.loss

    def step_optimizer(self):
        L = qlib()
        n = self.online.numel
        if self.fused_opt:  # clip + Adam + x3 repack in one launch from the norm partials
            if not self._ss_fresh:
                self.fast.sumsq_parts(self.grads.flat, self._ss)
            self._ss_fresh = False
            self.adam_step += 1
            h = evx_adam(lr=self.lr, beta1=self.betas[0], beta2=self.betas[1], eps=self.eps, weight_decay=0.0,
                         step=self.adam_step)
            self.fast.adam_step(self.online.flat, self.grads.flat, self.m, self.v, float(self.max_norm or 0.0), h,
                                self._ss, self.norm)
            return
        qcheck(L.evx_sumsq_norm(_p(self.grads.flat), n, _p(self.scratch), self.scratch.numel(), _p(self.norm),
                                _stream()), "sumsq")
        self.adam_step += 1
        h = evx_adam(lr=self.lr, beta1=self.betas[0], beta2=self.betas[1], eps=self.eps, weight_decay=0.0,
                     step=self.adam_step)
        qcheck(L.evx_clip_adam(_p(self.online.flat), _p(self.grads.flat), _p(self.m), _p(self.v), n,
                               _p(self.norm) if self.max_norm else None, float(self.max_norm or 0.0), C.byref(h),
                               _stream()), "clip_adam")
        if self.fast is not None:
            self.fast.repack()  # bf16 copies follow the fp32 master parameters

    def m_view(self, name: str) -> torch.Tensor:
        """Adam first moment of one parameter (torch's optimizer.state[p]["exp_avg"])."""
        return FlatParams(self.shapes, self.device, data=self.m)[name]

    def v_view(self, name: str) -> torch.Tensor:
        """Adam second moment of one parameter (torch's optimizer.state[p]["exp_avg_sq"])."""
        return FlatParams(self.shapes, self.device, data=self.v)[name]

    def sync_target(self):
        """DQNAgent.update_target_network (agents/dqn_agent.py:170-172)."""
        self.target.flat.copy_(self.online.flat)
        if self.fast_t is not None:
            self.fast_t.repack()

    def weights_written(self, target: bool = False):
        """Call after writing a network's fp32 parameters from outside the learner (a
        load_state_dict, a broadcast from another rank): the fused kernels read operand copies
        (bf16 hi / lo tiles) and, once attach_static ran, a per-centre act table of fc1 --
        the learner's online forward reads that table too -- and those are rebuilt only
        here, in sync_target and in the optimizer step."""
        fast = self.fast_t if target else self.fast
        if fast is not None:
            fast.repack()
