"""VITS stochastic duration predictor, inference direction (noise -> log
durations), for checkpoints that carry one (the public VITS / MMS-TTS
models; the random-init benchmark voice uses the deterministic predictor in
``vits.py``).

The predictor is a normalising flow over two channels conditioned on the
text encoder's hidden states (Kim et al., "Conditional Variational
Autoencoder with Adversarial Learning for End-to-End Text-to-Speech", 2021):

  cond  = proj(DDSConv(pre(h)))                       filter channels
  flows = [elementwise affine, conv flow x n]          forward order
  infer: z ~ N(0, noise_scale^2) over [B, 2, T]; for each flow in reverse
         order (the first conv flow skipped, as the published models do):
         flip channels, invert the flow; log w = channel 0

DDSConv: n layers of (depthwise conv, dilation k^i -> LayerNorm over channels
-> GELU -> 1x1 conv -> LayerNorm -> GELU), each added to its input. A conv
flow keeps channel 0 and maps channel 1 through a monotone rational-quadratic
spline on [-tail, tail] (identity outside) whose K bin widths, K heights and
K-1 inner knot slopes are predicted from channel 0 by a DDSConv stack
(Durkan et al., "Neural Spline Flows", 2019); the inverse solves the bin's
quadratic in closed form.

All of it runs at the phrase's symbol count (tens to hundreds of steps), so
it is plain fp32 tensor work; it is captured with the rest of the text phase
in the VITS graph runner.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

MIN_BIN_WIDTH = 1e-3
MIN_BIN_HEIGHT = 1e-3
MIN_DERIVATIVE = 1e-3


def _ln_channels(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """LayerNorm over the channel dim of a [B, C, T] tensor."""
    return F.layer_norm(x.transpose(1, 2), (x.shape[1],), w, b, eps).transpose(1, 2)


def dds_conv(x: torch.Tensor, mask: torch.Tensor, p: dict, kernel: int,
             cond: torch.Tensor | None = None) -> torch.Tensor:
    """Dilated depth-separable conv stack; x [B, C, T], mask [B, 1, T]."""
    if cond is not None:
        x = x + cond
    C = x.shape[1]
    for i, layer in enumerate(p["layers"]):
        dil = kernel ** i
        pad = (kernel * dil - dil) // 2
        y = F.conv1d(x * mask, layer["dw_w"], layer["dw_b"], padding=pad, dilation=dil, groups=C)
        y = F.gelu(_ln_channels(y, layer["n1_w"], layer["n1_b"]))
        y = F.conv1d(y, layer["pw_w"], layer["pw_b"])
        y = F.gelu(_ln_channels(y, layer["n2_w"], layer["n2_b"]))
        x = x + y
    return x * mask


def rq_spline_inverse(y: torch.Tensor, uw: torch.Tensor, uh: torch.Tensor, ud: torch.Tensor,
                      tail: float) -> torch.Tensor:
    """Inverse of the monotone rational-quadratic spline on [-tail, tail]
    (identity outside, unit slope at both ends). y [...]; uw, uh [..., K]
    unnormalised bin widths / heights; ud [..., K - 1] unnormalised inner
    knot slopes."""
    inside = (y >= -tail) & (y <= tail)
    K = uw.shape[-1]
    # boundary slopes of exactly 1: softplus(c) + min = 1
    c = math.log(math.exp(1.0 - MIN_DERIVATIVE) - 1.0)
    ud = F.pad(ud, (1, 1), value=c)
    widths = MIN_BIN_WIDTH + (1 - MIN_BIN_WIDTH * K) * torch.softmax(uw, -1)
    cw = F.pad(torch.cumsum(widths, -1), (1, 0), value=0.0) * (2 * tail) - tail
    cw[..., 0], cw[..., -1] = -tail, tail
    widths = cw[..., 1:] - cw[..., :-1]
    deriv = MIN_DERIVATIVE + F.softplus(ud)
    heights = MIN_BIN_HEIGHT + (1 - MIN_BIN_HEIGHT * K) * torch.softmax(uh, -1)
    ch = F.pad(torch.cumsum(heights, -1), (1, 0), value=0.0) * (2 * tail) - tail
    ch[..., 0], ch[..., -1] = -tail, tail
    heights = ch[..., 1:] - ch[..., :-1]
    yc = y.clamp(-tail, tail)
    # bin of each output value: the last knot with cumheight <= y
    edges = ch.clone()
    edges[..., -1] += 1e-6
    idx = (yc[..., None] >= edges).sum(-1, keepdim=True) - 1
    idx = idx.clamp(0, K - 1)
    g = lambda t: t.gather(-1, idx)[..., 0]     # noqa: E731
    x_k, w_k, y_k, h_k = g(cw[..., :-1]), g(widths), g(ch[..., :-1]), g(heights)
    d_k = g(deriv[..., :-1])
    d_k1 = g(deriv[..., 1:])
    s_k = h_k / w_k
    dy = yc - y_k
    # solve a xi^2 + b xi + c = 0 for the bin-relative position xi in [0, 1]
    a = dy * (d_k + d_k1 - 2 * s_k) + h_k * (s_k - d_k)
    b = h_k * d_k - dy * (d_k + d_k1 - 2 * s_k)
    cc = -s_k * dy
    disc = (b * b - 4 * a * cc).clamp_min(0.0)
    xi = (2 * cc) / (-b - torch.sqrt(disc))
    x = xi * w_k + x_k
    return torch.where(inside, x, y)


class StochasticDurationPredictor:
    """Inference-only stochastic duration predictor from checkpoint tensors
    (``p``: see ``loader.vits_from_state_dict``)."""

    def __init__(self, p: dict, *, kernel: int = 3, bins: int = 10, tail: float = 5.0):
        self.p, self.kernel, self.bins, self.tail = p, kernel, bins, tail

    def log_durations(self, h: torch.Tensor, mask: torch.Tensor, noise: torch.Tensor,
                      cond: torch.Tensor | None = None) -> torch.Tensor:
        """h [B, T, H] text hidden states, mask [B, T] bool, noise [B, 2, T]
        (already scaled by the noise scale), cond [B, H] (multi-speaker: the
        projected speaker vector, added after the input conv) -> log
        durations [B, T]."""
        p, k = self.p, self.kernel
        m = mask[:, None, :].float()
        x = h.float().transpose(1, 2)
        x = F.conv1d(x, p["pre_w"], p["pre_b"])
        if cond is not None:
            x = x + cond[:, :, None]
        x = dds_conv(x, m, p["dds"], k)
        cond = F.conv1d(x, p["proj_w"], p["proj_b"]) * m
        z = noise.float() * m
        flows = p["flows"]               # [affine, conv flow 1 .. n]
        # reverse order, the first conv flow skipped (the published models'
        # inference path drops it)
        for fl in list(reversed(flows[1:]))[:-1] + [flows[0]]:
            z = z.flip(1)
            if fl["kind"] == "affine":
                z = (z - fl["translate"][None]) * torch.exp(-fl["log_scale"][None]) * m
            else:
                z = self._conv_flow_inverse(z, m, cond, fl)
        return z[:, 0]

    def _conv_flow_inverse(self, z, m, cond, fl):
        k, K = self.kernel, self.bins
        x0, x1 = z[:, :1], z[:, 1:]
        h = F.conv1d(x0, fl["pre_w"], fl["pre_b"])
        h = dds_conv(h, m, fl["dds"], k, cond=cond)
        h = F.conv1d(h, fl["proj_w"], fl["proj_b"]) * m              # [B, 3K - 1, T]
        B, _, T = h.shape
        h = h.view(B, 1, 3 * K - 1, T).permute(0, 1, 3, 2)            # [B, 1, T, 3K - 1]
        fc = fl["pre_w"].shape[0]
        uw = h[..., :K] / math.sqrt(fc)
        uh = h[..., K:2 * K] / math.sqrt(fc)
        ud = h[..., 2 * K:]
        x1 = rq_spline_inverse(x1, uw, uh, ud, self.tail)
        return torch.cat([x0, x1], 1) * m
