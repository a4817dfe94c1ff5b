"""Causal streaming encode: a causal BigCodecEncoder (causal=True,
vq/module.py:11-48 CausalConv1d, left padding (K - stride) * dilation) fed chunk by chunk, with the
state a chunk boundary cuts carried on the device:

  * every causal conv keeps the last (K - stride) * dilation samples of its (activated) input and runs
    the next chunk over [context | chunk] with no padding, so each output sample sees exactly the
    inputs it sees in a whole-sequence pass;
  * the ResLSTM carries nn.LSTM's (h, c) per layer through bc_reslstm_fwd_state (the persistent kernel
    starts from the carried state and hands back the final one).

The reference has no streaming mode; its whole-sequence causal encoder defines the result: the
concatenation of the chunks' latents equals the encoder's output on the concatenated audio (bit for
bit in the exact-split x6 precision; in h3 the per-tile block scales differ between the two tilings, so
the outputs agree to fp32 rounding).  Chunks must be a multiple of the hop (prod(up_ratios)) samples.
Anti-aliased activations are not causal (act.py / resample.py look ahead), so antialias=True is refused.
Inside a chunk the ResidualUnits run as two conv launches (the one-launch kernel keeps input and output
lengths equal), and the carried contexts are prepended with torch.cat on the device.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import _lib
from .blocks import EncoderBlock, ResLSTM, _conv_of
from .modules import _as_input


class StreamingEncoder:
    """Wraps a causal BigCodecEncoder; `push(x (B, 1, n))` returns the latents (B, D, n / hop) of the
    chunk.  `reset()` starts a new stream.  The batch size is fixed per stream."""

    def __init__(self, encoder):
        convs = [m for m in encoder.modules() if hasattr(m, "causal_pad")]
        # every conv that looks at more than one input sample must be causal (the ResidualUnits' k=1
        # convs are plain, padding 0, in the reference too)
        if not convs or any(m.causal_pad is None and (m.kernel_size > 1 or m.padding) for m in convs):
            raise ValueError("streaming needs a causal encoder (causal=True)")
        if any(getattr(m, "antialias", False) for m in encoder.modules()):
            raise NotImplementedError("anti-aliased activations look ahead: not streamable")
        self.encoder = encoder
        self.hop = int(encoder.hop_length)
        self.reset()

    def reset(self):
        self._ctx: Dict[int, torch.Tensor] = {}
        self._lstm: Dict[int, tuple] = {}
        self.samples = 0

    def _conv(self, wrapper, xa, residual=None):
        c = _conv_of(wrapper)
        P = c.pad_left()
        if P == 0:
            return c.run(xa, residual)
        ctx = self._ctx.get(id(c))
        if ctx is None:
            ctx = torch.zeros((xa.shape[0], xa.shape[1], P), device=xa.device, dtype=torch.float32)
        xin = torch.cat([ctx, xa], dim=2)
        self._ctx[id(c)] = xin[:, :, -P:].contiguous()
        return c.run(xin, residual, pad_left=0)

    def _lstm_run(self, m: ResLSTM, h):
        y, state = m.run(h, state=self._lstm.get(id(m)), return_state=True)
        self._lstm[id(m)] = state
        return y

    def push(self, x) -> torch.Tensor:
        with _lib.status_scope():
            return self._push(x)

    def _push(self, x) -> torch.Tensor:
        x = _as_input(x)
        if x.shape[-1] % self.hop:
            raise ValueError(f"chunk of {x.shape[-1]} samples: must be a multiple of the hop ({self.hop})")
        blk = list(self.encoder.block)
        final_act, last_conv = blk[-2], blk[-1]
        h = self._conv(blk[0], x)
        for st in blk[1:-2]:
            if isinstance(st, EncoderBlock):
                sub = list(st.block)
                for ru in sub[:-2]:  # ResidualUnit: x + conv1(act2(conv7(act1(x))))
                    t = self._conv(ru.block[1], ru.block[0](h))
                    h = self._conv(ru.block[3], ru.block[2](t), residual=h)
                h = self._conv(sub[-1], sub[-2](h))
            elif isinstance(st, ResLSTM):
                h = self._lstm_run(st, h)
            else:
                raise NotImplementedError(f"unexpected encoder stage {type(st).__name__}")
        self.samples += x.shape[-1]
        out = self._conv(last_conv, final_act(h))
        _lib.check_status()
        return out

    def encode(self, x, chunk: int) -> torch.Tensor:
        """Whole input through `push` in chunks of `chunk` samples (the last may be shorter)."""
        self.reset()
        outs = [self.push(x[..., i:i + chunk]) for i in range(0, x.shape[-1], chunk)]
        return torch.cat(outs, dim=2)
