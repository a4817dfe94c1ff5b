"""Causal streaming encode and decode: a causal BigCodecEncoder (causal=True,
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

StreamingDecoder is the same for a causal BigCodecDecoder (vq/codec_decoder.py:15-94 with causal=True): latent
frames in, waveform out.  Its upsamplers are CausalConvTranspose1d (vq/module.py:50-57: ConvTranspose1d with
k = 2s, stride s, no padding, the last s outputs cropped), so output block t depends on input frames t and t - 1:
each carries its last input frame and runs the chunk over [frame | chunk] with padding s (which drops the s
outputs of the carried frame's own block on the left and the k - s look-ahead outputs on the right).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from audiotokenization_amd import _lib
from audiotokenization_amd import ops
from audiotokenization_amd.blocks import DecoderBlock, EncoderBlock, ResLSTM, _conv_of
from audiotokenization_amd.conv import CausalConvTranspose1d, ConvTranspose1dWN
from audiotokenization_amd.modules import _as_input


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


class StreamingDecoder(StreamingEncoder):
    """Wraps a causal BigCodecDecoder; `push(z (B, D, n))` (post-VQ embeddings, n frames) returns the waveform
    (B, 1, n * hop) of the chunk, equal to the whole-sequence causal decode of the concatenated frames.
    `tokens(codes (B, n, Nq) int64 device)` pushes a chunk of index frames (vq2emb first, codec_decoder.py:96-99).
    The carried state: every causal conv's input context, every upsampler's last input frame, the ResLSTM's
    (h, c)."""

    def __init__(self, decoder):
        convs = [m for m in decoder.modules() if hasattr(m, "causal_pad")]
        if not convs or any(m.causal_pad is None and (m.kernel_size > 1 or m.padding) for m in convs):
            raise ValueError("streaming needs a causal decoder (causal=True)")
        if any(isinstance(m, ConvTranspose1dWN) and not m.causal_crop for m in decoder.modules()):
            raise ValueError("streaming needs a causal decoder (causal=True): its upsamplers must be causal")
        if any(getattr(m, "antialias", False) for m in decoder.modules()):
            raise NotImplementedError("anti-aliased activations look ahead: not streamable")
        self.decoder = decoder
        self.hop = int(decoder.hop_length)
        self.reset()

    def _convT(self, wrapper, xa, out_snake=None):
        conv = wrapper.conv if isinstance(wrapper, CausalConvTranspose1d) else wrapper
        s, K = conv.stride, conv.kernel_size
        if K % s:
            raise NotImplementedError(f"streaming transposed conv needs kernel_size % stride == 0 (k={K}, s={s})")
        c = K // s - 1  # input frames of history an output block needs
        x = xa
        if c:
            ctx = self._ctx.get(id(conv))
            if ctx is None:
                ctx = torch.zeros((xa.shape[0], xa.shape[1], c), device=xa.device, dtype=torch.float32)
            x = torch.cat([ctx, xa], dim=2)
            self._ctx[id(conv)] = x[:, :, -c:].contiguous()
        phases, _, bias, cfg = conv.prepared(x.device)
        sa, sb = out_snake if out_snake is not None else (None, None)
        # full length (n + c - 1) s + K; padding c * s crops c * s on both sides: the n * s outputs of this chunk
        out = ops.load().conv_transpose1d(x, phases, bias, sa, sb, conv.out_channels, xa.shape[-1] * s, K, s, c * s,
                                          cfg, False)
        return out[0]

    def push(self, z) -> torch.Tensor:
        with _lib.status_scope():
            return self._push_dec(z)

    def tokens(self, codes) -> torch.Tensor:
        """codes (B, n, Nq) int64 on the device -> waveform chunk (B, 1, n * hop)."""
        return self.push(self.decoder.tokens_to_latent(codes))

    def _push_dec(self, z) -> torch.Tensor:
        z = _as_input(z)
        m = list(self.decoder.model)
        final_act, last_conv = m[-3], m[-2]
        h = self._conv(m[0], z)
        for st in m[1:-3]:
            if isinstance(st, ResLSTM):
                h = self._lstm_run(st, h)
            elif isinstance(st, DecoderBlock):
                sub = list(st.block)
                h = self._convT(sub[1], sub[0](h))
                for ru in sub[2:]:  # ResidualUnit: x + conv1(act2(conv7(act1(x))))
                    t = self._conv(ru.block[1], ru.block[0](h))
                    h = self._conv(ru.block[3], ru.block[2](t), residual=h)
            else:
                raise NotImplementedError(f"unexpected decoder stage {type(st).__name__}")
        self.samples += z.shape[-1] * self.hop
        out = self._conv_tanh(last_conv, final_act(h))
        _lib.check_status()
        return out

    def _conv_tanh(self, wrapper, xa):
        """The last conv with the decoder's nn.Tanh fused in its epilogue (codec_decoder.py:80)."""
        c = _conv_of(wrapper)
        P = c.pad_left()
        ctx = self._ctx.get(id(c))
        if ctx is None:
            ctx = torch.zeros((xa.shape[0], xa.shape[1], P), device=xa.device, dtype=torch.float32)
        xin = torch.cat([ctx, xa], dim=2)
        self._ctx[id(c)] = xin[:, :, -P:].contiguous()
        return c.run(xin, None, 1, pad_left=0)

    def decode(self, z, chunk: int) -> torch.Tensor:
        """Whole latent sequence through `push` in chunks of `chunk` frames (the last may be shorter)."""
        self.reset()
        outs = [self.push(z[..., i:i + chunk]) for i in range(0, z.shape[-1], chunk)]
        return torch.cat(outs, dim=2)
