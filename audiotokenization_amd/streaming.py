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
The carried contexts live on the device and every step of the state is one bc_stream_window launch: it writes the
[context | chunk] window (with the stage's Snake applied on the way) and the next context in one pass.  A
ResidualUnit the one-launch kernel serves (bc_resunit_fwd_snake_in: C = 48 / 96 in h3, x6, bf16) runs as ONE
launch over its raw window with its own causal padding: output column P + t sees window columns t … P + t, all
real samples, and its residual is the window's own column P + t; the first P = 6d outputs are dropped by taking the
view [P:] (no copy: the next window reads the strided view).  Other units run conv7 (Snake epilogue) and conv1
(residual add) over their activated window.  No torch compute kernel runs in a push.

StreamingDecoder is the same for a causal BigCodecDecoder (vq/codec_decoder.py:15-94 with causal=True): latent
frames in, waveform out.  Its upsamplers are CausalConvTranspose1d (vq/module.py:50-57: ConvTranspose1d with
k = 2s, stride s, no padding, the last s outputs cropped), so output block t depends on input frames t and t - 1:
each carries its last input frame and runs the chunk over [frame | chunk] with padding s (which drops the s
outputs of the carried frame's own block on the left and the k - s look-ahead outputs on the right).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import _lib
from . import ops
from .blocks import DecoderBlock, EncoderBlock, ResLSTM, _conv_of
from .conv import CausalConvTranspose1d, ConvTranspose1dWN
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
        # the precision the carried state belongs to: the fused and the two-launch ResidualUnit paths keep different
        # context (raw input vs activated input), and which one runs depends on the mode
        self._mode = _lib.precision_mode()

    def _check_mode(self):
        if _lib.precision_mode() != self._mode:
            raise RuntimeError(f"precision changed mid-stream ({self._mode} -> {_lib.precision_mode()}): the carried "
                               "context belongs to the old mode; reset() the stream first")

    def _window(self, key, x, P: int, act=None):
        """[carried context | x] (B, C, P + n), `act` (a Snake Activation1d or None) applied to x, as the input of a
        stage with P columns of causal history; the last P columns become the next chunk's context."""
        sa, sb = act.act.coeffs(x.device) if act is not None else (None, None)
        win, nctx = ops.load().stream_window(x, self._ctx.get(key) if P else None, sa, sb, P)
        if P:
            self._ctx[key] = nctx
        return win

    def _conv(self, wrapper, x, act=None, residual=None, out_snake=None, epilogue: int = 0):
        """A causal conv over [context | act(x)] with no padding: exactly the chunk's outputs."""
        c = _conv_of(wrapper)
        P = c.pad_left()
        if P == 0 and act is None and x.is_contiguous():
            return c.run(x, residual, epilogue, out_snake)
        return c.run(self._window(id(c), x, P, act), residual, epilogue, out_snake, pad_left=0)

    def _dense(self, h):
        """A contiguous copy of a strided chunk view (one launch), for the ops that take dense tensors."""
        return h if h.is_contiguous() else self._window(None, h, 0)

    def _unit(self, ru, h):
        """One ResidualUnit on a chunk: x + conv1(act2(conv7(act1(x)))) (vq/module.py:74-89)."""
        cfg = ru._fused_cfg()
        conv7 = _conv_of(ru.block[1])
        if cfg >= 0 and ru.snake_on_load():
            P = conv7.pad_left()  # 6d: the unit's whole history
            win = self._window(("ru", id(ru)), h, P)
            y = ru._flow_fused(cfg, win, None, True, None)[0]
            return y[:, :, P:]
        t = self._conv(ru.block[1], h, act=ru.block[0], out_snake=ru.block[2].act.coeffs(h.device))
        return self._conv(ru.block[3], t, residual=self._dense(h))

    def _lstm_run(self, m: ResLSTM, h):
        y, state = m.run(h, state=self._lstm.get(id(m)), return_state=True)
        self._lstm[id(m)] = state
        return y

    def push(self, x) -> torch.Tensor:
        self._check_mode()
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
                for ru in sub[:-2]:
                    h = self._unit(ru, h)
                h = self._conv(sub[-1], h, act=sub[-2])
            elif isinstance(st, ResLSTM):
                h = self._lstm_run(st, h)
            else:
                raise NotImplementedError(f"unexpected encoder stage {type(st).__name__}")
        self.samples += x.shape[-1]
        out = self._conv(last_conv, h, act=final_act)
        _lib.check_status()
        return out

    def graph(self, example) -> "StreamGraph":
        """This stream's push for chunks shaped like `example`, captured once in a HIP graph (StreamGraph)."""
        return StreamGraph(self, example)

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

    def _convT(self, wrapper, h, act):
        conv = wrapper.conv if isinstance(wrapper, CausalConvTranspose1d) else wrapper
        s, K = conv.stride, conv.kernel_size
        if K % s:
            raise NotImplementedError(f"streaming transposed conv needs kernel_size % stride == 0 (k={K}, s={s})")
        c = K // s - 1  # input frames of history an output block needs
        x = self._window(id(conv), h, c, act)
        phases, _, bias, cfg = conv.prepared(x.device, conv.phase_cfg(x.shape[0], x.shape[-1]))
        # full length (n + c - 1) s + K; padding c * s crops c * s on both sides: the n * s outputs of this chunk
        out = ops.load().conv_transpose1d(x, phases, bias, None, None, conv.out_channels, h.shape[-1] * s, K, s, c * s,
                                          cfg, False)
        return out[0]

    def push(self, z) -> torch.Tensor:
        self._check_mode()
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
                h = self._convT(sub[1], h, sub[0])
                for ru in sub[2:]:
                    h = self._unit(ru, h)
            else:
                raise NotImplementedError(f"unexpected decoder stage {type(st).__name__}")
        self.samples += z.shape[-1] * self.hop
        out = self._conv(last_conv, h, act=final_act, epilogue=1)  # the decoder's nn.Tanh in the epilogue
        _lib.check_status()
        return out

    def decode(self, z, chunk: int) -> torch.Tensor:
        """Whole latent sequence through `push` in chunks of `chunk` frames (the last may be shorter)."""
        self.reset()
        outs = [self.push(z[..., i:i + chunk]) for i in range(0, z.shape[-1], chunk)]
        return torch.cat(outs, dim=2)


class StreamGraph:
    """One push of a fixed chunk shape captured in a HIP graph (torch.cuda.CUDAGraph: hipStreamBeginCapture /
    hipGraphLaunch on ROCm) and replayed per chunk: the dozens of launches of a push (a window, a conv or a
    one-launch ResidualUnit per stage, the persistent ResLSTM) go to the device as ONE graph launch, so a stream
    of short chunks is no longer bound by host-side dispatch.  The carried state lives in static buffers: the
    graph reads them, its stages write the next state into graph-owned tensors, and the graph's last nodes copy
    those back into the static buffers.  The stream's current state is taken over at capture (the warm-up push
    that sizes every buffer is undone), and the stream continues from the graph's state afterwards.

    push(x) copies x into the static input, replays, and returns the graph's static output (overwritten by the next
    push: copy it to keep it).  check=True (the default) reads the ResLSTM status words after the replay (one
    host wait, as StreamingEncoder.push does); check=False skips it and check() reads them later.  The
    results equal the eager stream's bit for bit (tests/test_gpu_streaming.py)."""

    def __init__(self, stream: StreamingEncoder, example):
        example = _as_input(example)
        self.stream = stream
        self.input = example.clone()
        # one eager push sizes every carried state and warms the weight caches; then the state before it returns
        ctx0 = {k: v.clone() for k, v in stream._ctx.items()}
        lstm0 = {k: tuple(t.clone() for t in v) for k, v in stream._lstm.items()}
        samples0 = stream.samples
        with torch.no_grad():
            stream.push(self.input)
        self._ctx = {k: (ctx0[k] if k in ctx0 else torch.zeros_like(v)) for k, v in stream._ctx.items()}
        self._lstm = {k: (lstm0[k] if k in lstm0 else tuple(torch.zeros_like(t) for t in v))
                      for k, v in stream._lstm.items()}
        stream._ctx, stream._lstm, stream.samples = dict(self._ctx), dict(self._lstm), samples0
        torch.cuda.synchronize()
        self._graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), _lib.deferred_status() as ticket:
            with torch.cuda.graph(self._graph):
                self.output = stream.push(self.input)
                for k, v in stream._ctx.items():
                    self._ctx[k].copy_(v)
                for k, v in stream._lstm.items():
                    for dst, src in zip(self._lstm[k], v):
                        dst.copy_(src)
        self._status = ticket.items  # the graph's own status words, rewritten by every replay
        stream._ctx, stream._lstm, stream.samples = dict(self._ctx), dict(self._lstm), samples0
        self._n = example.shape[-1] * (stream.hop if isinstance(stream, StreamingDecoder) else 1)

    def push(self, x, check: bool = True) -> torch.Tensor:
        if tuple(x.shape) != tuple(self.input.shape):
            raise ValueError(f"this graph was captured for chunks of shape {tuple(self.input.shape)}, got {tuple(x.shape)}")
        self.input.copy_(x)
        self._graph.replay()
        self.stream.samples += self._n
        if check:
            self.check()
        return self.output

    def reset(self) -> None:
        """Start a new stream on this graph: the static state back to zeros (a fresh stream's context)."""
        for v in self._ctx.values():
            v.zero_()
        for v in self._lstm.values():
            for t in v:
                t.zero_()
        self.stream._ctx, self.stream._lstm, self.stream.samples = dict(self._ctx), dict(self._lstm), 0

    def check(self) -> None:
        """Raise BigCodecLibraryError if the last replay's persistent ResLSTM reported a failure (host wait)."""
        if self._status:
            _lib._raise_bad(self._status, torch.cat([t.reshape(-1) for t, _ in self._status]).cpu().tolist())
