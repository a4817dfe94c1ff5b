"""BigCodecEncoder / BigCodecDecoder (vq/codec_encoder.py:14-90, vq/codec_decoder.py:15-142) on the
HIP kernels, with the reference's constructor signatures, state_dict keys and call surface.

forward() runs the whole stack as one fused flow (blocks.py): every Snake is computed once in
the epilogue of the kernel producing its input, the ResLSTM writes the final Snake directly, and
the decoder's tanh is the last conv's epilogue."""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .blocks import DecoderBlock, EncoderBlock, ResLSTM, input_act, produce_conv
from .conv import WNConv1d
from .modules import FSQ, Activation1d, ResidualVQ, SnakeBeta, _as_input, _zeros


class _Tanh(nn.Module):
    """nn.Tanh (codec_decoder.py:80).  decode() runs it fused in the last conv's epilogue; called on its
    own (decoder.model used as the reference's nn.Sequential) it is bc_tanh_fwd."""

    def forward(self, x):
        return ops.load().tanh(_as_input(x))


class BigCodecEncoder(nn.Module):
    """vq/codec_encoder.py:14-90.  forward(x (B,1,T) f32 device) -> (B, out_channels, T/hop)."""

    def __init__(self, ngf=48, use_rnn=True, rnn_bidirectional=False, causal=False, antialias=False,
                 rnn_num_layers=2, up_ratios=(2, 2, 2, 5, 5), dilations=(1, 3, 9), out_channels=1024):
        super().__init__()
        self.hop_length = np.prod(up_ratios)
        self.ngf = ngf
        self.up_ratios = up_ratios
        if causal:
            assert not rnn_bidirectional
        d_model = ngf
        block = [WNConv1d(1, d_model, kernel_size=7, padding=3, causal=causal)]
        for stride in up_ratios:
            d_model *= 2
            block += [EncoderBlock(d_model, stride=stride, dilations=dilations, causal=causal, antialias=antialias)]
        if use_rnn:
            block += [ResLSTM(d_model, num_layers=rnn_num_layers, bidirectional=rnn_bidirectional)]
        block += [
            Activation1d(activation=SnakeBeta(d_model, alpha_logscale=True), antialias=antialias),
            WNConv1d(d_model, out_channels, kernel_size=3, padding=1, causal=causal),
        ]
        self.block = nn.Sequential(*block)
        self.enc_dim = d_model

    def forward(self, x):
        with L.status_scope():
            return self._forward(x)

    def _forward(self, x):
        x = _as_input(x)
        blk = list(self.block)
        final_act, last_conv = blk[-2], blk[-1]
        stages = blk[1:-2]  # EncoderBlocks [+ ResLSTM]
        # consumer activation of each stage's output
        def next_act_of(i):
            if i + 1 < len(stages):
                nxt = stages[i + 1]
                return input_act(nxt) if isinstance(nxt, EncoderBlock) else None  # ResLSTM takes raw
            return final_act
        y, ya = produce_conv(blk[0], x, None, want_raw=True, next_act=next_act_of(-1) if stages else final_act)
        for i, st in enumerate(stages):
            nact = next_act_of(i)
            want_raw = i + 1 < len(stages)  # the next stage needs the raw tensor (RU skip / LSTM input)
            if isinstance(st, EncoderBlock):
                y, ya = st.flow(y, ya, want_raw=want_raw, next_act=nact)
            else:
                y, ya = st.flow(y, want_raw=want_raw, next_act=nact)
        out = produce_conv(last_conv, ya, None, want_raw=True, next_act=None)[0]
        L.check_status()  # a failed persistent ResLSTM launch raises here, before the latent is used
        return out

    def inference(self, x):
        return self.forward(x)

    def remove_weight_norm(self):
        for m in self.modules():
            if m is not self and "weight_v" in m._parameters and hasattr(m, "remove_weight_norm"):
                m.remove_weight_norm()


class BigCodecDecoder(nn.Module):
    """vq/codec_decoder.py:15-142.  forward(x, vq=True) -> (z_q, codes (Nq,B,F), losses (Nq,));
    forward(x, vq=False) -> waveform (B, 1, T)."""

    def __init__(self, in_channels=1024, upsample_initial_channel=1536, ngf=48, use_rnn=True,
                 rnn_bidirectional=False, rnn_num_layers=2, up_ratios=(5, 5, 2, 2, 2), dilations=(1, 3, 9),
                 causal=False, antialias=False, fsq=False, fsq_levels=[4, 4, 4, 8], vq_num_quantizers=1,
                 vq_commit_weight=0.25, vq_weight_init=False, vq_full_commit_loss=False, codebook_size=8192,
                 codebook_dim=8):
        super().__init__()
        self.hop_length = np.prod(up_ratios)
        self.ngf = ngf
        self.up_ratios = up_ratios
        self.fsq = fsq
        if fsq:  # codec_decoder.py:41-47
            self.quantizer = FSQ(levels=fsq_levels, channel_first=True, dim=in_channels)
            assert codebook_size == np.prod(fsq_levels), "codebook_size must be equal to the product of fsq_levels"
        else:
            self.quantizer = ResidualVQ(num_quantizers=vq_num_quantizers, dim=in_channels,
                                        codebook_size=codebook_size, codebook_dim=codebook_dim,
                                        threshold_ema_dead_code=2, commitment=vq_commit_weight,
                                        weight_init=vq_weight_init, full_commit_loss=vq_full_commit_loss)
        channels = upsample_initial_channel
        layers = [WNConv1d(in_channels, channels, kernel_size=7, padding=3, causal=causal)]
        if use_rnn:
            layers += [ResLSTM(channels, num_layers=rnn_num_layers, bidirectional=rnn_bidirectional)]
        output_dim = channels
        for i, stride in enumerate(up_ratios):
            input_dim = channels // 2 ** i
            output_dim = channels // 2 ** (i + 1)
            layers += [DecoderBlock(input_dim, output_dim, stride, dilations, causal=causal, antialias=antialias)]
        layers += [
            Activation1d(activation=SnakeBeta(output_dim, alpha_logscale=True), antialias=antialias),
            WNConv1d(output_dim, 1, kernel_size=7, padding=3, causal=causal),
            _Tanh(),
        ]
        self.model = nn.Sequential(*layers)

    def decode(self, x):
        """self.model(x): fused flow; final Snake in the producer of the last conv's input, tanh in
        the last conv's epilogue."""
        with L.status_scope():
            return self._decode(x)

    def _decode(self, x):
        x = _as_input(x)
        m = list(self.model)
        final_act, last_conv = m[-3], m[-2]
        stages = m[1:-3]  # [ResLSTM] + DecoderBlocks

        def next_act_of(i):
            if i + 1 < len(stages):
                nxt = stages[i + 1]
                return nxt.first_act if isinstance(nxt, DecoderBlock) else None
            return final_act
        first_next = next_act_of(-1) if stages else final_act
        y, ya = produce_conv(m[0], x, None, want_raw=first_next is None, next_act=first_next)
        for i, st in enumerate(stages):
            nact = next_act_of(i)
            want_raw = nact is None
            if isinstance(st, DecoderBlock):
                y, ya = st.flow(y, ya, want_raw=want_raw, next_act=nact)
            else:
                y, ya = st.flow(y, want_raw=want_raw, next_act=nact)
        out = produce_conv(last_conv, ya, None, want_raw=True, next_act=None, epilogue=1)[0]
        L.check_status()
        return out

    def forward(self, x, vq=True):
        if vq is True:
            if self.fsq:  # codec_decoder.py:87-89
                x, q = self.quantizer(x)
                return x, q, _zeros(x.shape[0], x.device)
            return self.quantizer(x)
        return self.decode(x)

    def vq2emb(self, vq):
        self.quantizer = self.quantizer.eval()
        return self.quantizer.vq2emb(vq)

    def get_emb(self):
        self.quantizer = self.quantizer.eval()
        return self.quantizer.get_emb()

    def tokens_to_audio(self, vq):
        """Token -> audio: codes (B, T, Nq) int64 on the device (extract_indices' (F, Nq) files, batched)
        -> waveform (B, 1, T * hop): vq2emb (codec_decoder.py:96-99) -> transpose(1, 2) -> self(x, vq=False),
        with the embedding written straight in the decoder's (B, D, T) layout (bc_vq2emb_ct).  fsq=True decoders
        (whose vq2emb raises AttributeError in the reference: FSQ has none) take one index column through
        FSQ.indices_to_codes (finite_scalar_quantization.py:176-192, bc_fsq_codes), then the same decode."""
        return self.decode(self.tokens_to_latent(vq))

    def tokens_to_latent(self, vq):
        """codes (B, T, Nq) on the device -> the decoder's input (B, D, T) (see tokens_to_audio)."""
        if self.fsq:
            if vq.dim() != 3 or vq.shape[2] != 1:
                raise ValueError(f"an fsq=True decoder takes (B, T, 1) indices, got {tuple(vq.shape)}")
            return self.quantizer.indices_to_codes(vq[:, :, 0])
        return self.quantizer.vq2emb_ct(vq)

    def inference_vq(self, vq):
        return self.decode(vq[None, :, :])

    def inference_0(self, x):
        x, q, loss = self.quantizer(x)
        return self.decode(x), None

    def inference(self, x):
        return self.decode(x), None

    def remove_weight_norm(self):
        for m in self.modules():
            if m is not self and "weight_v" in m._parameters and hasattr(m, "remove_weight_norm"):
                m.remove_weight_norm()
