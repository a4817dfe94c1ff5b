"""CodecLightningModule-compatible inference shell (lightning_module.py:75-285).

It exposes every shape of the drop-in contract the reference callers use:
  * `.encoder`, `.decoder`, `.inference(wav)`            lightning_module.py:90,121,280-285
  * `.model['CodecEnc']`, `.model['generator']`           extract_indices.py:353-355, inference_full.py:558-559
    (`model` is a property, so it adds no duplicate state_dict keys and strict loading works)
  * `.encode(x)`, `.quantize(latent)` (5-tuple, codes at [1]), `.decode(z_q)`   extract_indices.py:361-363
Checkpoints: a Lightning dict with 'state_dict' (or 'model'), or a bare state_dict; keys of the
training-only submodules (discriminator., spec_discriminator., criteria., semantic heads) are ignored.
"""
from __future__ import annotations

from typing import Mapping

import torch
import torch.nn as nn

from .codec import BigCodecDecoder, BigCodecEncoder
from .config import AttrDict, decoder_kwargs, encoder_kwargs

_KEEP = ("encoder.", "decoder.")


class CodecLightningModule(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = AttrDict.wrap(cfg)
        self.construct_model()

    def construct_model(self):
        self.encoder = BigCodecEncoder(**encoder_kwargs(self.cfg.model.codec_encoder))
        self.decoder = BigCodecDecoder(**decoder_kwargs(self.cfg.model.codec_decoder))

    @property
    def model(self):
        return {"CodecEnc": self.encoder, "generator": self.decoder}

    # --- checkpoint handling ----------------------------------------------------------------------
    @staticmethod
    def codec_state_dict(checkpoint: Mapping) -> dict:
        if "state_dict" in checkpoint:
            sd = checkpoint["state_dict"]
        elif "model" in checkpoint:
            sd = checkpoint["model"]
        else:
            sd = checkpoint
        return {k: v for k, v in sd.items() if k.startswith(_KEEP)}

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        return super().load_state_dict(self.codec_state_dict(state_dict), strict=strict, assign=assign)

    @classmethod
    def from_checkpoint(cls, ckpt_path: str, cfg, map_location="cpu"):
        """torch.load with weights_only=True (a Lightning .ckpt of tensors and primitives loads)."""
        ckpt = torch.load(ckpt_path, map_location=map_location, weights_only=True)
        m = cls(cfg)
        m.load_state_dict(ckpt, strict=True)
        return m.eval()

    # --- inference surface ------------------------------------------------------------------------
    @torch.inference_mode()
    def inference(self, wav):
        vq_emb = self.encoder(wav.unsqueeze(1))
        vq_post_emb, vq_code, vq_loss = self.decoder(vq_emb, vq=True)
        return self.decoder(vq_post_emb, vq=False).squeeze(1)

    def forward(self, batch):
        wav = batch["wav"]
        vq_emb = self.encoder(wav.unsqueeze(1))
        vq_post_emb, vq_code, vq_loss = self.decoder(vq_emb, vq=True)
        y_ = self.decoder(vq_post_emb, vq=False)
        return {"gt_wav": wav.unsqueeze(1), "gen_wav": y_, "vq_loss": vq_loss, "vq_code": vq_code}

    def encode(self, x):
        return self.encoder(x)

    def quantize(self, latent):
        """(post_emb, codes (Nq,B,F), losses (Nq,), z_e-free placeholder, None) — codes at [1]."""
        post, codes, loss = self.decoder(latent, vq=True)
        return post, codes, loss, None, None

    def decode(self, z_q):
        return self.decoder(z_q, vq=False)
