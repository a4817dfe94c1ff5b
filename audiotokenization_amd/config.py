"""Hydra/OmegaConf-free config loading for the codec (the reference drivers re-read
`<save_path>/hydra/config.yaml` with OmegaConf, extract_indices.py:437 / inference_full.py:540).

Only `model.codec_encoder.*` and `model.codec_decoder.*` shape the hot path
(lightning_module.py:87-139); the rest of the file is carried through untouched."""
from __future__ import annotations

import os
from typing import Any, Mapping

import yaml


class AttrDict(dict):
    """dict with attribute access (enough of OmegaConf's DictConfig for the codec constructors)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    @staticmethod
    def wrap(obj: Any) -> Any:
        if isinstance(obj, Mapping):
            return AttrDict({k: AttrDict.wrap(v) for k, v in obj.items()})
        if isinstance(obj, list):
            return [AttrDict.wrap(v) for v in obj]
        return obj


def load_config(path: str) -> AttrDict:
    with open(path) as fh:
        return AttrDict.wrap(yaml.safe_load(fh))


def load_model_yaml(path: str) -> AttrDict:
    """A bare config/model/*.yaml (codec_encoder / codec_decoder / mpd / mstft) wrapped as cfg.model."""
    with open(path) as fh:
        model = yaml.safe_load(fh)
    return AttrDict.wrap({"model": model})


ENCODER_KEYS = ("ngf", "use_rnn", "rnn_bidirectional", "rnn_num_layers", "up_ratios", "dilations",
                "out_channels", "causal", "antialias")
DECODER_KEYS = ("in_channels", "upsample_initial_channel", "ngf", "use_rnn", "rnn_bidirectional",
                "rnn_num_layers", "up_ratios", "dilations", "causal", "antialias", "fsq", "fsq_levels",
                "vq_num_quantizers", "vq_commit_weight", "vq_full_commit_loss", "codebook_size",
                "codebook_dim")


def encoder_kwargs(enccfg: Mapping) -> dict:
    """lightning_module.py:89-99."""
    if enccfg.get("type", "bigcodec") != "bigcodec":
        raise NotImplementedError(f"codec encoder type {enccfg.get('type')!r} is out of scope (BigCodec only)")
    return {k: enccfg[k] for k in ENCODER_KEYS}


def decoder_kwargs(deccfg: Mapping) -> dict:
    """lightning_module.py:124-139 (note: the reference does not forward vq_weight_init)."""
    if deccfg.get("type", "bigcodec") != "bigcodec":
        raise NotImplementedError(f"codec decoder type {deccfg.get('type')!r} is out of scope (BigCodec only)")
    return {k: deccfg[k] for k in DECODER_KEYS}


# Model presets found in the reference configs.
PRESETS = {
    # config/model/default.yaml:1-32 (BigCodec paper, 159 M)
    "default": {
        "codec_encoder": dict(type="bigcodec", out_channels=1024, ngf=48, use_rnn=True, rnn_bidirectional=False,
                              rnn_num_layers=2, up_ratios=[2, 2, 2, 5, 5], dilations=[1, 3, 9], causal=False,
                              antialias=False),
        "codec_decoder": dict(type="bigcodec", in_channels=1024, upsample_initial_channel=1536, ngf=48, use_rnn=True,
                              rnn_bidirectional=False, rnn_num_layers=2, up_ratios=[5, 5, 2, 2, 2], dilations=[1, 3, 9],
                              causal=False, antialias=False, vq_num_quantizers=1, vq_commit_weight=0.25,
                              vq_weight_init=False, vq_full_commit_loss=False, fsq=False, fsq_levels=[4, 4, 4, 8],
                              codebook_size=8192, codebook_dim=8),
    },
    # cfgs/config8/model/base.yaml:1-31
    "base": {
        "codec_encoder": dict(type="bigcodec", out_channels=512, ngf=32, use_rnn=True, rnn_bidirectional=False,
                              rnn_num_layers=2, up_ratios=[2, 4, 5, 5], dilations=[1, 3, 9], causal=False,
                              antialias=False),
        "codec_decoder": dict(type="bigcodec", in_channels=512, upsample_initial_channel=512, ngf=32, use_rnn=True,
                              rnn_bidirectional=False, rnn_num_layers=2, up_ratios=[5, 5, 4, 2], dilations=[1, 3, 9],
                              causal=False, antialias=False, vq_num_quantizers=1, vq_commit_weight=0.25,
                              vq_weight_init=False, vq_full_commit_loss=False, fsq=False, fsq_levels=[4, 4, 4, 8],
                              codebook_size=8192, codebook_dim=8),
    },
    # config/model/debug.yaml:1-31 (what config/default.yaml:4 selects)
    "debug": {
        "codec_encoder": dict(type="bigcodec", out_channels=512, ngf=16, use_rnn=False, rnn_bidirectional=False,
                              rnn_num_layers=1, up_ratios=[2, 2, 4, 4, 5], dilations=[1, 3, 9], causal=False,
                              antialias=False),
        "codec_decoder": dict(type="bigcodec", in_channels=512, upsample_initial_channel=512, ngf=16, use_rnn=True,
                              rnn_bidirectional=False, rnn_num_layers=1, up_ratios=[5, 4, 4, 2, 2], dilations=[1, 3, 9],
                              causal=False, antialias=False, vq_num_quantizers=1, vq_commit_weight=0.25,
                              vq_weight_init=False, vq_full_commit_loss=False, fsq=False, fsq_levels=[4, 4, 4, 8],
                              codebook_size=8192, codebook_dim=8),
    },
}


def preset(name: str, **overrides) -> AttrDict:
    """cfg with cfg.model.codec_encoder / codec_decoder of a named preset; overrides apply to both
    (e.g. causal=True, antialias=True)."""
    p = {k: dict(v) for k, v in PRESETS[name].items()}
    for sec in p.values():
        for k, v in overrides.items():
            if k in sec:
                sec[k] = v
    return AttrDict.wrap({"model": p})


def find_checkpoint(save_path: str):
    """extract_indices.py:437-448: (config_path, ckpt_path or None)."""
    config_path = os.path.join(save_path, "hydra/config.yaml")
    for option in (os.path.join(save_path, "pl_log/last.ckpt"), os.path.join(save_path, "checkpoints/last.ckpt"),
                   os.path.join(save_path, "pl_log/checkpoints/last.ckpt"), os.path.join(save_path, "last.ckpt")):
        if os.path.exists(option):
            return config_path, option
    return config_path, None
