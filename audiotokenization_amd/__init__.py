"""audiotokenization_amd — the BigCodec audio-tokenization hot path of hoyso48/AudioTokenization,
rebuilt for AMD Instinct MI355X (gfx950): hand-written HIP kernels in libbigcodec_hip.so behind the
reference's own module interface.

    from audiotokenization_amd import BigCodecEncoder, BigCodecDecoder, CodecLightningModule
"""
from . import _lib  # noqa: F401
from .codec import BigCodecDecoder, BigCodecEncoder
from .config import AttrDict, load_config, preset
from .lightning_shim import CodecLightningModule
from .blocks import DecoderBlock, EncoderBlock, ResidualUnit, ResLSTM
from .conv import WNConv1d, WNConvTranspose1d
from .modules import Activation1d, FactorizedVectorQuantize, ResidualVQ, SnakeBeta

__all__ = [
    "BigCodecEncoder", "BigCodecDecoder", "CodecLightningModule", "AttrDict", "load_config", "preset",
    "Activation1d", "DecoderBlock", "EncoderBlock", "FactorizedVectorQuantize", "ResidualUnit", "ResidualVQ",
    "ResLSTM", "SnakeBeta",
]
__version__ = "0.1.0"
