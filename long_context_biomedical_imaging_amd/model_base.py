"""EncoderDecoderModel — drop-in for /root/reference/model/model_base.py (:18-83)."""
from __future__ import annotations

import torch.nn as nn

from .backbone_swin import custom_Swin
from .backbone_vit import ViT_with_alt_ops, custom_ViT
from .decoders import Identity, SwinLinear, SwinUNETR, UperNet2D, UperNet3D, ViTLinear, ViTUNETR


def identity_model(config, input_feature_channels):
    return Identity(), input_feature_channels


class EncoderDecoderModel(nn.Module):
    def __init__(self, config, encoder_name, decoder_name, input_feature_channels, output_feature_channels):
        super().__init__()
        self.config = config
        self.encoder_name = encoder_name
        self.decoder_name = decoder_name
        self.input_feature_channels = input_feature_channels
        self.output_feature_channels = output_feature_channels
        if encoder_name == "Identity":
            self.encoder, self.encoder_feature_channels = identity_model(config, input_feature_channels)
        elif encoder_name == "ViT":
            self.encoder, self.encoder_feature_channels = custom_ViT(config, input_feature_channels)
        elif encoder_name == "Swin":
            self.encoder, self.encoder_feature_channels = custom_Swin(config, input_feature_channels)
        else:
            raise NotImplementedError(f"Encoder not implemented: {encoder_name}")
        if decoder_name == "Identity":
            self.decoder, _ = identity_model(config, self.encoder_feature_channels)
        elif decoder_name == "ViTLinear":
            self.decoder = ViTLinear(config, self.encoder_feature_channels, output_feature_channels)
        elif decoder_name == "SwinLinear":
            self.decoder = SwinLinear(config, self.encoder_feature_channels, output_feature_channels)
        elif decoder_name == "ViTUNETR":
            self.decoder = ViTUNETR(config, self.encoder_feature_channels, output_feature_channels)
        elif decoder_name == "SwinUNETR":
            self.decoder = SwinUNETR(config, self.encoder_feature_channels, output_feature_channels)
        elif decoder_name == "UperNet2D":
            self.decoder = UperNet2D(config, self.encoder_feature_channels, output_feature_channels)
        elif decoder_name == "UperNet3D":
            self.decoder = UperNet3D(config, self.encoder_feature_channels, output_feature_channels)
        else:
            raise NotImplementedError(f"Decoder not implemented: {decoder_name}")
        # the encoder's hidden states this decoder reads (besides the input and the final output): the ViT encoder
        # is asked for those only (forward(x, keep_hidden=...): no sum kept alive only for the list); the argument
        # is passed per call, so the encoder called on its own still returns every hidden state
        taps = getattr(self.decoder, "hidden_taps", None)
        self._keep_hidden = frozenset(taps) if taps is not None and isinstance(self.encoder, ViT_with_alt_ops) \
            else None

    @property
    def device(self):
        return next(self.parameters()).device

    def forward(self, x):
        if self._keep_hidden is not None:
            return self.decoder(self.encoder(x, keep_hidden=self._keep_hidden))
        return self.decoder(self.encoder(x))
