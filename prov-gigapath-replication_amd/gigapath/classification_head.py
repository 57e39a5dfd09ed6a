"""Slide-level classifier over selected layer embeddings -- the slide encoder's caller in the
reference's fine-tuning and prediction code (reference gigapath/classification_head.py:18-92,
used by finetune/training.py and finetune/predict.py).

Same constructor and forward as the reference: ``feat_layer`` names the layer embeddings
(``all_layer_embed=True`` outputs, 0 = the input embedding, i = after layer i) that are
concatenated and fed to one ``nn.Linear``.  The MI355X slide encoder is inference-only, so the
encoder is always frozen here (its parameters get ``requires_grad=False`` and it stays in
eval mode); the linear classifier trains normally on its outputs.
"""
from __future__ import annotations

import torch
from torch import nn

from . import slide_encoder


def reshape_input(imgs, coords, pad_mask=None):
    """Drop a leading singleton dim of [1, B, N, D] / [1, B, N, 2] inputs (reference :7-15)."""
    if imgs.dim() == 4:
        imgs = imgs.squeeze(0)
    if coords.dim() == 4:
        coords = coords.squeeze(0)
    if pad_mask is not None and pad_mask.dim() != 2:
        pad_mask = pad_mask.squeeze(0)
    return imgs, coords, pad_mask


class ClassificationHead(nn.Module):
    def __init__(self, input_dim, latent_dim, feat_layer, n_classes=2, model_arch="gigapath_slide_enc12l768d",
                 pretrained="hf_hub:prov-gigapath/prov-gigapath", freeze=False, **kwargs):
        super().__init__()
        self.feat_layer = [int(x) for x in str(feat_layer).split("-")]
        self.feat_dim = len(self.feat_layer) * latent_dim
        self.slide_encoder = slide_encoder.create_model(pretrained, model_arch, in_chans=input_dim, **kwargs)
        if not freeze:
            print("MI355X slide encoder is inference-only: freezing it (the classifier still trains)")
        for p in self.slide_encoder.parameters():
            p.requires_grad = False
        self.slide_encoder.eval()
        self.classifier = nn.Sequential(nn.Linear(self.feat_dim, n_classes))

    def train(self, mode: bool = True):
        super().train(mode)
        self.slide_encoder.eval()            # the encoder never leaves eval mode
        return self

    def forward(self, images: torch.Tensor, coords: torch.Tensor) -> torch.Tensor:
        """images [B, N, D] (or [N, D]), coords [B, N, 2] -> logits [B, n_classes]."""
        if images.dim() == 2:
            images = images.unsqueeze(0)
        if coords.dim() == 2:
            coords = coords.unsqueeze(0)
        if images.dim() != 3:
            raise ValueError("images must be [B, N, D], got %s" % (tuple(images.shape),))
        with torch.no_grad():
            embeds = self.slide_encoder(images, coords, all_layer_embed=True)
        feats = torch.cat([embeds[i] for i in self.feat_layer], dim=-1)
        feats = feats.to(self.classifier[0].weight.dtype)
        return self.classifier(feats.reshape(-1, feats.size(-1)))


def get_model(**kwargs):
    return ClassificationHead(**kwargs)
