"""Embedding layers of spotlight/layers.py (reference :30-56): the initialisers
that fix the MF tables' starting point (N(0, 1/d) weights, zero biases)."""
import torch.nn as nn


class ScaledEmbedding(nn.Embedding):
    """nn.Embedding initialised to N(0, std = 1 / embedding_dim)."""

    def reset_parameters(self):
        self.weight.data.normal_(0, 1.0 / self.embedding_dim)
        if self.padding_idx is not None:
            self.weight.data[self.padding_idx].fill_(0)


class ZeroEmbedding(nn.Embedding):
    """nn.Embedding initialised to zero (biases)."""

    def reset_parameters(self):
        self.weight.data.zero_()
        if self.padding_idx is not None:
            self.weight.data[self.padding_idx].fill_(0)
