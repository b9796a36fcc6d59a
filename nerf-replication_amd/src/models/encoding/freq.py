"""Frequency positional encoding (reference: src/models/encoding/freq.py:7-32).

out = [x, sin(2^0 x), cos(2^0 x), ..., sin(2^{L-1} x), cos(2^{L-1} x)], L = num_freqs.
The training/rendering path never calls this: the same features are generated inside the
fused MLP kernel (csrc/mlp.hip, pe_tile) directly in MFMA operand layout.
"""
import torch


class Encoder:
    def __init__(self, include_input=True, input_dims=3, max_freq_log2=9, num_freqs=10, log_sampling=True):
        self.include_input = include_input
        self.input_dims = input_dims
        if log_sampling:
            self.freq_bands = 2.0 ** torch.linspace(0.0, max_freq_log2, steps=num_freqs)
        else:
            self.freq_bands = torch.linspace(1.0, 2.0 ** max_freq_log2, steps=num_freqs)
        self.out_dim = input_dims * (int(include_input) + 2 * num_freqs)

    def embed(self, x):
        parts = [x] if self.include_input else []
        for f in self.freq_bands.tolist():
            parts += [torch.sin(x * f), torch.cos(x * f)]
        return torch.cat(parts, -1)
