"""Encoder factory with the reference's interface (src/models/encoding/__init__.py:6-18).

Only the "frequency" encoder is on the lego path.  On the hot path the encoding is fused
into the first MLP layer of the gfx950 kernel; ``get_encoder`` still returns the
(callable, out_dim) pair the reference exposes as ``Network.embed_fn`` / ``input_ch``.
"""
from .freq import Encoder as FreqEncoder


def get_encoder(cfg):
    if cfg.type != "frequency":
        raise NotImplementedError(f"encoder {cfg.type!r} is not on the lego hot path (only 'frequency')")
    enc = FreqEncoder(include_input=True, input_dims=cfg.input_dim, max_freq_log2=cfg.freq - 1,
                      num_freqs=cfg.freq, log_sampling=True)
    return enc.embed, enc.out_dim
