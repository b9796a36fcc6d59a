"""make_renderer (reference: src/models/nerf/renderer/make_renderer.py:4-8)."""
from src.models.make_network import load_source


def make_renderer(cfg, network):
    return load_source(cfg.renderer_module, cfg.renderer_path).Renderer(network)
