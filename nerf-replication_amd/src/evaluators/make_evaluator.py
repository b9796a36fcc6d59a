"""make_evaluator (reference: src/evaluators/make_evaluator.py:5-15)."""
from src.models.make_network import load_source


def make_evaluator(cfg):
    if cfg.skip_eval:
        return None
    return load_source(cfg.evaluator_module, cfg.evaluator_path).Evaluator()
