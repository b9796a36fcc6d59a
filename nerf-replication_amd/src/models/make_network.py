"""make_network (reference: src/models/make_network.py:4-8): load cfg.network_path's
``Network`` through importlib (imp.load_source is gone in Python >= 3.12)."""
import importlib.util
import os
import sys


def load_source(module: str, path: str):
    if module in sys.modules and getattr(sys.modules[module], "__file__", None) and \
            os.path.abspath(sys.modules[module].__file__) == os.path.abspath(path):
        return sys.modules[module]
    if not os.path.exists(path):
        # resolve relative to the package root when not run from it
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        alt = os.path.join(root, path)
        path = alt if os.path.exists(alt) else path
    try:
        return importlib.import_module(module)
    except ImportError:
        spec = importlib.util.spec_from_file_location(module, path)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[module] = mod
        spec.loader.exec_module(mod)
        return mod


def make_network(cfg):
    return load_source(cfg.network_module, cfg.network_path).Network()
