"""Configuration with the reference's interface (src/config/config.py:8-209).

``from src.config import cfg, args`` yields the merged configuration; like the reference,
the command line (``--cfg_file``, ``--type``, ``--test``, ``--local_rank``, trailing
``key value`` overrides) is parsed at import time -- with ``parse_known_args`` so that
foreign argv (pytest, bench.py) does not break the import.  ``*_module`` strings become
``*_path`` file paths (config.py:172-174), which ``make_*`` load with importlib (the
reference's ``imp`` is gone in Python 3.12).

The CfgNode here is a small dict-backed node (attribute access, new keys allowed,
yaml merge, ``merge_from_list`` with literal values) -- the subset of yacs the hot path
and its entry points use.
"""
from __future__ import annotations

import argparse
import ast
import copy
import os

import yaml

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class CfgNode(dict):
    def __init__(self, init=None):
        super().__init__()
        for k, v in (init or {}).items():
            self[k] = self._wrap(v)

    @classmethod
    def _wrap(cls, v):
        return cls(v) if isinstance(v, dict) and not isinstance(v, CfgNode) else v

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name)

    def __setattr__(self, name, value):
        self[name] = self._wrap(value)

    def __deepcopy__(self, memo):
        return CfgNode({k: copy.deepcopy(v, memo) for k, v in self.items()})

    def clone(self):
        return copy.deepcopy(self)

    def merge_from_other_cfg(self, other):
        for k, v in other.items():
            if isinstance(v, dict) and isinstance(self.get(k), dict):
                self[k].merge_from_other_cfg(CfgNode._wrap(v))
            else:
                self[k] = self._wrap(copy.deepcopy(v))

    def merge_from_file(self, path):
        with open(path, "r") as f:
            self.merge_from_other_cfg(load_yaml(f))

    def merge_from_list(self, opts):
        if not opts:
            return
        if len(opts) % 2:
            raise ValueError(f"override list needs key/value pairs: {opts}")
        for key, val in zip(opts[0::2], opts[1::2]):
            node = self
            parts = key.split(".")
            for p in parts[:-1]:
                if p not in node:
                    node[p] = CfgNode()
                node = node[p]
            node[parts[-1]] = self._wrap(_decode(val))

    def dump(self):
        def plain(x):
            return {k: plain(v) for k, v in x.items()} if isinstance(x, dict) else x
        return yaml.safe_dump(plain(self))


def _decode_tree(x):
    """yacs decodes string leaves with literal_eval (so '5e-4' is a float)."""
    if isinstance(x, dict):
        return {k: _decode_tree(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_decode_tree(v) for v in x]
    return _decode(x)


def load_yaml(f) -> "CfgNode":
    return CfgNode(_decode_tree(yaml.safe_load(f) or {}))


def _decode(v):
    if not isinstance(v, str):
        return v
    try:
        return ast.literal_eval(v)
    except (ValueError, SyntaxError):
        return v


def default_cfg() -> CfgNode:
    """Defaults the hot path reads (config.py:8-131 subset + this build's knobs)."""
    return CfgNode({
        "task": "nerf_replication", "gpus": [0], "exp_name": "nerf", "exp_name_tag": "", "scene": "lego",
        "pretrain": "", "distributed": False, "resume": True, "fix_random": False, "skip_eval": False,
        "ep_iter": 500, "save_ep": 40, "save_latest_ep": 10, "eval_ep": 10, "log_interval": 10,
        "trained_model_dir": "data/trained_model", "trained_config_dir": "data/trained_config",
        "record_dir": "data/record", "result_dir": "data/result", "save_tag": "default",
        "task_arg": {},
        "train": {"epoch": 600, "num_workers": 0, "batch_size": 1, "lr": 5e-4, "weight_decay": 0.0,
                  "eps": 1e-8, "optim": "adam", "shuffle": True,
                  "scheduler": {"type": "exponential", "gamma": 0.1, "decay_epochs": 500}},
        "test": {"batch_size": 1, "epoch": -1},
        "eval": {"whole_img": True},
    })


def parse_cfg(cfg: CfgNode, args) -> None:
    """Directories and module paths (config.py:134-174); gpus are applied by the entry
    points (apply_gpus), not at import, so torchrun ranks keep their own devices."""
    if len(cfg.exp_name_tag) != 0:
        cfg.exp_name += "_" + cfg.exp_name_tag
    cfg.trained_model_dir = os.path.join(cfg.trained_model_dir, cfg.task, cfg.scene, cfg.exp_name)
    cfg.trained_config_dir = os.path.join(cfg.trained_config_dir, cfg.task, cfg.scene, cfg.exp_name)
    cfg.record_dir = os.path.join(cfg.record_dir, cfg.task, cfg.scene, cfg.exp_name)
    cfg.result_dir = os.path.join(cfg.result_dir, cfg.task, cfg.scene, cfg.exp_name, cfg.save_tag)
    cfg.local_rank = args.local_rank
    for key in [k for k in cfg if k.endswith("_module")]:
        cfg[key.replace("_module", "_path")] = cfg[key].replace(".", "/") + ".py"


def apply_gpus(cfg: CfgNode) -> None:
    """config.py:139-141 -- set CUDA_VISIBLE_DEVICES from cfg.gpus (single-process runs)."""
    if "LOCAL_RANK" in os.environ or "CUDA_VISIBLE_DEVICES" in os.environ:
        return
    if -1 not in cfg.gpus:
        os.environ["CUDA_VISIBLE_DEVICES"] = ", ".join(str(g) for g in cfg.gpus)


def resolve_cfg_file(path: str) -> str:
    if os.path.exists(path):
        return path
    alt = os.path.join(PKG_ROOT, path)
    if os.path.exists(alt):
        return alt
    raise FileNotFoundError(path)


def make_cfg(args) -> CfgNode:
    def merge(path, node):
        path = resolve_cfg_file(path)
        with open(path, "r") as f:
            cur = load_yaml(f)
        if "parent_cfg" in cur:
            node = merge(cur.parent_cfg, node)
        node.merge_from_other_cfg(cur)
        return node

    c = merge(args.cfg_file, default_cfg())
    opts = list(args.opts or [])
    if "other_opts" in opts:
        opts = opts[:opts.index("other_opts")]
    c.merge_from_list(opts)
    parse_cfg(c, args)
    return c


parser = argparse.ArgumentParser(add_help=False)
parser.add_argument("--cfg_file", default="configs/nerf/lego.yaml", type=str)
parser.add_argument("--test", action="store_true", dest="test", default=False)
parser.add_argument("--type", type=str, default="")
parser.add_argument("--det", type=str, default="")
parser.add_argument("--local_rank", type=int, default=0)
parser.add_argument("opts", default=None, nargs=argparse.REMAINDER)


def _parse_argv():
    # library use (bench.py, tests) sets NERF_AMD_NO_ARGV=1: defaults, argv untouched
    argv = [] if os.environ.get("NERF_AMD_NO_ARGV") else None
    a, _unknown = parser.parse_known_args(argv)
    opts = a.opts or []
    # keep only well-formed "key value" overrides (foreign argv such as pytest's is ignored)
    if len(opts) % 2 or any(str(o).startswith("-") for o in opts[0::2]):
        a.opts = []
    return a


args = _parse_argv()
try:
    cfg = make_cfg(args)
except FileNotFoundError:
    args.cfg_file = "configs/nerf/lego.yaml"
    args.opts = []
    cfg = make_cfg(args)
if len(args.type) > 0:
    cfg.task = "run" if cfg.get("task", "") == "" else cfg.task
