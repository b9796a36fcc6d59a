from .config import args, cfg  # noqa: F401
