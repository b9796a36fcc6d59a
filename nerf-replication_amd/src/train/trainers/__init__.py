from .make_trainer import make_trainer  # noqa: F401
