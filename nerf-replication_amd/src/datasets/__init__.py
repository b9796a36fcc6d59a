from .make_dataset import make_data_loader  # noqa: F401
