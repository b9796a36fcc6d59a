"""make_data_loader (reference: src/datasets/make_dataset.py:73-100).

Batches are produced on the GPU by the dataset itself (ray generation kernel), so the
"loader" is a plain iterator: ``max_iter`` random ray batches per epoch for training
(IterationBasedBatchSampler's role), one batch per image for testing.  There are no
worker processes, pinned host buffers or H2D copies on the training path.
"""
from src.models.make_network import load_source


class BatchLoader:
    def __init__(self, dataset, n_batches):
        self.dataset = dataset
        self.n = n_batches

    def __len__(self):
        return self.n

    def __iter__(self):
        for i in range(self.n):
            yield self.dataset[i]


def make_dataset(cfg, is_train=True):
    if is_train:
        module, path, kw = cfg.train_dataset_module, cfg.train_dataset_path, cfg.train_dataset
    else:
        module, path, kw = cfg.test_dataset_module, cfg.test_dataset_path, cfg.test_dataset
    return load_source(module, path).Dataset(**kw)


def make_data_loader(cfg, is_train=True, is_distributed=False, max_iter=-1):
    ds = make_dataset(cfg, is_train)
    if is_train:
        return BatchLoader(ds, max_iter if max_iter > 0 else cfg.ep_iter)
    return BatchLoader(ds, len(ds))
