"""CPU: the C-ABI library loads, exports every symbol include/nerf_amd.h declares, and its
host-side size helpers agree with the layout (no kernel launches: no GPU here)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nerf_amd.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nerf_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from nerf_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    return _lib.lib()


def test_header_declares_the_hot_path():
    names = declared_functions()
    for must in ("nerf_raygen", "nerf_sample_stratified", "nerf_sample_pdf", "nerf_composite_fwd",
                 "nerf_composite_bwd", "nerf_mlp_fwd", "nerf_mlp_bwd", "nerf_grid_index", "nerf_bake_points",
                 "nerf_march_gather", "nerf_adam_step", "nerf_searchsorted"):
        assert must in names


def test_every_declared_symbol_is_exported(lib):
    from nerf_amd import _lib
    for name in declared_functions():
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"


def test_sizes_and_layout(lib):
    assert lib.nerf_abi_version() == 3
    assert lib.nerf_mlp_net_params() == 595844
    # state_dict offsets: pts_linears.0.weight [256,63] then bias [256], ... rgb_linear.bias [3]
    assert lib.nerf_mlp_param_offset(0) == 0
    assert lib.nerf_mlp_param_offset(1) == 256 * 63
    assert lib.nerf_mlp_param_offset(24) == 595844
    assert lib.nerf_mlp_padded_samples(1) == 256
    assert lib.nerf_mlp_padded_samples(786432) == 786432
    assert lib.nerf_mlp_act_bytes(1, 256) == 2528 * 256 * 2
    assert lib.nerf_mlp_packed_bytes(1, 0) > 1185000 * 1 and lib.nerf_mlp_packed_bytes(0, 0) > 2 * 1185000
    assert lib.nerf_bake_num_points(128, 1) == 129 ** 3
    assert lib.nerf_bake_num_points(128, 0) == 128 ** 3 * 8


def test_argument_errors_are_reported_without_gpu(lib):
    from nerf_amd._lib import check
    with pytest.raises(RuntimeError, match="dtype"):
        check(lib.nerf_mlp_fwd(None, 7, None, None, 1, None, 10, 0, None, None, None, None), "nerf_mlp_fwd")
    with pytest.raises(RuntimeError, match="Sc"):
        check(lib.nerf_sample_pdf(None, None, 4, 65, 128, 1, None, None, 0, 0, None, None, None, None, None, None,
                                  None), "nerf_sample_pdf")


def test_product_path_rejects_cpu_tensors():
    import torch
    from nerf_amd import ops
    with pytest.raises(RuntimeError, match="GPU only"):
        ops.sample_stratified(torch.zeros(4, 6), 2.0, 6.0, 64, False)


def test_product_path_does_not_import_the_oracle():
    pkg = os.path.join(ROOT, "nerf-replication_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, flags=re.M), os.path.join(dirpath, f)
