"""Static checks on the gfx950 code hipcc emits for the MLP kernels (CPU; no GPU needed):
straight-line forward / dX kernels, every counted `s_waitcnt vmcnt(N)` + `s_barrier` weight
hand-off covering its LDS-DMA (N <= vector-memory ops issued after the last DMA), and no
scratch in the bf16 kernels.  The hand-off protocol is invisible to the compiler (the DMA is
inline asm), so a codegen change that reorders or adds stores is caught here, not as a
race on the GPU.  See tools/asm_check.py."""
import os
import re
import shutil
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="no hipcc")
def test_mlp_kernels_handoffs_and_registers(capsys):
    import asm_check
    # the two training kernels (the full list, fp32 included, is tools/asm_check.py's default)
    kernels = ["fwd_kernel<nerf::mlp::PBF16, true, false>", "dx_kernel<nerf::mlp::PBF16>"]
    with tempfile.TemporaryDirectory() as tmp:
        asm = asm_check.build_asm(tmp, kernels)
    bad = asm_check.check(asm)
    out = capsys.readouterr().out
    # fp32 kernels are the parity path: a small spill there is tolerated, not in bf16
    fatal = [l for l in out.splitlines() if l.startswith("BAD") and "PF32" not in l]
    assert not fatal, "\n" + out
    assert bad == len([l for l in out.splitlines() if l.startswith("BAD")])
    assert re.search(r"fwd_kernelINS0_5PBF16ELb1ELb0.*counted_waits=\d+ unsafe=0", out)
