"""The finish-part schedule model (csrc/mlp.hip FinishSchedule, round 6) on the CPU.

The round-5 finish-part sweep found bf16 builds whose training kernels wrote different masks / dZ on two
runs of one launch.  Two mechanisms, both found from the code and the emitted ISA:
  * a finish part clamped to the next unit's last step runs after the MFMA that reads the tile pair it
    writes (LRGB after LV, the dX stage bV after bRGB: 4-tile units) -- with 8 bf16 parts the dX read
    Hb[3] before its first write, i.e. uninitialised registers.  FinishSchedule simulates every group's
    steps and static_asserts the placement in every forward / dX instantiation;
  * an inline-asm VGPR write (v_pk_min_u16 of the ReLU mask bits) allocated to a dead accumulator lane
    of an MFMA still in flight (parts 2) -- removed, and tools/asm_check.py fails any such asm.
These tests pin the model: every shipped placement is sound, and the round-5 parts-8 placement fails to
compile."""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
MLP = os.path.join(ROOT, "nerf-replication_amd", "csrc", "mlp.hip")

pytestmark = pytest.mark.skipif(shutil.which(HIPCC) is None, reason="no hipcc")

CASES = [("PF32", 0, "false"), ("PF32", 0, "true"), ("PF32", 1, "false"),
         ("PBF16", 0, "false"), ("PBF16", 0, "true"), ("PBF16", 1, "false"),
         ("PBF3", 0, "false"), ("PBF3", 0, "true"), ("PBF3", 1, "false"), ("PBF6", 0, "false"),
         ("PBF3W", 2, "false"), ("PBF3W", 2, "true"),  # (the wide bf16x3 forward: 16-row units)
         ("PF32W", 2, "false"),  # (the wide fp32 training forward)
         ("PF32W", 3, "false"), ("PBF3W", 3, "false"), ("PBF16W", 3, "false")]  # (the wide dX: 16-row W^T units)


def _violations(tmp, defines):
    """finish_schedule_violation<P, DIR, DENSITY>() for every case, from a host program (constexpr)."""
    src = os.path.join(tmp, "sched.hip")
    with open(src, "w") as f:
        f.write("#define NERF_MLP_DEVICE_ONLY\n")
        f.write(f'#include "{MLP}"\n#include <cstdio>\nusing namespace nerf::mlp;\nint main() {{\n')
        for p, d, dens in CASES:
            f.write(f'  printf("%d\\n", finish_schedule_violation<{p}, {d}, {dens}>());\n')
        f.write("}\n")
    exe = os.path.join(tmp, "sched")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O0", "-std=c++17", "-fconstexpr-steps=33554432", f"-I{ROOT}/include", *defines, src, "-o", exe],
                   check=True, capture_output=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    return {c: int(v) for c, v in zip(CASES, out)}


def test_shipped_placements_are_sound():
    with tempfile.TemporaryDirectory() as tmp:
        v = _violations(tmp, [])
    assert all(x == 0 for x in v.values()), v


def test_round5_parts8_placement_is_caught():
    """8 bf16 finish parts: the forward (LRGB reading LV's tile 3) and the dX (bV reading bRGB's tile 3)
    read a pair before its part writes it (code 1); bf16x3's 8 parts (16-step units) stay sound."""
    with tempfile.TemporaryDirectory() as tmp:
        v = _violations(tmp, ["-DNERF_FINISH_PARTS_BF16=8", "-DNERF_FINISH_PARTS_BF3=8"])
    assert v[("PBF16", 0, "false")] == 1 and v[("PBF16", 1, "false")] == 1, v
    assert v[("PBF3", 0, "false")] == 0 and v[("PBF3", 1, "false")] == 0, v


def test_unsound_placement_fails_to_compile():
    """The static_assert in DxWave refuses a bf16 dX built with 8 finish parts."""
    with tempfile.TemporaryDirectory() as tmp:
        src = os.path.join(tmp, "k.hip")
        with open(src, "w") as f:
            f.write(f'#define NERF_MLP_DEVICE_ONLY\n#include "{MLP}"\n')
            f.write("template __global__ void nerf::mlp::dx_kernel<nerf::mlp::PBF16>(nerf::mlp::DxArgs);\n")
        bad = subprocess.run([HIPCC, "--offload-arch=gfx950", "-std=c++17", "-fconstexpr-steps=33554432", f"-I{ROOT}/include", "--cuda-device-only",
                              "-fsyntax-only", "-DNERF_FINISH_PARTS_BF16=8", src], capture_output=True, text=True)
        assert bad.returncode != 0 and "finish placement" in bad.stderr, bad.stderr[-2000:]
        good = subprocess.run([HIPCC, "--offload-arch=gfx950", "-std=c++17", "-fconstexpr-steps=33554432", f"-I{ROOT}/include", "--cuda-device-only",
                               "-fsyntax-only", "-DNERF_FINISH_PARTS_BF16=2", src], capture_output=True, text=True)
        assert good.returncode == 0, good.stderr[-2000:]


def test_pinned_knobs_refuse_unverified_values():
    """mlp.hip's knob policy: a tuning knob outside the schedule knobs builds only at its verified value."""
    with tempfile.TemporaryDirectory() as tmp:
        src = os.path.join(tmp, "k.hip")
        with open(src, "w") as f:
            f.write(f'#define NERF_MLP_DEVICE_ONLY\n#include "{MLP}"\n')
        for knob in ("-DNERF_DW_NBUF_BF16=2", "-DNERF_PACKED_MASK=0", "-DNERF_DMA_LEAN=0", "-DNERF_KEEP_PE_BF3=0"):
            bad = subprocess.run([HIPCC, "--offload-arch=gfx950", "-std=c++17", "-fconstexpr-steps=33554432", f"-I{ROOT}/include",
                                  "--cuda-device-only", "-fsyntax-only", knob, src], capture_output=True, text=True)
            assert bad.returncode != 0 and "knob policy" in bad.stderr, (knob, bad.stderr[-1500:])
