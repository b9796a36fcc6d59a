"""Static checks on the gfx950 assembly of the MLP kernels (hipcc --save-temps):
  * the forward / dX kernels are straight-line (no loop: a runtime walk of the constexpr
    layout tables would show up as one),
  * every counted `s_waitcnt vmcnt(N)` + s_barrier hand-off waits for the weight DMA:
    N <= vector-memory ops issued after the last global_load_lds before it,
  * no scratch (spills),
  * no compiler code touches M0 (the lean LDS-DMA sets it without saving it),
  * no inline asm writes a VGPR (round 6): hipcc's hazard recognizer does not model the MFMA hazards of
    an inline-asm VGPR write -- an asm output allocated to a dead lane of an accumulator whose MFMA is
    still in flight is overwritten by the MFMA's late write-back (the round-5 mask race), so every VGPR
    write must be compiler-placed (tools/mfma_war_scan.py measures the distances).
The finish-part placement (which MFMA reads which register tile pair after which finish part wrote it)
is a register dependence, invisible in the ISA as a hazard: it is checked at compile time by
FinishSchedule (csrc/mlp.hip), a static_assert on every forward / dX instantiation.
    python tools/asm_check.py            (exit status 1 on a violation)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# every MLP kernel instantiation the library builds: per precision the training, inference, density-only
# and persistent forwards, dX and dW; the bf16x3f training forward (bf16 stores) and the bf16x6 forward
# (the bf16x3 forwards are the wide PBF3W kernels since round 6; PBF3 keeps the bf16x3 dX / dW; the fp32 training
# forward is the wide PF32W one)
KERNELS = [f"fwd_kernel<nerf::mlp::{p}, {a}>" for p in ("PF32", "PBF16", "PBF3W")
           for a in ("true, false, false", "false, false, false", "false, true, false", "false, false, true")] + \
          ["fwd_kernel<nerf::mlp::PBF3W, true, false, false, true>", "fwd_kernel<nerf::mlp::PBF6, false, false, false>",
           "fwd_kernel<nerf::mlp::PF32W, true, false, false>"] + \
          [f"{k}_kernel<nerf::mlp::{p}>" for k in ("dx", "dw") for p in ("PF32", "PBF16", "PBF3")] + \
          ["dx_kernel<nerf::mlp::PF32W>", "dx_kernel<nerf::mlp::PBF3W>", "dx_kernel<nerf::mlp::PBF16W>"]  # (wide dX, r6)


def build_asm(tmp, kernels=None):
    """gfx950 assembly of the given kernel instantiations, one hipcc process per kernel (in
    parallel), concatenated."""
    kernels = kernels or KERNELS
    args = {"fwd": "(nerf::mlp::FwdArgs)", "dx_": "(nerf::mlp::DxArgs)", "dw_": "(nerf::mlp::DwArgs)"}
    procs = []
    for i, k in enumerate(kernels):
        src = os.path.join(tmp, f"k{i}.hip")
        with open(src, "w") as f:
            f.write("#define NERF_MLP_DEVICE_ONLY\n")
            f.write(f'#include "{ROOT}/nerf-replication_amd/csrc/mlp.hip"\n')
            f.write(f"template __global__ void nerf::mlp::{k}{args[k[:3]]};\n")
        extra = os.environ.get("NERF_ASM_EXTRA", "").split()  # variant -D flags (tools/build_variants.sh)
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                                       "-fconstexpr-steps=33554432", *extra,
                                       f"-I{ROOT}/include", "--cuda-device-only", "-S", src, "-o",
                                       os.path.join(tmp, f"k{i}.s")], cwd=tmp, stdout=subprocess.DEVNULL,
                                      stderr=subprocess.DEVNULL))
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("hipcc failed")
    asm = []
    for i, k in enumerate(kernels):
        text = open(os.path.join(tmp, f"k{i}.s")).read()
        # keep the instantiated kernel only (every file also carries the non-template reduce kernel)
        if "dw_reduce_kernel" not in k:
            text = re.sub(r"^_ZN4nerf3mlp16dw_reduce_kernel\w*:.*?s_endpgm", "", text, flags=re.S | re.M)
        asm.append(text)
    return "\n".join(asm)


def check(asm):
    bad = 0
    for name in re.findall(r"^(_Z\w+):", asm, re.M):
        body = asm[asm.index(name + ":"):]
        body = body[:body.index("s_endpgm")]
        lines = body.splitlines()
        labels = {m.group(1): i for i, l in enumerate(lines) for m in [re.match(r"^(\.LBB\w+):", l)] if m}
        loops = [i for i, l in enumerate(lines) for m in [re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)]
                 if m and m.group(1) in labels and labels[m.group(1)] < i]
        since, waits, unsafe = None, 0, 0
        # the lean LDS-DMA (NERF_DMA_LEAN) writes M0 without saving it: no compiler code of the
        # kernel may read or write M0 (every M0 access must sit inside an inline-asm statement)
        in_asm, m0_outside, asm_vgpr = False, 0, 0
        for l in lines:
            if ";;#ASMSTART" in l:
                in_asm = True
            elif ";;#ASMEND" in l:
                in_asm = False
            elif not in_asm and re.search(r"\bm0\b", l) and not l.strip().startswith(";"):
                m0_outside += 1
            elif in_asm and re.match(r"\s*v_\w+\s+v[\[\d]", l):
                asm_vgpr += 1  # an instruction inside inline asm whose destination is a VGPR
        for i, l in enumerate(lines):
            t = l.strip()
            if t.startswith("global_load_lds"):
                since = 0
            elif since is not None and re.match(r"(global_store|global_load|scratch_|buffer_|global_atomic)", t):
                since += 1
            m = re.match(r"s_waitcnt vmcnt\((\d+)\)", t)
            if m and i + 1 < len(lines) and "s_barrier" in lines[i + 1] and since is not None:
                waits += 1
                unsafe += int(m.group(1)) > since
        # the persistent inference forward (PERSIST = true) loops over its sample blocks: the block
        # loop (+ its guard) is its only backward branch
        persist = re.search(r"fwd_kernel\w*?ELb0ELb0ELb1E", name) is not None
        straight = "dw_kernel" in name or "dw_reduce" in name or not loops or (persist and len(loops) <= 2)
        ok = straight and not unsafe and not m0_outside and not asm_vgpr
        bad += not ok
        print(f"{'ok ' if ok else 'BAD'} {name[:70]:70s} loops={len(loops)} counted_waits={waits} unsafe={unsafe} "
              f"m0_outside_asm={m0_outside} asm_vgpr_writes={asm_vgpr}")
    for m in re.finditer(r"\.name:\s+(\S+)\n(?:.*\n){0,40}?\s+\.private_segment_fixed_size:\s+(\d+)", asm):
        if int(m.group(2)):
            bad += 1
            print(f"BAD scratch {m.group(2)} B in {m.group(1)}")
    return bad


if __name__ == "__main__":
    with tempfile.TemporaryDirectory() as tmp:
        sys.exit(1 if check(build_asm(tmp)) else 0)
