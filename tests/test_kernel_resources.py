"""Build-level guard (CPU, no GPU): kernels that issue their operand loads from inline asm with
hand-counted ``s_waitcnt vmcnt`` (csrc/igemm64.hip, csrc/wgrad_tr.hip) must not spill.  The compiler
treats an asm load's destination as written when the asm statement ends; under register pressure it
may spill or re-assign that VGPR while the load is still in flight, and the late write then lands on
whatever now lives there (a 32-row 128x128 weight-gradient variant spilled 36 bytes and faulted the GPU
with an address clobbered this way).  Every kernel in these files must report ScratchSize 0."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ASM_LOAD_FILES = ["igemm64.hip", "wgrad_tr.hip", "wgrad_halo.hip", "conv3_halo.hip"]


@pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which("true") is None, reason="hipcc not available")
@pytest.mark.parametrize("src", ASM_LOAD_FILES)
def test_inline_asm_load_kernels_do_not_spill(src, tmp_path):
    text = open(os.path.join(ROOT, "csrc", src)).read()
    assert 'asm volatile("global_load' in text or 'asm volatile("buffer_load' in text
    out = tmp_path / "k.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-I", os.path.join(ROOT, "csrc"), os.path.join(ROOT, "csrc", src), "-o", str(out)],
                   check=True, capture_output=True, timeout=600)
    asm = out.read_text()
    names = re.findall(r"^(_Z\S*kernel\S*):", asm, flags=re.M)
    scratch = [int(x) for x in re.findall(r"; ScratchSize: (\d+)", asm)]
    assert names and len(scratch) >= len(names)
    spilled = [n for n, s in zip(names, scratch) if s > 0]
    assert not spilled, f"kernels with scratch (spills) in {src}: {spilled}"


# kernels carrying the BatchNorm epilogue sums (csrc/bn_acc.h) or the FedSGD protocol: a guarded
# accumulate once kept its sums in scratch with a dynamic index (every igemm64 variant, 12 bytes)
NO_SCRATCH_FILES = ["bn.hip", "igemm.hip", "fedsgd_ps.hip", "async_ps.hip", "lenet_fused.hip"]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", NO_SCRATCH_FILES)
def test_epilogue_sum_kernels_do_not_use_scratch(src, tmp_path):
    out = tmp_path / "k.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-I", os.path.join(ROOT, "csrc"), os.path.join(ROOT, "csrc", src), "-o", str(out)],
                   check=True, capture_output=True, timeout=600)
    asm = out.read_text()
    names = re.findall(r"^(_Z\S*kernel\S*):", asm, flags=re.M)
    scratch = [int(x) for x in re.findall(r"; ScratchSize: (\d+)", asm)]
    assert names and len(scratch) >= len(names)
    spilled = [n for n, s in zip(names, scratch) if s > 0]
    assert not spilled, f"kernels with scratch in {src}: {spilled}"
