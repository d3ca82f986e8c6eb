"""Kernels that issue vector loads as inline asm, which the compiler neither counts nor waits for: compile every
csrc/*.hip holding such a load for gfx950 and check (tools/isa_audit.py) that no instruction of any kernel whose
text carries an inline-asm VGPR load touches a register such a load still has to write -- in the K loop (the register
sets are named at every wait) and after it (the last sets' loads are dead to the compiler, which reused their
registers for the epilogue until the final wait named them: a timing-dependent corruption of a few tiles of the deep
DiMP conv kernel, found by the layer3 golden in round 4).  The kernels are found from the assembly, not listed, so a
new inline-asm load anywhere is audited too."""
import glob
import os
import re
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "multi-modal-trakcing-bechmark_amd", "csrc")
sys.path.insert(0, os.path.join(REPO, "tools"))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
ASM_LOAD = re.compile(r'asm\s+volatile\s*\(\s*"(buffer|global)_load')


def _sources():
    return [p for p in sorted(glob.glob(os.path.join(CSRC, "*.hip"))) if ASM_LOAD.search(open(p).read())]


def _asm_vgpr_load_kernels(text):
    """Kernel symbols whose body holds an inline-asm load into VGPRs (not an LDS-DMA load)."""
    out = []
    for m in re.finditer(r"^(_Z\w+):", text, re.M):
        end = text.find(".Lfunc_end", m.end())
        body = text[m.end():end]
        if re.search(r";;#ASMSTART\s*\n\s*(buffer|global)_load\w*\s+v[\[\d](?![^\n]*\blds\b)", body):
            out.append(m.group(1))
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
def test_inline_asm_load_kernels_never_touch_pending_load_registers(tmp_path):
    import isa_audit
    srcs = _sources()
    assert any(p.endswith("dimpconv.hip") for p in srcs), srcs
    audited = {}
    for src in srcs:
        out = tmp_path / (os.path.basename(src) + ".s")
        subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", f"-I{REPO}/include",
                        "--cuda-device-only", "-S", src, "-o", str(out)], check=True, capture_output=True, timeout=600)
        text = out.read_text()
        for k in _asm_vgpr_load_kernels(text):
            audited[k] = isa_audit.audit(text, k)
    # the deep conv kernel's instances (the fused-downsample path included) are among them
    assert sum("conv_f16x3_deep_kernel" in k for k in audited) >= 4, sorted(audited)
    print(f"{len(audited)} kernels with inline-asm VGPR loads audited")
    bad = {k: v[:3] for k, v in audited.items() if v}
    assert not bad, bad
