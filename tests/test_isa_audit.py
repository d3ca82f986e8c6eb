"""The deep-pipelined DiMP conv kernel issues its activation loads as inline asm, which the compiler neither counts
nor waits for: compile dimpconv.hip for gfx950 and check (tools/isa_audit.py) that no instruction of any
conv_f16x3_deep_kernel instance touches a register such a load still has to write -- in the K loop (the register
sets are named at every wait) and after it (the last sets' loads are dead to the compiler, which reused their
registers for the epilogue until the final wait named them: a timing-dependent corruption of a few tiles)."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "multi-modal-trakcing-bechmark_amd", "csrc")
sys.path.insert(0, os.path.join(REPO, "tools"))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_deep_conv_kernel_never_touches_pending_load_registers(tmp_path):
    import isa_audit
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    out = tmp_path / "dimpconv.s"
    subprocess.run([hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", f"-I{REPO}/include",
                    "--cuda-device-only", "-S", os.path.join(CSRC, "dimpconv.hip"), "-o", str(out)],
                   check=True, capture_output=True, timeout=600)
    text = out.read_text()
    names = isa_audit.kernels(text, "conv_f16x3_deep_kernel")
    assert len(names) >= 4, names
    bad = {k: isa_audit.audit(text, k) for k in names}
    assert not any(bad.values()), {k: v[:3] for k, v in bad.items() if v}
