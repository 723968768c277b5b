"""Wait-state lint of the inline-asm MFMAs in the attention kernels (CPU: hipcc cross-compiles gfx950).

hipcc pads no hazard inside an `asm` statement, so a compiler-placed `v_accvgpr_write` right before an asm MFMA that
reads it, or a compiler instruction touching an asm MFMA's result too early, silently corrupts results on some waves.
`tools/check_mfma_asm_hazards.py` checks the generated assembly; this test builds it and requires zero findings."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
@pytest.mark.timeout(900)
def test_attention_asm_mfma_wait_states(tmp_path):
    src = os.path.join(ROOT, "accelerate_hpc_test_amd", "csrc", "kernels", "flash_attn.hip")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "kasm.sh"), src, str(tmp_path)], capture_output=True, text=True,
                       timeout=880)
    s_files = [f for f in os.listdir(tmp_path) if f.endswith("gfx950.s")]
    assert s_files, r.stdout + r.stderr
    asm = os.path.join(tmp_path, s_files[0])
    for kernel in ("attn_bwd_dq_w4_kernel", "attn_bwd_dkdv_w4_kernel"):
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_mfma_asm_hazards.py"), asm, kernel],
                             capture_output=True, text=True)
        assert out.returncode == 0, out.stdout[-3000:]


def _lint(tmp_path, body):
    asm = tmp_path / "k.s"
    asm.write_text("_Z6kernelv:\n" + body + ".Lfunc_end0:\n")
    return subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_mfma_asm_hazards.py"), str(asm), "kernel"],
                          capture_output=True, text=True)


def test_lint_flags_each_hazard_kind(tmp_path):
    """The lint itself on synthetic streams: a fresh AGPR operand, an early reader of the result, and the clean forms
    (the next MFMA of the same accumulation chain, a padded reader) that must pass."""
    mfma = "\t;;#ASMSTART\n\tv_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], a[0:3], v[0:15]\n\t;;#ASMEND\n"
    fresh = _lint(tmp_path, "\tv_accvgpr_write_b32 a1, v40\n" + mfma)
    assert fresh.returncode == 1 and "source read" in fresh.stdout
    early = _lint(tmp_path, mfma + "\tv_mul_f32_e32 v20, v3, v3\n")
    assert early.returncode == 1 and "result" in early.stdout
    chain = _lint(tmp_path, "\ts_nop 1\n" + mfma + mfma + "\ts_nop 7\n\ts_nop 7\n\tv_mul_f32_e32 v20, v3, v3\n")
    assert chain.returncode == 0, chain.stdout
