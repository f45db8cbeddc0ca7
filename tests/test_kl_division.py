"""The shared-sigma KL division of the fused loss kernel (correctly rounded reciprocal + one fma correction,
csrc/ppo_loss.hip) equals IEEE fp32 true division -- checked on the host by oracle/kl_division_check.c (plain C,
-ffp-contract=off), over policy-like and random-bit operands.  The GPU test
test_gpu_loss.py::test_shared_sigma_kl_fast_path_bit_exact compares the kernel's two paths bitwise."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_markstein_division_matches_true_division(tmp_path):
    exe = tmp_path / "kl_division_check"
    subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-fno-fast-math", "-o", str(exe),
                    os.path.join(ROOT, "oracle", "kl_division_check.c"), "-lm"], check=True)
    r = subprocess.run([str(exe), "4000", "2000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    tot, bad = (int(v) for v in r.stdout.split()[-3::2])
    assert tot > 7_000_000 and bad == 0, r.stdout
