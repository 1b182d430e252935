"""cell_floor's division (hn_common.h) against IEEE division on the CPU:
scripts/div_check.c compiled with gcc -ffp-contract=off (fmaf from libm is
the correctly rounded fused multiply-add, as v_fma_f32)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_cell_floor_division_exact(tmp_path):
    exe = tmp_path / "div_check"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), os.path.join(ROOT, "scripts", "div_check.c"),
                    "-lm"], check=True)
    r = subprocess.run([str(exe), "100000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout and " 0 floor mismatches" in r.stdout, r.stdout
