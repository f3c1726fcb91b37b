"""CPU check of the tracker's division by a constant divisor (tracker.hip div_const, Markstein's correction): the
device computes the reference's difference quotients / 0.02 and the lighting fit's / W^2 with a multiply and two
FMAs instead of a division; on random normal operands (and the infinities) it must give the IEEE quotient bit for
bit, which is what keeps the tracker bit-exact against the oracle (test_tracker_gpu.py)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_constant_division_is_correctly_rounded(tmp_path):
    exe = tmp_path / "cdc"
    src = os.path.join(ROOT, "tests", "native", "const_division_check.c")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", src, "-lm", "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "4000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
