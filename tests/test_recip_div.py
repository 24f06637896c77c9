"""The line sweeps' division (lssp_amd/csrc/linesweep_dev.h div_rcp): a / b
formed from the host's y = RN(1/b) by q0 = RN(a y) and two FMA corrections,
Markstein's construction, in place of the division's longer dependent chain.
The GPU tests compare whole sweeps against the oracle bit for bit; this CPU
test checks the arithmetic itself against IEEE division on 2e7 random and
adversarial operand pairs in the fast path's range (tests/native/recip_div_check.c,
built with gcc: fma() is the correctly rounded fused multiply-add)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_reciprocal_division_is_ieee_division(tmp_path):
    exe = tmp_path / "recip_div_check"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), os.path.join(HERE, "native", "recip_div_check.c"),
                    "-lm"], check=True)
    out = subprocess.run([str(exe), "20000000"], check=True, capture_output=True, text=True).stdout.split()
    n, bad = int(out[-2]), int(out[-1])
    assert n == 20000000 and bad == 0, out
