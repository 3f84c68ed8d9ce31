"""StrictMath (fdlibm 5.3) log / exp / log10: the product's device restatement
(guacamole_amd/csrc/gq_strictmath.h, compiled here for the host) and the oracle's
(oracle/strictmath.h) give identical bits, and both stay within 1 ulp of libm (log10: 4 ulps
near 1, a property of fdlibm's algorithm).  The somatic caller's knife-edge decisions
(SomaticStandardCaller.scala:220-236) depend on these bits."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_strictmath_product_equals_oracle(tmp_path):
    exe = str(tmp_path / "smcheck")
    src = os.path.join(ROOT, "tests", "native", "strictmath_check.cpp")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe, src])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 bit mismatches, 0 beyond" in out.stdout
