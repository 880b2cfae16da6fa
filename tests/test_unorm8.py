"""unorm8 (csrc/ctl_bsdf.h) replaces the reference's per-channel `float(b) /
255.0f` (Spectrum::fromRGBCOL via SpectrumConverter::COLORREFToFloat3,
Spectrum.h:528-532) with one product and one FMA correction step.  The input
domain is the 256 byte values, so the identity is proved exhaustively: the same
expression, compiled with gcc (no contraction, IEEE fmaf), equals the correctly
rounded quotient for every byte."""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BSDF = os.path.join(HERE, "..", "cudatracerlib_amd", "csrc", "ctl_bsdf.h")

SRC = r"""
#include <math.h>
#include <stdio.h>
static float unorm8(unsigned b) {
    const float x = (float)b, c = 1.0f / 255.0f;
    const float q0 = x * c;
    return fmaf(fmaf(-q0, 255.0f, x), c, q0);
}
int main(void) {
    int bad = 0;
    for (unsigned b = 0; b < 256; b++) {
        volatile float x = (float)b;
        if (unorm8(b) != x / 255.0f) bad++;
    }
    printf("%d\n", bad);
    return 0;
}
"""


def test_unorm8_is_the_product_code():
    text = open(BSDF).read()
    body = re.search(r"CTL_HD float unorm8\(uint32_t b\) \{(.*?)\n\}", text, re.S).group(1)
    assert "const float x = (float)b, c = 1.0f / 255.0f;" in body
    assert "const float q0 = x * c;" in body
    assert "return fmaf(fmaf(-q0, 255.0f, x), c, q0);" in body


def test_unorm8_equals_division_for_every_byte(tmp_path):
    gcc = "gcc"
    src = tmp_path / "unorm8.c"
    src.write_text(SRC)
    exe = tmp_path / "unorm8"
    try:
        subprocess.run([gcc, "-O2", "-ffp-contract=off", "-o", str(exe), str(src), "-lm"], check=True,
                       capture_output=True)
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f"no C compiler: {e}")
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.strip()
    assert out == "0"
