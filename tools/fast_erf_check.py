#!/usr/bin/env python3
"""Accuracy of the GEMM epilogues' fast erf (csrc/device_math.hpp), evaluated in fp32 with
the coefficients parsed from the header, against scipy's double-precision erf."""
import os
import re
import sys

import numpy as np
from scipy.special import erf

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "starpu-inference-server_amd", "csrc",
                   "device_math.hpp")


def coefficients(path=HDR, suffix=""):
    src = open(path).read()

    def arr(name):
        body = re.search(name + r"\[\d+\] = \{([^}]*)\}", src).group(1)
        return [float(v.strip().rstrip("f")) for v in body.split(",")]
    clamp = float(re.search(r"kErfClamp" + suffix + r" = ([0-9.]+)f", src).group(1))
    return arr("kErfP" + suffix), arr("kErfQ" + suffix), clamp


def fast_erf(x, p, q, clamp):
    x = np.clip(x.astype(np.float32), np.float32(-clamp), np.float32(clamp))
    x2 = x * x
    pp = np.full_like(x, np.float32(p[0]))
    for c in p[1:]:
        pp = pp * x2 + np.float32(c)
    qq = np.full_like(x, np.float32(q[0]))
    for c in q[1:]:
        qq = qq * x2 + np.float32(c)
    return x * pp * (np.float32(1) / qq)


def max_error(n=2_000_001, lim=8.0, suffix=""):
    """suffix "": the fp32-grade erf (gemm.hip); "16": the fp16-operand GEMM's (gemm256.hip)."""
    p, q, clamp = coefficients(suffix=suffix)
    x = np.linspace(-lim, lim, n).astype(np.float32)
    ref = erf(x.astype(np.float64))
    e_erf = float(np.abs(fast_erf(x, p, q, clamp) - ref).max())
    g = 0.5 * x * (1 + fast_erf(x / np.float32(np.sqrt(2)), p, q, clamp))
    e_gelu = float(np.abs(g - 0.5 * x.astype(np.float64) * (1 + ref_gelu(x))).max() / lim)
    return e_erf, e_gelu


def ref_gelu(x):
    return erf(x.astype(np.float64) / np.sqrt(2))


if __name__ == "__main__":
    e, g = max_error()
    e16, g16 = max_error(suffix="16")
    print(f"fast_erf max|err| = {e:.3e}; GELU max|err| / max|x| on [-8, 8] = {g:.3e}")
    print(f"fp16-GEMM erf max|err| = {e16:.3e}; GELU max|err| / max|x| = {g16:.3e}")
    sys.exit(0 if e < 5e-7 and e16 < 3e-6 else 1)
