"""The division-free requantizer of the HIP epilogues (qnn_internal.h quant_code_fast):
Markstein's correction q = fma(fma(-q0, s, t), RN(1/s), q0) must equal the IEEE
quotient RN(t/s) bit for bit, hence the same code as quantize.py:90-95.  Checked here
on the host (gcc + libm fmaf, the same IEEE binary32 operations) on quotients packed
around half-integers, where rint is sensitive, and on random ones."""
import os
import shutil
import subprocess

import pytest

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t st = 0x9E3779B97F4A7C15ull;
static inline uint64_t xr(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static inline float bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
int main(int argc, char** argv) {
  long n = atol(argv[1]), bad = 0;
  for (long it = 0; it < n; ++it) {
    float s = bits((uint32_t)((xr() & 0x7fffff) | ((uint32_t)(100 + (int)(xr() % 36)) << 23)));
    float inv = 1.0f / s, t;
    if ((it & 3) == 0) {
      t = ((float)(xr() >> 40) / 16777216.0f * 600.f - 300.f) * s;
    } else {
      float h = (float)((int)(xr() % 300) - 20) + 0.5f, tt = h * s;
      uint32_t tu; memcpy(&tu, &tt, 4); tu += (int)(xr() % 9) - 4; memcpy(&t, &tu, 4);
    }
    float ref = t / s, q0 = t * inv, q1 = fmaf(fmaf(-q0, s, t), inv, q0);
    if (memcmp(&q1, &ref, 4)) ++bad;
  }
  printf("%ld\n", bad);
  return 0;
}
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_markstein_quotient_is_ieee(tmp_path):
    c = tmp_path / "mk.c"
    c.write_text(SRC.replace("#include <string.h>", "#include <string.h>\n#include <stdlib.h>"))
    exe = tmp_path / "mk"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"], check=True)
    out = subprocess.run([str(exe), "20000000"], check=True, capture_output=True, text=True).stdout
    assert int(out.strip()) == 0


SRC_CLAMP = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint64_t st = 0x243F6A8885A308D3ull;
static inline uint64_t xr(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static inline float bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline float med3(float a, float lo, float hi) { return fminf(fmaxf(a, lo), hi); }
int main(int argc, char** argv) {
  long n = atol(argv[1]), bad = 0;
  for (long it = 0; it < n; ++it) {
    float s = bits((uint32_t)((xr() & 0x7fffff) | ((uint32_t)(100 + (int)(xr() % 36)) << 23)));
    float inv = 1.0f / s;
    /* quotients of magnitude 2^-2 .. 2^31, either sign, mantissa random */
    float mag = ldexpf(1.0f + (float)(xr() >> 40) / 16777216.0f, (int)(xr() % 34) - 2);
    float t = ((xr() & 1) ? mag : -mag) * s;
    if (!isfinite(t)) continue;
    float ref = rintf(med3(t / s, 0.0f, 255.0f));
    float q0 = t * inv, q = fmaf(fmaf(-q0, s, t), inv, q0);
    float fast = rintf(med3(q, 0.0f, 255.0f));
    if (memcmp(&fast, &ref, 4)) ++bad;
    /* the product form (qnn_internal.h qclamp2): q0 clamped to +-2^20 first */
    float q0c = med3(q0, -1048576.0f, 1048576.0f), qc = fmaf(fmaf(-q0c, s, t), inv, q0c);
    float fc = rintf(med3(qc, 0.0f, 255.0f));
    if (memcmp(&fc, &ref, 4)) ++bad;
  }
  /* t * inv overflowing: tiny scales (normal and subnormal), finite t up to FLT_MAX, either sign,
     and infinite t; the unclamped form gives NaN there, the clamped one the IEEE code */
  for (long it = 0; it < n / 16; ++it) {
    float s = bits((uint32_t)(xr() % 0x0f000000u) + 1u);
    float inv = 1.0f / s;
    if (!isfinite(inv)) continue;
    float t = bits((uint32_t)((xr() & 0x7fffff) | ((uint32_t)(200 + (int)(xr() % 55)) << 23)));
    if ((it & 7) == 7) t = INFINITY;
    if (xr() & 1) t = -t;
    float ref = rintf(med3(t / s, 0.0f, 255.0f));
    float q0 = t * inv;
    float q0c = med3(q0, -1048576.0f, 1048576.0f), qc = fmaf(fmaf(-q0c, s, t), inv, q0c);
    float fc = rintf(med3(qc, 0.0f, 255.0f));
    if (memcmp(&fc, &ref, 4)) ++bad;
  }
  printf("%ld\n", bad);
  return 0;
}
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_clamp_free_quantizer_codes_are_ieee(tmp_path):
    """The Markstein quotient clamped to [0, 255] and rounded half to even equals the IEEE
    division's code for every finite quotient, including those far beyond 2^20 where q0 and the
    corrected q differ; and qnn_internal.h qclamp2's form (q0 clamped to +-2^20 first) does so
    also where t * inv overflows (tiny scales, |t| up to FLT_MAX, infinite t), where the
    unclamped correction would give fma(-inf, inv, inf) = NaN."""
    c = tmp_path / "cf.c"
    c.write_text(SRC_CLAMP)
    exe = tmp_path / "cf"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"], check=True)
    out = subprocess.run([str(exe), "20000000"], check=True, capture_output=True, text=True).stdout
    assert int(out.strip()) == 0
