"""The BLS step direction's quotient (irm_kernels_impl.hpp, div_rcp with rcp_rn_of): with r = RN(1/b),
q = RN(a·r) and RN(q + (a − q·b)·r) must be the IEEE quotient RN(a/b) — optimizer_BLS.py:165's
ĝ = g / norm.  And r itself: one Newton step RN(y + y·RN(1 − b·y)) from either faithful rounding y of 1/b
(v_rcp_f32 is faithful) must give RN(1/b) for every divisor mantissa but all-ones, where rcp_rn_of selects
RN(1/b) by its bit pattern 0x7F000000 − bits(b).  Checked on the host in C (fmaf, -ffp-contract=off) for every divisor mantissa
(2^23 values) against 16 dividends each, and for 2^26 random pairs over exponents far beyond
what the kernel sees (‖G‖ from 2^-40 to 2^40, |ĝ| = |G|/‖G‖ from 2^-60 to 4 — |ĝ| ≤ 1 up to ‖G‖'s
rounding).  Markstein's theorem needs the remainder a − q·b to be a normal number: below |a| ≈ 2^-100
(a G element of ~1e-31) the formula can differ; the device check counts the kernel's actual quotients; the IRM_DIV_CHECK device build
counts the kernel's own mismatches (tools/div_check.py)."""
import os
import subprocess

import pytest

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static inline uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline float fb(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline float divq(float a, float b, float r) { const float q = a * r; return fmaf(fmaf(-q, b, a), r, q); }
int main(void) {
    long long bad = 0, n = 0;
    for (uint32_t m = 0; m < (1u << 23); ++m) {          /* every divisor mantissa */
        const float b = fb(0x3f800000u | m), r = 1.0f / b;
        for (int k = 0; k < 16; ++k) {
            const float a = fb(0x3f800000u | (uint32_t)(xr() & 0x7fffff)) * ((k & 1) ? -1.f : 1.f);
            bad += divq(a, b, r) != a / b; ++n;
        }
    }
    for (long long i = 0; i < (1ll << 26); ++i) {        /* b in [2^-40, 2^40), |a/b| in [2^-60, 2^2) */
        const uint64_t x = xr();
        const int eb = (int)((x >> 32) % 80) - 40, eq = (int)(x % 62) - 60;
        const float b = fb(((uint32_t)(127 + eb) << 23) | (uint32_t)((x >> 40) & 0x7fffff));
        const float a = fb(((uint32_t)(127 + eb + eq) << 23) | (uint32_t)((x >> 8) & 0x7fffff)) * ((x >> 63) ? -1.f : 1.f);
        const float r = 1.0f / b;
        bad += divq(a, b, r) != a / b; ++n;
    }
    long long rbad = 0;                                  /* the reciprocal: y faithful -> Newton step is RN(1/b) */
    for (int e = -30; e <= 30; ++e) {                    /* all-ones mantissa: RN(1/b) has the bits 0x7F000000 - bits(b) */
        const float b = ldexpf(fb(0x3fffffffu), e);
        uint32_t ub; memcpy(&ub, &b, 4);
        rbad += fb(0x7F000000u - ub) != 1.0f / b;
    }
    for (uint32_t m = 0; m < (1u << 23) - 1; ++m) {      /* (all-ones mantissa excluded: selected above) */
        const float b = fb(0x3f800000u | m), cr = 1.0f / b;
        const double ex = 1.0 / (double)b;
        const float lo = (double)cr <= ex ? cr : nextafterf(cr, 0.f), hi = (double)cr >= ex ? cr : nextafterf(cr, 2.f);
        const float ys[2] = {lo, hi};
        for (int k = 0; k < 2; ++k) rbad += fmaf(fmaf(-b, ys[k], 1.f), ys[k], ys[k]) != cr;
    }
    printf("%lld %lld %lld\n", n, bad, rbad);
    return 0;
}
"""


def test_markstein_quotient_is_the_ieee_division(tmp_path):
    c = tmp_path / "div.c"
    c.write_text(SRC)
    exe = tmp_path / "div"
    try:
        subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"])
    except (OSError, subprocess.CalledProcessError):
        pytest.skip("no host C compiler")
    n, bad, rbad = map(int, subprocess.check_output([str(exe)], timeout=300).split())
    print(f"{n} quotients, {bad} differ from a/b; refined reciprocals off RN(1/b): {rbad}")
    assert n > 2 ** 27 and bad == 0 and rbad == 0
