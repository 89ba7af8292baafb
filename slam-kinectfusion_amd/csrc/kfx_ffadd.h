// Exact fast-forward of a repeated float addition (integrate's vc replay).
//
// The reference accumulates a column's camera-space position by n float adds,
// x <- RN(x + s) (tsdf_volume.cu:53-55); a z-chunk or a Z-slab that starts at
// slice n must reproduce that value bit for bit.  Inside one binade of |x|,
// [2^E, 2^(E+1)), every float is an integer multiple X of u = 2^(E-23), so
// while the exact sum x + s stays in the binade, RN(x + s) = (X + R) u with
// R = the integer nearest to s / u: the sequence is an arithmetic progression
// in integers, and m steps of it are (X + m R) u.  Ties (s / u a
// half-integer) round to even: after at most one plain step X is even and
// every step adds the same even integer, again a progression.  Steps that leave the
// binade, values near zero and extreme or non-finite values take plain float
// adds.  Integer and float arithmetic only (a handful of registers: the loop
// runs in integrate's prologue).  Checked against the plain loop on millions
// of cases (tests/test_ffadd.py) and bit for bit inside the GPU parity tests.
// Host and device share this code.
#pragma once
#include <cstdint>
#include <cstring>

#if defined(__HIPCC__)
#define KFX_HD __host__ __device__
#else
#define KFX_HD
#endif

namespace kfx {

KFX_HD inline uint32_t ff_f_bits(float f) {
  uint32_t b;
  std::memcpy(&b, &f, 4);
  return b;
}
KFX_HD inline float ff_pow2f(int e) {  // 2^e as a float, -126 <= e <= 127
  const uint32_t b = (uint32_t)(e + 127) << 23;
  float f;
  std::memcpy(&f, &b, 4);
  return f;
}

// n repeated x <- RN(x + s) (binary32, round to nearest even), exactly.
KFX_HD inline float ff_add(float x, float s, int n) {
  const float as = s < 0.f ? -s : s;
  if (n > 0 && as == 0.f) return x + s;  // adding zero: one add settles -0 and NaN
  while (n > 0) {
    const float ax = x < 0.f ? -x : x;
    // plain step: |x| within four steps of zero (tiny binades: one add each
    // is cheaper), extreme or non-finite values, s == 0
    if (!(ax >= 4.f * as) || !(ax >= 0x1p-90f) || !(ax < 0x1p90f) || !(as >= 0x1p-90f)) {
      x = x + s;
      --n;
      continue;
    }
    const uint32_t bx = ff_f_bits(ax);
    const int E = (int)((bx >> 23) & 0xffu) - 127;              // |x| in [2^E, 2^(E+1))
    const int X = (int)((bx & 0x7fffffu) | 0x800000u);          // |x| / u in [2^23, 2^24)
    const float su = (x < 0.f ? -s : s) * ff_pow2f(23 - E);     // s / u toward |x|: exact, |su| <= 2^22
    const float rf = __builtin_rintf(su);
    const float f = su - rf;                                    // exact
    const int R = (int)rf;
    if (f == 0.5f || f == -0.5f) {
      // tie: 2 su = Q is odd, so X + Q/2 is a half-integer and rounds to the
      // even one of X + lo, X + hi (lo = (Q-1)/2, hi = lo + 1).  From an even
      // X every step adds the same c = the even one of lo, hi; an odd X takes
      // one plain step first (its result is even).  Step k stays in the
      // binade's rounding while X + k c + Q/2 lies in [2^23 + 1/2, 2^24 - 1/2]
      // (a result of 2^24 u = 2^(E+1) is still exact).
      const int Q = 2 * R + (f > 0.f ? 1 : -1), lo = (Q - 1) / 2, hi = lo + 1;
      if ((X & 1) == 0) {
        const int c = (lo & 1) == 0 ? lo : hi;
        int m;
        if (c > 0) {  // Q >= 3: the lower bound holds
          const int num = 0x1000000 - X - hi;
          m = num >= 0 ? num / c + 1 : 0;
        } else if (c < 0) {  // Q <= -3: the upper bound holds
          const int num = X + lo - 0x800000;
          m = num >= 0 ? num / -c + 1 : 0;
        } else {  // Q = +-1: X is a fixed point while its sum stays in range
          if (X + lo >= 0x800000 && X + hi <= 0x1000000) return x;
          m = 0;
        }
        if (m > 0) {
          if (m > n) m = n;
          const float xn = (float)(X + m * c) * ff_pow2f(E - 23);  // exact
          x = x < 0.f ? -xn : xn;
          n -= m;
          continue;
        }
      }
      x = x + s;
      --n;
      continue;
    }
    // the sum X + R + f must stay in [2^23, 2^24): X + R in [lb, ub]
    const int lb = 0x800000 + (f < 0.f ? 1 : 0), ub = 0x1000000 - (f < 0.f ? 0 : 1);
    if (X + R < lb || X + R > ub) {  // the step leaves the binade
      x = x + s;
      --n;
      continue;
    }
    if (R == 0) return x;  // |s| < u/2: x is a fixed point while in the binade
    // the most steps with X + m R in [lb, ub]: D / |R| (D < 2^24, exact in
    // float) from a reciprocal estimate, then corrected
    const int D = R > 0 ? ub - X : X - lb, aR = R > 0 ? R : -R;
    int m = (int)((float)D * (1.f / (float)aR));
    while (m > 0 && m * aR > D) --m;
    while ((m + 1) * aR <= D) ++m;
    if (m > n) m = n;
    const float xn = (float)(X + m * R) * ff_pow2f(E - 23);  // exact
    x = x < 0.f ? -xn : xn;
    n -= m;
  }
  return x;
}

// ff_add out of line (ff_add_fast's rare fallback: one copy of the loop per
// kernel instead of one per call site)
KFX_HD __attribute__((noinline)) inline float ff_add_call(float x, float s, int n) { return ff_add(x, s, n); }

// ff_add when all n steps stay in x's binade without a tie (the common case
// of a ray's next few hundred samples): ff_add's first iteration with no loop
// (X + R and X + n R both in range: the progression in between is too), a
// fixed branch-light sequence; anything else takes ff_add.  Same results.
KFX_HD inline float ff_add_fast(float x, float s, int n) {
  const float as = s < 0.f ? -s : s, ax = x < 0.f ? -x : x;
  if (n > 0 && ax >= 4.f * as && ax >= 0x1p-90f && ax < 0x1p90f && as >= 0x1p-90f) {
    const uint32_t bx = ff_f_bits(ax);
    const int E = (int)((bx >> 23) & 0xffu) - 127;
    const int X = (int)((bx & 0x7fffffu) | 0x800000u);
    const float su = (x < 0.f ? -s : s) * ff_pow2f(23 - E);  // exact, |su| <= 2^22
    const float rf = __builtin_rintf(su);
    const float f = su - rf;
    if (f != 0.5f && f != -0.5f) {
      const int R = (int)rf;
      const int lb = 0x800000 + (f < 0.f ? 1 : 0), ub = 0x1000000 - (f < 0.f ? 0 : 1);
      const long long Xn = (long long)X + (long long)n * R;
      if (X + R >= lb && X + R <= ub && Xn >= lb && Xn <= ub) {
        const float xn = (float)(int)Xn * ff_pow2f(E - 23);  // exact
        return x < 0.f ? -xn : xn;
      }
    }
  }
#if !defined(KFX_FF_NOINLINE) || KFX_FF_NOINLINE
  return ff_add_call(x, s, n);
#else
  return ff_add(x, s, n);
#endif
}

}  // namespace kfx
