// Exhaustive check of sqrt_le_bound (kfx_kernels.hip, a copy of the host function
// below): for every non-negative float x, (sqrtf(x) <= t) == (x <= bound(t)).
// build: g++ -O2 -ffp-contract=off tools/sqrt_bound_check.cpp -o /tmp/sqrt_bound_check
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdint>
#include <limits>
float sqrt_le_bound(float t) {
  if (std::isnan(t)) return t;
  if (t < 0.f) return -1.f;
  if (std::isinf(t)) return t;
  float x = t * t;
  if (std::isinf(x)) x = std::numeric_limits<float>::max();
  while (x > 0.f && std::sqrt(x) > t) x = std::nextafter(x, 0.f);
  for (;;) {
    const float n = std::nextafter(x, std::numeric_limits<float>::infinity());
    if (std::isinf(n) || std::sqrt(n) > t) break;
    x = n;
  }
  return x;
}
int main() {
  float ts[] = {0.015f, std::sin(30.f * 0.017453293f), 0.f, 1e-30f, 3.f, 1e30f, 0.1f, 0.5f};
  for (float t : ts) {
    float b = sqrt_le_bound(t);
    long bad = 0;
    for (uint64_t u = 0; u < 0x80000000ull; ++u) {  // every non-negative float incl. inf/NaN
      uint32_t w = (uint32_t)u; float x; memcpy(&x, &w, 4);
      if ((std::sqrt(x) <= t) != (x <= b)) ++bad;
    }
    printf("t=%g bound=%a mismatches=%ld\n", t, b, bad);
  }
}
