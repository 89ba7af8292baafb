// Brute-force check of kfx::ff_add and ff_add_fast (csrc/kfx_ffadd.h) against the plain loop
// of float adds it fast-forwards.  argv: seed cases.  Prints "bad <count>".
#include "kfx_ffadd.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

int main(int argc, char** argv) {
  const unsigned seed = argc > 1 ? (unsigned)std::atoi(argv[1]) : 7u;
  const long cases = argc > 2 ? std::atol(argv[2]) : 100000;
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  long bad = 0;
  for (long it = 0; it < cases; ++it) {
    float x, s;
    switch (it % 11) {
      case 0: x = U(g) * 3.f; s = U(g) * 0.01f; break;                  // camera-space columns
      case 1: x = U(g) * 0.01f; s = U(g) * 0.004f; break;               // crossing zero
      case 2: x = U(g) * 1000.f; s = U(g) * 1e-5f; break;               // fixed points
      case 3:                                                           // exact binary values and ties
        x = std::ldexp(1.f, (int)(g() % 20) - 10) * (float)(1 + g() % 3);
        s = std::ldexp(1.f, (int)(g() % 30) - 35) * ((g() & 1) ? 1.5f : 1.f) * ((g() & 2) ? -1.f : 1.f);
        break;
      case 4: x = U(g) * 2.f; s = -x / (float)(1 + g() % 500); break;  // runs into zero
      case 5: x = U(g) * 1.2f; s = U(g) * 3e-4f; break;
      case 6: x = 1.0f + U(g) * 0.5f; s = 0.004f + U(g) * 1e-4f; break;
      case 7: x = std::ldexp(U(g), (int)(g() % 200) - 100); s = std::ldexp(U(g), (int)(g() % 200) - 100); break;
      case 8: case 9: {                                                 // steps with trailing-zero mantissas: ties
        x = U(g) * 4.f;
        s = U(g) * 0.01f;
        uint32_t b;
        std::memcpy(&b, &s, 4);
        b &= ~((1u << (g() % 21)) - 1u);
        if (g() % 16 == 0) b &= 0x80000000u;                            // +-0 steps
        std::memcpy(&s, &b, 4);
        break;
      }
      default: x = (g() & 1) ? INFINITY : NAN; s = U(g); break;          // non-finite
    }
    const int n = (int)(g() % 2100);
    float a = x;
    for (int k = 0; k < n; ++k) a = a + s;
    const float b = kfx::ff_add(x, s, n), c = kfx::ff_add_fast(x, s, n);
    if (std::memcmp(&a, &b, 4) != 0 && !(std::isnan(a) && std::isnan(b))) {
      if (bad < 10) std::printf("x=%a s=%a n=%d loop %a ff %a\n", x, s, n, a, b);
      ++bad;
    }
    if (std::memcmp(&a, &c, 4) != 0 && !(std::isnan(a) && std::isnan(c))) {
      if (bad < 10) std::printf("x=%a s=%a n=%d loop %a ff_fast %a\n", x, s, n, a, c);
      ++bad;
    }
  }
  std::printf("bad %ld\n", bad);
  return bad != 0;
}
