// Random-pair check of the FMA (Markstein) division x/d = fma(fma(-q0,d,x),y,q0),
// q0 = RN(x*y), y = RN(1/d), for GENERAL divisors (the projection vc.x / vc.z
// in k_integrate): random x, d over wide exponent ranges + d with extreme
// significands (1.0, 1.111..1, near powers of two).
// gcc -O2 -ffp-contract=off -mfma -fopenmp tools/markstein_general.c -lm -o /tmp/mg && /tmp/mg 2000
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>
static float bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
int main(int argc, char **argv) {
  const long millions = argc > 1 ? atol(argv[1]) : 100;
  long bad = 0, tot = 0;
#pragma omp parallel reduction(+ : bad, tot)
  {
    uint64_t s = 88172645463325252ULL ^ (uint64_t)(size_t)&bad ^ ((uint64_t)omp_get_thread_num() << 40);
#define RND() (s ^= s << 13, s ^= s >> 7, s ^= s << 17, (uint32_t)s)
#pragma omp for
    for (long it = 0; it < millions; ++it) {
      for (int k = 0; k < 1000000; ++k) {
        // d, x: exponents in [2^-40, 2^40], any significand; a quarter with extreme significands
        uint32_t dm = RND() & 0x7fffffu;
        const uint32_t sel = RND() & 7u;
        if (sel == 0) dm = 0x7fffffu - (RND() & 0xffu);
        if (sel == 1) dm = RND() & 0xffu;
        const uint32_t de = 127 - 40 + (RND() % 81);
        const float d = bits((de << 23) | dm) * ((RND() & 1) ? -1.f : 1.f);
        const uint32_t xe = 127 - 40 + (RND() % 81);
        const float x = bits((xe << 23) | (RND() & 0x7fffffu)) * ((RND() & 1) ? -1.f : 1.f);
        const float y = 1.0f / d;
        const float q0 = x * y;
        const float r = fmaf(-q0, d, x);
        const float q1 = fmaf(r, y, q0);
        const float e = x / d;
        ++tot;
        if (memcmp(&q1, &e, 4)) {
          ++bad;
          if (bad < 5) printf("mismatch x=%a d=%a got %a want %a\n", x, d, q1, e);
        }
      }
    }
  }
  printf("tested %ld, mismatches %ld\n", tot, bad);
  return bad != 0;
}
