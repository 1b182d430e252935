/* Checks cell_floor (hn_common.h): the quotient num / g from RN(1/g) with one
 * fma correction step equals IEEE division for num >= 2^-100, and its floor
 * equals the IEEE quotient's floor for every num >= 0, over the grid sizes of
 * six boxes x three finest resolutions (num uniform over the box, within 4 ulp
 * of cell boundaries, and tiny).  usage: div_check [trials per level]
 * Exit status 1 on any mismatch.  (tests/test_div_check.py runs it.) */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static uint64_t s = 88172645463325252ull;
static inline uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline float u01(void) { return (float)((rnd() >> 40) * (1.0 / 16777216.0)); }
static inline float nextf(float x, int k) { uint32_t u; memcpy(&u, &x, 4); u += k; memcpy(&x, &u, 4); return x; }
int main(int argc, char** argv) {
  const long per = argc > 1 ? atol(argv[1]) : 2000000;
  /* grid sizes as HashEmbedder computes them: (bmax - bmin) / res, res = floor(16 * b^l) */
  const float boxes[][2] = {{-4.f, 4.f}, {-4.f, 3.3f}, {-3.4f, 3.3f}, {-1.f, 1.f}, {-1.5f, 1.5f}, {-2.f, 2.f}};
  const int finest[] = {512, 1024, 2048};
  long long n = 0, bad = 0, badfloor = 0;
  for (int bi = 0; bi < 6; ++bi)
    for (int fi = 0; fi < 3; ++fi) {
      const float lo = boxes[bi][0], hi = boxes[bi][1];
      const double b = exp((log((double)finest[fi]) - log(16.0)) / 15.0);
      for (int l = 0; l < 16; ++l) {
        const float res = floorf((float)(16.0 * pow(b, l)));
        const float gs = (hi - lo) / res;
        const float y = 1.f / gs;
        for (long t = 0; t < per; ++t) {
          float num;
          const int mode = t % 4;
          if (mode == 0) num = u01() * (hi - lo);
          else if (mode == 1) { int k = (int)(u01() * res); num = nextf((float)k * gs, (int)(rnd() % 9) - 4); }
          else if (mode == 2) { int k = (int)(u01() * res); num = nextf((float)k * gs + gs, (int)(rnd() % 9) - 4); }
          else num = ldexpf(u01(), -(int)(rnd() % 60));
          if (!(num >= 0)) continue;
          float q = num * y;
          float r = fmaf(-gs, q, num);
          q = fmaf(r, y, q);
          const float ref = num / gs;
          ++n;
          if (floorf(q) != floorf(ref)) ++badfloor;
          if (q != ref && num >= 0x1p-100f) { if (bad < 10) printf("mismatch gs=%a num=%a fast=%a ref=%a\n", gs, num, q, ref); ++bad; }
        }
      }
    }
  printf("%lld trials, %lld mismatches (num >= 2^-100), %lld floor mismatches (any num)\n", n, bad, badfloor);
  return bad || badfloor;
}
