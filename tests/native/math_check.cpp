// Host check of sfrt_math.h against the host libm (glibc 2.35 atanf/atan2f/asinf/acosf).
// Built and run by tests/test_math_exhaustive.py:
//   g++ -O2 -std=c++17 -ffp-contract=off -fopenmp math_check.cpp -o math_check
//   ./math_check asinf|atanf|acosf      -> every binary32 input
//   ./math_check atan2f <npairs> <seed> -> random + structured pairs
//   ./math_check atan2f_x1 | atan2f_y1  -> atan2f(y, 1) / atan2f(1, x) for every binary32
//   ./math_check divpi                  -> q/PI2 + 1 and q/PI + 0.5 for every finite q
//   ./math_check divrecip <n>           -> div_recip(a, b, 1/b) == a/b on n random pairs
// Prints "<fn> checked=<n> mismatches=<m>" and the first mismatches.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <math.h>

#include "../../sfml-software-raytracer_amd/csrc/sfrt_math.h"

static inline uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float fl(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline bool same(float a, float b) {
  if (std::isnan(a) && std::isnan(b)) return true;  // NaN payloads not compared
  return bits(a) == bits(b);
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const char* fn = argv[1];
  unsigned long long bad = 0, checked = 0;
  if (!strcmp(fn, "asinf") || !strcmp(fn, "atanf") || !strcmp(fn, "acosf")) {
    const int which = !strcmp(fn, "asinf") ? 0 : !strcmp(fn, "atanf") ? 1 : 2;
#pragma omp parallel for reduction(+ : bad, checked) schedule(static)
    for (long long hi = 0; hi < 65536; hi++) {
      for (uint32_t lo = 0; lo < 65536; lo++) {
        const float x = fl((uint32_t)(hi << 16) | lo);
        const float want = which == 0 ? ::asinf(x) : which == 1 ? ::atanf(x) : ::acosf(x);
        const float got = which == 0 ? sfrt_math::asinf(x)
                          : which == 1 ? sfrt_math::atanf(x) : sfrt_math::acosf(x);
        checked++;
        if (!same(want, got)) {
          if (bad < 5) {
#pragma omp critical
            printf("MISMATCH %s(%a [0x%08x]) libm=%a sfrt=%a\n", fn, x, bits(x), want, got);
          }
          bad++;
        }
      }
    }
  } else if (!strcmp(fn, "atan2f_x1") || !strcmp(fn, "atan2f_y1") || !strcmp(fn, "divpi")) {
    const int mode = !strcmp(fn, "atan2f_x1") ? 0 : !strcmp(fn, "atan2f_y1") ? 1 : 2;
#pragma omp parallel for reduction(+ : bad, checked) schedule(static)
    for (long long hi = 0; hi < 65536; hi++) {
      for (uint32_t lo = 0; lo < 65536; lo++) {
        const float v = fl((uint32_t)(hi << 16) | lo);
        bool ok;
        if (mode == 0) {
          ok = same(::atan2f(v, 1.0f), sfrt_math::atan2f(v, 1.0f));
        } else if (mode == 1) {
          ok = same(::atan2f(1.0f, v), sfrt_math::atan2f(1.0f, v));
        } else {
          if (!std::isfinite(v)) continue;
          ok = same(v / 6.28318530718f + 1.0f, sfrt_math::div_pi2_plus_1(v)) &&
               same(v / 3.1415926535f + 0.5f, sfrt_math::div_pi_plus_half(v));
        }
        checked++;
        if (!ok) {
          if (bad < 5) {
#pragma omp critical
            printf("MISMATCH %s(%a)\n", fn, v);
          }
          bad++;
        }
      }
    }
  } else if (!strcmp(fn, "atan2f")) {
    const long long n = argc > 2 ? atoll(argv[2]) : 100000000LL;
    const unsigned seed = argc > 3 ? (unsigned)atoi(argv[3]) : 1u;
    static const float specials[] = {0.0f, -0.0f, 1.0f, -1.0f, INFINITY, -INFINITY, NAN,
                                     1e-45f, -1e-45f, 1e30f, -1e30f, 3.0f, -3.0f, 0.5f};
    const int ns = sizeof(specials) / sizeof(specials[0]);
    for (int a = 0; a < ns; a++)
      for (int b = 0; b < ns; b++) {
        const float y = specials[a], x = specials[b];
        checked++;
        if (!same(::atan2f(y, x), sfrt_math::atan2f(y, x))) {
          if (bad < 5) printf("MISMATCH atan2f(%a, %a)\n", y, x);
          bad++;
        }
      }
#pragma omp parallel for reduction(+ : bad, checked) schedule(static)
    for (long long k = 0; k < n; k++) {
      // splitmix64 -> two floats; half the pairs drawn from the scene domain
      uint64_t z = (uint64_t)k * 0x9E3779B97F4A7C15ULL + seed * 0xD1B54A32D192ED03ULL;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
      z ^= z >> 31;
      float y, x;
      if (k & 1) {
        y = fl((uint32_t)z);
        x = fl((uint32_t)(z >> 32));
      } else {  // |coords| < 64, the range hit points live in
        y = ((float)(uint32_t)z / 4294967296.0f - 0.5f) * 128.0f;
        x = ((float)(uint32_t)(z >> 32) / 4294967296.0f - 0.5f) * 128.0f;
      }
      const float want = ::atan2f(y, x), got = sfrt_math::atan2f(y, x);
      checked++;
      if (!same(want, got)) {
        if (bad < 5) {
#pragma omp critical
          printf("MISMATCH atan2f(%a, %a) libm=%a sfrt=%a\n", y, x, want, got);
        }
        bad++;
      }
    }
  } else if (!strcmp(fn, "divrecip")) {
    // sfrt_math::div_recip(a, b, 1/b) == a / b over random normal pairs and the
    // voxel DDA domain (b in (2^-14, 1.5], a in [-0.25, 1.25]).
    const long long n = argc > 2 ? atoll(argv[2]) : 100000000LL;
#pragma omp parallel for reduction(+ : bad, checked) schedule(static)
    for (long long k = 0; k < n; k++) {
      uint64_t z = (uint64_t)k * 0x9E3779B97F4A7C15ULL + 77;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
      z ^= z >> 31;
      float a, b;
      if (k & 1) {
        const uint32_t eb = 127 - 60 + (uint32_t)((z >> 40) % 121);
        const uint32_t ea = eb - 40 + (uint32_t)((z >> 48) % 81);
        b = fl((eb << 23) | ((uint32_t)z & 0x7fffffu) | (uint32_t)((z >> 63) << 31));
        a = fl((ea << 23) | ((uint32_t)(z >> 20) & 0x7fffffu) | (uint32_t)(((z >> 62) & 1) << 31));
      } else {
        b = 1.5f * ((float)((uint32_t)z >> 8) / 16777216.0f);
        if (b < 0x1.0p-14f) b = 0x1.0p-14f;
        a = -0.25f + 1.5f * ((float)((uint32_t)(z >> 32) >> 8) / 16777216.0f);
      }
      checked++;
      if (!same(a / b, sfrt_math::div_recip(a, b, 1.0f / b))) {
        if (bad < 5) {
#pragma omp critical
          printf("MISMATCH divrecip a=%a b=%a\n", a, b);
        }
        bad++;
      }
    }
  } else {
    return 2;
  }
  printf("%s checked=%llu mismatches=%llu\n", fn, checked, bad);
  return bad ? 1 : 0;
}
