// Device check of sfrt_math.h on gfx950 against the host libm (glibc 2.35).
// Built and run by tests/test_gpu_parity.py::test_device_math_matches_libm:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fopenmp math_gpu_check.hip
//   ./math_gpu_check asinf|atanf|acosf [stride] -> every stride-th binary32 pattern
//   ./math_gpu_check atan2f <npairs>        -> random + scene-range pairs
//   ./math_gpu_check sqrt_div [stride]      -> correctly rounded sqrtf and x/y vs the host
//   ./math_gpu_check divpi                  -> x/PI2 + 1 and x/PI + 0.5 (fma form) for every finite x
//   ./math_gpu_check atan2f_x1              -> atan2f(y, 1) for every binary32 y
//   ./math_gpu_check atan2f_wave <npairs>   -> sfrt::atan2f_wave (sfrt_device.h) on waves of
//                                              random bits, mixed scene-range pairs, pairs
//                                              sharing one atanf interval, and smooth sweeps
// Prints "<fn> checked=<n> mismatches=<m>".
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../sfml-software-raytracer_amd/csrc/sfrt_device.h"
#include "../../sfml-software-raytracer_amd/csrc/sfrt_math.h"

#pragma clang fp contract(off)

__global__ void k_eval(int fn, const float* __restrict__ x, const float* __restrict__ y,
                       float* __restrict__ out, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float r;
  switch (fn) {
    case 0: r = sfrt_math::asinf(x[i]); break;
    case 1: r = sfrt_math::atanf(x[i]); break;
    case 2: r = sfrt_math::atan2f(x[i], y[i]); break;
    case 3: r = __builtin_sqrtf(x[i]); break;
    case 4: r = x[i] / y[i]; break;
    case 5: r = sfrt_math::div_pi2_plus_1(x[i]); break;
    case 6: r = sfrt_math::div_pi_plus_half(x[i]); break;
    case 8: r = sfrt_math::acosf(x[i]); break;
    case 9: r = sfrt::atan2f_wave(x[i], y[i]); break;
    default: r = sfrt_math::atan2f(x[i], 1.0f); break;
  }
  out[i] = r;
}

static float host_eval(int fn, float x, float y) {
  switch (fn) {
    case 0: return ::asinf(x);
    case 1: return ::atanf(x);
    case 2: return ::atan2f(x, y);
    case 3: return std::sqrt(x);
    case 4: return x / y;
    case 5: return std::isfinite(x) ? x / 6.28318530718f + 1.0f : NAN;
    case 6: return std::isfinite(x) ? x / 3.1415926535f + 0.5f : NAN;
    case 8: return ::acosf(x);
    case 9: return ::atan2f(x, y);
    default: return ::atan2f(x, 1.0f);
  }
}

static inline uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float fl(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  int fn;
  if (!strcmp(argv[1], "asinf")) fn = 0;
  else if (!strcmp(argv[1], "atanf")) fn = 1;
  else if (!strcmp(argv[1], "atan2f")) fn = 2;
  else if (!strcmp(argv[1], "sqrt_div")) fn = 3;
  else if (!strcmp(argv[1], "divpi")) fn = 5;
  else if (!strcmp(argv[1], "atan2f_x1")) fn = 7;
  else if (!strcmp(argv[1], "acosf")) fn = 8;
  else if (!strcmp(argv[1], "atan2f_wave")) fn = 9;
  else return 2;
  const long long total = (fn == 2 || fn == 9) ? (argc > 2 ? atoll(argv[2]) : 100000000LL)
                                  : (4294967296LL / (argc > 2 ? atoll(argv[2]) : 1));
  const long long stride = (fn == 2 || fn == 9) ? 1 : (argc > 2 ? atoll(argv[2]) : 1);
  const long chunk = 1L << 26;
  std::vector<float> hx(chunk), hy(chunk), hout(chunk);
  float *dx, *dy, *dout;
  if (hipMalloc(&dx, chunk * 4) || hipMalloc(&dy, chunk * 4) || hipMalloc(&dout, chunk * 4)) {
    printf("hipMalloc failed\n");
    return 3;
  }
  unsigned long long checked = 0, bad = 0;
  const int passes = (fn == 3 || fn == 5) ? 2 : 1;  // sqrt_div: sqrtf, x/y; divpi: PI2, PI
  for (int pass = 0; pass < passes; pass++) {
    const int f = (fn == 3 || fn == 5) ? fn + pass : fn;
    for (long long base = 0; base < total; base += chunk) {
      const long n = (long)((total - base) < chunk ? (total - base) : chunk);
#pragma omp parallel for schedule(static)
      for (long i = 0; i < n; i++) {
        const long long k = base + i;
        if (f == 9) {
          // 64-lane blocks (one wave each): 0 random bits, 1 mixed scene-range pairs,
          // 2 one atanf interval per wave (ratios inside it, either sign), 3 smooth sweeps
          const long long b = k >> 6;
          const uint64_t z = mix((uint64_t)k * 0x9E3779B97F4A7C15ULL + 11);
          const uint64_t zb = mix((uint64_t)b * 0xD1B54A32D192ED03ULL + 5);
          const float u0 = (float)(uint32_t)z / 4294967296.0f;
          const float u1 = (float)(uint32_t)(z >> 32) / 4294967296.0f;
          switch (b & 3) {
            case 0: hx[i] = fl((uint32_t)z); hy[i] = fl((uint32_t)(z >> 32)); break;
            case 1: hx[i] = (u0 - 0.5f) * 128.0f; hy[i] = (u1 - 0.5f) * 128.0f; break;
            case 2: {
              static const float edges[6] = {0x1p-29f, 0.4375f, 0.6875f, 1.1875f, 2.4375f, 0x1p25f};
              const int id = (int)((zb >> 8) % 5);
              const float lo = edges[id], hi = edges[id + 1];
              const float rho = lo * std::pow(hi / lo, u0);
              const float xx = (0.25f + u1 * 60.0f) * ((zb & 1) ? -1.0f : 1.0f);
              hy[i] = xx;
              hx[i] = xx * rho * (((zb >> 1) & 1) ? -1.0f : 1.0f);
              if ((z & 1023) == 0) hx[i] = lo * xx;  // interval edges
              break;
            }
            default: {
              const float th = (float)((zb >> 11) % 6283) * 1e-3f + (float)(k & 63) * 1e-4f;
              const float sc = 1.0f + (float)((zb >> 24) % 1000);
              hx[i] = std::sin(th) * sc;
              hy[i] = std::cos(th) * sc;
            }
          }
        } else if (f == 2 || f == 4) {
          const uint64_t z = mix((uint64_t)k * 0x9E3779B97F4A7C15ULL + 7);
          if (k & 1) {
            hx[i] = fl((uint32_t)z);
            hy[i] = fl((uint32_t)(z >> 32));
          } else {
            hx[i] = ((float)(uint32_t)z / 4294967296.0f - 0.5f) * 128.0f;
            hy[i] = ((float)(uint32_t)(z >> 32) / 4294967296.0f - 0.5f) * 128.0f;
          }
        } else {
          hx[i] = fl((uint32_t)(k * stride));
          hy[i] = 0.0f;
        }
      }
      if (hipMemcpy(dx, hx.data(), n * 4, hipMemcpyHostToDevice) ||
          hipMemcpy(dy, hy.data(), n * 4, hipMemcpyHostToDevice))
        return 3;
      hipLaunchKernelGGL(k_eval, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, f, dx, dy, dout, n);
      if (hipMemcpy(hout.data(), dout, n * 4, hipMemcpyDeviceToHost)) return 3;
      unsigned long long b = 0;
#pragma omp parallel for reduction(+ : b) schedule(static)
      for (long i = 0; i < n; i++) {
        const float want = host_eval(f, hx[i], hy[i]);
        const float got = hout[i];
        const bool skip = (f == 5 || f == 6) && !std::isfinite(hx[i]);  // finite inputs only
        const bool ok = skip || (std::isnan(want) && std::isnan(got)) || bits(want) == bits(got);
        if (!ok) b++;
      }
      if (b && bad < 1) {
        for (long i = 0; i < n; i++) {
          const float want = host_eval(f, hx[i], hy[i]);
          const bool skip = (f == 5 || f == 6) && !std::isfinite(hx[i]);
          if (!skip && !((std::isnan(want) && std::isnan(hout[i])) || bits(want) == bits(hout[i]))) {
            printf("MISMATCH fn=%d x=%a y=%a host=%a gpu=%a\n", f, hx[i], hy[i], want, hout[i]);
            break;
          }
        }
      }
      bad += b;
      checked += n;
    }
  }
  printf("%s checked=%llu mismatches=%llu\n", argv[1], checked, bad);
  return bad ? 1 : 0;
}
