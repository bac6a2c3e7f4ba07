// gfx950 check of sfrt_math::div_recip(a, b, 1.0f / b) == a / b (correctly
// rounded division, classes 0-2) and of sfrt::div_inrange(a, b) == a / b (the
// compiler's division sequence without its range scaling, classes 3-4), bit for
// bit, entirely on the device (no host compare).
// Built and run by tests/test_gpu_parity.py::test_device_div_recip:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off div_check.hip -o div_check
//   ./div_check <log2 pairs per class>
// Classes: random normal b in [2^-60, 2^60] with random a keeping a/b normal;
// the voxel DDA domain (b in (2^-14, 1.5], a in [-0.25, 1.25]); b with
// all-ones / one-ulp-off-a-power-of-two significands and dense a in [0, 2).
// div_inrange: random a, b with |a|, |b| in [2^-40, 2^40) (every 64th a = +0 with
// b > 0); b with hard significands in the same range and random a.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../sfml-software-raytracer_amd/csrc/sfrt_device.h"
#include "../../sfml-software-raytracer_amd/csrc/sfrt_math.h"

#pragma clang fp contract(off)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float u01(uint32_t u) { return (float)(u >> 8) * (1.0f / 16777216.0f); }

__global__ void k_check(int cls, unsigned long long iters, unsigned long long* bad,
                        float* example) {
  const unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long nt = (unsigned long long)gridDim.x * blockDim.x;
  unsigned long long nbad = 0;
  for (unsigned long long k = t; k < iters; k += nt) {
    const uint64_t z = mix(k * 0x9E3779B97F4A7C15ULL + 0x1234567ULL * (cls + 1));
    float a, b;
    if (cls == 0) {        // random normal operands, quotient kept normal
      const uint32_t eb = 127 - 60 + (uint32_t)((z >> 40) % 121);
      const uint32_t ea = eb - 40 + (uint32_t)((z >> 48) % 81);
      b = sfrt_math::u2f((eb << 23) | ((uint32_t)z & 0x7fffffu) | ((z >> 63) << 31));
      a = sfrt_math::u2f((ea << 23) | ((uint32_t)(z >> 20) & 0x7fffffu) | (((z >> 62) & 1) << 31));
    } else if (cls == 1) { // voxel DDA domain
      b = 1.5f * u01((uint32_t)z);
      if (b < 0x1.0p-14f) b = 0x1.0p-14f;
      a = -0.25f + 1.5f * u01((uint32_t)(z >> 32));
    } else if (cls == 3 || cls == 4) {  // div_inrange operands: |a|, |b| in [2^-40, 2^40)
      const uint32_t eb = 127 - 40 + (uint32_t)((z >> 40) % 80);
      const uint32_t ea = 127 - 40 + (uint32_t)((z >> 48) % 80);
      uint32_t mant = (uint32_t)z & 0x7fffffu;
      if (cls == 4) {
        const uint32_t kind = (uint32_t)(z >> 61);
        mant = kind < 2 ? 0x7fffffu : (kind < 4 ? 0x000001u : (kind < 6 ? 0x7ffffeu : 0u));
      }
      b = sfrt_math::u2f((eb << 23) | mant | ((z >> 63) << 31));
      a = sfrt_math::u2f((ea << 23) | ((uint32_t)(z >> 20) & 0x7fffffu) | (((z >> 62) & 1) << 31));
      if (cls == 3 && ((z >> 8) & 63) == 0) {  // +0 over a positive b
        a = 0.0f;
        b = fabsf(b);
      }
    } else {               // hard significands for b, dense a
      const uint32_t kind = (uint32_t)(z >> 61);
      const uint32_t eb = 127 - 20 + (uint32_t)((z >> 50) % 41);
      uint32_t mant = kind < 2 ? 0x7fffffu : (kind < 4 ? 0x000001u : (kind < 6 ? 0x7ffffeu : (uint32_t)(z >> 24) & 0x7fffffu));
      b = sfrt_math::u2f((eb << 23) | mant);
      a = sfrt_math::u2f((uint32_t)(127u << 23) | ((uint32_t)z & 0x7fffffu)) - 1.0f + u01((uint32_t)(z >> 32));
    }
    const float want = a / b;
    const float got = cls >= 3 ? sfrt::div_inrange(a, b) : sfrt_math::div_recip(a, b, 1.0f / b);
    const bool same = (want != want && got != got) || sfrt_math::f2u(want) == sfrt_math::f2u(got);
    if (!same) {
      nbad++;
      example[0] = a;
      example[1] = b;
    }
  }
  if (nbad) atomicAdd(bad, nbad);
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 33;
  const unsigned long long iters = 1ull << lg;
  unsigned long long* d_bad;
  float* d_ex;
  if (hipMalloc(&d_bad, 8) || hipMalloc(&d_ex, 8)) return 3;
  unsigned long long total_bad = 0, total = 0;
  for (int cls = 0; cls < 5; cls++) {
    unsigned long long zero = 0;
    float ex[2] = {0, 0};
    hipMemcpy(d_bad, &zero, 8, hipMemcpyHostToDevice);
    hipMemcpy(d_ex, ex, 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check, dim3(256 * 64), dim3(256), 0, 0, cls, iters, d_bad, d_ex);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    unsigned long long b = 0;
    hipMemcpy(&b, d_bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(ex, d_ex, 8, hipMemcpyDeviceToHost);
    if (b) printf("MISMATCH class %d: %llu, e.g. a=%a b=%a\n", cls, b, ex[0], ex[1]);
    total_bad += b;
    total += iters;
  }
  printf("div_recip/div_inrange checked=%llu mismatches=%llu\n", total, total_bad);
  return total_bad ? 1 : 0;
}
