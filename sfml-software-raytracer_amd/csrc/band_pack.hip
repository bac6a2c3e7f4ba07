// band_pack.hip -- the transfer format of a row band on its way to rank 0
// (the path's one exchange step; DESIGN.md 7 "Packed bands").
//
// A band crosses xGMI once per frame and at N >= 2 rank 0's ingress bounds the
// step.  A frame pixel is (texel.rgb * brightness, texel.a) (SphereWorld.cpp:
// 376-381, stored by :109), so its alpha is a texel's alpha; the reference's
// textures hold alpha 0 or 255 only (Floor.png, sfrt_world_alpha_binary checks
// the loaded ones).  Such a band packs losslessly into 3 bytes of RGB plus one
// alpha bit per pixel: 3.125 B instead of 4 (22% fewer bytes over the link).
//
// Layout for P pixels, B = ceil(P / 256) blocks, B * 800 bytes in two planes (the
// RGB of every block first, then every block's alpha bits):
//   [0, 768 B * B)            RGB plane, pixel p at bytes 3p .. 3p+2 (R, G, B);
//                             bytes past pixel P in the last block are zero;
//   [768 B * B, 800 B * B)    alpha plane, bit p of the little-endian bit string =
//                             pixel p's alpha is 255 (0 = alpha 0); bits past P are zero.
// Both kernels are HBM-streaming: a lane moves 4 pixels (16 B in, 12 B + 4 bits
// out, or back), a wave one 256-pixel block.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sfrt.h"
#include "sfrt_host.h"

namespace {

constexpr int kBlockPx = 256;        // pixels per wave (4 per lane)
constexpr int kBlockRgb = 3 * kBlockPx;
constexpr int kThreads = 256;        // 4 waves per workgroup

__global__ __launch_bounds__(kThreads) void k_band_pack(const uint32_t* __restrict__ rgba,
                                                        int64_t pixels, int64_t blocks,
                                                        uint32_t* __restrict__ rgb,
                                                        uint64_t* __restrict__ bits) {
  const int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (t >= blocks * 64) return;  // whole waves only (blocks * 64 lanes)
  const int64_t p0 = t * 4;
  uint32_t px[4];
  if (p0 + 3 < pixels) {
#pragma unroll
    for (int i = 0; i < 4; i++) px[i] = __builtin_nontemporal_load(rgba + p0 + i);
  } else {
#pragma unroll
    for (int i = 0; i < 4; i++) px[i] = p0 + i < pixels ? rgba[p0 + i] : 0u;
  }
  rgb[3 * t + 0] = (px[0] & 0xffffffu) | (px[1] << 24);
  rgb[3 * t + 1] = ((px[1] >> 8) & 0xffffu) | (px[2] << 16);
  rgb[3 * t + 2] = ((px[2] >> 16) & 0xffu) | (px[3] << 8);
  uint32_t nib = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) nib |= (uint32_t)((px[i] >> 24) == 0xffu) << i;
  // 16 lanes -> one 64-bit word: lane l's nibble at bits 4 (l % 16) .. +3
  const int l16 = (int)(t & 15);
  uint64_t word = (uint64_t)nib << (4 * l16);
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) word |= (uint64_t)__shfl_xor((unsigned long long)word, m, 16);
  if (l16 == 0) bits[t >> 4] = word;
}

struct Rgb4 {  // one lane's 12 bytes of RGB (one dwordx3 load)
  uint32_t w0, w1, w2;
};

// A16: the RGBA destination is 16-byte aligned, so a lane's 4 pixels are one dwordx4 store.
template <bool A16>
__global__ __launch_bounds__(kThreads) void k_band_unpack(const Rgb4* __restrict__ rgb,
                                                          const uint64_t* __restrict__ bits,
                                                          int64_t pixels,
                                                          uint32_t* __restrict__ rgba) {
  const int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const int64_t p0 = t * 4;
  if (p0 >= pixels) return;
  const Rgb4 v = rgb[t];
  const uint32_t w0 = v.w0, w1 = v.w1, w2 = v.w2;
  const uint32_t nib = (uint32_t)(bits[t >> 4] >> (4 * (int)(t & 15)));
  const uint32_t a = 0xff000000u;
  uint32_t px[4];
  px[0] = (w0 & 0xffffffu) | ((nib & 1u) ? a : 0u);
  px[1] = (w0 >> 24) | ((w1 & 0xffffu) << 8) | ((nib & 2u) ? a : 0u);
  px[2] = (w1 >> 16) | ((w2 & 0xffu) << 16) | ((nib & 4u) ? a : 0u);
  px[3] = (w2 >> 8) | ((nib & 8u) ? a : 0u);
  if (A16 && p0 + 3 < pixels) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 q = {px[0], px[1], px[2], px[3]};
    __builtin_nontemporal_store(q, (u32x4*)(rgba + p0));
  } else if (p0 + 3 < pixels) {
#pragma unroll
    for (int i = 0; i < 4; i++) __builtin_nontemporal_store(px[i], rgba + p0 + i);
  } else {
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (p0 + i < pixels) rgba[p0 + i] = px[i];
  }
}

int64_t blocks_of(int64_t pixels) { return (pixels + kBlockPx - 1) / kBlockPx; }

// RGBA pixels are dwords; the packed buffer's bit words are 8-byte words at an offset of
// a multiple of 768 B, so the buffer itself must be 8-byte aligned.
bool args_ok(const void* rgba, int64_t pixels, const void* packed) {
  if (pixels < 0) return false;
  if (pixels == 0) return true;
  return rgba && packed && ((uintptr_t)rgba & 3u) == 0 && ((uintptr_t)packed & 7u) == 0;
}

}  // namespace

extern "C" {

int64_t sfrt_band_packed_bytes(int64_t pixels) {
  if (pixels < 0) return SFRT_E_INVALID;
  return blocks_of(pixels) * (kBlockRgb + kBlockPx / 8);
}

int sfrt_band_pack(const void* dev_rgba, int64_t pixels, void* dev_packed, void* hip_stream) {
  if (!args_ok(dev_rgba, pixels, dev_packed)) return SFRT_E_INVALID;
  if (pixels == 0) return SFRT_OK;
  const int64_t blocks = blocks_of(pixels);
  uint32_t* rgb = (uint32_t*)dev_packed;
  uint64_t* bits = (uint64_t*)((uint8_t*)dev_packed + blocks * kBlockRgb);
  const int64_t grid = (blocks * 64 + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(k_band_pack, dim3((unsigned)grid), dim3(kThreads), 0, (hipStream_t)hip_stream,
                     (const uint32_t*)dev_rgba, pixels, blocks, rgb, bits);
  HIP_TRY(hipGetLastError());
  return SFRT_OK;
}

int sfrt_band_unpack(const void* dev_packed, int64_t pixels, void* dev_rgba, void* hip_stream) {
  if (!args_ok(dev_rgba, pixels, dev_packed)) return SFRT_E_INVALID;
  if (pixels == 0) return SFRT_OK;
  const int64_t blocks = blocks_of(pixels);
  const Rgb4* rgb = (const Rgb4*)dev_packed;
  const uint64_t* bits = (const uint64_t*)((const uint8_t*)dev_packed + blocks * kBlockRgb);
  const int64_t grid = (blocks * 64 + kThreads - 1) / kThreads;
  if (((uintptr_t)dev_rgba & 15u) == 0)
    hipLaunchKernelGGL(k_band_unpack<true>, dim3((unsigned)grid), dim3(kThreads), 0,
                       (hipStream_t)hip_stream, rgb, bits, pixels, (uint32_t*)dev_rgba);
  else
    hipLaunchKernelGGL(k_band_unpack<false>, dim3((unsigned)grid), dim3(kThreads), 0,
                       (hipStream_t)hip_stream, rgb, bits, pixels, (uint32_t*)dev_rgba);
  HIP_TRY(hipGetLastError());
  return SFRT_OK;
}

}  // extern "C"
