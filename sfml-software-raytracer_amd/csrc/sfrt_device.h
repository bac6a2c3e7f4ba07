// sfrt_device.h -- gfx950 device helpers shared by the trace kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "sfrt_math.h"

#pragma clang fp contract(off)

namespace sfrt {

// v, unchanged, through an empty asm: arithmetic on the result cannot be hoisted above the
// asm, nor the asm speculated.  Used at the head of a wave-uniform fallback branch (a
// ballot found some lane outside a fast path's domain) to keep it a branch: left to itself
// the compiler if-converts such branches -- computing BOTH the fallback and the fast path
// for every wave and selecting -- which cost ~5 % of the frame kernel's VALU.
__device__ __forceinline__ float keep_branch(float v) {
  __asm__ volatile("; keep_branch" : "+v"(v));  // (the comment marks rare paths for tools/)
  return v;
}

// A 64-bit value made wave-uniform (SGPR pair) from lane 0's copy.  The
// builtin returns int: each half goes through uint32_t so the low word is
// zero-extended, not sign-extended into the high word.
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Wave-wide min / max of unsigned words, all in DPP: the row reduction
// (quad_perm, half-mirror, mirror; each step one v_min_u32_dpp), then
// row_bcast:15 into rows 1 and 3 and row_bcast:31 into rows 2 and 3, so lane
// 63 holds the wave's result.  For binary32 values >= +0 (no NaN) the bit
// patterns order like the values, so these also reduce non-negative floats
// with no canonicalising VALU ops.  Call with the whole wave active (DPP
// reads inactive lanes' stale values).
// IDENTITY (the op's neutral value) fills lanes whose row is masked off, so
// the compiler folds each mov_dpp into the min / max itself.
template <int CTRL, int ROW_MASK, uint32_t IDENTITY>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)IDENTITY, (int)x, CTRL, ROW_MASK, 0xf, false);
}

template <bool MAX>
__device__ __forceinline__ uint32_t wave_reduce_u32(uint32_t v) {
  constexpr uint32_t I = MAX ? 0u : 0xffffffffu;
  auto op = [](uint32_t a, uint32_t b) {
    return MAX ? __builtin_elementwise_max(a, b) : __builtin_elementwise_min(a, b);
  };
  v = op(v, dpp_u32<0xB1, 0xf, I>(v));   // quad_perm [1,0,3,2]
  v = op(v, dpp_u32<0x4E, 0xf, I>(v));   // quad_perm [2,3,0,1]
  v = op(v, dpp_u32<0x141, 0xf, I>(v));  // row_half_mirror
  v = op(v, dpp_u32<0x140, 0xf, I>(v));  // row_mirror
  v = op(v, dpp_u32<0x142, 0xa, I>(v));  // row_bcast:15 -> rows 1, 3
  v = op(v, dpp_u32<0x143, 0xc, I>(v));  // row_bcast:31 -> rows 2, 3
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) { return wave_reduce_u32<false>(v); }
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) { return wave_reduce_u32<true>(v); }

// sqrtf(x) correctly rounded for x >= 2^-96 (not denormal/tiny): the raw
// v_sqrt_f32 (within 1 ulp) corrected by the two fma residual tests that the
// compiler's own correctly rounded lowering uses -- minus its tiny-input
// rescaling and special-value selects, which these inputs never need.
__device__ __forceinline__ float sqrt_cr_normal(float x) {
  const float r = __builtin_amdgcn_sqrtf(x);
  const float rm = sfrt_math::u2f(sfrt_math::f2u(r) - 1u);
  const float rp = sfrt_math::u2f(sfrt_math::f2u(r) + 1u);
  float q = __builtin_fmaf(-rm, r, x) <= 0.0f ? rm : r;
  q = __builtin_fmaf(-rp, r, x) > 0.0f ? rp : q;
  return q;
}

// a / b, correctly rounded, for operands that need none of the hardware division's
// range handling.  hipcc lowers a binary32 `a / b` on gfx950 to
//   d = v_div_scale(b, b, a); y0 = v_rcp(d); y = fma(fma(-d, y0, 1), y0, y0);
//   n = v_div_scale(a, b, a); q = n*y; q = fma(fma(-d, q, n), y, q);
//   v_div_fixup(v_div_fmas(fma(-d, q, n), y, q), b, a)
// (11 VALU).  v_div_scale returns its operand unchanged and clears VCC -- so
// v_div_fmas is a plain fma -- unless a or b is zero, denormal, inf or NaN, 1/b
// or a/b is denormal, |a| < 2^-103 or a's exponent exceeds b's by 96 or more;
// v_div_fixup returns the quotient unchanged when it is finite, normal and
// neither operand is special.  For finite normal a, b with a/b normal, and
// |b| < 2^126, all of that holds, and div_seed(b) + div_inrange(a, b, y) run
// the same operations on the same values (2 + 5 VALU, the seed shared by every
// division by b).  Also exact for a = +0 with b > 0 (every step yields +0).
// Checked against `/` on gfx950 (tests/native/div_check.hip, classes 3-4).
__device__ __forceinline__ float div_seed(float b) {
  const float y0 = __builtin_amdgcn_rcpf(b);
  return __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
}
__device__ __forceinline__ float div_inrange(float a, float b, float y) {
  float q = a * y;
  q = __builtin_fmaf(__builtin_fmaf(-b, q, a), y, q);
  return __builtin_fmaf(__builtin_fmaf(-b, q, a), y, q);
}
__device__ __forceinline__ float div_inrange(float a, float b) { return div_inrange(a, b, div_seed(b)); }

// |v| in [2^-40, 2^40) (so finite, non-zero, normal): two quotients of such
// values are normal and every precondition of div_inrange holds.  Two compares
// with |v| as a source modifier (NaN fails both), combined in the SGPR masks.
__device__ __forceinline__ bool div_operand_ok(float v) {
  return __builtin_fabsf(v) >= 0x1.0p-40f && __builtin_fabsf(v) < 0x1.0p40f;
}

// The wave's lanes whose v fails div_operand_ok, as the OR of one ballot per compare: a
// ballot of a combined condition costs two more VALU (the compiler turns the lane mask back
// into a value and compares it again), a ballot of one compare is that compare's own mask.
__device__ __forceinline__ uint64_t ballot_bad_operand(float v) {
  return __builtin_amdgcn_ballot_w64(!(__builtin_fabsf(v) >= 0x1.0p-40f)) |
         __builtin_amdgcn_ballot_w64(!(__builtin_fabsf(v) < 0x1.0p40f));
}

// a[i] / b for N numerators sharing one divisor, correctly rounded (the bits of `/`): one
// reciprocal seed for all when every lane's operands lie in [2^-40, 2^40) (div_inrange's
// domain, checked per compare: ballot_bad_operand); a wave with any other operand -- a zero
// numerator among them -- divides plainly.
template <int N>
__device__ __forceinline__ void div_shared(const float (&a)[N], float b, float (&q)[N]) {
  uint64_t bad = ballot_bad_operand(b);
#pragma unroll
  for (int i = 0; i < N; i++) bad |= ballot_bad_operand(a[i]);
  if (bad == 0) {
    const float y = div_seed(b);
#pragma unroll
    for (int i = 0; i < N; i++) q[i] = div_inrange(a[i], b, y);
  } else {
    const float bb = keep_branch(b);
#pragma unroll
    for (int i = 0; i < N; i++) q[i] = a[i] / bb;
  }
}

// c / 255.0f for an integer c in [0, 255], correctly rounded: RN(c * RN(1/255)) corrected once
// by Markstein's fma step (exact for all 256 c: tests/test_math_exhaustive.py::test_div255_exact, exact rationals).
__device__ __forceinline__ float div255(float c) {
  const float y = 0x1.010102p-8f;  // RN(1/255)
  const float q = c * y;
  return __builtin_fmaf(__builtin_fmaf(-255.0f, q, c), y, q);
}

// atan2f(y, x), bit for bit sfrt_math::atan2f (= glibc's e_atan2f.c), with a
// cheaper path for the waves the renderers produce.  When every lane of the
// wave has finite non-zero x and y and |y/x| in [2^-29, 2^25), no special case
// of e_atan2f.c / s_atanf.c can fire: the |y|/x < -2^60 and |y/x| > 2^60
// overrides need an exponent gap above 60, the tiny and huge atanf branches an
// argument outside that range.  Then atanf runs on the positive |y/x| (no sign
// handling), and when all lanes also share the argument-reduction interval,
// only that interval's code runs (a uniform branch; one division, none for
// |y/x| < 7/16).  The quadrant fix-up uses (z + pi_lo) - pi == -(pi - (z + pi_lo))
// (round-to-nearest is symmetric).  Any other wave takes sfrt_math::atan2f.
__device__ __forceinline__ float atan2f_wave(float y, float x) {
  using sfrt_math::f2u;
  using sfrt_math::u2f;
  const uint32_t hx = f2u(x), hy = f2u(y);
  // |x|, |y| in [2^-40, 2^40): y / x through div_inrange (a wave with other operands,
  // all rare, takes the general code, like one with |y/x| outside [2^-29, 2^25))
  const float q = div_inrange(y, x);
  const uint32_t iq = f2u(q) & 0x7fffffffu;
  // (ballot_bad_operand: one ballot per compare)
  if (ballot_bad_operand(x) | ballot_bad_operand(y) |
      __builtin_amdgcn_ballot_w64(!(iq - 0x31000000u < 0x4c000000u - 0x31000000u)))
    return sfrt_math::atan2f(y, x);
  const float a = u2f(iq);
  const int id = iq < 0x3ee00000u ? -1
               : iq < 0x3f300000u ? 0
               : iq < 0x3f980000u ? 1
               : iq < 0x401c0000u ? 2
               : 3;
  // The reduction divisions below use div_inrange: a in [2^-29, 2^25) makes every
  // denominator lie in [1, 1.5 * 2^25 + 1] and every numerator +0 (a = 0.5, 1, 1.5)
  // or of magnitude >= 2^-29 (a multiple of a's ulp, or a itself over 1).
  // s_atanf.c tail for the reduced argument xr: (s1 + s2) * xr and the final sum
  auto poly = [](float xr) {
    const float z = xr * xr;
    const float w = z * z;
    float s1 = u2f(0x3c8569d7u) * w + u2f(0x3d4bda59u);
    s1 = s1 * w + u2f(0x3d886b35u);
    s1 = s1 * w + u2f(0x3dba2e6eu);
    s1 = s1 * w + u2f(0x3e124925u);
    s1 = s1 * w + u2f(0x3eaaaaabu);
    s1 = s1 * z;
    float s2 = u2f(0xbd15a221u) * w - u2f(0x3d6ef16bu);
    s2 = s2 * w - u2f(0x3d9d8795u);
    s2 = s2 * w - u2f(0x3de38e38u);
    s2 = s2 * w - u2f(0x3e4ccccdu);
    s2 = s2 * w;
    return (s1 + s2) * xr;
  };
  float zr;
  const int id0 = __builtin_amdgcn_readfirstlane(id);
  if (__builtin_amdgcn_ballot_w64(id != id0) == 0) {
    // one reduction interval for the whole wave (uniform branch)
    if (id0 < 0) {
      zr = a - poly(a);
    } else {
      float xr, hi, lo;
      if (id0 == 0) {
        xr = div_inrange((a + a) - 1.0f, a + 2.0f);
        hi = u2f(0x3eed6338u); lo = u2f(0x31ac3769u);
      } else if (id0 == 1) {
        xr = div_inrange(a - 1.0f, a + 1.0f);
        hi = u2f(0x3f490fdau); lo = u2f(0x33222168u);
      } else if (id0 == 2) {
        xr = div_inrange(a - 1.5f, a * 1.5f + 1.0f);
        hi = u2f(0x3f7b985eu); lo = u2f(0x33140fb4u);
      } else {
        xr = div_inrange(-1.0f, a);
        hi = u2f(0x3fc90fdau); lo = u2f(0x33a22168u);
      }
      zr = hi - ((poly(xr) - lo) - xr);
    }
  } else {
    float num = a, den = 1.0f;
    if (id == 0) { num = (a + a) - 1.0f; den = a + 2.0f; }
    if (id == 1) { num = a - 1.0f; den = a + 1.0f; }
    if (id == 2) { num = a - 1.5f; den = a * 1.5f + 1.0f; }
    if (id == 3) { num = -1.0f; den = a; }
    const float xr = div_inrange(num, den);
    const float xs = poly(xr);
    float hi = u2f(0x3fc90fdau), lo = u2f(0x33a22168u);
    if (id == 0) { hi = u2f(0x3eed6338u); lo = u2f(0x31ac3769u); }
    if (id == 1) { hi = u2f(0x3f490fdau); lo = u2f(0x33222168u); }
    if (id == 2) { hi = u2f(0x3f7b985eu); lo = u2f(0x33140fb4u); }
    zr = id < 0 ? xr - xs : hi - ((xs - lo) - xr);
  }
  // e_atan2f.c quadrants: m = 0: z, 1: -z, 2: pi - (z + pi_lo), 3: (z + pi_lo) - pi
  const float r = (int32_t)hx < 0 ? u2f(0x40490fdbu) - (zr + u2f(0x33bbbd2eu)) : zr;
  return u2f(f2u(r) ^ (hy & 0x80000000u));
}

// ---- adaptive tile order (DESIGN.md 5 "Tile order"; host side sfrt_sched.h) ----
constexpr int kTileBuckets = 16;  // march-step classes

// Tile-order bucket of a tile's march steps, longest first: 16 classes, finer
// where most tiles are (steps 4..16 at 4K).
__device__ __forceinline__ uint32_t tile_bucket(uint32_t steps) {
  const uint32_t c = steps < 16u ? (steps < 4u ? 0u : (steps - 2u) >> 1)  // 0..6
                     : steps < 32u ? 7u + ((steps - 16u) >> 2)             // 7..10
                     : steps < 40u ? 11u : steps < 48u ? 12u : steps < 64u ? 13u
                     : steps < 96u ? 14u : 15u;
  return (uint32_t)(kTileBuckets - 1) - c;
}

// Where the order array keeps the tile of dispatch slot `slot` (0 = longest) of an n-tile launch.
// Slot s runs in workgroup s + 1 (workgroup 0 is the sorter), and workgroups are dealt to the 8
// XCDs round-robin (observed placement): the entries of the slots one XCD runs are
// stored together, so each XCD's L2 fetches only its eighth of the array.  Row-major storage had
// every XCD fetch every line of it -- at 4K 8 x 518 KB for the GLSL kernel's 129,600 tiles, 4.1 MB of
// the launch's reads.  A bijection of [0, n) into [0, n + 8) (sfrt_sched.h
// order_capacity).
__device__ __forceinline__ uint32_t order_index(int slot, int n) {
  const uint32_t d = (uint32_t)slot + 1u;
  const uint32_t per = ((uint32_t)n >> 3) + 1u;  // >= ceil((n + 1) / 8)
  return (d & 7u) * per + (d >> 3);
}

// An order entry: the tile in the low kOrderTileBits bits and, above them, the tile's class in
// the cost buffer the order was sorted from (its own, undilated).  That buffer is the one the
// launch reading the order records into (sfrt_sched.h), so a wave whose class is unchanged need
// not store it again (TileSchedPtrs::cost_diff): with a still camera no launch stores any.  The
// cost stores are one byte per tile from every XCD, so each XCD's L2 wrote back a partial copy of
// the whole array -- at 4K ~1 MB of the GLSL launch's writes.  Chains take grids of
// fewer than 2^28 tiles (sfrt_sched.h kOrderMaxTiles).
constexpr int kOrderTileBits = 28;
constexpr uint32_t kOrderTileMask = (1u << kOrderTileBits) - 1u;
static_assert(kTileBuckets <= (1 << (32 - kOrderTileBits)), "a class fits above the tile");

// The tile of dispatch slot `slot` of an n-tile launch and the class its order entry carries
// (kTileBuckets when there is none: row-major launches, a corrupt entry).
__device__ __forceinline__ int slot_tile(const uint32_t* order, int slot, int n, uint32_t& cls) {
  cls = (uint32_t)kTileBuckets;
  if (!order) return slot;
  const uint32_t e = order[order_index(slot, n)];
  const int t = (int)(e & kOrderTileMask);
  if (t >= n) return slot;  // never outside the grid
  cls = e >> kOrderTileBits;
  return t;
}

// Records tile `tile`'s class c, unless diff is set and the order entry already had it (cls).
__device__ __forceinline__ void store_cost(uint8_t* cost, int tile, uint32_t c, uint32_t cls, int diff) {
  if (!diff || c != cls) cost[tile] = (uint8_t)c;
}

// Stable counting sort of n tiles by bucket (longest first; ties in tile
// order), by one wave, into the slot layout of order_index.  Each lane owns one contiguous chunk of tiles, read 16
// buckets per 16-byte load with eight loads in flight (the passes are bound by
// load latency), and its own column of a [bucket][lane] histogram in LDS, so
// counting and ranking need no atomics; the exclusive scan runs bucket-major
// over (bucket, lane), which keeps chunk order -- tile order -- within a bucket.
// (Per-lane counters: LDS atomics without conflicts.)
// dilate (a moving camera): tile t is ranked by the longest of tiles t - 1, t,
// t + 1 (its row neighbours; across a row end the neighbour is the other row's
// end tile, a harmless over-estimate): content that a turning camera moves by
// less than a tile between the recorded frame and the one the order serves
// stays inside that window, so a tile that turns long is not left for the end.
__device__ __forceinline__ void sort_tiles(const uint8_t* __restrict__ cost, int n,
                                           uint32_t* __restrict__ order, bool dilate = false) {
  __shared__ uint32_t cnt[kTileBuckets][64];
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int b = 0; b < kTileBuckets; b++) cnt[b][lane] = 0u;
  const int nvec = n >> 4;
  const int per = (nvec + 63) >> 6;  // 16-byte vectors per lane
  const int v0 = lane * per < nvec ? lane * per : nvec;
  const int v1 = v0 + per < nvec ? v0 + per : nvec;
  // the n % 16 tail tiles go to the last lane's chunk end (after vector nvec - 1)
  const bool tail = lane == 63;
  const uint4* __restrict__ cv = reinterpret_cast<const uint4*>(cost);
  auto at = [&](int t) { return (uint32_t)cost[t < 0 ? 0 : t >= n ? n - 1 : t]; };
  // D loads in flight: 8, or 4 when dilating (its three bytes per tile would otherwise
  // lift the kernel past 64 VGPRs -- one wave per SIMD fewer for every render wave)
  auto pass = [&](auto d_tag, auto&& one) {
    constexpr int D = decltype(d_tag)::value;
    uint32_t prev = dilate && v0 < v1 ? at(16 * v0 - 1) : 0u;  // bucket of the tile before
    for (int v = v0; v < v1; v += D) {
      uint4 q[D];
#pragma unroll
      for (int u = 0; u < D; u++) q[u] = v + u < v1 ? cv[v + u] : make_uint4(0, 0, 0, 0);
      const uint32_t after = dilate ? at(16 * (v + D < v1 ? v + D : v1)) : 0u;
#pragma unroll
      for (int u = 0; u < D; u++) {
        if (v + u >= v1) break;
        const uint32_t w[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
        if (!dilate) {
#pragma unroll
          for (int e = 0; e < 16; e++) {
            const uint32_t c = (w[e >> 2] >> (8 * (e & 3))) & 0xffu;
            one(c, (v + u) * 16 + e, c);
          }
          continue;
        }
        const uint32_t nxt = u + 1 < D && v + u + 1 < v1 ? (q[u + 1].x & 0xffu) : after;
        uint32_t cur = w[0] & 0xffu;
#pragma unroll
        for (int e = 0; e < 16; e++) {
          const uint32_t right = e < 15 ? (w[(e + 1) >> 2] >> (8 * ((e + 1) & 3))) & 0xffu : nxt;
          uint32_t m = prev < cur ? prev : cur;  // bucket 0 = longest: the minimum
          m = right < m ? right : m;
          one(m, (v + u) * 16 + e, cur);
          prev = cur;
          cur = right;
        }
      }
    }
    if (tail)
      for (int t = nvec * 16; t < n; t++) {
        const uint32_t c = at(t);
        uint32_t m = c;
        if (dilate) {
          const uint32_t l = at(t - 1), r = at(t + 1);
          m = l < m ? l : m;
          m = r < m ? r : m;
        }
        one(m, t, c);
      }
  };
  // LDS atomics on the lane's own counters: no conflicts, and the count pass's
  // need no return (a plain read-modify-write would wait on every read)
  auto count = [&](uint32_t b, int, uint32_t) { atomicAdd(&cnt[b][lane], 1u); };
  if (dilate) pass(std::integral_constant<int, 4>{}, count);
  else pass(std::integral_constant<int, 8>{}, count);
  uint32_t run = 0;  // exclusive scan over (bucket, lane), bucket-major
#pragma unroll
  for (int b = 0; b < kTileBuckets; b++) {
    const uint32_t c = cnt[b][lane];
    uint32_t incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t up = (uint32_t)__shfl_up((int)incl, off, 64);
      if (lane >= off) incl += up;
    }
    cnt[b][lane] = run + incl - c;
    run += (uint32_t)__shfl((int)incl, 63, 64);
  }
  auto place = [&](uint32_t b, int t, uint32_t c) {
    order[order_index((int)atomicAdd(&cnt[b][lane], 1u), n)] = (uint32_t)t | (c << kOrderTileBits);
  };
  if (dilate) pass(std::integral_constant<int, 4>{}, place);
  else pass(std::integral_constant<int, 8>{}, place);
}

constexpr float kTinySqrtArg = 0x1.0p-96f;

// Correctly rounded sqrtf for any x: the short form unless some lane of the
// wave has a tiny argument (then the compiler's full lowering for all lanes).
__device__ __forceinline__ float sqrt_cr(float x) {
  if (__builtin_amdgcn_ballot_w64(x < kTinySqrtArg)) return __builtin_sqrtf(keep_branch(x));
  return sqrt_cr_normal(x);
}

}  // namespace sfrt
