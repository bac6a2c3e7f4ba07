// sfrt_sched.h -- host side of the adaptive tile order ("Tile order")
// shared by the one-wave-per-tile renderers (sphere_trace.hip, voxel_trace.hip;
// device side: sfrt_device.h sort_tiles).
//
// Launch k of a chain (consecutive launches of one renderer object with one tile
// grid) reads order[k % 2] (built by launch k-1 from launch k-2's costs), records
// its per-tile march-step classes into cost[k % 2], and -- from its extra
// workgroup 0 -- sorts cost[(k+1) % 2] (launch k-1's) into order[(k+1) % 2].
// Consecutive launches are ordered by their stream; before a launch on another
// stream than the previous one, the host waits for the device (below).  An order is
// used only when the two launches before had the same grid (key).  Scheduling
// only: every tile is rendered once whatever the order.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sfrt {

// Entries of an n-tile order array: its slot layout (sfrt_device.h order_index) maps the n slots
// into [0, n + 8).
inline long long order_capacity(long long n) { return n + 8; }
// Order entries keep the tile in 28 bits (sfrt_device.h kOrderTileBits): larger grids render
// row-major.
constexpr long long kOrderMaxTiles = 1ll << 28;

struct TileSchedPtrs {
  const uint32_t* tile_order = nullptr;  // slot -> tile (nullptr: row-major)
  uint8_t* tile_cost = nullptr;          // this launch's per-tile classes (nullptr: no chain)
  const uint8_t* prev_cost = nullptr;    // launch k-1's, to sort (nullptr: no sorter workgroup)
  uint32_t* next_order = nullptr;        // the sorter's output, for launch k+1
  // tile_order's entries carry the classes now in tile_cost (the buffer they were sorted from,
  // untouched since): the launch stores only the classes that changed
  bool cost_diff = false;
};

struct TileSched {
  uint32_t* order[2] = {};
  uint8_t* cost[2] = {};
  long long cap = 0;
  int64_t k = 0;
  long long key_prev = 0;        // tile grid of launch k-1 (0: none)
  bool sorted_prev = false;      // launch k-1 sorted launch k-2's tiles into order[k % 2]
  long long pending_key = 0;     // begin() -> end(): the launch being queued
  bool pending_sorted = false;
  bool committed = false;        // the last end() advanced the chain
  hipStream_t last_stream = nullptr;
  bool have_last = false;
  uint64_t used = 0;             // TileChains: when the chain last took a launch
  bool probed = false;           // a timing-probe launch rewrote cost[k % 2] since k last moved

  void release() {
    for (int q = 0; q < 2; q++) {
      (void)hipFree(order[q]);
      (void)hipFree(cost[q]);
      order[q] = nullptr;
      cost[q] = nullptr;
    }
    cap = 0;
  }

  // Link a launch on s with tile grid `key` (0: takes no part) of `tiles` tiles
  // into the chain.  mode: 1 = adaptive; 2 = timing probe (reuse the last order,
  // no sorter, the chain does not advance).  The chain state moves only in end(),
  // once the launch is known to be queued.
  hipError_t begin(long long key, long long tiles, hipStream_t s, int mode, TileSchedPtrs& p) {
    p = TileSchedPtrs{};
    pending_key = 0;
    if (key == 0 || mode == 0 || tiles >= kOrderMaxTiles) return hipSuccess;
    hipError_t e;
    // A launch on another stream than the chain's last one (TileChains: a stream beyond the
    // kChains in use took this chain over).  That stream's handle must not be used: the caller
    // may have destroyed it since (hipStreamQuery on a destroyed stream's handle crashed,
    // tools/gpu/probe_dead_stream.py, profiles/r6y_dead_stream.txt), so the host waits for the
    // whole device -- which also covers that stream's launches -- and the chain continues on s.
    if (have_last && last_stream != s) {
      if ((e = hipDeviceSynchronize()) != hipSuccess) return e;
      have_last = false;
    }
    if (tiles > cap) {  // (re)allocate; a new chain starts
      // Stream-ordered, no device-wide wait (a hipDeviceSynchronize here had made the first draw
      // on a new stream wait for every other stream's work): the old buffers were last used on s
      // (above), so they are freed and the new ones allocated in the order of s.
      for (int q = 0; q < 2; q++) {
        if (order[q] && (e = hipFreeAsync(order[q], s)) != hipSuccess) return e;
        if (cost[q] && (e = hipFreeAsync(cost[q], s)) != hipSuccess) return e;
        order[q] = nullptr;
        cost[q] = nullptr;
      }
      cap = 0;
      reset();
      for (int q = 0; q < 2; q++) {
        if ((e = hipMallocAsync((void**)&order[q], sizeof(uint32_t) * (size_t)order_capacity(tiles),
                                s)) != hipSuccess)
          return e;
        if ((e = hipMallocAsync((void**)&cost[q], (size_t)tiles, s)) != hipSuccess) return e;
      }
      cap = tiles;
    }
    const bool same = key_prev == key;  // launch k-1 had this tile grid
    p.tile_order = (same && sorted_prev) ? order[k & 1] : nullptr;
    p.tile_cost = cost[k & 1];
    p.prev_cost = same ? cost[(k + 1) & 1] : nullptr;
    p.next_order = order[(k + 1) & 1];
    if (mode == 2 && sorted_prev && same) {
      p.prev_cost = nullptr;
      probed = true;  // it stores every class: cost[k % 2] no longer matches order[k % 2]
      return hipSuccess;  // nothing to commit
    }
    p.cost_diff = p.tile_order != nullptr && !probed;
    pending_key = key;
    pending_sorted = same;
    return hipSuccess;
  }

  // After the launch that took part (p.tile_cost set) was queued on s (queued =
  // false: it failed).  A failed launch restarts the chain: its cost buffer was
  // never written, so no later launch may sort it or read an order built from it.
  hipError_t end(const TileSchedPtrs& p, hipStream_t s, bool queued = true) {
    committed = false;  // also for a launch outside the chain (no stale "committed")
    if (!p.tile_cost) return hipSuccess;
    if (!queued) {
      reset();
      return hipSuccess;
    }
    committed = pending_key != 0;
    if (pending_key) {
      sorted_prev = pending_sorted;
      key_prev = pending_key;
      k++;
      pending_key = 0;
      probed = false;
    }
    last_stream = s;
    have_last = true;
    return hipSuccess;
  }

  void reset() {
    k = 0;
    key_prev = 0;
    sorted_prev = false;
    pending_key = 0;
    probed = false;
  }
};

// One chain per stream (up to kChains streams): launches on different streams share no
// cost or order buffer, so nothing orders them against each other -- two frames in flight
// on two streams overlap, the second starting while the first drains.  Each chain orders
// its launches by the march steps of its own launch two back.  A further stream takes the
// least recently used chain, whose begin() then waits for the device (a stream handle is
// kept only to be compared, never passed to HIP: its owner may destroy it).  Sixteen chains
// cover a render thread per stream (the reference renders with eight threads, Source.cpp:13);
// a chain's buffers are allocated by its first launch.
struct TileChains {
  static constexpr int kChains = 16;
  TileSched chain[kChains];
  uint64_t clock = 0;

  int pick(hipStream_t s) {
    int lru = 0;
    for (int q = 0; q < kChains; q++)
      if (chain[q].have_last && chain[q].last_stream == s) return touch(q);
    for (int q = 0; q < kChains; q++)
      if (!chain[q].have_last) return touch(q);
    for (int q = 1; q < kChains; q++)
      if (chain[q].used < chain[lru].used) lru = q;
    return touch(lru);
  }
  int touch(int q) {
    chain[q].used = ++clock;
    return q;
  }
  void release() {
    for (auto& c : chain) c.release();
  }
};

}  // namespace sfrt
