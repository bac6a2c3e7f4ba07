"""Patch glsl_trace.hip in place with per-wave work counters (revert with git checkout)."""
import sys
p = sys.argv[1]
s = open(p).read()
s = s.replace('''template <bool LDS>
__device__ __forceinline__ void fragment(''', '''__device__ unsigned long long g_stats[8];
#define STAT(k) do { if ((threadIdx.x & 63) == __builtin_ffsll(__builtin_amdgcn_read_exec()) - 1) atomicAdd(&g_stats[k], 1ull); } while (0)
template <bool LDS>
__device__ __forceinline__ void fragment(''')
s = s.replace('''  const float fx = (float)i + 0.5f;''', '''  STAT(0);
  const float fx = (float)i + 0.5f;''')
s = s.replace('''    if (__builtin_amdgcn_ballot_w64(inside)) {
''', '''    if (__builtin_amdgcn_ballot_w64(inside)) {
      STAT(1);
''')
s = s.replace('''    if (++steps > kGlslMarchCap) {''', '''    STAT(2);
    if (++steps > kGlslMarchCap) {''')
s = s.replace('''      if (!__builtin_amdgcn_ballot_w64(!dominated)) continue;''', '''      STAT(4);
      if (!__builtin_amdgcn_ballot_w64(!dominated)) continue;
      STAT(3);''')
s = s.replace('''        if (!__builtin_amdgcn_ballot_w64(!(near && cosang <= P.cos_lit))) continue;''', '''        STAT(6);
        if (!__builtin_amdgcn_ballot_w64(!(near && cosang <= P.cos_lit))) continue;
        STAT(5);''')
s = s.replace('''    draw = inside ? k : draw;
''', '''    STAT(7);
    draw = inside ? k : draw;
''')
s = s.replace('''}  // namespace

int launch_glsl(''', '''}  // namespace

extern "C" __attribute__((visibility("default"))) int sfrt_glsl_stats(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stats), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  if (reset) { unsigned long long z[8] = {}; (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stats), z, sizeof z); }
  return 0;
}

int launch_glsl(''')
assert s.count("STAT(") >= 8, s.count("STAT(")
open(p, "w").write(s)
