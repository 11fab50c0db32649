// wk_region_prof.h -- the wave-level region profile of the split rollout kernels (probe builds
// only: -DWK_REGION_PROF; scripts/region_prof.py).  In the product build every hook below is an
// empty inline function or macro, so the kernels carry no profiling code.
//
// Wave-level: every mark is executed by the lanes that run the code it ends,
// and the wave's FIRST ACTIVE lane charges the s_memtime delta since the wave's previous mark --
// whichever lanes executed that one -- to the region the mark names, in a per-wave LDS record.
// So a region's time is the time the WAVE spent executing it (whatever its lane mask), and 'other'
// is only the code between regions (slot selection, joins, the env-step tail).  Each mark also
// adds the number of active lanes, so lanes / count is the region's mean active lanes.
#pragma once
#include "wk_common.h"

namespace wk {

enum { RP_JOINT, RP_INTEG, RP_AABB_LL, RP_AABB_LF, RP_AABB_BF, RP_SAT_LL, RP_SAT_LF, RP_SAT_BF,
       RP_CON_LL, RP_CON_LF, RP_CON_BF, RP_IMP_LL, RP_IMP_LF, RP_IMP_BF, RP_POLICY, RP_OTHER, RP_N };
#ifdef WK_REGION_PROF
static __device__ unsigned long long g_region_prof[3 * RP_N];  // ticks, lane sums, counts
struct WaveProf { unsigned long long acc[RP_N]; unsigned long long lanes[RP_N]; unsigned cnt[RP_N]; unsigned long long t; };
struct RegionProf { WaveProf* w; };
// deps: values the region computes -- the empty asm makes them ready before the stamp, so the
// scheduler cannot sink the region's arithmetic past its mark into the next region
__device__ __forceinline__ void rp_dep(float v) { asm volatile("" ::"v"(v)); }
template <class... T>
__device__ __forceinline__ void rp_mark(RegionProf* p, int r, T... deps) {
  if (!p) return;
  (rp_dep((float)deps), ...);
  const uint64_t ex = __builtin_amdgcn_read_exec();
  const int lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if (lane == __builtin_ffsll((long long)ex) - 1) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    p->w->acc[r] += t - p->w->t;
    p->w->t = t;
    p->w->lanes[r] += (unsigned long long)__builtin_popcountll(ex);
    p->w->cnt[r] += 1u;
  }
}
__device__ __forceinline__ void rp_begin(RegionProf* p) {
  if ((threadIdx.x & 63) == 0) {
    for (int r = 0; r < RP_N; r++) { p->w->acc[r] = 0; p->w->lanes[r] = 0; p->w->cnt[r] = 0; }
    p->w->t = __builtin_amdgcn_s_memtime();
  }
}
__device__ __forceinline__ void rp_end(RegionProf* p) {
  if ((threadIdx.x & 63) == 0)
    for (int r = 0; r < RP_N; r++) {
      atomicAdd(&g_region_prof[r], p->w->acc[r]);
      atomicAdd(&g_region_prof[RP_N + r], p->w->lanes[r]);
      atomicAdd(&g_region_prof[2 * RP_N + r], (unsigned long long)p->w->cnt[r]);
    }
}
// in a kernel of NW waves per block: declares `rp`, the wave's profile record
#define RP_KERNEL_BEGIN(NW)                     \
  __shared__ WaveProf rp_waves_[NW];            \
  RegionProf rp_rec_{&rp_waves_[threadIdx.x >> 6]}; \
  RegionProf* rp = &rp_rec_;                    \
  rp_begin(rp)
#define RP_KERNEL_END() rp_end(rp)
#else
struct RegionProf {};
template <class... T>
__device__ __forceinline__ void rp_mark(RegionProf*, int, T...) {}
#ifdef WK_WAVE_CLOCK
// -DWK_WAVE_CLOCK (probe builds only): every wave's start and end on the 100 MHz constant clock
// (s_memrealtime: one clock for the whole device) with its HW_ID and XCC_ID, per launched wave
// [start, end, hw_id, xcc_id] -- the spread of wave durations and of their ends within one launch
static __device__ unsigned long long g_wave_clock[4 * 8192];
#define RP_KERNEL_BEGIN(NW)                                       \
  RegionProf* rp = nullptr;                                       \
  const unsigned long long wc_t0_ = __builtin_amdgcn_s_memrealtime()
#define RP_KERNEL_END()                                                                         \
  do {                                                                                          \
    (void)rp;                                                                                   \
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();                             \
    const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;                            \
    if ((threadIdx.x & 63) == 0 && w < 8192) {                                                  \
      g_wave_clock[4 * w] = wc_t0_;                                                             \
      g_wave_clock[4 * w + 1] = t1;                                                             \
      g_wave_clock[4 * w + 2] = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);           \
      g_wave_clock[4 * w + 3] = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);          \
    }                                                                                           \
  } while (0)
#else
#define RP_KERNEL_BEGIN(NW) RegionProf* rp = nullptr
#define RP_KERNEL_END() ((void)rp)
#endif
#endif

}  // namespace wk

#ifdef WK_REGION_PROF
// host: the accumulated [ticks, lane sums, counts] x RP_N (scripts/region_prof.py)
#define RP_HOST_READER                                                                          \
  extern "C" int wk_region_prof(unsigned long long* out, int reset) {                          \
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(wk::g_region_prof),                                \
                            sizeof(unsigned long long) * 3 * wk::RP_N) != hipSuccess)          \
      return -1;                                                                                \
    if (reset) {                                                                                \
      unsigned long long z[3 * wk::RP_N] = {};                                                  \
      if (hipMemcpyToSymbol(HIP_SYMBOL(wk::g_region_prof), z, sizeof(z)) != hipSuccess) return -1; \
    }                                                                                           \
    return 0;                                                                                   \
  }
#elif defined(WK_WAVE_CLOCK)
#define RP_HOST_READER                                                                          \
  extern "C" int wk_wave_clock(unsigned long long* out) {                                      \
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(wk::g_wave_clock), sizeof(unsigned long long) * 4 * 8192) \
               == hipSuccess ? 0 : -1;                                                          \
  }
#else
#define RP_HOST_READER
#endif
