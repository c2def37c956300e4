// TOOLS ONLY -- never linked into libfrcnn_amd.so.  The RoIAlign kernel variants
// measured on the way to the product kernels (DESIGN.md §4 records each result),
// kept for the micro-benchmarks (tools/bench_roi_align.py, tools/bench_roi_bwd.py,
// tools/probe/) and the variant-equality test (tests/test_tools_variants.py).
// Built by tools/build_tools.py into tools/lib/libfrcnn_tools.so.
#include <stdlib.h>

#include <algorithm>

#include "roi_kernels.h"

namespace frh {


// ---------------------------------------------------------------------------
// One wave, one RoI, channels [c0, c1): the RoI's tap rows (dense window
// [y0, y1] when it has <= 4*ph rows, else the (y_lo, y_hi) list of its 2*ph
// y-samples) x columns [x0 & ~(kV-1), x1] are staged channel by channel into
// the wave's slab by LDS-DMA (kV floats per lane), two batches in flight with
// counted vmcnt waits; lane = bin evaluates from LDS.  Slabs beyond kSlab /
// 2 are gathered per bin.  Used where a group's union does not fit.
template <int kSlab, int kV>
__device__ __forceinline__ void roi_segment(const RoiLevels& lv, const RoiCfg& c, float* __restrict__ out, float* slab,
                                            int64_t k, int c0, int c1, int lane) {
  constexpr int SR = 2;
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw, nsy = c.ph * SR;
  const int sy = (int)lv.sy[l], sx = (int)lv.sx[l], scs = (int)lv.sc[l];
  const bool active = lane < nbins;
  const int bin = active ? lane : 0;
  const int py = bin / c.pw, px = bin - py * c.pw;
  Tap ty[SR], tx[SR];
#pragma unroll
  for (int i = 0; i < SR; ++i) {  // sampling 2: the "/ gh" of the sample position is an exact halving
    ty[i] = make_tap(g.start_h + (float)py * g.bin_h + ((float)i + 0.5f) * g.bin_h * 0.5f, H);
    tx[i] = make_tap(g.start_w + (float)px * g.bin_w + ((float)i + 0.5f) * g.bin_w * 0.5f, W);
  }
  int ylo = 1 << 30, yhi = -1, xlo = 1 << 30, xhi = -1;
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    if (active && ty[i].valid) ylo = min(ylo, ty[i].lo), yhi = max(yhi, ty[i].hi);
    if (active && tx[i].valid) xlo = min(xlo, tx[i].lo), xhi = max(xhi, tx[i].hi);
  }
  const int y0 = __builtin_amdgcn_readfirstlane(wave_min_i32(ylo)), y1 = __builtin_amdgcn_readfirstlane(wave_max_i32(yhi));
  const int x0 = __builtin_amdgcn_readfirstlane(wave_min_i32(xlo)), x1 = __builtin_amdgcn_readfirstlane(wave_max_i32(xhi));
  const bool any = y1 >= y0 && x1 >= x0;
  const int xs0 = x0 & ~(kV - 1);
  const int ws = kV == 1 ? ((x1 - x0 + 1) | 1) : ((x1 - xs0 + kV) & ~(kV - 1));
  const bool dense = any && y1 - y0 + 1 <= 2 * nsy;
  const int nrows = !any ? 0 : dense ? y1 - y0 + 1 : 2 * nsy;
  const int R = (nrows * ws + kV * kWave - 1) / (kV * kWave);
  const int Rr = R <= 1 ? 1 : R <= 2 ? 2 : R <= 4 ? 4 : R <= 8 ? 8 : 16;
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l];
  const int64_t extent = ((int64_t)(c.C - 1) * scs + (int64_t)(H - 1) * sy + (int64_t)(W - 1) * sx + 1) * 4;
  const __amdgpu_buffer_rsrc_t fr = uniform_rsrc(base, extent);
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + k * c.C * nbins, (int64_t)c.C * nbins * 4);
  const int cstep = scs * 4, ostep = nbins * 4;
  const int ovoff = active ? lane * 4 : 0x40000000;  // idle lanes: dropped by the range check
  if (!any) {
    for (int ch = c0; ch < c1; ++ch) __builtin_amdgcn_raw_buffer_store_b32(0u, orr, ovoff, ch * ostep, 0);
    return;
  }
  bool ok[SR][SR];
  float wt[SR][SR][4];
#pragma unroll
  for (int iy = 0; iy < SR; ++iy)
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap a = ty[iy], b = tx[ix];
      ok[iy][ix] = a.valid && b.valid;
      wt[iy][ix][0] = a.h * b.h;
      wt[iy][ix][1] = a.h * b.l;
      wt[iy][ix][2] = a.l * b.h;
      wt[iy][ix][3] = a.l * b.l;
    }
  auto combine = [&](const float (&v)[SR][SR][4]) {
    float acc = 0.0f;
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        float val = ((wt[iy][ix][0] * v[iy][ix][0] + wt[iy][ix][1] * v[iy][ix][1]) + wt[iy][ix][2] * v[iy][ix][2]) +
                    wt[iy][ix][3] * v[iy][ix][3];
        acc = acc + (ok[iy][ix] ? val : 0.0f);
      }
    return acc * 0.25f;
  };
  if (Rr * kV * kWave * 2 > kSlab) {
    // window larger than half the slab: per-bin gather, two channels in flight
    int off[SR][SR][4];
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        const bool v = ok[iy][ix];
        const int r0 = v ? ty[iy].lo * sy : 0, r1 = v ? ty[iy].hi * sy : 0;
        const int q0 = v ? tx[ix].lo * sx : 0, q1 = v ? tx[ix].hi * sx : 0;
        off[iy][ix][0] = (r0 + q0) * 4;
        off[iy][ix][1] = (r0 + q1) * 4;
        off[iy][ix][2] = (r1 + q0) * 4;
        off[iy][ix][3] = (r1 + q1) * 4;
      }
    for (int ch = c0; ch < c1; ch += 2) {
      const int chb = min(ch + 1, c1 - 1);
      float va[SR][SR][4], vb[SR][SR][4];
#pragma unroll
      for (int iy = 0; iy < SR; ++iy)
#pragma unroll
        for (int ix = 0; ix < SR; ++ix)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            va[iy][ix][q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(fr, off[iy][ix][q], ch * cstep, 0));
            vb[iy][ix][q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(fr, off[iy][ix][q], chb * cstep, 0));
          }
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(combine(va)), orr, ovoff, ch * ostep, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(combine(vb)), orr, ch + 1 < c1 ? ovoff : 0x40000000,
                                            (ch + 1) * ostep, 0);
    }
    return;
  }
  // slab byte offsets of this bin's taps: [iy][row lo/hi][ix][col lo/hi]
  int sa[SR][2][SR][2];
#pragma unroll
  for (int iy = 0; iy < SR; ++iy)
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap a = ty[iy], b = tx[ix];
      const bool v = ok[iy][ix];
      const int rlo = dense ? a.lo - y0 : 2 * (py * SR + iy), rhi = dense ? a.hi - y0 : 2 * (py * SR + iy) + 1;
      sa[iy][0][ix][0] = v ? (rlo * ws + (b.lo - xs0)) * 4 : 0;
      sa[iy][0][ix][1] = v ? (rlo * ws + (b.hi - xs0)) * 4 : 0;
      sa[iy][1][ix][0] = v ? (rhi * ws + (b.lo - xs0)) * 4 : 0;
      sa[iy][1][ix][1] = v ? (rhi * ws + (b.hi - xs0)) * 4 : 0;
    }
  auto bin_value = [&](const char* sl) {
    float v[SR][SR][4];
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        v[iy][ix][0] = *reinterpret_cast<const float*>(sl + sa[iy][0][ix][0]);
        v[iy][ix][1] = *reinterpret_cast<const float*>(sl + sa[iy][0][ix][1]);
        v[iy][ix][2] = *reinterpret_cast<const float*>(sl + sa[iy][1][ix][0]);
        v[iy][ix][3] = *reinterpret_cast<const float*>(sl + sa[iy][1][ix][1]);
      }
    return combine(v);
  };
  // sparse rows: entry 2i / 2i+1 = y_lo / y_hi of y-sample i = ty[i % 2] of lane (i / 2) * pw
  const int tyl0 = ty[0].valid ? ty[0].lo : y0, tyh0 = ty[0].valid ? ty[0].hi : y0;
  const int tyl1 = ty[1].valid ? ty[1].lo : y0, tyh1 = ty[1].valid ? ty[1].hi : y0;
  const int n = nrows * ws;
  auto run = [&](auto rb) {
    constexpr int RB = decltype(rb)::value;
    constexpr int kB0 = kSlab / (2 * RB * kV * kWave);
    constexpr int kB = kB0 < 1 ? 1 : (kB0 < 16 ? kB0 : 16);  // channels per batch
    constexpr int F = RB * kV * kWave * 4;                     // slab bytes per channel
    static_assert(kB * (RB + 1) < 64, "batch too large for vmcnt");
    if (kB0 < 1) return;  // excluded by the gather test above
    int goff[RB];
    {
      const int step = kV * kWave, dr = step / ws, dc = step - dr * ws;
      int r = (kV * lane) / ws, col = kV * lane - r * ws;
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        const int e = kV * lane + j * step;
        const int rs = min(r, 2 * nsy - 1), src = (rs >> 2) * c.pw;
        const int a0 = __shfl(tyl0, src, kWave), a1 = __shfl(tyh0, src, kWave);
        const int b0 = __shfl(tyl1, src, kWave), b1 = __shfl(tyh1, src, kWave);
        const int srow = (rs & 2) ? ((rs & 1) ? b1 : b0) : ((rs & 1) ? a1 : a0);
        const int fy = dense ? y0 + r : srow;
        // columns past the row end only fill slab cells no tap reads; lanes past the slab
        // re-read its first element (no extra line)
        const int fx = kV == 1 ? min(xs0 + col, W - 1) : xs0 + col;
        goff[j] = e < n ? (fy * sy + fx * sx) * 4 : (y0 * sy + xs0 * sx) * 4;
        r += dr;
        col += dc;
        if (col >= ws) col -= ws, ++r;
      }
    }
    const int nb = (c1 - c0 + kB - 1) / kB;
    auto issue = [&](int b) {  // batch b -> slot b & 1; channels past c1 re-read the last one
      const int slot = (b & 1) * kB;
#pragma unroll
      for (int s = 0; s < kB; ++s) {
        const int ch = min(c0 + b * kB + s, c1 - 1);
#pragma unroll
        for (int j = 0; j < RB; ++j)
          lds_dma<4 * kV>(fr, slab + (slot + s) * (F / 4) + j * kV * kWave, goff[j], ch * cstep);
      }
    };
    issue(0);
    if (nb > 1) issue(1);
    for (int b = 0; b < nb; ++b) {
      // retire batch b: younger than it are batch b-1's kB stores and batch b+1's DMAs
      if (b + 1 < nb) {
        if (b == 0)
          wait_vmcnt<kB * RB>();
        else
          wait_vmcnt<kB * RB + kB>();
      } else {
        wait_vmcnt<0>();
      }
      const char* sl = reinterpret_cast<const char*>(slab + (b & 1) * kB * (F / 4));
#pragma unroll
      for (int s = 0; s < kB; ++s) {
        const int ch = c0 + b * kB + s;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bin_value(sl + s * F)), orr,
                                              ch < c1 ? ovoff : 0x40000000, ch * ostep, 0);
      }
      if (b + 2 < nb) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot b & 1 fully read before it is refilled
        issue(b + 2);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  if (Rr == 1)
    run(std::integral_constant<int, 1>{});
  else if (Rr == 2)
    run(std::integral_constant<int, 2>{});
  else if (Rr == 4)
    run(std::integral_constant<int, 4>{});
  else if (Rr == 8)
    run(std::integral_constant<int, 8>{});
  else
    run(std::integral_constant<int, 16>{});
}

// ---------------------------------------------------------------------------
// Measured slower (variants 38, 52, 53) -- kept here, out of the product.
// Dynamic item scheduling for the pair kernel (kSingle, chunk-major): kDynWaves waves per
// XCD list stay resident and take (channel chunk, RoI) items of their XCD's list from a
// per-list counter, so the launch has no tail of late long items, and each wave fetches
// the NEXT item's index and RoI while it works on the current one (its prologue loses
// the memory round trips).  Counters: g_roi_dyn[x * 64] (next item of list x) and
// [x * 64 + 32] (waves of list x that have left); the last wave out of a list resets
// both, so stream-ordered launches start from zero.  (Two launches of this kernel must
// not run concurrently on different streams: they would share the counters.)
static __device__ uint32_t g_roi_dyn[8 * 64];

__device__ __forceinline__ uint32_t lane0_fetch_add(uint32_t* p, uint32_t v) {  // one atomic per wave
  uint32_t r = 0;
  if ((threadIdx.x & (kWave - 1)) == 0) r = __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return r;  // lane 0 holds it: read with __builtin_amdgcn_readfirstlane
}

// kStatic: no counters -- wave j of a list takes items j, j + P, j + 2P, ... (P = waves per
// list), still with the next item's RoI fetched before the current item's work.
template <int kPW = kPairWave, int kHalf = kPairHalf, int kStAux = kCpolNT, bool kStatic = false>
__global__ void __launch_bounds__(kWave) roi_align_fwd_pair_dyn_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out,
                                                                       uint32_t waves_per_list) {
  __shared__ __attribute__((aligned(16))) float slab[kHalf];
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)slab);
  const uint32_t x = blockIdx.x & 7u;
  const uint32_t G = (uint32_t)(c.C + 2 * kPW - 1) / (uint32_t)(2 * kPW), K32 = (uint32_t)c.K;
  const uint32_t total = K32 * G, per = (total + 7u) / 8u;
  const uint32_t lo = x * per, n = min(lo + per, total) > lo ? min(lo + per, total) - lo : 0u;
  uint32_t* cnt = g_roi_dyn + x * 64u;
  uint32_t* left = g_roi_dyn + x * 64u + 32u;
  const uint32_t wj = blockIdx.x >> 3;
  auto next_index = [&](uint32_t cur) -> uint32_t {  // dynamic: lane 0 holds it; static: uniform
    return kStatic ? cur + waves_per_list : lane0_fetch_add(cnt, 1u);
  };
  uint32_t i0 = kStatic ? wj : __builtin_amdgcn_readfirstlane(lane0_fetch_add(cnt, 1u));
  if (i0 < n) {
    auto kc = [&](uint32_t i, int64_t* k, int* ch) {
      const uint32_t w = lo + i;
      *ch = (int)(w / K32);
      *k = (int64_t)(w - (uint32_t)*ch * K32);
    };
    int64_t k0;
    int ch0;
    kc(i0, &k0, &ch0);
    RoiRaw r0 = roi_fetch(c, k0);
    uint32_t i1v = next_index(i0);  // in flight while item i0 runs
    while (true) {
      const uint32_t i1 = kStatic ? i1v : __builtin_amdgcn_readfirstlane(i1v);
      int64_t k1 = k0;
      int ch1 = ch0;
      RoiRaw r1 = r0;
      uint32_t i2v = 0;
      if (i1 < n) {  // the next item's RoI and the one after's index, before this item's work
        kc(i1, &k1, &ch1);
        r1 = roi_fetch(c, k1);
        i2v = next_index(i1);
      }
      // the lane index through an opaque copy: lane-only values of the item (bin, DMA slots)
      // are recomputed per item instead of hoisted out of the loop into live registers
      int lane = threadIdx.x & (kWave - 1);
      asm volatile("" : "+v"(lane));
      pair_item<kPW, kHalf, kStAux, 0, false, true, true>(lv, c, out, k0, ch0, lo + i0, r0, sbase, 0, lane);
      if (i1 >= n) break;
      i0 = i1;
      k0 = k1;
      ch0 = ch1;
      r0 = r1;
      i1v = i2v;
    }
  }
  if (kStatic) return;
  // leave: the last wave of this list resets its counters (every other wave of the list has
  // made its final counter add before its own add to `left`)
  __builtin_amdgcn_s_waitcnt(0);
  const uint32_t out_n = __builtin_amdgcn_readfirstlane(lane0_fetch_add(left, 1u));
  if (out_n == waves_per_list - 1u && (threadIdx.x & (kWave - 1)) == 0) {
    __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(left, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Persistent channel-pair forward (variant 25).  The staging and evaluation of
// the channel-pair kernel above, but a grid of resident single-wave workgroups
// walks the items (RoI, kStrPairs channel pairs): wave w takes items w, w + G,
// w + 2G, ...  The two-buffer LDS ring never drains between items: before the
// last stage of item i is evaluated, item i+1's RoI / level / descriptor loads,
// its tap window and DMA offsets are set up and its first stage is issued, so
// the per-item setup and first-load latency (about half of a channel-pair
// wave's life) overlap the previous item's evaluation.  Stage
// shapes (D pairs per stage) may change from item to item; the vmcnt waits
// count the DMAs and stores issued after the stage being retired (in-order
// completion) and round down to a supported immediate (waiting for fewer
// outstanding operations is always safe).  Bit-identical to the other kernels.
constexpr int kStrPairs = 8;         // channel pairs per item
constexpr int kStrGoff = PairLayout<1>::RP;

struct StrItem {
  int64_t k;
  int ok, D, nst, npairs, cw0, scs4;
  int H, W, y0, x0, dy, dx, Cs2;
  float sh, sw, bh, bw;
  __amdgpu_buffer_rsrc_t fr, orr;
  int goff[kStrGoff];
};

__device__ __forceinline__ int str_dma_count(int D) { return D >= 4 ? 24 : 26; }

// s_waitcnt vmcnt(N') for the largest supported N' <= n
__device__ __forceinline__ void wait_vmcnt_le(int n) {
  if (n >= 42) wait_vmcnt<42>();
  else if (n >= 40) wait_vmcnt<40>();
  else if (n >= 34) wait_vmcnt<34>();
  else if (n >= 32) wait_vmcnt<32>();
  else if (n >= 30) wait_vmcnt<30>();
  else if (n >= 28) wait_vmcnt<28>();
  else if (n >= 26) wait_vmcnt<26>();
  else if (n >= 24) wait_vmcnt<24>();
  else if (n >= 16) wait_vmcnt<16>();
  else if (n >= 8) wait_vmcnt<8>();
  else if (n >= 4) wait_vmcnt<4>();
  else if (n >= 2) wait_vmcnt<2>();
  else wait_vmcnt<0>();
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// DMA-side setup of item t (uniform over the wave except goff)
__device__ __forceinline__ void str_setup(StrItem& it, const RoiLevels& lv, const RoiCfg& c, float* out, int64_t t,
                                          int G) {
  constexpr int SR = 2;
  const int lane = threadIdx.x;
  it.k = t / G;
  it.cw0 = (int)(t - it.k * G) * 2 * kStrPairs;
  it.npairs = min(kStrPairs, (c.C - it.cw0) / 2);
  const RoiGeom g = roi_geom(c, lv, it.k);
  const int l = g.lvl;
  it.H = lv.h[l];
  it.W = lv.w[l];
  it.sh = g.start_h;
  it.sw = g.start_w;
  it.bh = g.bin_h;
  it.bw = g.bin_w;
  const int sy = (int)lv.sy[l], sx = (int)lv.sx[l], scs = (int)lv.sc[l];
  it.scs4 = scs * 4;
  const int nbins = c.ph * c.pw;
  it.orr = uniform_rsrc(out + (it.k * c.C + it.cw0) * nbins, (int64_t)2 * it.npairs * nbins * 4);
  auto pos_y = [&](int p, int i) { return it.sh + (float)p * it.bh + ((float)i + 0.5f) * it.bh * 0.5f; };
  auto pos_x = [&](int p, int i) { return it.sw + (float)p * it.bw + ((float)i + 0.5f) * it.bw * 0.5f; };
  const int nly = 2 * SR * c.ph, nlx = 2 * SR * c.pw;
  int yrow = -1, xcol = -1, ylo = 1 << 30, yhi = -1, xlo = 1 << 30, xhi = -1;
  if (lane < nly) {
    const int s = lane >> 1;
    const Tap tp = make_tap(pos_y(s >> 1, s & 1), it.H);
    if (tp.valid) yrow = (lane & 1) ? tp.hi : tp.lo, ylo = tp.lo, yhi = tp.hi;
  }
  if (lane < nlx) {
    const int s = lane >> 1;
    const Tap tp = make_tap(pos_x(s >> 1, s & 1), it.W);
    if (tp.valid) xcol = (lane & 1) ? tp.hi : tp.lo, xlo = tp.lo, xhi = tp.hi;
  }
  const int y0 = __builtin_amdgcn_readfirstlane(wave_min_i32(ylo)), y1 = __builtin_amdgcn_readfirstlane(wave_max_i32(yhi));
  const int x0 = __builtin_amdgcn_readfirstlane(wave_min_i32(xlo)), x1 = __builtin_amdgcn_readfirstlane(wave_max_i32(xhi));
  it.ok = y1 >= y0 && x1 >= x0;
  it.y0 = y0;
  it.x0 = x0;
  it.dy = y1 - y0 + 1 <= nly;
  it.dx = x1 - x0 + 1 <= nlx;
  const int R = it.dy ? y1 - y0 + 1 : nly, Cs = it.dx ? x1 - x0 + 1 : nlx;
  it.Cs2 = Cs | 1;
  const int ncell = R * it.Cs2;
  it.D = ncell <= PairLayout<8>::kCells ? 8 : ncell <= PairLayout<4>::kCells ? 4 : ncell <= PairLayout<2>::kCells ? 2 : 1;
  it.nst = (it.npairs + it.D - 1) / it.D;
  if (!it.ok) return;
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l];
  const int64_t extent = ((int64_t)(c.C - 1) * scs + (int64_t)(it.H - 1) * sy + (int64_t)(it.W - 1) * sx + 1) * 4;
  it.fr = uniform_rsrc(base, extent);
  const int rsrc = (it.dy ? y0 + min(lane, R - 1) : (yrow >= 0 ? yrow : y0)) * sy * 4;
  const int csrc = (it.dx ? x0 + min(lane, Cs - 1) : (xcol >= 0 ? xcol : x0)) * sx * 4;
  const uint32_t inv = (65536u + (uint32_t)it.Cs2 - 1u) / (uint32_t)it.Cs2;
  const int RS = it.D == 8 ? PairLayout<8>::RS : it.D == 4 ? PairLayout<4>::RS : it.D == 2 ? PairLayout<2>::RS
                                                                                               : PairLayout<1>::RS;
  const int RP = RS / kWave;
#pragma unroll
  for (int j = 0; j < kStrGoff; ++j) {
    int e = (j * kWave + lane) >> 1;
    e = e < ncell ? e : 0;
    const int r = (int)(((uint32_t)e * inv) >> 16), col = min(e - r * it.Cs2, Cs - 1);
    const int v = __shfl(rsrc, r, kWave) + __shfl(csrc, col, kWave) + (lane & 1) * it.scs4;
    it.goff[j] = j < RP ? v : 0;
  }
}

// eval-side setup: this lane's bin weights (zero for invalid samples) and LDS tap addresses
__device__ __forceinline__ void str_taps(const StrItem& it, const RoiCfg& c, uint32_t lbase, uint32_t (&ta)[2][2][4],
                                         float (&wt)[2][2][4]) {
  constexpr int SR = 2;
  const int lane = threadIdx.x;
  const int nbins = c.ph * c.pw;
  const int bin = lane < nbins ? lane : 0;
  const int py = (int)(((uint32_t)bin * ((65536u + (uint32_t)c.pw - 1u) / (uint32_t)c.pw)) >> 16), px = bin - py * c.pw;
  auto pos_y = [&](int p, int i) { return it.sh + (float)p * it.bh + ((float)i + 0.5f) * it.bh * 0.5f; };
  auto pos_x = [&](int p, int i) { return it.sw + (float)p * it.bw + ((float)i + 0.5f) * it.bw * 0.5f; };
#pragma unroll
  for (int iy = 0; iy < SR; ++iy) {
    const Tap a = make_tap(pos_y(py, iy), it.H);
    const int r0 = it.dy ? a.lo - it.y0 : 2 * (py * SR + iy), r1 = it.dy ? a.hi - it.y0 : 2 * (py * SR + iy) + 1;
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap b = make_tap(pos_x(px, ix), it.W);
      const int q0 = it.dx ? b.lo - it.x0 : 2 * (px * SR + ix), q1 = it.dx ? b.hi - it.x0 : 2 * (px * SR + ix) + 1;
      const bool ok = a.valid && b.valid;
      wt[iy][ix][0] = ok ? a.h * b.h : 0.f;
      wt[iy][ix][1] = ok ? a.h * b.l : 0.f;
      wt[iy][ix][2] = ok ? a.l * b.h : 0.f;
      wt[iy][ix][3] = ok ? a.l * b.l : 0.f;
      ta[iy][ix][0] = lbase + (ok ? 8u * (uint32_t)(r0 * it.Cs2 + q0) : 0u);
      ta[iy][ix][1] = lbase + (ok ? 8u * (uint32_t)(r0 * it.Cs2 + q1) : 0u);
      ta[iy][ix][2] = lbase + (ok ? 8u * (uint32_t)(r1 * it.Cs2 + q0) : 0u);
      ta[iy][ix][3] = lbase + (ok ? 8u * (uint32_t)(r1 * it.Cs2 + q1) : 0u);
    }
  }
}

template <int D>
__device__ __forceinline__ void str_issue(const StrItem& it, float* slab, int b, int s) {
  constexpr int RS = PairLayout<D>::RS, RP = PairLayout<D>::RP;
  float* buf = slab + b * kPairHalf;
#pragma unroll
  for (int d = 0; d < D; ++d) {  // pairs past the last re-read it (their stores are dropped)
    const int soff = (it.cw0 + 2 * min(s * D + d, it.npairs - 1)) * it.scs4;
#pragma unroll
    for (int j = 0; j < RP; ++j) lds_dma<4>(it.fr, buf + d * RS + j * kWave, it.goff[j], soff);
  }
}

__device__ __forceinline__ void str_issue_dyn(const StrItem& it, float* slab, int b, int s) {
  switch (it.D) {
    case 8: str_issue<8>(it, slab, b, s); break;
    case 4: str_issue<4>(it, slab, b, s); break;
    case 2: str_issue<2>(it, slab, b, s); break;
    default: str_issue<1>(it, slab, b, s); break;
  }
}

template <int D, int kBuf>
__device__ __forceinline__ void str_eval(const StrItem& it, int s, int ovoff, int ostep, const uint32_t (&ta)[2][2][4],
                                         const float (&wt)[2][2][4]) {
  constexpr int SR = 2, RS = PairLayout<D>::RS;
  f32x2 v[2][8];
  f32x2 acc = {0.0f, 0.0f};
  auto load = [&](auto hh) {
    constexpr int h = decltype(hh)::value, d = h >> 1, iy = h & 1, OFF = 4 * (kBuf * kPairHalf + d * RS);
#pragma unroll
    for (int ix = 0; ix < SR; ++ix)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[h & 1][ix * 4 + q] = lds_read_b64<OFF>(ta[iy][ix][q]);
  };
  load(std::integral_constant<int, 0>{});
  static_for<0, 2 * D>([&](auto hh) {
    constexpr int h = decltype(hh)::value, d = h >> 1, iy = h & 1;
    if constexpr (h + 1 < 2 * D) {
      load(std::integral_constant<int, h + 1>{});
      lds_wait<8>(v[h & 1]);
    } else {
      lds_wait<0>(v[h & 1]);
    }
    if (iy == 0) acc = f32x2{0.0f, 0.0f};
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const float* w = wt[iy][ix];
      const f32x2* x = &v[h & 1][ix * 4];
      const f32x2 val = ((f32x2(w[0]) * x[0] + f32x2(w[1]) * x[1]) + f32x2(w[2]) * x[2]) + f32x2(w[3]) * x[3];
      acc = acc + val;
    }
    if (iy == 1) {
      const f32x2 r = acc * 0.25f;
      const int p = s * D + d;
      const int vo = p < it.npairs ? ovoff : 0x40000000;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.x), it.orr, vo, 2 * p * ostep, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.y), it.orr, vo, (2 * p + 1) * ostep, 0);
    }
  });
}

__device__ __forceinline__ void str_eval_dyn(const StrItem& it, int b, int s, int ovoff, int ostep,
                                             const uint32_t (&ta)[2][2][4], const float (&wt)[2][2][4]) {
  if (b == 0) {
    switch (it.D) {
      case 8: str_eval<8, 0>(it, s, ovoff, ostep, ta, wt); break;
      case 4: str_eval<4, 0>(it, s, ovoff, ostep, ta, wt); break;
      case 2: str_eval<2, 0>(it, s, ovoff, ostep, ta, wt); break;
      default: str_eval<1, 0>(it, s, ovoff, ostep, ta, wt); break;
    }
  } else {
    switch (it.D) {
      case 8: str_eval<8, 1>(it, s, ovoff, ostep, ta, wt); break;
      case 4: str_eval<4, 1>(it, s, ovoff, ostep, ta, wt); break;
      case 2: str_eval<2, 1>(it, s, ovoff, ostep, ta, wt); break;
      default: str_eval<1, 1>(it, s, ovoff, ostep, ta, wt); break;
    }
  }
}

// an item with no valid sample: every bin of its channels is 0
__device__ __forceinline__ void str_zero(const StrItem& it, int ovoff, int ostep) {
  for (int ch = 0; ch < 2 * it.npairs; ++ch) __builtin_amdgcn_raw_buffer_store_b32(0u, it.orr, ovoff, ch * ostep, 0);
}

template <int kWpe = 0>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kWpe > 0 ? kWpe : 1))) roi_align_fwd_stream_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out,
                                                                      int64_t nitems, int G) {
  __shared__ __attribute__((aligned(16))) float slab[2 * kPairHalf];
  const int lane = threadIdx.x;
  const int nbins = c.ph * c.pw;
  const int ovoff = lane < nbins ? lane * 4 : 0x40000000;  // idle lanes: dropped by the range check
  const int ostep = nbins * 4;
  const uint32_t lbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)slab);
  int64_t t = blockIdx.x;
  if (t >= nitems) return;
  StrItem cur;
  for (;;) {  // first item with a valid sample
    str_setup(cur, lv, c, out, t, G);
    if (cur.ok) break;
    str_zero(cur, ovoff, ostep);
    t += gridDim.x;
    if (t >= nitems) return;
  }
  str_issue_dyn(cur, slab, 0, 0);
  int bt = 0, prev_st = 0;
  uint32_t ta[2][2][4];
  float wt[2][2][4];
  str_taps(cur, c, lbase, ta, wt);
  for (;;) {
    for (int s = 0; s + 1 < cur.nst; ++s) {
      str_issue_dyn(cur, slab, bt ^ 1, s + 1);
      wait_vmcnt_le(str_dma_count(cur.D) + prev_st);
      wave_sync();
      str_eval_dyn(cur, bt, s, ovoff, ostep, ta, wt);
      prev_st = 2 * cur.D;
      wave_sync();
      bt ^= 1;
    }
    // last stage of this item: first set up and issue the next item's stage 0
    StrItem nxt;
    bool have = false;
    int extra = 0;
    int64_t t2 = t;
    for (;;) {
      t2 += gridDim.x;
      if (t2 >= nitems) break;
      str_setup(nxt, lv, c, out, t2, G);
      if (nxt.ok) {
        have = true;
        break;
      }
      str_zero(nxt, ovoff, ostep);
      extra += 2 * nxt.npairs;
    }
    int dn = 0;
    if (have) {
      str_issue_dyn(nxt, slab, bt ^ 1, 0);
      dn = str_dma_count(nxt.D);
    }
    wait_vmcnt_le(dn + prev_st + extra);
    wave_sync();
    str_eval_dyn(cur, bt, cur.nst - 1, ovoff, ostep, ta, wt);
    prev_st = 2 * cur.D;
    wave_sync();
    bt ^= 1;
    if (!have) break;
    cur = nxt;
    t = t2;
    str_taps(cur, c, lbase, ta, wt);
  }
}

// ---------------------------------------------------------------------------
// Wide-staged forward (variant 30).  Workgroup = (RoI, 64 channels), wave = 16
// channels, lane = bin, as the per-RoI LDS kernel -- but every RoI is staged:
// the slab is the RoI's tap rows (the dense window [y0, y1] when it has at most
// 4*ph rows, else the list of the 2*ph samples' (lo, hi) rows) x the columns
// [x0 & ~3, x1 + 1] rounded up to whole 16-B quads, copied with 16-B loads
// (one buffer_load_dwordx4 per lane per 64 quads: a quarter of the load
// instructions of 4-B staging, which is what bound staging large windows) and
// ds_write_b128.  The x-pair (x_lo, x_lo + 1) of a sample row is one
// ds_read2_b32 into a register pair, and both products of the pair run as one
// v_pk_mul_f32 (the sum keeps the reference order, so results stay
// bit-identical).  A round stages 8 / RB channel windows (RB = 16-B loads per
// lane per window); the next round's loads are in flight while this round is
// evaluated.  Invalid samples have zero weights and read cell 0.  Windows
// beyond kX4Slab floats (none at 7x7 sampling 2 below 28 x 36) take the block
// gather.
constexpr int kX4Slab = 2048;  // floats per wave: 8 quads per lane

// kXcd: XCD x (= linear block id % 8) takes the x-th contiguous eighth of the
// (RoI, chunk) items, so RoIs that are neighbours in the input order share an L2.
template <int kSkip = 0, bool kXcd = false, int kWpe = 0>
__global__ void __launch_bounds__(kRoiThreads) __attribute__((amdgpu_waves_per_eu(kWpe > 0 ? kWpe : 1)))
roi_align_fwd_x4_kernel(RoiLevels lv, RoiCfg c,
                                                                       float* __restrict__ out) {
  constexpr int SR = 2;
  constexpr int kWC = kRoiChanChunk / (kRoiThreads / kWave);  // 16 channels per wave
  __shared__ __attribute__((aligned(16))) float slab_all[kRoiThreads / kWave][kX4Slab];
  int64_t k = blockIdx.x;
  int chunk = blockIdx.y;
  if (kXcd) {
    const int64_t total = (int64_t)gridDim.x * gridDim.y, per = (total + 7) / 8;
    const int64_t lin = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    const int64_t w = (lin % 8) * per + lin / 8;
    if (w >= total) return;
    k = w / gridDim.y;
    chunk = (int)(w - k * gridDim.y);
  }
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
  const int cw0 = chunk * kRoiChanChunk + wave * kWC;
  const int nch = min(kWC, c.C - cw0);
  float* slab = slab_all[wave];
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw;
  const int sy = (int)lv.sy[l], scs = (int)lv.sc[l];  // sx == 1 (host check)
  auto pos_y = [&](int p, int i) { return g.start_h + (float)p * g.bin_h + ((float)i + 0.5f) * g.bin_h * 0.5f; };
  auto pos_x = [&](int p, int i) { return g.start_w + (float)p * g.bin_w + ((float)i + 0.5f) * g.bin_w * 0.5f; };
  const int nly = 2 * SR * c.ph;  // row list: entry i = row (i & 1 ? hi : lo) of y-sample i / 2
  int yrow = -1, ylo = 1 << 30, yhi = -1, xlo = 1 << 30, xhi = -1;
  if (lane < nly) {
    const int s = lane >> 1;
    const Tap t = make_tap(pos_y(s >> 1, s & 1), H);
    if (t.valid) yrow = (lane & 1) ? t.hi : t.lo, ylo = t.lo, yhi = t.hi;
  }
  if (lane < SR * c.pw) {
    const Tap t = make_tap(pos_x(lane >> 1, lane & 1), W);
    if (t.valid) xlo = t.lo, xhi = t.hi;
  }
  const int y0 = __builtin_amdgcn_readfirstlane(wave_min_i32(ylo)), y1 = __builtin_amdgcn_readfirstlane(wave_max_i32(yhi));
  const int x0 = __builtin_amdgcn_readfirstlane(wave_min_i32(xlo)), x1 = __builtin_amdgcn_readfirstlane(wave_max_i32(xhi));
  const bool any = y1 >= y0 && x1 >= x0;
  const bool dy = y1 - y0 + 1 <= nly;
  const int R = !any ? 0 : dy ? y1 - y0 + 1 : nly;
  const int xs0 = x0 & ~3, wq = any ? (x1 + 2 - xs0 + 3) >> 2 : 0;  // quads per slab row (covers x1 + 1)
  const int Wr = 4 * wq, nq = R * wq;
  if (4 * nq > kX4Slab) {  // uniform over the block (one RoI)
    if (kSkip != 2 && kSkip != 3) fwd_buf_block<2>(lv, c, out, k, chunk * kRoiChanChunk, g);
    return;
  }
  const int RB = (nq + kWave - 1) / kWave;
  if ((kSkip == 1 || kSkip == 2) && (kSkip == 1) == (RB <= 1)) return;
  if (nch <= 0) return;
  const bool active = lane < nbins;
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + (k * c.C + cw0) * nbins, (int64_t)nch * nbins * 4);
  const int ovoff = active ? lane * 4 : 0x40000000;  // idle lanes: dropped by the range check
  const int ostep = nbins * 4;
  if (!any) {
    for (int ch = 0; ch < nch; ++ch) __builtin_amdgcn_raw_buffer_store_b32(0u, orr, ovoff, ch * ostep, 0);
    return;
  }
  // one descriptor per channel plane: quads past the plane's last element read 0
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l] + (int64_t)cw0 * scs;
  const int64_t plane = ((int64_t)(H - 1) * sy + W) * 4;
  // this lane's bin: weights (zero for invalid samples) and slab offsets of its x-pairs
  const int bin = active ? lane : 0;
  const int py = (int)(((uint32_t)bin * ((65536u + (uint32_t)c.pw - 1u) / (uint32_t)c.pw)) >> 16), px = bin - py * c.pw;
  f32x2 wlo[SR][SR], whi[SR][SR];  // (w_ll, w_lh), (w_hl, w_hh)
  int sa[SR][SR][2];               // slab floats of the (x_lo, x_lo + 1) pair in rows lo / hi
#pragma unroll
  for (int iy = 0; iy < SR; ++iy) {
    const Tap a = make_tap(pos_y(py, iy), H);
    const int r0 = dy ? a.lo - y0 : 2 * (py * SR + iy), r1 = dy ? a.hi - y0 : 2 * (py * SR + iy) + 1;
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap b = make_tap(pos_x(px, ix), W);
      const bool ok = a.valid && b.valid;
      wlo[iy][ix] = ok ? f32x2{a.h * b.h, a.h * b.l} : f32x2{0.f, 0.f};
      whi[iy][ix] = ok ? f32x2{a.l * b.h, a.l * b.l} : f32x2{0.f, 0.f};
      sa[iy][ix][0] = ok ? r0 * Wr + (b.lo - xs0) : 0;
      sa[iy][ix][1] = ok ? r1 * Wr + (b.lo - xs0) : 0;
    }
  }
  auto bin_value = [&](const float* sl) {
    float acc = 0.0f;
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        const f32x2 lo = {sl[sa[iy][ix][0]], sl[sa[iy][ix][0] + 1]};
        const f32x2 hi = {sl[sa[iy][ix][1]], sl[sa[iy][ix][1] + 1]};
        const f32x2 p = wlo[iy][ix] * lo, q = whi[iy][ix] * hi;
        acc = acc + (((p.x + p.y) + q.x) + q.y);
      }
    return acc * 0.25f;
  };
  // quad e = lane + 64 j of a window  <-  feature row (dense: y0 + e / wq; list: row e / wq), columns xs0 + 4 (e % wq)
  const uint32_t invq = (65536u + (uint32_t)wq - 1u) / (uint32_t)wq;
  auto run = [&](auto rb) {
    constexpr int RBc = decltype(rb)::value, D = 8 / RBc;  // D channel windows per round, 8 loads per lane
    int goff[RBc];
#pragma unroll
    for (int j = 0; j < RBc; ++j) {
      int e = lane + j * kWave;
      e = e < nq ? e : 0;  // lanes past the window re-read its first quad
      const int r = (int)(((uint32_t)e * invq) >> 16), m = e - r * wq;
      const int fy = dy ? y0 + r : __shfl(yrow >= 0 ? yrow : y0, r, kWave);
      goff[j] = (fy * sy + xs0 + 4 * m) * 4;
    }
    u32x4 st[D][RBc];
    auto issue = [&](int c0r) {
#pragma unroll
      for (int d = 0; d < D; ++d)
#pragma unroll
        for (int j = 0; j < RBc; ++j)
          st[d][j] = __builtin_amdgcn_raw_buffer_load_b128(
              uniform_rsrc(base + (int64_t)min(c0r + d, nch - 1) * scs, plane), goff[j], 0, 0);
    };
    issue(0);
    for (int i = 0; i < nch; i += D) {
#pragma unroll
      for (int d = 0; d < D; ++d)
#pragma unroll
        for (int j = 0; j < RBc; ++j)
          *reinterpret_cast<u32x4*>(slab + ((d * RBc + j) * kWave + lane) * 4) = st[d][j];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (i + D < nch) issue(i + D);
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if (i + d < nch) {
          if (kSkip == 3) {  // diagnostics: evaluate, do not store
            const float v = bin_value(slab + d * RBc * kWave * 4);
            asm volatile("" ::"v"(v));
          } else {
            const float v = kSkip == 4 ? 0.0f : bin_value(slab + d * RBc * kWave * 4);  // 4: store, do not evaluate
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), orr, ovoff, (i + d) * ostep, 0);
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  };
  if (RB <= 1)
    run(std::integral_constant<int, 1>{});
  else if (RB <= 2)
    run(std::integral_constant<int, 2>{});
  else if (RB <= 4)
    run(std::integral_constant<int, 4>{});
  else
    run(std::integral_constant<int, 8>{});
}

// ---------------------------------------------------------------------------
// Grouped forward (opt-in: frh_roi_align_fwd_ws).  Measured on cfg2 (1024 RoIs):
// 76-85 us vs 55 us for the per-RoI kernel -- each workgroup is a serial chain
// of a ~6 us dependent-load prologue plus ~2 us per 4-channel step (DESIGN.md
// §4); it moves half the L2 lines but does not yet hide the latency.
//
// roi_group_plan_kernel (one workgroup, K <= 8192): counting sort of the RoIs
// by (image, level, 128-px tile of the RoI centre), then the sorted sequence is
// cut into groups of kGrp consecutive RoIs of one (image, level).  Output:
// order [K], gstart [ngroups + 1], ngroups.
//
// roi_align_fwd_group_kernel: workgroup = (group, 64 channels), wave w = the
// group's RoI w.  The union of the group's tap rows (a bitmask over feature
// rows) x the union of their columns is staged per channel into a three-slot
// LDS ring by LDS-DMA (all 512 threads, fixed per-thread offsets), one barrier
// per channel; wave w evaluates RoI w's 49 bins from the slot.  A feature line
// shared by several RoIs of the group is fetched once, not once per RoI (the
// RoI-by-RoI kernels are bound by the L1-miss line rate: ~3.1M mostly partial
// lines for cfg2 vs ~1.6M here).  Groups whose union exceeds a slot fall back
// to roi_segment per wave.  XCD x (= block % 8) takes the x-th eighth of the
// groups, so neighbouring groups share an L2.
constexpr int kGrp = 8;                    // RoIs per group = waves per workgroup
constexpr int kGrpThreads = kGrp * kWave;  // 512
constexpr int kGrpChans = 64;              // channels per workgroup
constexpr int kGrpRing = 18432;            // LDS ring floats (72 KB: two workgroups per CU)
constexpr int kRowWords = 32;              // union row bitmask: feature maps up to 1024 rows
constexpr int kMaxURows = 512;
constexpr int kPlanThreads = 1024, kPlanMaxRois = 8192, kPlanBuckets = 4096;

struct GroupPlan {
  const int32_t* order;    // [K] RoI ids, grouped
  const int32_t* gstart;   // [maxg + 1]; gstart[ngroups] = K
  const int32_t* ngroups;  // [1]
};

// block-wide exclusive scan (sum or max) of one value per thread
template <bool kMax>
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  auto op = [](uint32_t a, uint32_t b) { return kMax ? (a > b ? a : b) : a + b; };
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, kWave);
    if (lane >= o) inc = op(inc, u);
  }
  if (lane == kWave - 1) wsum[w] = inc;
  __syncthreads();
  uint32_t base = 0, all = 0;
  for (int i = 0; i < (int)(blockDim.x / kWave); ++i) {
    if (i < w) base = op(base, wsum[i]);
    all = op(all, wsum[i]);
  }
  *total = all;
  __syncthreads();
  // exclusive: the inclusive value of the previous lane, folded into the earlier waves' total
  const uint32_t prev = __shfl_up(inc, 1, kWave);
  return lane == 0 ? base : op(base, prev);
}

__global__ void __launch_bounds__(kPlanThreads) roi_group_plan_kernel(const float* rois, const int64_t* levels,
                                                                      int32_t K, int32_t* order, int32_t* gstart,
                                                                      int32_t* ngroups) {
  __shared__ uint32_t cnt[kPlanBuckets];
  __shared__ uint16_t keys[kPlanMaxRois];
  __shared__ uint16_t pkey[kPlanMaxRois];
  __shared__ uint32_t wsum[kPlanThreads / kWave];
  const int t = threadIdx.x;
  for (int b = t; b < kPlanBuckets; b += kPlanThreads) cnt[b] = 0;
  __syncthreads();
  for (int k = t; k < K; k += kPlanThreads) {
    const float* r = rois + (int64_t)k * 5;
    const int lvl = levels ? (int)levels[k] : 0;
    const float xc = 0.5f * (r[1] + r[3]), yc = 0.5f * (r[2] + r[4]);
    const int ty = yc < 0.0f ? 0 : (yc >= 896.0f ? 7 : (int)(yc * (1.0f / 128.0f)));
    const int tx = xc < 0.0f ? 0 : (xc >= 896.0f ? 7 : (int)(xc * (1.0f / 128.0f)));
    const uint16_t key = (uint16_t)((((int)r[0] & 15) << 8) | ((lvl & 3) << 6) | (ty << 3) | tx);
    keys[k] = key;
    atomicAdd(&cnt[key], 1u);
  }
  __syncthreads();
  constexpr int P = kPlanBuckets / kPlanThreads;
  uint32_t loc[P], s = 0, tot;
#pragma unroll
  for (int i = 0; i < P; ++i) {
    loc[i] = s;
    s += cnt[t * P + i];
  }
  const uint32_t base = block_exscan<false>(s, wsum, &tot);
#pragma unroll
  for (int i = 0; i < P; ++i) cnt[t * P + i] = base + loc[i];
  __syncthreads();
  for (int k = t; k < K; k += kPlanThreads) {
    const uint32_t pos = atomicAdd(&cnt[keys[k]], 1u);  // order inside a bucket: arbitrary
    order[pos] = k;
    pkey[pos] = keys[k];
  }
  __syncthreads();
  // groups: runs of equal (image, level) = pkey >> 6, cut every kGrp positions
  constexpr int Q = kPlanMaxRois / kPlanThreads;
  uint32_t segs[Q], lastseg = 0;
#pragma unroll
  for (int i = 0; i < Q; ++i) {
    const int p = t * Q + i;
    const bool head = p < K && (p == 0 || (pkey[p] >> 6) != (pkey[p - 1] >> 6));
    if (head) lastseg = (uint32_t)p;
    segs[i] = lastseg;  // running segment start inside this thread's span (0 = none yet)
  }
  const uint32_t carry = block_exscan<true>(lastseg, wsum, &tot);  // latest head before this span
  uint32_t nhead = 0;
  bool gflag[Q];
#pragma unroll
  for (int i = 0; i < Q; ++i) {
    const int p = t * Q + i;
    const uint32_t ss = segs[i] > carry ? segs[i] : carry;
    gflag[i] = p < K && ((uint32_t)p - ss) % kGrp == 0;
    nhead += gflag[i];
  }
  const uint32_t gbase = block_exscan<false>(nhead, wsum, &tot);
  uint32_t gid = gbase;
#pragma unroll
  for (int i = 0; i < Q; ++i)
    if (gflag[i]) gstart[gid++] = t * Q + i;
  if (t == 0) {
    gstart[tot] = K;
    ngroups[0] = (int32_t)tot;
  }
}

// kDiag (timing diagnostics only, variant 51): thread 0 of every workgroup writes
// int64 [start, union ready, end, path | U << 8] past the K*C*ph*pw results.
template <int kV, int kDiag = 0>
__global__ void __launch_bounds__(kGrpThreads) roi_align_fwd_group_kernel(RoiLevels lv, RoiCfg c, GroupPlan gp,
                                                                          float* __restrict__ out) {
  const uint64_t t_start = kDiag ? __builtin_amdgcn_s_memrealtime() : 0;
  constexpr int SR = 2;
  __shared__ float ring[kGrpRing];
  __shared__ uint32_t umask[kRowWords], upre[kRowWords + 1];
  __shared__ uint16_t urows[kMaxURows];
  __shared__ int ux[2];
  const int t = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(t / kWave), lane = t & (kWave - 1);
  const int ng = __builtin_amdgcn_readfirstlane(gp.ngroups[0]);
  const int gq = (ng + 7) >> 3;  // groups per XCD slice
  const int nchunk = (c.C + kGrpChans - 1) / kGrpChans;
  const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
  const int chunk = gq ? j / gq : 0, gi = j - chunk * gq;
  const int grp = xcd * gq + gi;
  if (gq == 0 || chunk >= nchunk || grp >= ng) return;  // uniform over the block
  const int gs = __builtin_amdgcn_readfirstlane(gp.gstart[grp]);
  const int gn = __builtin_amdgcn_readfirstlane(gp.gstart[grp + 1]) - gs;
  const bool has = wave < gn;  // waves past the group mirror its first RoI and store nothing
  const int64_t k = __builtin_amdgcn_readfirstlane(gp.order[gs + (has ? wave : 0)]);
  const int c0 = chunk * kGrpChans, c1 = min(c.C, c0 + kGrpChans);
  if (t < kRowWords) umask[t] = 0;
  if (t == 0) ux[0] = 1 << 30, ux[1] = -1;
  __syncthreads();
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw;
  const int sy = (int)lv.sy[l], sx = (int)lv.sx[l], scs = (int)lv.sc[l];
  const bool active = lane < nbins;
  const int bin = active ? lane : 0;
  const int py = bin / c.pw, px = bin - py * c.pw;
  Tap ty[SR], tx[SR];
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    ty[i] = make_tap(g.start_h + (float)py * g.bin_h + ((float)i + 0.5f) * g.bin_h * 0.5f, H);
    tx[i] = make_tap(g.start_w + (float)px * g.bin_w + ((float)i + 0.5f) * g.bin_w * 0.5f, W);
  }
  // the union: every row a tap reads, and the column span
  int xlo = 1 << 30, xhi = -1;
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    if (active && ty[i].valid && ty[i].hi < kRowWords * 32) {
      atomicOr(&umask[ty[i].lo >> 5], 1u << (ty[i].lo & 31));
      atomicOr(&umask[ty[i].hi >> 5], 1u << (ty[i].hi & 31));
    }
    if (active && tx[i].valid) xlo = min(xlo, tx[i].lo), xhi = max(xhi, tx[i].hi);
  }
  const int wx0 = wave_min_i32(xlo), wx1 = wave_max_i32(xhi);
  if (lane == 0 && wx1 >= 0) {
    atomicMin(&ux[0], wx0);
    atomicMax(&ux[1], wx1);
  }
  __syncthreads();
  if (wave == 0) {  // prefix counts of the row mask, and the union's row list
    const uint32_t w = lane < kRowWords ? umask[lane] : 0u;
    uint32_t inc = __popc(w);
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, kWave);
      if (lane >= o) inc += u;
    }
    const uint32_t ex = inc - __popc(w);
    if (lane < kRowWords) upre[lane] = ex;
    if (lane == kRowWords - 1) upre[kRowWords] = inc;
    uint32_t m = w, r = ex;
    while (m) {
      const int b = __ffs(m) - 1;
      if (r < (uint32_t)kMaxURows) urows[r] = (uint16_t)(lane * 32 + b);
      ++r;
      m &= m - 1;
    }
  }
  __syncthreads();
  const uint64_t t_union = kDiag ? __builtin_amdgcn_s_memrealtime() : 0;
  auto stamp = [&](int path, int U) {
    if (kDiag && t == 0) {
      int64_t* d = reinterpret_cast<int64_t*>(out + c.K * c.C * c.ph * c.pw) + (int64_t)blockIdx.x * 4;
      d[0] = (int64_t)t_start;
      d[1] = (int64_t)t_union;
      d[2] = (int64_t)__builtin_amdgcn_s_memrealtime();
      d[3] = path | ((int64_t)U << 8);
    }
  };
  const int nr = (int)upre[kRowWords];
  const int ux0 = ux[0], ux1 = ux[1];
  const int xs0 = ux0 & ~(kV - 1);
  const int uw = kV == 1 ? ((ux1 - ux0 + 1) | 1) : ((ux1 - xs0 + kV) & ~(kV - 1));
  const int U = nr * uw;
  bool rows_ok = H <= kRowWords * 32;
  const int nbig = __builtin_amdgcn_readfirstlane((int)(ux1 < 0 ? 0 : 1));
  if (nbig == 0 || !rows_ok || nr > kMaxURows || 3 * U > kGrpRing - 2 * kV * kWave * kGrp) {
    // no valid tap anywhere, or a union too large for three slots: each wave on its own RoI
    if (has) roi_segment<kGrpRing / kGrp, kV>(lv, c, out, ring + wave * (kGrpRing / kGrp), k, c0, c1, lane);
    if (kDiag) {
      __syncthreads();
      stamp(1, U);
    }
    return;
  }
  bool ok[SR][SR];
  float wt[SR][SR][4];
  int sa[SR][2][SR][2];
  auto ridx = [&](int y) { return (int)upre[y >> 5] + __popc(umask[y >> 5] & ((1u << (y & 31)) - 1u)); };
#pragma unroll
  for (int iy = 0; iy < SR; ++iy) {
    const int rl = ty[iy].valid ? ridx(ty[iy].lo) : 0, rh = ty[iy].valid ? ridx(ty[iy].hi) : 0;
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap a = ty[iy], b = tx[ix];
      const bool v = a.valid && b.valid;
      ok[iy][ix] = v;
      wt[iy][ix][0] = a.h * b.h;
      wt[iy][ix][1] = a.h * b.l;
      wt[iy][ix][2] = a.l * b.h;
      wt[iy][ix][3] = a.l * b.l;
      sa[iy][0][ix][0] = v ? (rl * uw + (b.lo - xs0)) * 4 : 0;
      sa[iy][0][ix][1] = v ? (rl * uw + (b.hi - xs0)) * 4 : 0;
      sa[iy][1][ix][0] = v ? (rh * uw + (b.lo - xs0)) * 4 : 0;
      sa[iy][1][ix][1] = v ? (rh * uw + (b.hi - xs0)) * 4 : 0;
    }
  }
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l];
  const int64_t extent = ((int64_t)(c.C - 1) * scs + (int64_t)(H - 1) * sy + (int64_t)(W - 1) * sx + 1) * 4;
  const __amdgpu_buffer_rsrc_t fr = uniform_rsrc(base, extent);
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + k * c.C * nbins, (int64_t)c.C * nbins * 4);
  const int cstep = scs * 4, ostep = nbins * 4;
  const int ovoff = (has && active) ? lane * 4 : 0x40000000;  // dropped by the range check
  // Staging: a channel's union is Q wave-instructions of kV*64 floats; instruction q is
  // issued by wave q % 8 (round q / 8).  Every wave issues the same J rounds per
  // channel (rounds past Q load a dummy into a junk block), so one counted vmcnt fits
  // all waves.  A step is B channels (B slots of Q*kV*64 floats); three step buffers,
  // two steps in flight ahead of the one being read, one barrier per step.
  constexpr int kPiece = kV * kWave;  // floats per DMA wave-instruction
  constexpr int kRing = kGrpRing - kPiece;
  const int Q = (U + kPiece - 1) / kPiece;
  const int SF = Q * kPiece;
  float* junk = ring + kRing;
  auto run = [&](auto jj, auto bb, auto ddp) {
    constexpr int J = decltype(jj)::value;   // DMA rounds per wave per channel
    constexpr int B = decltype(bb)::value;   // channels per step
    constexpr int D = decltype(ddp)::value;  // steps in flight ahead of the one being read
    constexpr int NB = D + 1;                // step buffers
    static_assert(B * (J + 1) * (D - 1) < 64 && B * J * D < 64, "vmcnt range");
    int goff[J], dst[J];
#pragma unroll
    for (int q = 0; q < J; ++q) {
      const int piece = wave + q * kGrp;
      const int e = kV * lane + piece * kPiece;
      const int r = e / uw, col = e - r * uw;
      const int fx = kV == 1 ? min(xs0 + col, W - 1) : xs0 + col;
      const bool real = piece < Q;
      goff[q] = real && e < U ? ((int)urows[r] * sy + fx * sx) * 4 : ((int)urows[0] * sy + xs0 * sx) * 4;
      dst[q] = real ? piece * kPiece : -1;
    }
    const int nch = c1 - c0, nst = (nch + B - 1) / B;
    auto issue = [&](int st) {  // step st: channels c0 + B*st + b (clamped) -> buffer st % NB
      float* sb = ring + (st % NB) * (B * SF);
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const int ch = c0 + min(st * B + b, nch - 1);
#pragma unroll
        for (int q = 0; q < J; ++q) lds_dma<4 * kV>(fr, dst[q] >= 0 ? sb + b * SF + dst[q] : junk, goff[q], ch * cstep);
      }
    };
    for (int st = 0; st < D && st < nst; ++st) issue(st);
    for (int st = 0; st < nst; ++st) {
      // retire step st: younger than its DMAs are, for each of the D-1 steps issued after
      // it, B stores and B*J DMAs (the first step has no stores before; the tail waits all)
      if (st + D - 1 < nst) {
        if (st == 0)
          wait_vmcnt<B * J * (D - 1)>();
        else
          wait_vmcnt<B * (J + 1) * (D - 1)>();
      } else {
        wait_vmcnt<0>();
      }
      const uint64_t t_w = kDiag ? __builtin_amdgcn_s_memrealtime() : 0;
      asm volatile("s_barrier" ::: "memory");  // every wave's share of step st has landed
      const uint64_t t_b = kDiag ? __builtin_amdgcn_s_memrealtime() : 0;
      const char* sb = reinterpret_cast<const char*>(ring + (st % NB) * (B * SF));
      float acc[B];
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const char* sl = sb + b * SF * 4;
        float v[SR][SR][4];
#pragma unroll
        for (int iy = 0; iy < SR; ++iy)
#pragma unroll
          for (int ix = 0; ix < SR; ++ix) {
            v[iy][ix][0] = *reinterpret_cast<const float*>(sl + sa[iy][0][ix][0]);
            v[iy][ix][1] = *reinterpret_cast<const float*>(sl + sa[iy][0][ix][1]);
            v[iy][ix][2] = *reinterpret_cast<const float*>(sl + sa[iy][1][ix][0]);
            v[iy][ix][3] = *reinterpret_cast<const float*>(sl + sa[iy][1][ix][1]);
          }
        float a = 0.0f;
#pragma unroll
        for (int iy = 0; iy < SR; ++iy)
#pragma unroll
          for (int ix = 0; ix < SR; ++ix) {
            float val = ((wt[iy][ix][0] * v[iy][ix][0] + wt[iy][ix][1] * v[iy][ix][1]) + wt[iy][ix][2] * v[iy][ix][2]) +
                        wt[iy][ix][3] * v[iy][ix][3];
            a = a + (ok[iy][ix] ? val : 0.0f);
          }
        acc[b] = a * 0.25f;
      }
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const int ci = st * B + b;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[b]), orr, ci < nch ? ovoff : 0x40000000,
                                              (c0 + ci) * ostep, 0);
      }
      // buffer (st + D) % NB was last read in step st - 1, which every wave finished before this step's barrier
      if (st + D < nst) issue(st + D);
      if (kDiag && lane == 0 && blockIdx.x < 64 && st < 20 && (wave == 0 || wave == 7)) {
        int64_t* d = reinterpret_cast<int64_t*>(out + c.K * c.C * c.ph * c.pw) + 8192 +
                     ((int64_t)(blockIdx.x * 2 + (wave ? 1 : 0)) * 20 + st) * 4;
        d[0] = (int64_t)t_w;
        d[1] = (int64_t)t_b;
        d[2] = (int64_t)__builtin_amdgcn_s_memrealtime();
        d[3] = B * 100 + D;
      }
    }
  };
  const int J = (Q + kGrp - 1) / kGrp;
  // deepest pipeline the ring holds: B channels per step, D steps ahead
  // B channels per step, D steps ahead: the deepest pipeline the ring holds within vmcnt range
  const int n4 = kRing / (4 * SF), n2 = kRing / (2 * SF), n1 = kRing / SF;  // step buffers that fit
  const int shape = n4 >= 7 ? 0 : n4 >= 5 ? 1 : n4 >= 3 ? 2 : n2 >= 5 ? 3 : n2 >= 3 ? 4 : n1 >= 5 ? 5 : 6;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;
  using I6 = std::integral_constant<int, 6>;
  auto with_bd = [&](auto jj) {
    constexpr int Jc = decltype(jj)::value;
    constexpr bool f46 = 4 * (Jc + 1) * 5 < 64, f44 = 4 * (Jc + 1) * 3 < 64;
    if (shape == 0 && f46)
      run(jj, I4{}, std::conditional_t<f46, I6, I2>{});
    else if (shape <= 1 && f44)
      run(jj, I4{}, std::conditional_t<f44, I4, I2>{});
    else if (shape <= 2)
      run(jj, I4{}, I2{});
    else if (shape == 3)
      run(jj, I2{}, I4{});
    else if (shape == 4)
      run(jj, I2{}, I2{});
    else if (shape == 5)
      run(jj, I1{}, I4{});
    else
      run(jj, I1{}, I2{});
  };
  if (J <= 1)
    with_bd(std::integral_constant<int, 1>{});
  else if (J <= 2)
    with_bd(std::integral_constant<int, 2>{});
  else if (J <= 3)
    with_bd(std::integral_constant<int, 3>{});
  else  // only the 4-byte staging (kV = 1) gets here
    run(std::integral_constant<int, 16>{}, std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{});
  if (kDiag) {
    __syncthreads();
    stamp(2 + J * 4, U);
  }
}
// ---------------------------------------------------------------------------
// Backward into a channels-last gradient (sampling 2, ph*pw <= 64, C % 16 == 0):
// the default.  Global float atomics execute at the memory side as 64-B
// requests (MI355X_MICROARCH.md, global float atomics): the NCHW flush above
// adds window rows of a few cells -- mostly partial 64-B requests -- and runs
// at a fraction of the atomic byte rate.  Here the gradient is accumulated in
// a [B, H, W, C] buffer (zeroed by the caller; the autograd wrapper returns it
// as a channels_last view): each wave owns 16 channels of the RoI, sums its
// taps into an LDS band of the tap window laid out [cell][16 channels] (row
// stride 17: conflict-free both ways), and flushes each window cell's 16
// channels as ONE full 64-B atomic request.  Windows taller than a band of
// kClBandCells cells are done band by band.  Contributions are the reference's
// grad * w / count (count = 4: an exact * 0.25); float atomics make the
// summation order run-dependent, as in torchvision's own CUDA backward.
// Measured (tools/bench_roi_bwd.py, cfg2 RoIs, incl. clearing): 1.38 ms vs 1.19 ms
// for the NCHW kernel, so the NCHW kernel stays the default (ops.ROI_ALIGN_BWD);
// this one runs whenever the caller hands a channels_last gradient.
constexpr int kClChans = 16;      // channels per wave = floats per flushed 64-B segment
constexpr int kClBandCells = 256;  // window cells per LDS band
constexpr int kClStride = kClChans + 1;

__global__ void __launch_bounds__(kRoiThreads) roi_align_bwd_cl_kernel(RoiLevels lv, RoiCfg c,
                                                                       const float* __restrict__ gout) {
  constexpr int SR = 2;
  __shared__ float band_all[kRoiThreads / kWave][kClBandCells * kClStride];  // 68 KB
  const int64_t k = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
  const int cw0 = blockIdx.y * kRoiChanChunk + wave * kClChans;
  if (cw0 >= c.C) return;  // host: C % 16 == 0
  float* band = band_all[wave];
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw;
  const bool active = lane < nbins;
  const int bin = active ? lane : 0;
  const int py = bin / c.pw, px = bin - py * c.pw;
  Tap ty[SR], tx[SR];
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    ty[i] = make_tap(g.start_h + (float)py * g.bin_h + ((float)i + 0.5f) * g.bin_h * 0.5f, H);
    tx[i] = make_tap(g.start_w + (float)px * g.bin_w + ((float)i + 0.5f) * g.bin_w * 0.5f, W);
  }
  int ylo = 1 << 30, yhi = -1, xlo = 1 << 30, xhi = -1;
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    if (active && ty[i].valid) ylo = min(ylo, ty[i].lo), yhi = max(yhi, ty[i].hi);
    if (active && tx[i].valid) xlo = min(xlo, tx[i].lo), xhi = max(xhi, tx[i].hi);
  }
  const int y0 = __builtin_amdgcn_readfirstlane(wave_min_i32(ylo)), y1 = __builtin_amdgcn_readfirstlane(wave_max_i32(yhi));
  const int x0 = __builtin_amdgcn_readfirstlane(wave_min_i32(xlo)), x1 = __builtin_amdgcn_readfirstlane(wave_max_i32(xhi));
  if (y1 < y0 || x1 < x0) return;  // no valid tap: no gradient
  const int WW = x1 - x0 + 1;      // host: every level's width <= kClBandCells
  const int RB = kClBandCells / WW;  // window rows per band
  const int64_t sy = lv.sy[l], sx = lv.sx[l];
  float* gbase = lv.grad[l] + (int64_t)g.b * lv.sb[l] + (int64_t)cw0 * lv.sc[l];
  const float* go = gout + (k * c.C + cw0) * nbins;
  bool ok[SR][SR];
  float wt[SR][SR][4];
  int row[SR][SR][4], col[SR][SR][4];
#pragma unroll
  for (int iy = 0; iy < SR; ++iy)
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap a = ty[iy], b = tx[ix];
      ok[iy][ix] = active && a.valid && b.valid;
      wt[iy][ix][0] = a.h * b.h;
      wt[iy][ix][1] = a.h * b.l;
      wt[iy][ix][2] = a.l * b.h;
      wt[iy][ix][3] = a.l * b.l;
      row[iy][ix][0] = row[iy][ix][1] = a.lo - y0;
      row[iy][ix][2] = row[iy][ix][3] = a.hi - y0;
      col[iy][ix][0] = col[iy][ix][2] = b.lo - x0;
      col[iy][ix][1] = col[iy][ix][3] = b.hi - x0;
    }
  float gq[kClChans];  // grad * 0.25 per channel: (g * w) / 4 == (g * 0.25) * w exactly
#pragma unroll
  for (int ch = 0; ch < kClChans; ++ch) gq[ch] = active ? go[ch * nbins + bin] * 0.25f : 0.0f;
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  for (int r0 = 0; r0 <= y1 - y0; r0 += RB) {
    const int nr = min(RB, y1 - y0 + 1 - r0), ncell = nr * WW;
    for (int e = lane; e < ncell * kClStride; e += kWave) band[e] = 0.0f;
    wave_sync();
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rr = row[iy][ix][q] - r0;
          if (ok[iy][ix] && rr >= 0 && rr < nr) {
            float* cell = band + (rr * WW + col[iy][ix][q]) * kClStride;
            const float w = wt[iy][ix][q];
#pragma unroll
            for (int ch = 0; ch < kClChans; ++ch) atomicAdd(cell + ch, gq[ch] * w);
          }
        }
    wave_sync();
    // flush: lane = (cell, channel); the 16 channels of a cell are one 64-B segment
    for (int e = lane; e < ncell * kClChans; e += kWave) {
      const int ce = e / kClChans, ch = e - ce * kClChans;
      const float v = band[ce * kClStride + ch];
      const int y = y0 + r0 + ce / WW, x = x0 + ce % WW;
      if (v != 0.0f) atomicAdd(gbase + (int64_t)ch * lv.sc[l] + (int64_t)y * sy + (int64_t)x * sx, v);
    }
    wave_sync();  // the band is re-zeroed only after every lane read it
  }
}

// ---------------------------------------------------------------------------
// Backward, tiled gather (sampling 2, ph*pw <= 64): the default.  The
// window-accumulated kernel above still ends in one global float atomic per
// (RoI, channel, window cell) -- ~45 M for a cfg2 batch, bound by the L2
// atomic rate (1.24 ms per train step).  Here the feature gradient is built
// tile by tile with no global atomics:
//   bin_count : per RoI, the tap window (as the forward) -> the 16x16-cell
//               tiles of its level it overlaps; count per tile
//   bin_scan  : one workgroup: tile list offsets
//   bin_fill  : per RoI, append its id to each overlapped tile's list
//   tile      : workgroup = (tile, 32 channels), wave = 8 channels; the wave
//               zeroes an LDS copy of the tile for its channels, walks the
//               tile's RoIs (lane = bin) adding grad * w / count of every tap
//               that falls in the tile with ds_add_f32, then stores the tile --
//               every cell of every level written once (zeros where no RoI
//               reaches), so the caller need not clear the gradient.
// Contributions are the reference's grad * w / count, as the kernels above;
// the order of the RoIs within a tile follows the fill atomics, so the last
// bits are run-dependent like torchvision's own CUDA backward.
// Measured (tools/bench_roi_bwd.py, cfg2 RoIs): SLOWER than the atomic kernel --
// a RoI overlaps 4.4 tiles on average and every (RoI, tile) pair evaluates all
// 16 x 49 taps, and the positives around one ground truth pile up to 100 RoIs
// on one tile (one workgroup's serial list).  Opt-in (ops.ROI_ALIGN_BWD).

constexpr int kBwdTile = 16;                 // tile side in cells
constexpr int kBwdTileCells = kBwdTile * kBwdTile;
constexpr int kBwdTileChans = 32;            // channels per workgroup
constexpr int kBwdWaveChans = kBwdTileChans / (kRoiThreads / kWave);  // 8

struct TileMap {
  int nty[FRH_MAX_LEVELS], ntx[FRH_MAX_LEVELS];
  int64_t base[FRH_MAX_LEVELS + 1];  // first tile id of each level (images level-major inside)
  int B;
};

struct TileLists {
  uint32_t* count;  // [T]
  uint32_t* off;    // [T + 1]
  uint32_t* fill;   // [T]
  int4* win;        // [K]: tile rows ty0..ty1, cols tx0..tx1 (ty0 > ty1: none)
  int32_t* list;    // [cap]
  int64_t cap;
};

// the RoI's tap window at its level (forward's make_tap over all 2*ph / 2*pw samples)
__device__ __forceinline__ int4 roi_tap_window(const RoiCfg& c, const RoiLevels& lv, int64_t k, int* lvl, int* img) {
  const RoiGeom g = roi_geom(c, lv, k);
  const int H = lv.h[g.lvl], W = lv.w[g.lvl];
  int y0 = 1 << 30, y1 = -1, x0 = 1 << 30, x1 = -1;
  for (int p = 0; p < c.ph; ++p)
    for (int i = 0; i < 2; ++i) {
      const Tap t = make_tap(g.start_h + (float)p * g.bin_h + ((float)i + 0.5f) * g.bin_h * 0.5f, H);
      if (t.valid) y0 = min(y0, t.lo), y1 = max(y1, t.hi);
    }
  for (int p = 0; p < c.pw; ++p)
    for (int i = 0; i < 2; ++i) {
      const Tap t = make_tap(g.start_w + (float)p * g.bin_w + ((float)i + 0.5f) * g.bin_w * 0.5f, W);
      if (t.valid) x0 = min(x0, t.lo), x1 = max(x1, t.hi);
    }
  *lvl = g.lvl;
  *img = g.b;
  if (y1 < y0 || x1 < x0) return make_int4(1, 0, 1, 0);
  return make_int4(y0 / kBwdTile, y1 / kBwdTile, x0 / kBwdTile, x1 / kBwdTile);
}

__device__ __forceinline__ int64_t tile_id(const TileMap& tm, int l, int b, int ty, int tx) {
  return tm.base[l] + ((int64_t)b * tm.nty[l] + ty) * tm.ntx[l] + tx;
}

__global__ void roi_bwd_bin_count_kernel(RoiLevels lv, RoiCfg c, TileMap tm, TileLists tl) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= c.K) return;
  int l, b;
  const int4 w = roi_tap_window(c, lv, k, &l, &b);
  tl.win[k] = w;
  for (int ty = w.x; ty <= w.y; ++ty)
    for (int tx = w.z; tx <= w.w; ++tx) atomicAdd(&tl.count[tile_id(tm, l, b, ty, tx)], 1u);
}

__global__ void __launch_bounds__(1024) roi_bwd_bin_scan_kernel(TileLists tl, int64_t T) {
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (T + 1023) / 1024, s = t * per, e = min(T, s + per);
  uint32_t sum = 0;
  for (int64_t i = s; i < e; ++i) sum += tl.count[i];
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (int64_t i = s; i < e; ++i) {
    tl.off[i] = run;
    run += tl.count[i];
  }
  if (t == 1023) tl.off[T] = part[1023];
}

__global__ void roi_bwd_bin_fill_kernel(RoiLevels lv, RoiCfg c, TileMap tm, TileLists tl) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= c.K) return;
  const int4 w = tl.win[k];
  if (w.x > w.y) return;
  const float* r = c.rois + k * 5;
  const int b = (int)r[0], l = c.levels ? (int)c.levels[k] : 0;
  for (int ty = w.x; ty <= w.y; ++ty)
    for (int tx = w.z; tx <= w.w; ++tx) {
      const int64_t t = tile_id(tm, l, b, ty, tx);
      const uint32_t pos = tl.off[t] + atomicAdd(&tl.fill[t], 1u);
      if (pos < tl.cap) tl.list[pos] = (int32_t)k;
    }
}

__global__ void __launch_bounds__(kRoiThreads) roi_align_bwd_tile_kernel(RoiLevels lv, RoiCfg c, TileMap tm,
                                                                         TileLists tl, const float* __restrict__ gout) {
  constexpr int SR = 2;
  __shared__ float tile_all[kRoiThreads / kWave][kBwdWaveChans * kBwdTileCells];  // 32 KB
  const int64_t t = blockIdx.x;
  int l = 0;
  while (l + 1 < lv.L && t >= tm.base[l + 1]) ++l;
  const int64_t lt = t - tm.base[l];
  const int per_img = tm.nty[l] * tm.ntx[l];
  const int b = (int)(lt / per_img), rem = (int)(lt - (int64_t)b * per_img);
  const int tyi = rem / tm.ntx[l], txi = rem - tyi * tm.ntx[l];
  const int H = lv.h[l], W = lv.w[l];
  const int Y0 = tyi * kBwdTile, X0 = txi * kBwdTile;
  const int th = min(kBwdTile, H - Y0), tw = min(kBwdTile, W - X0);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
  const int cw0 = blockIdx.y * kBwdTileChans + wave * kBwdWaveChans;
  const int nch = min(kBwdWaveChans, c.C - cw0);
  if (nch <= 0) return;
  float* tile = tile_all[wave];
  for (int e = lane; e < kBwdWaveChans * kBwdTileCells; e += kWave) tile[e] = 0.0f;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int nbins = c.ph * c.pw;
  const bool active = lane < nbins;
  const int bin = active ? lane : 0;
  const int py = bin / c.pw, px = bin - py * c.pw;
  const uint32_t i0 = tl.off[t], i1 = min((int64_t)tl.off[t + 1], tl.cap);
  for (uint32_t i = i0; i < i1; ++i) {
    const int64_t k = tl.list[i];
    const RoiGeom g = roi_geom(c, lv, k);
    Tap ty[SR], tx[SR];
#pragma unroll
    for (int s = 0; s < SR; ++s) {
      ty[s] = make_tap(g.start_h + (float)py * g.bin_h + ((float)s + 0.5f) * g.bin_h * 0.5f, H);
      tx[s] = make_tap(g.start_w + (float)px * g.bin_w + ((float)s + 0.5f) * g.bin_w * 0.5f, W);
    }
    // tile cells of this bin's 16 taps (-1: outside the tile or invalid sample) and weights
    int cell[SR][SR][4];
    float wt[SR][SR][4];
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        const Tap a = ty[iy], bb = tx[ix];
        const bool ok = active && a.valid && bb.valid;
        const int ylo = a.lo - Y0, yhi = a.hi - Y0, xlo = bb.lo - X0, xhi = bb.hi - X0;
        const bool iyl = ylo >= 0 && ylo < th, iyh = yhi >= 0 && yhi < th;
        const bool ixl = xlo >= 0 && xlo < tw, ixh = xhi >= 0 && xhi < tw;
        cell[iy][ix][0] = ok && iyl && ixl ? ylo * kBwdTile + xlo : -1;
        cell[iy][ix][1] = ok && iyl && ixh ? ylo * kBwdTile + xhi : -1;
        cell[iy][ix][2] = ok && iyh && ixl ? yhi * kBwdTile + xlo : -1;
        cell[iy][ix][3] = ok && iyh && ixh ? yhi * kBwdTile + xhi : -1;
        wt[iy][ix][0] = a.h * bb.h;
        wt[iy][ix][1] = a.h * bb.l;
        wt[iy][ix][2] = a.l * bb.h;
        wt[iy][ix][3] = a.l * bb.l;
      }
    const float* go = gout + (k * c.C + cw0) * nbins + bin;
    float gv[kBwdWaveChans];
#pragma unroll
    for (int ch = 0; ch < kBwdWaveChans; ++ch) gv[ch] = (active && ch < nch) ? go[ch * nbins] : 0.0f;
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = cell[iy][ix][q];
          if (e >= 0) {
#pragma unroll
            for (int ch = 0; ch < kBwdWaveChans; ++ch)
              atomicAdd(&tile[ch * kBwdTileCells + e], gv[ch] * wt[iy][ix][q] * 0.25f);
          }
        }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float* gbase = lv.grad[l] + (int64_t)b * lv.sb[l] + (int64_t)cw0 * lv.sc[l];
  for (int e = lane; e < nch * kBwdTileCells; e += kWave) {
    const int ch = e / kBwdTileCells, cl = e - ch * kBwdTileCells;
    const int y = cl / kBwdTile, x = cl - y * kBwdTile;
    if (y < th && x < tw) gbase[(int64_t)ch * lv.sc[l] + (int64_t)(Y0 + y) * lv.sy[l] + (int64_t)(X0 + x) * lv.sx[l]] =
        tile[e];
  }
}
// resident single-wave workgroups of the persistent forward: CUs x the occupancy the
// kernel's LDS and registers allow (FRH_STR_WAVES overrides the per-CU count)
template <int kWpe>
static int64_t stream_grid_waves() {
  static int64_t cached[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
  if (!cached[dev]) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, roi_align_fwd_stream_kernel<kWpe>, kWave, 0) !=
            hipSuccess ||
        per <= 0)
      per = 8;
    if (const char* e = getenv("FRH_STR_WAVES")) per = std::max(1, atoi(e));
    cached[dev] = (int64_t)cus * per;
  }
  return cached[dev];
}

static int32_t group_bound(int64_t num_rois) { return (int32_t)((num_rois + kGrp - 1) / kGrp + 64); }

}  // namespace frh

using namespace frh;

// variant: 0 = direct gather, 10 = per-RoI LDS windows (9, 11, 12, 15-19: its
// stage-size / chunk / occupancy variants), 20 = channel pairs (the product default;
// FRH_PAIR_PW = 4 / 16 / 32 / 64 pairs per wave instead of 8; 21 chunk-major XCD order), 25 / 26 = persistent
// item-walking pair waves, 30-37 = wide-staged (31-34 diagnostics, 35 XCD order,
// 36 / 37 occupancy), 50 / 51 = grouped union staging (needs the workspace of
// frh_roi_align_workspace; 51 stamps), -1 = the product's choice.
extern "C" int32_t frh_roi_align_fwd_variant(int32_t variant, int32_t num_levels, const float* const* feats,
                                             const int32_t* feat_hw, const int64_t* strides, const float* scales,
                                             int32_t batch, int32_t channels, const float* rois,
                                             const int64_t* roi_levels, int64_t num_rois, int32_t pooled_h,
                                             int32_t pooled_w, int32_t sampling_ratio, int32_t aligned, float* out,
                                             void* workspace, size_t ws_bytes, void* stream) {
  int32_t r = roi_common_checks(batch, channels, num_rois, pooled_h, pooled_w, rois);
  if (r) return r;
  FRH_REQUIRE((feats && out) || num_rois == 0, "null pointer argument");
  RoiLevels lv;
  r = make_levels(num_levels, feats, nullptr, feat_hw, strides, scales, &lv);
  if (r) return r;
  if (num_rois == 0) return FRH_OK;
  RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned};
  const FwdCaps f = fwd_caps(lv, channels, pooled_h, pooled_w, sampling_ratio);
  const bool grp_ok = f.lds && num_rois <= kPlanMaxRois && workspace &&
                      ws_bytes >= ((size_t)num_rois + group_bound(num_rois) + 2) * sizeof(int32_t);
  const bool pok = pair_ok(f, channels, pooled_h, pooled_w);
  if (variant == -2) variant = grp_ok ? 50 : -1;
  if (variant < 0) variant = pok ? 20 : (f.lds ? 10 : 0);
  bool x4_ok = f.lds && 4 * pooled_h <= kWave;
  for (int l = 0; l < lv.L; ++l) x4_ok = x4_ok && lv.sx[l] == 1 && lv.sy[l] % 4 == 0 && lv.sc[l] % 4 == 0 &&
                                         lv.sb[l] % 4 == 0 && (reinterpret_cast<uintptr_t>(lv.feat[l]) & 15) == 0;
  FRH_REQUIRE(variant == 0 || ((variant >= 9 && variant <= 19 && variant != 13 && variant != 14) && f.lds) ||
                  ((variant == 50 || variant == 51) && grp_ok) || (((variant >= 20 && variant <= 29) || (variant >= 38 && variant <= 49) || variant == 52 || variant == 53 || variant == 55) && pok) ||
                  (variant >= 30 && variant <= 37 && x4_ok),
              "roi_align variant %d unsupported here", variant);
  const dim3 grid((unsigned)num_rois, (unsigned)((channels + kRoiChanChunk - 1) / kRoiChanChunk));
  if (variant == 50 || variant == 51) {
    int32_t* order = static_cast<int32_t*>(workspace);
    int32_t* ngroups = order + num_rois;
    int32_t* gstart = ngroups + 1;
    hipLaunchKernelGGL(roi_group_plan_kernel, dim3(1), dim3(kPlanThreads), 0, as_stream(stream), rois, roi_levels,
                       (int32_t)num_rois, order, gstart, ngroups);
    r = check_launch("frh_roi_align_fwd (plan)");
    if (r) return r;
    const GroupPlan gp{order, gstart, ngroups};
    const int64_t nchunk = (channels + kGrpChans - 1) / kGrpChans;
    const dim3 g((unsigned)(8 * ((group_bound(num_rois) + 7) / 8) * nchunk));
    if (variant == 51)
      hipLaunchKernelGGL((roi_align_fwd_group_kernel<4, 1>), g, dim3(kGrpThreads), 0, as_stream(stream), lv, c, gp, out);
    else if (f.x4)
      hipLaunchKernelGGL(roi_align_fwd_group_kernel<4>, g, dim3(kGrpThreads), 0, as_stream(stream), lv, c, gp, out);
    else
      hipLaunchKernelGGL(roi_align_fwd_group_kernel<1>, g, dim3(kGrpThreads), 0, as_stream(stream), lv, c, gp, out);
  } else if (variant == 20) {
    const int pw = getenv("FRH_PAIR_PW") ? atoi(getenv("FRH_PAIR_PW")) : kPairWave;
    const dim3 g2((unsigned)num_rois, (unsigned)((channels + 2 * pw - 1) / (2 * pw)));
    if (pw == 64) hipLaunchKernelGGL((roi_align_fwd_pair_kernel<64>), g2, dim3(kWave), 0, as_stream(stream), lv, c, out);
    else if (pw == 32) hipLaunchKernelGGL((roi_align_fwd_pair_kernel<32>), g2, dim3(kWave), 0, as_stream(stream), lv, c, out);
    else if (pw == 16) hipLaunchKernelGGL((roi_align_fwd_pair_kernel<16>), g2, dim3(kWave), 0, as_stream(stream), lv, c, out);
    else if (pw == 4) hipLaunchKernelGGL((roi_align_fwd_pair_kernel<4>), g2, dim3(kWave), 0, as_stream(stream), lv, c, out);
    else hipLaunchKernelGGL((roi_align_fwd_pair_kernel<8>), g2, dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else if (variant == 21) {  // pairs, chunk-major XCD order (roi_kernels.h kOrder 1)
    const int64_t total = num_rois * ((channels + 2 * kPairWave - 1) / (2 * kPairWave));
    hipLaunchKernelGGL((roi_align_fwd_pair_kernel<kPairWave, kPairHalf, 1>), dim3((unsigned)(8 * ((total + 7) / 8))),
                       dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else if (variant == 38 || variant == 52 || variant == 53) {
    // 38: dynamic item scheduling (roi_align_fwd_pair_dyn_kernel), 512 waves per XCD list;
    // 52 / 53: static strided items with the next RoI prefetched, 512 / 256 waves per list
    const uint32_t wpl = variant == 53 ? 256 : 512;
    if (variant == 38)
      hipLaunchKernelGGL((roi_align_fwd_pair_dyn_kernel<kPairWave, kPairHalf, kCpolNT>), dim3(8 * wpl), dim3(kWave), 0,
                         as_stream(stream), lv, c, out, wpl);
    else
      hipLaunchKernelGGL((roi_align_fwd_pair_dyn_kernel<kPairWave, kPairHalf, kCpolNT, true>), dim3(8 * wpl), dim3(kWave),
                         0, as_stream(stream), lv, c, out, wpl);
  } else if (variant == 55) {  // the default with the lean tap state (kLean)
    const int64_t total = num_rois * ((channels + 2 * kPairWave - 1) / (2 * kPairWave));
    hipLaunchKernelGGL((roi_align_fwd_pair_kernel<kPairWave, kPairHalf, 1, kCpolNT, 0, false, true, 1, true, 1, true>),
                       dim3((unsigned)(8 * ((total + 7) / 8))), dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else if (variant == 29) {  // product kernel (single buffer, nt stores) with two items per wave
    const int64_t total = num_rois * ((channels + 2 * kPairWave - 1) / (2 * kPairWave));
    const int64_t per = (total + 7) / 8;
    hipLaunchKernelGGL((roi_align_fwd_pair_kernel<kPairWave, kPairHalf, 1, kCpolNT, 0, false, true, 1, true, 2>),
                       dim3((unsigned)(8 * ((per + 1) / 2))), dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else if (variant == 49 || variant == 39) {  // single buffer, no tap read-ahead: 49 registers for 5 waves per SIMD, 39 unconstrained
    const int pw = 8;
    const int64_t total = num_rois * ((channels + 2 * pw - 1) / (2 * pw));
    const dim3 g1((unsigned)(8 * ((total + 7) / 8)));
    if (variant == 49)
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<8, kPairHalf, 1, 2, 0, false, true, 5, false>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
    else
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<8, kPairHalf, 1, 2, 0, false, true, 1, false>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else if (variant >= 46 && variant <= 48) {  // single slab buffer: 46 16 pairs, 47 8 pairs, 48 = 46 stamped
    const int pw = variant == 47 ? 8 : 16;
    const int64_t total = num_rois * ((channels + 2 * pw - 1) / (2 * pw));
    const dim3 g1((unsigned)(8 * ((total + 7) / 8)));
    if (variant == 46)
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<16, kPairHalf, 1, 2, 0, false, true>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
    else if (variant == 47)
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<8, kPairHalf, 1, 2, 0, false, true>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
    else
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<16, kPairHalf, 1, 2, 0, true, true>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else if (variant == 44 || variant == 45) {  // stamped timing builds of variants 40 / 23 (8 int64 per item after out)
    const int pw = variant == 44 ? 16 : 8;
    const int64_t total = num_rois * ((channels + 2 * pw - 1) / (2 * pw));
    const dim3 g1((unsigned)(8 * ((total + 7) / 8)));
    if (variant == 44)
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<16, kPairHalf, 1, 2, 0, true>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
    else
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<8, kPairHalf, 1, 2, 0, true>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else if (variant == 40 || variant == 41) {  // chunk-major pairs, nt stores, 16 / 32 pairs per wave
    const int pw = variant == 40 ? 16 : 32;
    const int64_t total = num_rois * ((channels + 2 * pw - 1) / (2 * pw));
    const dim3 g1((unsigned)(8 * ((total + 7) / 8)));
    if (variant == 40)
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<16, kPairHalf, 1, 2, 0>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
    else
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<32, kPairHalf, 1, 2, 0>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else if (variant == 27 || variant == 28) {  // chunk-major pairs at 4 / 16 pairs per wave
    const int pw = variant == 27 ? 4 : 16;
    const int64_t total = num_rois * ((channels + 2 * pw - 1) / (2 * pw));
    const dim3 g1((unsigned)(8 * ((total + 7) / 8)));
    if (variant == 27)
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<4, kPairHalf, 1>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
    else
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<16, kPairHalf, 1>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else if (variant >= 22 && variant <= 24) {  // chunk-major pairs, cache policy: 22 sc1 stores, 23 nt stores, 24 nt loads
    const int64_t total = num_rois * ((channels + 2 * kPairWave - 1) / (2 * kPairWave));
    const dim3 g1((unsigned)(8 * ((total + 7) / 8)));
    if (variant == 22)
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<kPairWave, kPairHalf, 1, 16, 0>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
    else if (variant == 23)
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<kPairWave, kPairHalf, 1, 2, 0>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
    else
      hipLaunchKernelGGL((roi_align_fwd_pair_kernel<kPairWave, kPairHalf, 1, 0, 2>), g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else if (variant == 25 || variant == 26) {  // 26: registers for 3 waves per SIMD (spills)
    const int G = (channels + 2 * kStrPairs - 1) / (2 * kStrPairs);
    const int64_t nitems = num_rois * G;
    if (variant == 25)
      hipLaunchKernelGGL(roi_align_fwd_stream_kernel<0>,
                         dim3((unsigned)std::min<int64_t>(nitems, stream_grid_waves<0>())), dim3(kWave), 0,
                         as_stream(stream), lv, c, out, nitems, G);
    else
      hipLaunchKernelGGL(roi_align_fwd_stream_kernel<3>,
                         dim3((unsigned)std::min<int64_t>(nitems, stream_grid_waves<3>())), dim3(kWave), 0,
                         as_stream(stream), lv, c, out, nitems, G);
  } else if (variant >= 30 && variant <= 37) {  // diagnostics: 31 / 32 skip large / small windows, 33 no stores, 34 no evaluation
    if (variant == 30)
      hipLaunchKernelGGL(roi_align_fwd_x4_kernel<0>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else if (variant == 36)
      hipLaunchKernelGGL((roi_align_fwd_x4_kernel<0, false, 8>), grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else if (variant == 37)
      hipLaunchKernelGGL((roi_align_fwd_x4_kernel<0, false, 6>), grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else if (variant == 35)
      hipLaunchKernelGGL((roi_align_fwd_x4_kernel<0, true>), grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else if (variant == 33)
      hipLaunchKernelGGL(roi_align_fwd_x4_kernel<3>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else if (variant == 34)
      hipLaunchKernelGGL(roi_align_fwd_x4_kernel<4>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else if (variant == 31)
      hipLaunchKernelGGL(roi_align_fwd_x4_kernel<2>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else
      hipLaunchKernelGGL(roi_align_fwd_x4_kernel<1>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  } else if (variant >= 9 && variant <= 19) {
    if (variant == 10)
      hipLaunchKernelGGL(roi_align_fwd_lds_kernel<256>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else if (variant == 15)  // occupancy: registers for 8 waves per SIMD
      hipLaunchKernelGGL((roi_align_fwd_lds_kernel<256, kRoiChanChunk, 8>), grid, dim3(kRoiThreads), 0,
                         as_stream(stream), lv, c, out);
    else if (variant == 16)  // occupancy: registers for 6 waves per SIMD
      hipLaunchKernelGGL((roi_align_fwd_lds_kernel<256, kRoiChanChunk, 6>), grid, dim3(kRoiThreads), 0,
                         as_stream(stream), lv, c, out);
    else if (variant == 11)
      hipLaunchKernelGGL(roi_align_fwd_lds_kernel<512>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else if (variant == 17)
      hipLaunchKernelGGL((roi_align_fwd_lds_kernel<256, 128>), dim3((unsigned)num_rois, (unsigned)((channels + 127) / 128)),
                         dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else if (variant == 18)
      hipLaunchKernelGGL((roi_align_fwd_lds_kernel<256, 256>), dim3((unsigned)num_rois, (unsigned)((channels + 255) / 256)),
                         dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else if (variant == 19)
      hipLaunchKernelGGL((roi_align_fwd_lds_kernel<1024, 256>), dim3((unsigned)num_rois, (unsigned)((channels + 255) / 256)),
                         dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else if (variant == 9)
      hipLaunchKernelGGL((roi_align_fwd_lds_kernel<1024, 128>), dim3((unsigned)num_rois, (unsigned)((channels + 127) / 128)),
                         dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
    else
      hipLaunchKernelGGL(roi_align_fwd_lds_kernel<1024>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  } else {
    hipLaunchKernelGGL(roi_align_fwd_kernel, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  }
  return check_launch("frh_roi_align_fwd_variant");
}

// Backward into a channels-last gradient with 64-B atomic segments (measured slower
// than the product's separable kernel).
extern "C" int32_t frh_roi_align_bwd_cl(int32_t num_levels, float* const* grad_feats, const int32_t* feat_hw,
                                        const int64_t* strides, const float* scales, int32_t batch, int32_t channels,
                                        const float* rois, const int64_t* roi_levels, int64_t num_rois,
                                        int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio, int32_t aligned,
                                        const float* grad_out, void* stream) {
  int32_t r = roi_common_checks(batch, channels, num_rois, pooled_h, pooled_w, rois);
  if (r) return r;
  RoiLevels lv;
  r = make_levels(num_levels, nullptr, grad_feats, feat_hw, strides, scales, &lv);
  if (r) return r;
  if (num_rois == 0) return FRH_OK;
  bool cl = sampling_ratio == 2 && pooled_h * pooled_w <= 64 && channels % kClChans == 0;
  for (int l = 0; l < lv.L; ++l) cl = cl && lv.sc[l] == 1 && lv.w[l] <= kClBandCells;
  FRH_REQUIRE(cl, "channels-last backward needs sampling 2, <= 64 bins, C %% 16 == 0, unit channel stride");
  RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned};
  const dim3 grid((unsigned)num_rois, (unsigned)((channels + kRoiChanChunk - 1) / kRoiChanChunk));
  hipLaunchKernelGGL(roi_align_bwd_cl_kernel, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, grad_out);
  return check_launch("frh_roi_align_bwd_cl");
}

extern "C" size_t frh_roi_align_workspace(int64_t num_rois) {
  if (num_rois <= 0 || num_rois > kPlanMaxRois) return 0;
  return ((size_t)num_rois + group_bound(num_rois) + 2) * sizeof(int32_t);
}

extern "C" int32_t frh_roi_align_fwd_ws(int32_t num_levels, const float* const* feats, const int32_t* feat_hw,
                                        const int64_t* strides, const float* scales, int32_t batch, int32_t channels,
                                        const float* rois, const int64_t* roi_levels, int64_t num_rois,
                                        int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio, int32_t aligned,
                                        float* out, void* workspace, size_t ws_bytes, void* stream) {
  return frh_roi_align_fwd_variant(-2, num_levels, feats, feat_hw, strides, scales, batch, channels, rois,
                                   roi_levels, num_rois, pooled_h, pooled_w, sampling_ratio, aligned, out, workspace,
                                   ws_bytes, stream);
}

static TileMap tile_map(int32_t L, const int32_t* feat_hw, int32_t batch, int64_t* max_tiles) {
  TileMap tm{};
  tm.B = batch;
  tm.base[0] = 0;
  *max_tiles = 1;
  for (int l = 0; l < L; ++l) {
    tm.nty[l] = (feat_hw[2 * l] + kBwdTile - 1) / kBwdTile;
    tm.ntx[l] = (feat_hw[2 * l + 1] + kBwdTile - 1) / kBwdTile;
    tm.base[l + 1] = tm.base[l] + (int64_t)batch * tm.nty[l] * tm.ntx[l];
    *max_tiles = std::max<int64_t>(*max_tiles, (int64_t)tm.nty[l] * tm.ntx[l]);
  }
  return tm;
}

struct BwdLayout {
  size_t count, off, fill, win, list, total;
  int64_t cap;
};

static BwdLayout bwd_layout(int32_t L, const int32_t* feat_hw, int32_t batch, int64_t num_rois) {
  int64_t mt;
  const TileMap tm = tile_map(L, feat_hw, batch, &mt);
  const int64_t T = tm.base[L];
  auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
  BwdLayout z;
  z.cap = num_rois * mt;
  z.count = 0;
  z.off = z.count + al(T * 4);
  z.fill = z.off + al((T + 1) * 4);
  z.win = z.fill + al(T * 4);
  z.list = z.win + al(num_rois * 16);
  z.total = z.list + al(z.cap * 4);
  return z;
}

extern "C" size_t frh_roi_align_bwd_workspace(int32_t num_levels, const int32_t* feat_hw, int32_t batch,
                                              int64_t num_rois) {
  if (num_levels < 1 || num_levels > FRH_MAX_LEVELS || !feat_hw || batch < 1 || num_rois < 0) return 0;
  return bwd_layout(num_levels, feat_hw, batch, num_rois).total;
}

extern "C" int32_t frh_roi_align_bwd_tiled(int32_t num_levels, float* const* grad_feats, const int32_t* feat_hw,
                                           const int64_t* strides, const float* scales, int32_t batch,
                                           int32_t channels, const float* rois, const int64_t* roi_levels,
                                           int64_t num_rois, int32_t pooled_h, int32_t pooled_w,
                                           int32_t sampling_ratio, int32_t aligned, const float* grad_out,
                                           void* workspace, size_t ws_bytes, void* stream) {
  int32_t r = roi_common_checks(batch, channels, num_rois, pooled_h, pooled_w, rois);
  if (r) return r;
  FRH_REQUIRE(sampling_ratio == 2 && pooled_h * pooled_w <= kWave, "tiled backward needs sampling_ratio 2 and "
              "pooled_h * pooled_w <= 64 (got %d, %dx%d)", sampling_ratio, pooled_h, pooled_w);
  RoiLevels lv;
  r = make_levels(num_levels, nullptr, grad_feats, feat_hw, strides, scales, &lv);
  if (r) return r;
  FRH_REQUIRE(grad_feats && (grad_out || num_rois == 0), "null pointer argument");
  const BwdLayout z = bwd_layout(num_levels, feat_hw, batch, num_rois);
  FRH_REQUIRE(workspace && ws_bytes >= z.total, "workspace too small (%zu < %zu)", ws_bytes, z.total);
  int64_t mt;
  const TileMap tm = tile_map(num_levels, feat_hw, batch, &mt);
  const int64_t T = tm.base[num_levels];
  char* ws = static_cast<char*>(workspace);
  TileLists tl{reinterpret_cast<uint32_t*>(ws + z.count), reinterpret_cast<uint32_t*>(ws + z.off),
               reinterpret_cast<uint32_t*>(ws + z.fill), reinterpret_cast<int4*>(ws + z.win),
               reinterpret_cast<int32_t*>(ws + z.list), z.cap};
  hipStream_t st = as_stream(stream);
  RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned};
  FRH_HIP(hipMemsetAsync(ws + z.count, 0, z.off - z.count, st));
  FRH_HIP(hipMemsetAsync(ws + z.fill, 0, z.win - z.fill, st));
  if (num_rois > 0) {
    const unsigned nb = (unsigned)((num_rois + 255) / 256);
    hipLaunchKernelGGL(roi_bwd_bin_count_kernel, dim3(nb), dim3(256), 0, st, lv, c, tm, tl);
  }
  hipLaunchKernelGGL(roi_bwd_bin_scan_kernel, dim3(1), dim3(1024), 0, st, tl, T);
  if (num_rois > 0) {
    const unsigned nb = (unsigned)((num_rois + 255) / 256);
    hipLaunchKernelGGL(roi_bwd_bin_fill_kernel, dim3(nb), dim3(256), 0, st, lv, c, tm, tl);
  }
  dim3 grid((unsigned)T, (unsigned)((channels + kBwdTileChans - 1) / kBwdTileChans));
  hipLaunchKernelGGL(roi_align_bwd_tile_kernel, grid, dim3(kRoiThreads), 0, st, lv, c, tm, tl, grad_out);
  return check_launch("frh_roi_align_bwd_tiled");
}

// dense-layout convenience entry points (header): layout 0 = NCHW, 1 = NHWC
