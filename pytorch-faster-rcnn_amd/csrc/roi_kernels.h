// RoIAlign kernels shared by the product library (csrc/roi_align.hip) and the
// tools-only variant library (tools/csrc/roi_variants.hip).  See roi_align.hip.
#pragma once
#include <math.h>
#include <stdlib.h>

#include <algorithm>

#include <type_traits>

#include "roi_common.h"

namespace frh {

constexpr int kRoiThreads = 256;
constexpr int kRoiChanChunk = 64;
constexpr int kMaxSamplesPerDim = 1024;

// true when the separable tables fit in LDS (always for fixed sampling ratios;
// adaptive grids on huge RoIs fall back to computing taps per sample)
__device__ __forceinline__ bool taps_fit(const RoiGeom& g, const RoiCfg& c) {
  return c.ph * g.gh <= kMaxSamplesPerDim && c.pw * g.gw <= kMaxSamplesPerDim;
}

__device__ __forceinline__ void fill_taps(const RoiGeom& g, const RoiCfg& c, int H, int W, Tap* ty, Tap* tx) {
  if (!taps_fit(g, c)) return;
  const int ny = c.ph * g.gh, nx = c.pw * g.gw;
  for (int e = threadIdx.x; e < ny + nx; e += blockDim.x) {
    if (e < ny) {
      int p = e / g.gh, i = e - p * g.gh;
      ty[e] = make_tap(sample_y(g, p, i), H);
    } else {
      int q = e - ny;
      int p = q / g.gw, i = q - p * g.gw;
      tx[q] = make_tap(sample_x(g, p, i), W);
    }
  }
}

static __global__ void __launch_bounds__(kRoiThreads) roi_align_fwd_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out) {
  __shared__ Tap ty[kMaxSamplesPerDim], tx[kMaxSamplesPerDim];
  const int64_t k = blockIdx.x;
  const int c0 = blockIdx.y * kRoiChanChunk;
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  fill_taps(g, c, H, W, ty, tx);
  __syncthreads();
  const int nbins = c.ph * c.pw;
  const int nch = min(kRoiChanChunk, c.C - c0);
  const bool tab = taps_fit(g, c);
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l];
  const int64_t sy = lv.sy[l], sx = lv.sx[l], scs = lv.sc[l];
  float* o = out + (k * c.C + c0) * nbins;
  for (int item = threadIdx.x; item < nch * nbins; item += blockDim.x) {
    const int cl = item / nbins, bin = item - cl * nbins;
    const int py = bin / c.pw, px = bin - py * c.pw;
    const float* f = base + (int64_t)(c0 + cl) * scs;
    float acc = 0.0f;
    for (int iy = 0; iy < g.gh; ++iy) {
      const Tap a = tab ? ty[py * g.gh + iy] : make_tap(sample_y(g, py, iy), H);
      for (int ix = 0; ix < g.gw; ++ix) {
        const Tap bx = tab ? tx[px * g.gw + ix] : make_tap(sample_x(g, px, ix), W);
        float val = 0.0f;
        if (a.valid && bx.valid) {
          float w1 = a.h * bx.h, w2 = a.h * bx.l, w3 = a.l * bx.h, w4 = a.l * bx.l;
          float v1 = f[a.lo * sy + bx.lo * sx], v2 = f[a.lo * sy + bx.hi * sx];
          float v3 = f[a.hi * sy + bx.lo * sx], v4 = f[a.hi * sy + bx.hi * sx];
          val = ((w1 * v1 + w2 * v2) + w3 * v3) + w4 * v4;
        }
        acc = acc + val;
      }
    }
    o[item] = acc / g.count;
  }
}


// Buffer-descriptor variant (sampling ratio 2, ph*pw <= 256; the default).
// Lane (bin, channel group cg) keeps its bin's 16 tap offsets in VGPRs as
// 32-bit byte offsets into a descriptor over this (image, level, channel
// chunk) slice; the channel walk moves only the wave-uniform soffset, so the
// loop carries no per-lane address arithmetic.  When every x-sample of the
// wave has x_hi = x_lo + 1 (all but right-border clamped samples) the taps of
// a sample row are one 8-byte load: 8 loads per (bin, channel) instead of 16.
// The 1/count of SR=2 is an exact power of two, so acc * 0.25 == acc / 4.
// Results identical to the direct kernel.
template <int U>
__device__ __forceinline__ void fwd_buf_block(const RoiLevels& lv, const RoiCfg& c, float* __restrict__ out,
                                              int64_t k, int c0, const RoiGeom& g) {
  constexpr int SR = 2;
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw;
  const int groups = kRoiThreads / nbins;
  const int t = threadIdx.x;
  if (t >= groups * nbins) return;
  const int bin = t % nbins, cg = t / nbins;
  const int py = bin / c.pw, px = bin - py * c.pw;
  Tap ty[SR], tx[SR];
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    ty[i] = make_tap(sample_y(g, py, i), H);
    tx[i] = make_tap(sample_x(g, px, i), W);
  }
  const int sy = (int)lv.sy[l], sx = (int)lv.sx[l], scs = (int)lv.sc[l];
  const int nch = min(kRoiChanChunk, c.C - c0);
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l] + (int64_t)c0 * scs;
  const int64_t extent = ((int64_t)(nch - 1) * scs + (int64_t)(H - 1) * sy + (int64_t)(W - 1) * sx + 1) * 4;
  const __amdgpu_buffer_rsrc_t fr = uniform_rsrc(base, extent);
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + (k * c.C + c0) * nbins, (int64_t)nch * nbins * 4);
  const int cstep = groups * scs * 4, ostep = groups * nbins * 4;
  bool ok[SR][SR];
  float wt[SR][SR][4];
  int row[SR][2], col[SR][2];
  bool pair = sx == 1;
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    row[i][0] = (cg * scs + (ty[i].valid ? ty[i].lo * sy : 0)) * 4;
    row[i][1] = (cg * scs + (ty[i].valid ? ty[i].hi * sy : 0)) * 4;
    col[i][0] = tx[i].valid ? tx[i].lo * sx * 4 : 0;
    col[i][1] = tx[i].valid ? tx[i].hi * sx * 4 : 0;
    pair = pair && (!tx[i].valid || tx[i].hi == tx[i].lo + 1);
  }
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
  auto bin_value = [&](const float (&v)[SR][SR][4]) {
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
  // wave-uniform trip counts (soffset must stay scalar): every lane has a
  // channel in the first nch / groups steps, the tail step is lane-guarded
  const int full = nch / groups, iters = (nch + groups - 1) / groups;
  const bool tail_ok = cg + full * groups < nch;
  if (__all(pair)) {
    int off[SR][2][SR];
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) off[iy][r][ix] = row[iy][r] + col[ix][0];
    int it = 0;
    for (; it + U <= full; it += U) {
      u32x2 rv[U][SR][2][SR];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int iy = 0; iy < SR; ++iy)
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int ix = 0; ix < SR; ++ix)
              rv[u][iy][r][ix] = __builtin_amdgcn_raw_buffer_load_b64(fr, off[iy][r][ix], (it + u) * cstep, 0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float v[SR][SR][4];
#pragma unroll
        for (int iy = 0; iy < SR; ++iy)
#pragma unroll
          for (int ix = 0; ix < SR; ++ix) {
            v[iy][ix][0] = __uint_as_float(rv[u][iy][0][ix].x);
            v[iy][ix][1] = __uint_as_float(rv[u][iy][0][ix].y);
            v[iy][ix][2] = __uint_as_float(rv[u][iy][1][ix].x);
            v[iy][ix][3] = __uint_as_float(rv[u][iy][1][ix].y);
          }
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bin_value(v)), orr, t * 4, (it + u) * ostep, 0);
      }
    }
    for (; it < iters; ++it) {
      if (it == full && !tail_ok) break;
      float v[SR][SR][4];
#pragma unroll
      for (int iy = 0; iy < SR; ++iy)
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) {
          const u32x2 a = __builtin_amdgcn_raw_buffer_load_b64(fr, off[iy][0][ix], it * cstep, 0);
          const u32x2 b = __builtin_amdgcn_raw_buffer_load_b64(fr, off[iy][1][ix], it * cstep, 0);
          v[iy][ix][0] = __uint_as_float(a.x);
          v[iy][ix][1] = __uint_as_float(a.y);
          v[iy][ix][2] = __uint_as_float(b.x);
          v[iy][ix][3] = __uint_as_float(b.y);
        }
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bin_value(v)), orr, t * 4, it * ostep, 0);
    }
  } else {
    for (int it = 0; it < iters; ++it) {
      if (it == full && !tail_ok) break;
      float v[SR][SR][4];
#pragma unroll
      for (int iy = 0; iy < SR; ++iy)
#pragma unroll
        for (int ix = 0; ix < SR; ++ix)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            v[iy][ix][q] = __uint_as_float(
                __builtin_amdgcn_raw_buffer_load_b32(fr, row[iy][q >> 1] + col[ix][q & 1], it * cstep, 0));
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bin_value(v)), orr, t * 4, it * ostep, 0);
    }
  }
}


// Wave-staged variant (sampling ratio 2, ph*pw <= 64, 2*ph and 2*pw <= 64).
// Every tap of a RoI lies in the window [y0, y1] x [x0, x1] of its level;
// after FPN level mapping that window is a few to ~30 cells per side.  Each
// wave owns 16 channels of the RoI and, per channel, copies the window into
// its own LDS slab with lane-contiguous loads (every feature line fetched
// once per RoI-channel, instead of 8 gathers per bin hitting the same lines),
// then lane = bin reads its 16 taps from LDS.  The loads of channel i+1 are
// in flight while channel i is evaluated.  The slab row has one extra column
// holding a copy of the window's last feature column, so a right-border
// clamped tap (x_lo = x_hi = W-1) reads (x_lo, x_lo + 1) like every other
// sample.  No block barriers: waves are independent.  Windows above
// kWinMax floats take the per-wave gather path.  Results identical to the
// direct kernel.
constexpr int kWinMax = 1024;
constexpr int kWinR = kWinMax / kWave;

// kChunk: channels per workgroup (kChunk / 4 per wave).
// kWpe: minimum waves per SIMD the register allocation must allow (0: compiler's choice).
template <int kStageMax, int kChunk = kRoiChanChunk, int kWpe = 0>
__global__ void __launch_bounds__(kRoiThreads) __attribute__((amdgpu_waves_per_eu(kWpe > 0 ? kWpe : 1)))
roi_align_fwd_lds_kernel(RoiLevels lv, RoiCfg c,
                                                                        float* __restrict__ out) {
  constexpr int SR = 2;
  __shared__ float slab_all[kRoiThreads / kWave][kWinMax];
  const int64_t k = blockIdx.x;
  // readfirstlane: the wave index is uniform, and the compiler must know it (soffset operands)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
  constexpr int kWC = kChunk / (kRoiThreads / kWave);
  const int cw0 = blockIdx.y * kChunk + wave * kWC;
  const int nch = min(kWC, c.C - cw0);
  float* slab = slab_all[wave];
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw;
  const int sy = (int)lv.sy[l], sx = (int)lv.sx[l], scs = (int)lv.sc[l];
  // window of the valid taps: lane i evaluates y sample i and x sample i
  int ylo = 1 << 30, yhi = -1, xlo = 1 << 30, xhi = -1;
  if (lane < c.ph * SR) {
    const Tap t = make_tap(sample_y(g, lane / SR, lane % SR), H);
    if (t.valid) ylo = t.lo, yhi = t.hi;
  }
  if (lane < c.pw * SR) {
    const Tap t = make_tap(sample_x(g, lane / SR, lane % SR), W);
    if (t.valid) xlo = t.lo, xhi = t.hi;
  }
  const int y0 = __builtin_amdgcn_readfirstlane(wave_min_i32(ylo)), y1 = __builtin_amdgcn_readfirstlane(wave_max_i32(yhi));
  const int x0 = __builtin_amdgcn_readfirstlane(wave_min_i32(xlo)), x1 = __builtin_amdgcn_readfirstlane(wave_max_i32(xhi));
  const bool any = y1 >= y0 && x1 >= x0;
  // odd slab row stride: the 4 tap rows of a wave's bins spread over the LDS banks
  const int ws = (x1 - x0 + 2) | 1, n = any ? (y1 - y0 + 1) * ws : 0;
  if (n > kStageMax) {  // uniform over the block (one RoI): large windows take the block gather path
    for (int cc = 0; cc < kChunk && blockIdx.y * kChunk + cc < c.C; cc += kRoiChanChunk)
      fwd_buf_block<2>(lv, c, out, k, blockIdx.y * kChunk + cc, g);
    return;
  }
  if (nch <= 0) return;
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l] + (int64_t)cw0 * scs;
  const int64_t extent = ((int64_t)(nch - 1) * scs + (int64_t)(H - 1) * sy + (int64_t)(W - 1) * sx + 1) * 4;
  const __amdgpu_buffer_rsrc_t fr = uniform_rsrc(base, extent);
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + (k * c.C + cw0) * nbins, (int64_t)nch * nbins * 4);
  const int cstep = scs * 4, ostep = nbins * 4;
  // this lane's bin: taps, weights, validity
  const int bin = lane < nbins ? lane : 0;
  const int py = bin / c.pw, px = bin - py * c.pw;
  Tap ty[SR], tx[SR];
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    ty[i] = make_tap(sample_y(g, py, i), H);
    tx[i] = make_tap(sample_x(g, px, i), W);
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
  auto bin_value = [&](const float (&v)[SR][SR][4]) {
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
  const bool active = lane < nbins;
  if (n <= kStageMax) {
    // slab addresses of this bin's sample rows (x_lo, x_lo + 1 pairs)
    int sa[SR][2][SR];
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        const bool v = ok[iy][ix];
        sa[iy][0][ix] = v ? (ty[iy].lo - y0) * ws + (tx[ix].lo - x0) : 0;
        sa[iy][1][ix] = v ? (ty[iy].hi - y0) * ws + (tx[ix].lo - x0) : 0;
      }
    // staging: slab element e = lane + 64 j  <-  feature (y0 + e / ws, min(x0 + e % ws, W - 1));
    // the j loop is specialised on RB = 64-element rounds (1, 2, 4, 8, 16) so it unrolls branch-free
    auto run = [&](auto rb) {
      constexpr int RB = decltype(rb)::value, D = kWinR / RB;  // D channel windows per round, 16 loads/lane
      int goff[RB];
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        const int e = lane + j * kWave;
        const int r = e / ws, cc = e - r * ws;
        // lanes past the window re-read its first element: no extra cache line per round
        goff[j] = e < n ? ((y0 + r) * sy + min(x0 + cc, W - 1) * sx) * 4 : (y0 * sy + x0 * sx) * 4;
      }
      float st[D][RB];
      auto issue = [&](int c0r) {
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
          for (int j = 0; j < RB; ++j)
            st[d][j] = __uint_as_float(
                __builtin_amdgcn_raw_buffer_load_b32(fr, goff[j], min(c0r + d, nch - 1) * cstep, 0));
      };
      issue(0);
      for (int i = 0; i < nch; i += D) {
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
          for (int j = 0; j < RB; ++j) slab[(d * RB + j) * kWave + lane] = st[d][j];  // [n, 64 RB) junk, unread
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (i + D < nch) issue(i + D);
        if (active) {
#pragma unroll
          for (int d = 0; d < D; ++d) {
            if (i + d < nch) {
              const float* sl = slab + d * RB * kWave;
              float v[SR][SR][4];
#pragma unroll
              for (int iy = 0; iy < SR; ++iy)
#pragma unroll
                for (int ix = 0; ix < SR; ++ix) {
                  v[iy][ix][0] = sl[sa[iy][0][ix]];
                  v[iy][ix][1] = sl[sa[iy][0][ix] + 1];
                  v[iy][ix][2] = sl[sa[iy][1][ix]];
                  v[iy][ix][3] = sl[sa[iy][1][ix] + 1];
                }
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bin_value(v)), orr, lane * 4, (i + d) * ostep, 0);
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    };
    const int R = (n + kWave - 1) / kWave;
    if (R <= 1)
      run(std::integral_constant<int, 1>{});
    else if (R <= 2 || kStageMax <= 2 * kWave)
      run(std::integral_constant<int, 2>{});
    else if (R <= 4 || kStageMax <= 4 * kWave)
      run(std::integral_constant<int, 4>{});
    else if (R <= 8 || kStageMax <= 8 * kWave)
      run(std::integral_constant<int, 8>{});
    else
      run(std::integral_constant<int, kWinR>{});
  }
}


// ---------------------------------------------------------------------------
// Channel-pair forward (the default).  One wave per (RoI, 16 channels = 8 channel
// pairs), lane = bin.  The RoI's tap grid is staged into the wave's LDS slab by 4-B
// LDS-DMA with the two channels of a pair interleaved ([cell][2]), so every tap of a
// bin is ONE aligned ds_read_b64 and the bilinear sums run as packed f32
// (v_pk_mul_f32 / v_pk_add_f32) on both channels at once.  Each slab dimension is
// either the dense tap window [y0, y1] (at most 4*ph rows) or the list of the 2*ph
// samples' (lo, hi) taps, so every RoI fits (<= 28 x 29 cells at 7x7) and large RoIs
// need no per-bin gather.  A DMA round moves 32 consecutive cells of one pair.  ONE
// slab buffer of kPairHalf dwords per wave (6.5 KB: 20 resident waves per CU, the
// register count's cap); a stage is the D pairs (D = 8, 4, 2, 1, as the cell count
// allows) it holds; the tap reads of half-sample-row h+1 are in flight while h is
// summed.  Lean tap state: per-sample weight factors and tap bases, the 16 weights
// and addresses rebuilt per half-row behind an opaque copy (95 VGPRs).
// Invalid samples have zero weights and read cell 0 (finite features: +0, the
// reference's own 0 * feature term).  Same operation order as torchvision:
// bit-identical to the other kernels.
//
// The per-wave prologue (RoI geometry, tap window, per-bin tap state) is the same for
// the 16 channel chunks of a RoI and is still recomputed by each: loading it from a
// per-RoI descriptor written by a first launch measured slower (under
// this kernel's memory load the descriptor's loads take longer than the ~450
// instructions they replace).
constexpr int kPairWave = 8;                    // channel pairs per wave (= workgroup): 16 channels
constexpr int kPairHalf = 1664;                 // dwords per slab buffer (6.5 KB)
constexpr int kPairChunk = 2 * kPairWave;       // channels per workgroup

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// ds_read_b64 by hand: the compiler would pair two of them into ds_read2_b64,
// which runs at half the rate (8 LDS cycles instead of 2 x 2, MI355X_MICROARCH
// §LDS).  The caller waits with lds_wait<N>, which also orders the values.
template <int OFF>
__device__ __forceinline__ f32x2 lds_read_b64(uint32_t addr) {
  f32x2 v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void lds_wait(f32x2 (&v)[8]) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
               : "i"(N)
               : "memory");
}

template <int D, int kHalf = kPairHalf>
struct PairLayout {
  static constexpr int RS = (kHalf / D) / kWave * kWave;  // dwords per pair region
  static constexpr int RP = RS / kWave;                       // DMA rounds per pair
  static constexpr int kCells = RS / 2;
  static_assert(D * RP + 2 * D < 64, "vmcnt is 6 bits");
};

// The RoI's wave-uniform slab geometry and the feature plane it reads.
struct PairGeom {
  int empty;             // no valid sample: every bin is 0
  int y0, x0, R, Cs, Cs2;
  int dy, dx;            // dense window rows / columns (else the sample tap lists)
  int sy, sx, scs;       // feature element strides (row, column, channel)
  uint32_t inv;          // e / Cs2 == (e * inv) >> 16 for e < 1024
  uint32_t extent;       // feature bytes addressable from base
  const float* base;     // image b of the RoI's level
};

// This lane's share: the slab-row / column source offsets of its tap-list entries and
// its bin's lean tap state (tap bases relative to the slab start).
struct PairLane {
  int rsrc, csrc;
  float fyh[2], fyl[2], fxh[2], fxl[2];
  uint32_t tb0[2][2], tdq[2], tdr[2];
  int rlo, rhi;  // slab rows of the bin's valid samples (INT_MAX / -1: none, or an idle lane)
  uint32_t vmask;  // bit 2 iy + ix: sample (iy, ix) valid (tb0 meaningful)
};

// kUnit: bytes of one cell's entry in a slab region (8: a channel pair; 16: a quad).
template <int kUnit = 8>
__device__ __forceinline__ void pair_setup(const RoiLevels& lv, const RoiCfg& c, const RoiRaw& raw, int lane,
                                           PairGeom& G, PairLane& P) {
  constexpr int SR = 2;
  const RoiGeom g = roi_geom_raw(c, lv, raw);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw;
  G.sy = (int)lv.sy[l];
  G.sx = (int)lv.sx[l];
  G.scs = (int)lv.sc[l];
  // sample positions (sampling ratio 2: the reference's "/ 2" is an exact halving)
  auto pos_y = [&](int p, int i) { return g.start_h + (float)p * g.bin_h + ((float)i + 0.5f) * g.bin_h * 0.5f; };
  auto pos_x = [&](int p, int i) { return g.start_w + (float)p * g.bin_w + ((float)i + 0.5f) * g.bin_w * 0.5f; };
  const int nly = 2 * SR * c.ph, nlx = 2 * SR * c.pw;  // tap lists: entry i = tap (i & 1 ? hi : lo) of sample i / 2
  int yrow = -1, xcol = -1, ylo = 1 << 30, yhi = -1, xlo = 1 << 30, xhi = -1;
  if (lane < nly) {
    const int s = lane >> 1;
    const Tap t = make_tap(pos_y(s >> 1, s & 1), H);
    if (t.valid) yrow = (lane & 1) ? t.hi : t.lo, ylo = t.lo, yhi = t.hi;
  }
  if (lane < nlx) {
    const int s = lane >> 1;
    const Tap t = make_tap(pos_x(s >> 1, s & 1), W);
    if (t.valid) xcol = (lane & 1) ? t.hi : t.lo, xlo = t.lo, xhi = t.hi;
  }
  const int y0 = __builtin_amdgcn_readfirstlane(wave_min_i32(ylo)), y1 = __builtin_amdgcn_readfirstlane(wave_max_i32(yhi));
  const int x0 = __builtin_amdgcn_readfirstlane(wave_min_i32(xlo)), x1 = __builtin_amdgcn_readfirstlane(wave_max_i32(xhi));
  G.empty = !(y1 >= y0 && x1 >= x0);
  G.y0 = y0;
  G.x0 = x0;
  const bool dy = y1 - y0 + 1 <= nly, dx = x1 - x0 + 1 <= nlx;
  G.dy = dy;
  G.dx = dx;
  G.R = dy ? y1 - y0 + 1 : nly;
  G.Cs = dx ? x1 - x0 + 1 : nlx;
  // slab row stride: odd, so the tap reads of a wave spread over the banks
  G.Cs2 = G.Cs | 1;
  // feature byte offsets of slab row / column `lane`
  P.rsrc = (dy ? y0 + min(lane, G.R - 1) : (yrow >= 0 ? yrow : y0)) * G.sy * 4;
  P.csrc = (dx ? x0 + min(lane, G.Cs - 1) : (xcol >= 0 ? xcol : x0)) * G.sx * 4;
  // this lane's bin: per-sample factors (zeroed for invalid samples: the same products, or +0)
  // and tap bases + row / column deltas
  const int bin = lane < nbins ? lane : 0;
  const int py = (int)(((uint32_t)bin * ((65536u + (uint32_t)c.pw - 1u) / (uint32_t)c.pw)) >> 16), px = bin - py * c.pw;
  P.rlo = 0x7fffffff;
  P.rhi = -1;
  P.vmask = 0u;
#pragma unroll
  for (int iy = 0; iy < SR; ++iy) {
    const Tap a = make_tap(pos_y(py, iy), H);
    P.fyh[iy] = a.valid ? a.h : 0.f;
    P.fyl[iy] = a.valid ? a.l : 0.f;
    const int r0 = dy ? a.lo - y0 : 2 * (py * SR + iy), r1 = dy ? a.hi - y0 : 2 * (py * SR + iy) + 1;
    if (a.valid && lane < nbins) {
      P.rlo = min(P.rlo, r0);
      P.rhi = max(P.rhi, r1);
    }
    P.tdr[iy] = (uint32_t)kUnit * (uint32_t)((r1 - r0) * G.Cs2);
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap b = make_tap(pos_x(px, ix), W);
      const int q0 = dx ? b.lo - x0 : 2 * (px * SR + ix), q1 = dx ? b.hi - x0 : 2 * (px * SR + ix) + 1;
      if (iy == 0) {
        P.fxh[ix] = b.valid ? b.h : 0.f;
        P.fxl[ix] = b.valid ? b.l : 0.f;
        P.tdq[ix] = (uint32_t)kUnit * (uint32_t)(q1 - q0);
      }
      P.tb0[iy][ix] = (a.valid && b.valid) ? (uint32_t)kUnit * (uint32_t)(r0 * G.Cs2 + q0) : 0u;
      P.vmask |= (a.valid && b.valid) ? 1u << (2 * iy + ix) : 0u;
    }
  }
  G.base = lv.feat[l] + (int64_t)g.b * lv.sb[l];
  G.extent = (uint32_t)(((int64_t)(c.C - 1) * G.scs + (int64_t)(H - 1) * G.sy + (int64_t)(W - 1) * G.sx + 1) * 4);
  G.inv = (65536u + (uint32_t)G.Cs2 - 1u) / (uint32_t)G.Cs2;
}

// One item: RoI k, channel chunk `chunk` (16 channels).  kStAux / kLdAux: cache policy
// of the output stores / staging loads (cdna.h).  kStamp (tools-only timing builds):
// lane 0 writes 8 int64 per item after the output -- s_memrealtime at start / setup
// done / first stage landed / end, D, cells, RoI record landed, XCD.
template <int kStAux, int kLdAux, bool kStamp>
__device__ __forceinline__ void pair_item(const RoiLevels& lv, const RoiCfg& c, float* __restrict__ out, int64_t k,
                                          int chunk, int64_t item, uint32_t sbase, int64_t t_start, int lane) {
  constexpr int SR = 2, kPW = kPairWave, kHalf = kPairHalf;
  int64_t t_setup = 0, t_land = 0, t_fetched = 0;
  const int cw0 = chunk * 2 * kPW;
  const int npairs = min(kPW, (c.C - cw0) / 2);  // host: C even
  const int nbins = c.ph * c.pw;
  PairGeom G;
  PairLane P;
  const RoiRaw raw = roi_fetch(c, k);
  if (kStamp) t_fetched = (int64_t)__builtin_amdgcn_s_memrealtime();
  pair_setup(lv, c, raw, lane, G, P);
  const bool active = lane < nbins;
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + (k * c.C + cw0) * nbins, (int64_t)2 * npairs * nbins * 4);
  const int ovoff = active ? lane * 4 : 0x40000000;  // idle lanes: dropped by the range check
  const int ostep = nbins * 4;
  if (G.empty) {  // no valid sample: all bins 0
    for (int ch = 0; ch < 2 * npairs; ++ch) __builtin_amdgcn_raw_buffer_store_b32(0u, orr, ovoff, ch * ostep, kStAux);
    return;
  }
  const int y0 = G.y0, x0 = G.x0, R = G.R, Cs = G.Cs, Cs2 = G.Cs2, sy = G.sy, sx = G.sx, scs = G.scs;
  const bool dy = G.dy, dx = G.dx;
  const int ncell = R * Cs2;
  const bool small = ncell <= PairLayout<8, kHalf>::kCells;
  const int rsrc = P.rsrc, csrc = P.csrc;
  const __amdgpu_buffer_rsrc_t fr = uniform_rsrc(G.base, (int64_t)G.extent);
  const uint32_t inv = G.inv;
  if (kStamp) t_setup = (int64_t)__builtin_amdgcn_s_memrealtime();
  int stamp_d = 0;

  auto run = [&](auto dd) {
    constexpr int D = decltype(dd)::value, RS = PairLayout<D, kHalf>::RS, RP = PairLayout<D, kHalf>::RP;
    const int nst = (npairs + D - 1) / D;
    // region dword j * 64 + lane of every pair  <-  channel (lane & 1) of cell (j * 64 + lane) / 2
    auto goff_at = [&](int j) {
      int e = (j * kWave + lane) >> 1;
      e = e < ncell ? e : 0;
      const int r = (int)(((uint32_t)e * inv) >> 16), col = min(e - r * Cs2, Cs - 1);
      // dense window: slab cell (r, col) is feature (y0 + r, x0 + col), no lane exchange
      return (dy && dx) ? ((y0 + r) * sy + (x0 + col) * sx + (lane & 1) * scs) * 4
                        : __shfl(rsrc, r, kWave) + __shfl(csrc, col, kWave) + (lane & 1) * scs * 4;
    };
    int goff[RP];
#pragma unroll
    for (int j = 0; j < RP; ++j) goff[j] = goff_at(j);
    auto issue = [&](int s) {  // pairs past the last re-read it (their stores are dropped)
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int soff = (cw0 + 2 * min(s * D + d, npairs - 1)) * scs * 4;
#pragma unroll
        for (int j = 0; j < RP; ++j) lds_dma_at<4, kLdAux>(fr, sbase + 4u * (uint32_t)(d * RS + j * kWave), goff[j], soff);
      }
    };
    auto eval = [&](int s) {
      // half-rows h = 2 d + iy: 8 tap reads each; the reads of h + 1 in flight while h is summed
      f32x2 v[2][8];
      f32x2 acc = {0.0f, 0.0f};
      // the factors pass through an opaque copy per stage, so the products and sums below are
      // computed here and not hoisted out of the stage loop into live registers
      float ly_h[SR], ly_l[SR], lx_h[SR], lx_l[SR];
      uint32_t lb[SR][SR], ldq[SR], ldr[SR];
#pragma unroll
      for (int i = 0; i < SR; ++i) {
        ly_h[i] = P.fyh[i], ly_l[i] = P.fyl[i], lx_h[i] = P.fxh[i], lx_l[i] = P.fxl[i], ldq[i] = P.tdq[i],
        ldr[i] = P.tdr[i];
        asm volatile("" : "+v"(ly_h[i]), "+v"(ly_l[i]), "+v"(lx_h[i]), "+v"(lx_l[i]), "+v"(ldq[i]), "+v"(ldr[i]));
#pragma unroll
        for (int j = 0; j < SR; ++j) {
          lb[i][j] = sbase + P.tb0[i][j];
          asm volatile("" : "+v"(lb[i][j]));
        }
      }
      auto tap = [&](int iy, int ix, int q) -> uint32_t {
        return lb[iy][ix] + ((q & 1) ? ldq[ix] : 0u) + ((q & 2) ? ldr[iy] : 0u);
      };
      auto load = [&](auto hh) {
        constexpr int h = decltype(hh)::value, d = h >> 1, iy = h & 1, OFF = 4 * (d * RS);
#pragma unroll
        for (int ix = 0; ix < SR; ++ix)
#pragma unroll
          for (int q = 0; q < 4; ++q) v[h & 1][ix * 4 + q] = lds_read_b64<OFF>(tap(iy, ix, q));
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
          const float w[4] = {ly_h[iy] * lx_h[ix], ly_h[iy] * lx_l[ix], ly_l[iy] * lx_h[ix], ly_l[iy] * lx_l[ix]};
          const f32x2* x = &v[h & 1][ix * 4];
          const f32x2 val = ((f32x2(w[0]) * x[0] + f32x2(w[1]) * x[1]) + f32x2(w[2]) * x[2]) + f32x2(w[3]) * x[3];
          acc = acc + val;
        }
        if (iy == 1) {
          const f32x2 r = acc * 0.25f;
          const int p = s * D + d;
          const int vo = p < npairs ? ovoff : 0x40000000;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.x), orr, vo, 2 * p * ostep, kStAux);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.y), orr, vo, (2 * p + 1) * ostep, kStAux);
        }
      });
    };
    stamp_d = D;
    for (int s = 0; s < nst; ++s) {
      issue(s);  // the previous stage's tap reads completed (lds_wait<0> + barrier below)
      wait_vmcnt<0>();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (kStamp && s == 0) t_land = (int64_t)__builtin_amdgcn_s_memrealtime();
      eval(s);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  };
  if (small)
    run(std::integral_constant<int, 8>{});
  else if (ncell <= PairLayout<4, kHalf>::kCells)
    run(std::integral_constant<int, 4>{});
  else if (ncell <= PairLayout<2, kHalf>::kCells)
    run(std::integral_constant<int, 2>{});
  else
    run(std::integral_constant<int, 1>{});
  if (kStamp && lane == 0) {
    int64_t* st = reinterpret_cast<int64_t*>(out + c.K * c.C * nbins) + item * 8;
    const int64_t t_end = (int64_t)__builtin_amdgcn_s_memrealtime();
    st[0] = t_start;
    st[1] = t_setup;
    st[2] = t_land;
    st[3] = t_end;
    st[4] = stamp_d;
    st[5] = ncell;
    st[6] = t_fetched;
    st[7] = blockIdx.x & 7;
  }
}

// A 1-D grid of 8 * ceil(K * chunks / 8) single-wave workgroups in which XCD x
// (= linear id % 8) takes the x-th eighth of the chunk-major (chunk, RoI) item list,
// so each XCD's L2 holds the feature planes of its own channel chunks.  32-bit item
// arithmetic (host: K * chunks < 2^31).
template <int kStAux = kCpolNT, bool kStamp = false, bool kSpan = false>
__global__ void __launch_bounds__(kWave) roi_align_fwd_pair_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out) {
  const int64_t t_start = (kStamp || kSpan) ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  __shared__ __attribute__((aligned(16))) float slab[kPairHalf];
  // the slab as an LDS byte address (integer: no generic-pointer casts)
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)slab);
  const uint32_t G = (uint32_t)(c.C + kPairChunk - 1) / (uint32_t)kPairChunk, K32 = (uint32_t)c.K;
  const uint32_t total = K32 * G, per = (total + 7u) / 8u;
  const uint32_t w = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  const uint32_t wend = min((blockIdx.x & 7u) * per + per, total);
  if (w >= wend) return;
  const int ch0 = (int)(w / K32);
  const int64_t k0 = (int64_t)(w - (uint32_t)ch0 * K32);
  pair_item<kStAux, 0, kStamp>(lv, c, out, k0, ch0, w, sbase, t_start, threadIdx.x & (kWave - 1));
  if (kSpan && threadIdx.x == 0) record_span(c, t_start);
}


// ---------------------------------------------------------------------------
// Channel-quad forward for channels-last features (unit channel stride: the FPN's NHWC
// outputs).  The pair kernel's structure -- one wave per (RoI, 16 channels), lane = bin,
// per-bin tap state computed once per item, the RoI's tap cells staged in LDS, packed-f32
// bilinear sums -- with the staging matched to NHWC: slab region d holds channel quad d
// (4 channels = 16 B) of every staged cell, filled by 16-B LDS-DMA (lane = cell: one
// instruction stages 64 cells of a quad; the 4 quads of an item read each cell's 64
// contiguous bytes), and every tap is ONE ds_read_b128 giving 4 channels.  A stage holds
// the D quads (D = 4, 2, 1) whose regions fit the slab.  The slab is 13 KB: 832 cells,
// so the largest tap grid of 7x7 bins at sampling 2 -- 28 rows (a dense window of <= 28
// rows or the 28-entry tap list) by 29 columns (28, rounded up to the odd row stride)
// = 812 cells -- is staged whole (VOC-sized RoIs: about a fifth of them; an 8-KB slab sent
// those to per-lane global gathers, 3.6x slower per launch).  12 slabs per CU = the
// 3 waves per SIMD the kernel's registers are sized for.  Same operation order:
// bit-identical to the other kernels.
constexpr int kQuadWave = 4;     // channel quads per wave (= workgroup): 16 channels
constexpr int kQuadSlab = 3328;  // dwords per slab (13 KB = 13 whole 64-cell DMA rounds of one quad)
constexpr int kQuadChunk = 4 * kQuadWave;

template <int D, int kSlab = kQuadSlab>
struct QuadLayout {
  static constexpr int RS = (kSlab / D) / 256 * 256;  // dwords per quad region: whole 64-cell DMA rounds
  static constexpr int RP = RS / 256;                  // DMA rounds per region
  static constexpr int kCells = RS / 4;
  static_assert(D * RP < 64, "vmcnt is 6 bits");
};

// the largest tap grid of ph x pw bins at sampling 2 (rows x odd row stride): what the
// quad kernel's D = 1 region must hold
constexpr int quad_max_cells(int ph, int pw) { return (4 * ph) * ((4 * pw) | 1); }
static_assert(quad_max_cells(7, 7) <= QuadLayout<1>::kCells, "7x7 tap grids must fit one slab");

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int OFF>
__device__ __forceinline__ f32x4 lds_read_b128(uint32_t addr) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void lds_wait4(f32x4 (&v)[8]) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
               : "i"(N)
               : "memory");
}

// torchvision's per-sample sum for 4 channels: ((w1 v1 + w2 v2) + w3 v3) + w4 v4, as two
// packed halves
__device__ __forceinline__ f32x4 quad_val(const float (&w)[4], const f32x4* x) {
  f32x2 lo = ((f32x2(w[0]) * x[0].xy + f32x2(w[1]) * x[1].xy) + f32x2(w[2]) * x[2].xy) + f32x2(w[3]) * x[3].xy;
  f32x2 hi = ((f32x2(w[0]) * x[0].zw + f32x2(w[1]) * x[1].zw) + f32x2(w[2]) * x[2].zw) + f32x2(w[3]) * x[3].zw;
  return f32x4{lo.x, lo.y, hi.x, hi.y};
}

// kQW: channel quads per item (4: 16 channels).  kOut: 0 = per-channel 4-B stores of the
// bin row (lane = bin), 1 = [channel][bin] staged in LDS (obuf), then 16-B stores of the
// item's contiguous output block, 2 = no stores (tools-only diagnostic).
// kOpt bit 1 (kFwdTrim): lanes past the window's cells load nothing (an out-of-range offset:
// no memory request) and DMA rounds past the window are not issued.
// kOpt bit 4 (kFwdSorted, tools-only experiment): item k reads record k of c.rec (a spatial
// processing order, tools/csrc/roi_lab_kernels.h roi_sort_kernel) and writes the output row the
// record names.
constexpr int kFwdTrim = 1, kFwdIlvRot = 2, kFwdSorted = 4;
template <int kStAux, bool kStamp, int kQW = kQuadWave, int kOut = 0, int kSlab = kQuadSlab, bool kOnly4 = false,
          int kOpt = 0>
__device__ __forceinline__ void quad_body(const PairGeom& G, const PairLane& P, const RoiCfg& c,
                                          float* __restrict__ out, int64_t k, int chunk, int64_t item, uint32_t sbase,
                                          int64_t t_start, int lane, float* obuf);

template <int kStAux, bool kStamp, int kQW = kQuadWave, int kOut = 0, int kSlab = kQuadSlab>
__device__ __forceinline__ void quad_item(const RoiLevels& lv, const RoiCfg& c, float* __restrict__ out, int64_t k,
                                          int chunk, int64_t item, uint32_t sbase, int64_t t_start, int lane,
                                          float* obuf = nullptr) {
  PairGeom G;
  PairLane P;
  const RoiRaw raw = roi_fetch(c, k);
  pair_setup<16>(lv, c, raw, lane, G, P);
  quad_body<kStAux, kStamp, kQW, kOut, kSlab>(G, P, c, out, k, chunk, item, sbase, t_start, lane, obuf);
}

// the item after its setup (G, P): staging, evaluation, stores.  The host admits only
// shapes whose largest tap grid fits one region (quad_ok: quad_max_cells <= kCells of D = 1).
template <int kStAux, bool kStamp, int kQW, int kOut, int kSlab, bool kOnly4, int kOpt>
__device__ __forceinline__ void quad_body(const PairGeom& G, const PairLane& P, const RoiCfg& c,
                                          float* __restrict__ out, int64_t k, int chunk, int64_t item, uint32_t sbase,
                                          int64_t t_start, int lane, float* obuf) {
  constexpr int SR = 2;
  int64_t t_setup = 0, t_land = 0;
  const int cw0 = chunk * 4 * kQW;
  const int nquads = min(kQW, (c.C - cw0) / 4);  // host: C % 4 == 0
  const int nbins = c.ph * c.pw;
  const bool active = lane < nbins;
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + (k * c.C + cw0) * nbins, (int64_t)4 * nquads * nbins * 4);
  const int ovoff = active ? lane * 4 : 0x40000000;  // idle lanes: dropped by the range check
  const int ostep = nbins * 4;
  if (G.empty) {  // no valid sample: all bins 0
    for (int ch = 0; ch < 4 * nquads; ++ch) __builtin_amdgcn_raw_buffer_store_b32(0u, orr, ovoff, ch * ostep, kStAux);
    return;
  }
  const int y0 = G.y0, x0 = G.x0, Cs = G.Cs, Cs2 = G.Cs2, sy = G.sy, sx = G.sx;
  const bool dy = G.dy, dx = G.dx;
  const int ncell = G.R * Cs2;
  const int rsrc = P.rsrc, csrc = P.csrc;
  const __amdgpu_buffer_rsrc_t fr = uniform_rsrc(G.base, (int64_t)G.extent);
  const uint32_t inv = G.inv;
  if (kStamp) t_setup = (int64_t)__builtin_amdgcn_s_memrealtime();
  int stamp_d = 0;
  auto store4 = [&](int q, f32x4 r) {
    if constexpr (kOut == 2) {
      if (r.x == 1234.5f) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.y), orr, ovoff, 0, kStAux);
      return;
    }
    if constexpr (kOut == 1) {
      if (q < nquads && active) {
        obuf[(4 * q) * nbins + lane] = r.x;
        obuf[(4 * q + 1) * nbins + lane] = r.y;
        obuf[(4 * q + 2) * nbins + lane] = r.z;
        obuf[(4 * q + 3) * nbins + lane] = r.w;
      }
      return;
    }
    const int vo = q < nquads ? ovoff : 0x40000000;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.x), orr, vo, (4 * q) * ostep, kStAux);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.y), orr, vo, (4 * q + 1) * ostep, kStAux);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.z), orr, vo, (4 * q + 2) * ostep, kStAux);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.w), orr, vo, (4 * q + 3) * ostep, kStAux);
  };
  auto run = [&](auto dd) {
    constexpr int D = decltype(dd)::value, RS = QuadLayout<D, kSlab>::RS, RP = QuadLayout<D, kSlab>::RP;
    const int nst = (nquads + D - 1) / D;
    // region 16-B unit j * 64 + lane of every quad  <-  that quad of cell j * 64 + lane
    auto goff_at = [&](int j) {
      int e = j * kWave + lane;
      const bool in = e < ncell;
      e = in ? e : 0;
      const int r = (int)(((uint32_t)e * inv) >> 16), col = min(e - r * Cs2, Cs - 1);
      const int o = (dy && dx) ? ((y0 + r) * sy + (x0 + col) * sx) * 4 : __shfl(rsrc, r, kWave) + __shfl(csrc, col, kWave);
      return ((kOpt & kFwdTrim) && !in) ? 0x40000000 : o;
    };
    int goff[RP];
#pragma unroll
    for (int j = 0; j < RP; ++j) goff[j] = goff_at(j);
    const int nr = (kOpt & kFwdTrim) ? (ncell + kWave - 1) / kWave : RP;  // rounds holding cells (uniform)
    auto issue = [&](int s) {  // quads past the last re-read it (their stores are dropped)
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int soff = (cw0 + 4 * min(s * D + d, nquads - 1)) * 4;
#pragma unroll
        for (int j = 0; j < RP; ++j)
          if (j < nr) lds_dma_at<16, 0>(fr, sbase + 4u * (uint32_t)(d * RS + j * 256), goff[j], soff);
      }
    };
    auto eval = [&](int s) {
      f32x4 v[2][8];
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
      float ly_h[SR], ly_l[SR], lx_h[SR], lx_l[SR];
      uint32_t lb[SR][SR], ldq[SR], ldr[SR];
#pragma unroll
      for (int i = 0; i < SR; ++i) {
        ly_h[i] = P.fyh[i], ly_l[i] = P.fyl[i], lx_h[i] = P.fxh[i], lx_l[i] = P.fxl[i], ldq[i] = P.tdq[i],
        ldr[i] = P.tdr[i];
        asm volatile("" : "+v"(ly_h[i]), "+v"(ly_l[i]), "+v"(lx_h[i]), "+v"(lx_l[i]), "+v"(ldq[i]), "+v"(ldr[i]));
#pragma unroll
        for (int j = 0; j < SR; ++j) {
          lb[i][j] = sbase + P.tb0[i][j];
          asm volatile("" : "+v"(lb[i][j]));
        }
      }
      auto tap = [&](int iy, int ix, int q) -> uint32_t {
        return lb[iy][ix] + ((q & 1) ? ldq[ix] : 0u) + ((q & 2) ? ldr[iy] : 0u);
      };
      auto load = [&](auto hh) {
        constexpr int h = decltype(hh)::value, d = h >> 1, iy = h & 1, OFF = 4 * (d * RS);
#pragma unroll
        for (int ix = 0; ix < SR; ++ix)
#pragma unroll
          for (int q = 0; q < 4; ++q) v[h & 1][ix * 4 + q] = lds_read_b128<OFF>(tap(iy, ix, q));
      };
      load(std::integral_constant<int, 0>{});
      static_for<0, 2 * D>([&](auto hh) {
        constexpr int h = decltype(hh)::value, d = h >> 1, iy = h & 1;
        if constexpr (h + 1 < 2 * D) {
          load(std::integral_constant<int, h + 1>{});
          lds_wait4<8>(v[h & 1]);
        } else {
          lds_wait4<0>(v[h & 1]);
        }
        if (iy == 0) acc = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) {
          const float w[4] = {ly_h[iy] * lx_h[ix], ly_h[iy] * lx_l[ix], ly_l[iy] * lx_h[ix], ly_l[iy] * lx_l[ix]};
          acc = acc + quad_val(w, &v[h & 1][ix * 4]);
        }
        if (iy == 1) store4(s * D + d, acc * 0.25f);  // count 4: / 4 == * 0.25
      });
    };
    stamp_d = D;
    for (int s = 0; s < nst; ++s) {
      issue(s);  // the previous stage's tap reads completed (lds_wait4<0> + barrier below)
      wait_vmcnt<0>();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (kStamp && s == 0) t_land = (int64_t)__builtin_amdgcn_s_memrealtime();
      eval(s);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  };
  if constexpr (kOnly4) {  // the caller took ncell <= kCells of D = 4
    run(std::integral_constant<int, 4>{});
  } else {
    if (ncell <= QuadLayout<4, kSlab>::kCells)
      run(std::integral_constant<int, 4>{});
    else if (ncell <= QuadLayout<2, kSlab>::kCells)
      run(std::integral_constant<int, 2>{});
    else  // ncell <= quad_max_cells(ph, pw) <= QuadLayout<1, kSlab>::kCells (quad_ok)
      run(std::integral_constant<int, 1>{});
  }
  if constexpr (kOut == 1) {  // the item's [channel][bin] block: contiguous, 16-B stores
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int n4 = 4 * nquads * nbins / 4;
    const float4* o4 = reinterpret_cast<const float4*>(obuf);
    for (int e = lane; e < n4; e += kWave) {
      const float4 q = o4[e];
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{__float_as_uint(q.x), __float_as_uint(q.y), __float_as_uint(q.z), __float_as_uint(q.w)}, orr, e * 16,
          0, kStAux);
    }
  }
  if (kStamp && lane == 0) {
    int64_t* st = reinterpret_cast<int64_t*>(out + c.K * c.C * nbins) + item * 8;
    const int64_t t_end = (int64_t)__builtin_amdgcn_s_memrealtime();
    st[0] = t_start;
    st[1] = t_setup;
    st[2] = t_land;
    st[3] = t_end;
    st[4] = stamp_d;
    st[5] = ncell;
    st[6] = t_setup;
    st[7] = blockIdx.x & 7;
  }
}

// 1-D grid of 8 * ceil(K * chunks / 8) single-wave workgroups; XCD x takes the x-th eighth
// of the item list (as the pair kernel: the two 16-channel chunks of a 128-B line share an
// XCD).  kOrder 0: chunk-major (chunk, RoI); 1: chunk-pair-major, the pair's two chunks of
// a RoI adjacent (2p, k), (2p + 1, k) -- the two waves reading the two halves of the same
// lines run together, so the second finds them in L2.
template <int kStAux = kCpolNT, bool kStamp = false, int kWpe = 3, int kQW = kQuadWave, int kOut = 0,
          bool kSpan = false, int kSlab = kQuadSlab, int kOrder = 0>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kWpe))) roi_align_fwd_quad_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out) {
  const int64_t t_start = (kStamp || kSpan) ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  __shared__ __attribute__((aligned(16))) float slab[kSlab];
  __shared__ __attribute__((aligned(16))) float obuf[kOut == 1 ? 4 * kQW * kWave : 4];  // [channel][bin], <= 64 bins
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)slab);
  const uint32_t G = (uint32_t)(c.C + 4 * kQW - 1) / (uint32_t)(4 * kQW), K32 = (uint32_t)c.K;
  const uint32_t total = K32 * G, per = (total + 7u) / 8u;
  const uint32_t w = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  const uint32_t wend = min((blockIdx.x & 7u) * per + per, total);
  if (w >= wend) return;
  int ch0;
  int64_t k0;
  if (kOrder == 0) {
    ch0 = (int)(w / K32);
    k0 = (int64_t)(w - (uint32_t)ch0 * K32);
  } else {
    const uint32_t p = w / (2u * K32), r = w - p * 2u * K32;
    if (2u * p + 1u < G) {
      ch0 = (int)(2u * p + (r & 1u));
      k0 = (int64_t)(r >> 1);
    } else {  // odd chunk count: the last chunk alone
      ch0 = (int)(2u * p);
      k0 = (int64_t)r;
    }
  }
  quad_item<kStAux, kStamp, kQW, kOut, kSlab>(lv, c, out, k0, ch0, w, sbase, t_start, threadIdx.x & (kWave - 1), obuf);
  if (kSpan && threadIdx.x == 0) record_span(c, t_start);
}

// ---------------------------------------------------------------------------
// Channel-quad forward with coalesced band staging (channels-last features).  The quad
// kernel stages one channel quad of every window cell per LDS-DMA instruction: lane =
// cell, 16 B from each of 64 cells 1 KB apart, so every lane is its own L2 request --
// VOC-sized windows (hundreds of cells) made the launch L2-request-rate bound (24 M
// 16-B requests for 410 MB staged, 93 % L2 hits, 111 us).  Here lane = 4 x cell + quad:
// the four lanes of a cell read its 64 contiguous bytes (the item's 16 channels), one
// 64-B request, and the slab holds [cell][16 channels] (64 B per cell).  A window larger
// than the slab is staged in row bands: each band holds the rows of the next bin rows
// whose samples fit (rows of the lowest pending bin first; every bin's rows span <= 5
// <= kSlabCells / 29), evaluated by the lanes (bins) of those rows; windows within the slab
// are one band (the random-init RoIs of the bench: all of them).  Tap reads: lane l reads
// quad (d + l) mod 4 at step d, so the 16 lanes of a ds_read_b128 group spread over the
// 64 banks (a fixed quad would put them on the 4 bank groups of cell mod 4); its stores
// go to those quads' channels.  Same operation order per output: bit-identical to the
// other kernels.
template <int kSlabCells>
struct BandLayout {
  static_assert(kSlabCells % 16 == 0, "whole 16-cell DMA instructions");
  static constexpr int kMaxDma = kSlabCells / 16;
  static_assert(kMaxDma < 64, "vmcnt is 6 bits");
};

// kRot: 0 = every lane reads quad d at step d (bank conflicts: 4 bank groups per quad);
// 1 = lane l reads quad (d + l) mod 4, results kept and stored per channel after the 4 steps
// (each store instruction writes one channel plane, 49 contiguous floats); 2 = as 1 but
// each step's quad stored at once (lane-dependent channel planes: 4 partial lines each);
// 3 = as 0, the results kept until the last band and stored by every bin at once (a band's
// own stores cover only its bins' part of each channel row: partial lines).
// Whole-window stages of two channel quads, cell-interleaved: the slab holds [cell][2 quads]
// (32 B per cell), the two lanes of a cell read its 32 contiguous bytes (one request for two
// quads, the quad layout's [quad][cell] takes two), quads {0, 1} then {2, 3}.  G / P carry the
// quad layout's 16-B tap offsets (pair_setup<16>); every lane evaluates every stage (no band
// masking) and stores whole channel rows.  For windows of up to kSlabCells * 2 cells.
// kOpt bit 2 (kFwdIlvRot, D = 2): at step d lane l reads quad (d + l) & 1 of its cells, so the
// 16 lanes of a ds_read_b128 group use both 16-B halves of the 32-B cells (16 bank slots
// instead of 8); the two results are stored per channel after both steps.
template <int kStAux, int kSlabCells, int D = 2, bool kStamp = false, int kOpt = 0>
__device__ __forceinline__ void ilv_body(const PairGeom& G, const PairLane& P, const RoiCfg& c,
                                          float* __restrict__ out, int64_t k, int chunk, uint32_t sbase, int lane,
                                          int64_t item = 0, int64_t t_start = 0) {
  constexpr int SR = 2;
  const int cw0 = chunk * 4 * kQuadWave;
  const int nquads = min(kQuadWave, (c.C - cw0) / 4);  // host: C % 4 == 0
  const int nbins = c.ph * c.pw;
  const bool active = lane < nbins;
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + (k * c.C + cw0) * nbins, (int64_t)4 * nquads * nbins * 4);
  const int ovoff = active ? lane * 4 : 0x40000000;
  const int ostep = nbins * 4;
  const int y0 = G.y0, x0 = G.x0, Cs = G.Cs, Cs2 = G.Cs2, sy = G.sy, sx = G.sx;
  const bool dense = G.dy && G.dx;
  const int ncell = G.R * Cs2;
  constexpr int kLg = D == 4 ? 2 : 1;
  const int nj = (ncell + (kWave / D - 1)) >> (6 - kLg);  // 64 / D cells per DMA instruction
  const __amdgpu_buffer_rsrc_t fr = uniform_rsrc(G.base, (int64_t)G.extent);
  const uint32_t inv = G.inv;
  const int soff = cw0 * 4;
  for (int s = 0; s < 4 / D; ++s) {
    const int dq = min(D * s + (lane & (D - 1)), nquads - 1);
    for (int j = 0; j < nj; ++j) {
      int e = (kWave / D) * j + (lane >> kLg);
      const bool in = e < ncell;
      e = in ? e : 0;
      const int r = (int)(((uint32_t)e * inv) >> 16), col = min(e - r * Cs2, Cs - 1);
      const int goff = dense ? ((y0 + r) * sy + (x0 + col) * sx) * 4 : __shfl(P.rsrc, r, kWave) + __shfl(P.csrc, col, kWave);
      lds_dma_at<16, 0>(fr, sbase + 1024u * (uint32_t)j, ((kOpt & kFwdTrim) && !in) ? 0x40000000 : goff + dq * 16, soff);
    }
    wait_vmcnt<0>();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    f32x4 v[2][8];
    float ly_h[SR], ly_l[SR], lx_h[SR], lx_l[SR];
    uint32_t lb[SR][SR], ldq[SR], ldr[SR];
#pragma unroll
    for (int i = 0; i < SR; ++i) {  // 16*D-B cells: the quad layout's offsets times D
      ly_h[i] = P.fyh[i], ly_l[i] = P.fyl[i], lx_h[i] = P.fxh[i], lx_l[i] = P.fxl[i], ldq[i] = P.tdq[i] << kLg,
      ldr[i] = P.tdr[i] << kLg;
      asm volatile("" : "+v"(ly_h[i]), "+v"(ly_l[i]), "+v"(lx_h[i]), "+v"(lx_l[i]), "+v"(ldq[i]), "+v"(ldr[i]));
#pragma unroll
      for (int jx = 0; jx < SR; ++jx) {
        lb[i][jx] = sbase + (P.tb0[i][jx] << kLg);
        asm volatile("" : "+v"(lb[i][jx]));
      }
    }
    auto tap = [&](int iy, int ix, int q) -> uint32_t {
      return lb[iy][ix] + ((q & 1) ? ldq[ix] : 0u) + ((q & 2) ? ldr[iy] : 0u);
    };
    constexpr bool kRotI = (kOpt & kFwdIlvRot) != 0 && D == 2;
    f32x4 rr0 = {}, rr1 = {};  // kRotI: the results of steps 0 / 1
    static_for<0, D>([&](auto dd) {
      constexpr int d = decltype(dd)::value;
      const uint32_t qo = kRotI ? 16u * (uint32_t)((d + lane) & 1) : 0u;  // kRotI: this lane's quad at step d
      auto load = [&](auto hh) {
        constexpr int iy = decltype(hh)::value;
#pragma unroll
        for (int ix = 0; ix < SR; ++ix)
#pragma unroll
          for (int q = 0; q < 4; ++q) v[iy][ix * 4 + q] = lds_read_b128<kRotI ? 0 : 16 * d>(tap(iy, ix, q) + qo);
      };
      load(std::integral_constant<int, 0>{});
      load(std::integral_constant<int, 1>{});
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
      lds_wait4<8>(v[0]);
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        const float w[4] = {ly_h[0] * lx_h[ix], ly_h[0] * lx_l[ix], ly_l[0] * lx_h[ix], ly_l[0] * lx_l[ix]};
        acc = acc + quad_val(w, &v[0][ix * 4]);
      }
      lds_wait4<0>(v[1]);
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        const float w[4] = {ly_h[1] * lx_h[ix], ly_h[1] * lx_l[ix], ly_l[1] * lx_h[ix], ly_l[1] * lx_l[ix]};
        acc = acc + quad_val(w, &v[1][ix * 4]);
      }
      const f32x4 r4 = acc * 0.25f;  // count 4: / 4 == * 0.25
      if constexpr (kRotI) {
        if constexpr (d == 0) rr0 = r4;
        else rr1 = r4;
      } else {
        const int Q = D * s + d;
        const int vo = Q < nquads ? ovoff : 0x40000000;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.x), orr, vo, (4 * Q) * ostep, kStAux);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.y), orr, vo, (4 * Q + 1) * ostep, kStAux);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.z), orr, vo, (4 * Q + 2) * ostep, kStAux);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.w), orr, vo, (4 * Q + 3) * ostep, kStAux);
      }
    });
    if constexpr (kRotI) {  // quad q of the stage was computed at step (q - lane) & 1
      const bool sw = (lane & 1) != 0;  // odd lanes: step 0 read quad 1
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x4 r4 = (q == 0) != sw ? rr0 : rr1;
        const int Q = 2 * s + q;
        const int vo = Q < nquads ? ovoff : 0x40000000;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.x), orr, vo, (4 * Q) * ostep, kStAux);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.y), orr, vo, (4 * Q + 1) * ostep, kStAux);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.z), orr, vo, (4 * Q + 2) * ostep, kStAux);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.w), orr, vo, (4 * Q + 3) * ostep, kStAux);
      }
    }
    // this stage's tap reads are complete (lds_wait4<0>) before the next stage's DMA
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (kStamp && lane == 0) {  // tools timing build: [4] = -D marks this path
    int64_t* st = reinterpret_cast<int64_t*>(out + c.K * c.C * nbins) + item * 8;
    st[0] = t_start;
    st[1] = st[2] = st[6] = 0;
    st[3] = (int64_t)__builtin_amdgcn_s_memrealtime();
    st[4] = -D;
    st[5] = ncell;
    st[7] = blockIdx.x & 7;
  }
}

// kHybrid = D > 0: windows that the quad kernel stages D quads at a time (at most
// QuadLayout<D, kSlabCells * 16>::kCells cells: every random-init RoI of the bench but a few,
// most small RoIs) take its path instead -- lane = cell, 64 cells and one address per DMA
// instruction: fewer instructions where the window is small and the L2 request rate is not
// the bound -- the rest the bands.
// band_body: one item (RoI k, 16 channels from chunk) after its RoI setup (G, P of
// pair_setup<16> when kHybrid or kIlv, else pair_setup<64>); P by value: the band path rescales it.
template <int kStAux, bool kStamp, int kSlabCells, int kRot = 1, int kHybrid = 0, int kHybridHi = 0,
          int kIlv = 0, int kOpt = 0>
__device__ __forceinline__ void band_body(const RoiCfg& c, float* __restrict__ out, int64_t k, int chunk,
                                          int64_t item, uint32_t sbase, int64_t t_start, int lane, const PairGeom& G,
                                          PairLane P) {
  constexpr int SR = 2;
  int64_t t_setup = 0, t_land = 0;
  if constexpr (kHybrid > 0 || kIlv > 0) {
    if constexpr (kHybrid > 0) {
      if (!G.empty && G.R * G.Cs2 <= QuadLayout<kHybrid, kSlabCells * 16>::kCells) {
        quad_body<kStAux, kStamp, kQuadWave, 0, kSlabCells * 16, kHybrid == 4, kOpt>(G, P, c, out, k, chunk, item,
                                                                                    sbase, t_start, lane, nullptr);
        return;
      }
    }
    if constexpr ((kIlv & 1) != 0) {  // up to kSlabCells cells: one whole-window stage of [cell][4 quads]
      if (!G.empty && G.R * G.Cs2 <= kSlabCells) {
        ilv_body<kStAux, kSlabCells, 4, kStamp, kOpt>(G, P, c, out, k, chunk, sbase, lane, item, t_start);
        return;
      }
    }
    if constexpr ((kIlv & 2) != 0) {  // up to 2 * kSlabCells cells: two whole-window stages of [cell][2 quads]
      if (!G.empty && G.R * G.Cs2 <= 2 * kSlabCells) {
        ilv_body<kStAux, kSlabCells, 2, kStamp, kOpt>(G, P, c, out, k, chunk, sbase, lane, item, t_start);
        return;
      }
    }
    if constexpr (kHybridHi > 0) {  // windows of many bands: the quad kernel's D = 2 / 1 stages instead
      if (!G.empty && G.R * G.Cs2 > kHybridHi) {
        quad_body<kStAux, kStamp, kQuadWave, 0, kSlabCells * 16, false, kOpt>(G, P, c, out, k, chunk, item, sbase,
                                                                             t_start, lane, nullptr);
        return;
      }
    }
#pragma unroll
    for (int i = 0; i < SR; ++i) {  // the band layout's 64-B cells
      P.tdq[i] <<= 2;
      P.tdr[i] <<= 2;
#pragma unroll
      for (int j = 0; j < SR; ++j) P.tb0[i][j] <<= 2;
    }
  }
  const int cw0 = chunk * 4 * kQuadWave;
  const int nquads = min(kQuadWave, (c.C - cw0) / 4);  // host: C % 4 == 0
  const int nbins = c.ph * c.pw;
  const bool active = lane < nbins;
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + (k * c.C + cw0) * nbins, (int64_t)4 * nquads * nbins * 4);
  const int ostep = nbins * 4;
  if (G.empty) {  // no valid sample: all bins 0
    const int vo = active ? lane * 4 : 0x40000000;
    for (int ch = 0; ch < 4 * nquads; ++ch) __builtin_amdgcn_raw_buffer_store_b32(0u, orr, vo, ch * ostep, kStAux);
    return;
  }
  if (kStamp) t_setup = (int64_t)__builtin_amdgcn_s_memrealtime();
  const int y0 = G.y0, x0 = G.x0, Cs = G.Cs, Cs2 = G.Cs2, sy = G.sy, sx = G.sx, R = G.R;
  const bool dense = G.dy && G.dx;
  const __amdgpu_buffer_rsrc_t fr = uniform_rsrc(G.base, (int64_t)G.extent);
  const uint32_t inv = G.inv;
  const int rows_cap = kSlabCells / Cs2;
  // this lane's share of a DMA instruction: cell (lane >> 2) of the instruction's 16, quad lane & 3
  const int dq = min(lane & 3, nquads - 1);
  const int soff = cw0 * 4;
  bool pending = active;
  int nbands = 0;
  f32x4 res0 = {}, res1 = {}, res2 = {}, res3 = {};  // kRot 1 / 3: the step results (named: no indexed array)
  while (true) {
    const uint64_t pend = __ballot(pending);
    if (!pend) break;
    // the band: rows [rs, re) -- from the lowest row of a pending bin, the bins whose rows all fit
    const int rmin = __builtin_amdgcn_readfirstlane(wave_min_i32(pending ? P.rlo : 0x7fffffff));
    const int rs = rmin == 0x7fffffff ? 0 : max(0, rmin);  // only bins without a valid row left: one row
    const int rcap = min(rs + rows_cap, R);
    bool in = pending && P.rhi < rcap;
    if (!__ballot(in)) in = pending;  // unreachable by the rows bound (host: 5 rows fit); never loops forever
    const int re = min(R, max(rs + 1, __builtin_amdgcn_readfirstlane(wave_max_i32(in ? P.rhi + 1 : 0))));
    const int nb = (re - rs) * Cs2;
    const int nj = (nb + 15) >> 4;
    // stage rows [rs, re): instruction j, lane -> cell 16 j + (lane >> 2) of the band, quad dq
    for (int j = 0; j < nj; ++j) {
      int e = 16 * j + (lane >> 2);
      const bool inb = e < nb;
      e = inb ? e : 0;
      const int r = (int)(((uint32_t)e * inv) >> 16), col = min(e - r * Cs2, Cs - 1);
      const int goff = dense ? ((y0 + rs + r) * sy + (x0 + col) * sx) * 4
                             : __shfl(P.rsrc, rs + r, kWave) + __shfl(P.csrc, col, kWave);
      lds_dma_at<16, 0>(fr, sbase + 1024u * (uint32_t)j, ((kOpt & kFwdTrim) && !inb) ? 0x40000000 : goff + dq * 16,
                        soff);
    }
    wait_vmcnt<0>();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (kStamp && nbands == 0) t_land = (int64_t)__builtin_amdgcn_s_memrealtime();
    if (in) {
      const uint32_t boff = 64u * (uint32_t)(rs * Cs2);
      f32x4 v[2][8];
      float ly_h[SR], ly_l[SR], lx_h[SR], lx_l[SR];
      uint32_t lb[SR][SR], ldq[SR], ldr[SR];
#pragma unroll
      for (int i = 0; i < SR; ++i) {
        ly_h[i] = P.fyh[i], ly_l[i] = P.fyl[i], lx_h[i] = P.fxh[i], lx_l[i] = P.fxl[i], ldq[i] = P.tdq[i],
        ldr[i] = P.tdr[i];
#pragma unroll
        for (int jx = 0; jx < SR; ++jx)  // invalid samples read band cell 0 (finite) with zero weights
          lb[i][jx] = sbase + (((P.vmask >> (2 * i + jx)) & 1u) ? P.tb0[i][jx] - boff : 0u);
      }
      static_for<0, kQuadWave>([&](auto dd) {
        constexpr int d = decltype(dd)::value;
        const int qq = kRot == 1 || kRot == 2 ? (d + lane) & 3 : d;  // this lane's quad at step d
        const uint32_t qo = 16u * (uint32_t)qq;
        uint32_t lq[SR][SR];
#pragma unroll
        for (int iy = 0; iy < SR; ++iy)
#pragma unroll
          for (int ix = 0; ix < SR; ++ix) lq[iy][ix] = lb[iy][ix] + qo;
        auto tap = [&](int iy, int ix, int q) -> uint32_t {
          return lq[iy][ix] + ((q & 1) ? ldq[ix] : 0u) + ((q & 2) ? ldr[iy] : 0u);
        };
        auto load = [&](auto hh) {
          constexpr int iy = decltype(hh)::value;
#pragma unroll
          for (int ix = 0; ix < SR; ++ix)
#pragma unroll
            for (int q = 0; q < 4; ++q) v[iy][ix * 4 + q] = lds_read_b128<0>(tap(iy, ix, q));
        };
        load(std::integral_constant<int, 0>{});
        load(std::integral_constant<int, 1>{});
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
        lds_wait4<8>(v[0]);
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) {
          const float w[4] = {ly_h[0] * lx_h[ix], ly_h[0] * lx_l[ix], ly_l[0] * lx_h[ix], ly_l[0] * lx_l[ix]};
          acc = acc + quad_val(w, &v[0][ix * 4]);
        }
        lds_wait4<0>(v[1]);
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) {
          const float w[4] = {ly_h[1] * lx_h[ix], ly_h[1] * lx_l[ix], ly_l[1] * lx_h[ix], ly_l[1] * lx_l[ix]};
          acc = acc + quad_val(w, &v[1][ix * 4]);
        }
        const f32x4 r4 = acc * 0.25f;  // count 4: / 4 == * 0.25
        if constexpr (kRot == 1 || kRot == 3) {
          if constexpr (d == 0) res0 = r4;
          if constexpr (d == 1) res1 = r4;
          if constexpr (d == 2) res2 = r4;
          if constexpr (d == 3) res3 = r4;
        } else {
          const int vo = qq < nquads ? lane * 4 + 4 * qq * ostep : 0x40000000;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.x), orr, vo, 0, kStAux);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.y), orr, vo, ostep, kStAux);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.z), orr, vo, 2 * ostep, kStAux);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.w), orr, vo, 3 * ostep, kStAux);
        }
      });
      if constexpr (kRot == 1) {  // quad Q was computed at step (Q - lane) mod 4: one channel plane per store
#pragma unroll
        for (int Q = 0; Q < kQuadWave; ++Q) {
          const int sel = (Q - lane) & 3;
          const bool s0 = sel == 0, s1 = sel == 1, s2 = sel == 2;
          const float o[4] = {s0 ? res0.x : s1 ? res1.x : s2 ? res2.x : res3.x,
                              s0 ? res0.y : s1 ? res1.y : s2 ? res2.y : res3.y,
                              s0 ? res0.z : s1 ? res1.z : s2 ? res2.z : res3.z,
                              s0 ? res0.w : s1 ? res1.w : s2 ? res2.w : res3.w};
          const int vo = Q < nquads ? lane * 4 : 0x40000000;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o[e]), orr, vo, (4 * Q + e) * ostep, kStAux);
        }
      }
      pending = false;
    }
    ++nbands;
    // the band's tap reads are complete (lds_wait4<0>) before the next band's DMA overwrites it
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if constexpr (kRot == 3) {  // every bin's 16 channels after the last band: whole channel rows per store
    const int vo = active ? lane * 4 : 0x40000000;
    static_for<0, kQuadWave>([&](auto qd) {
      constexpr int Q = decltype(qd)::value;
      const f32x4 r4 = Q == 0 ? res0 : Q == 1 ? res1 : Q == 2 ? res2 : res3;
      const int v = Q < nquads ? vo : 0x40000000;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.x), orr, v, (4 * Q) * ostep, kStAux);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.y), orr, v, (4 * Q + 1) * ostep, kStAux);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.z), orr, v, (4 * Q + 2) * ostep, kStAux);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4.w), orr, v, (4 * Q + 3) * ostep, kStAux);
    });
  }
  if (kStamp && lane == 0) {
    int64_t* st = reinterpret_cast<int64_t*>(out + c.K * c.C * nbins) + item * 8;
    st[0] = t_start;
    st[1] = t_setup;
    st[2] = t_land;
    st[3] = (int64_t)__builtin_amdgcn_s_memrealtime();
    st[4] = nbands;
    st[5] = R * Cs2;
    st[6] = t_setup;
    st[7] = blockIdx.x & 7;
  }
}

template <int kStAux, bool kStamp, int kSlabCells, int kRot = 1, int kHybrid = 0, int kHybridHi = 0,
          int kIlv = 0, int kOpt = 0>
__device__ __forceinline__ void band_item(const RoiLevels& lv, const RoiCfg& c, float* __restrict__ out, int64_t k,
                                          int chunk, int64_t item, uint32_t sbase, int64_t t_start, int lane) {
  PairGeom G;
  PairLane P;
  int64_t ko = k;
  const RoiRaw raw = (kOpt & kFwdSorted) ? roi_fetch_rec(c, k, &ko) : roi_fetch(c, k);
  pair_setup<(kHybrid || kIlv) ? 16 : 64>(lv, c, raw, lane, G, P);
  band_body<kStAux, kStamp, kSlabCells, kRot, kHybrid, kHybridHi, kIlv, kOpt>(c, out, ko, chunk, item, sbase, t_start,
                                                                              lane, G, P);
}

// 1-D grid of 8 * ceil(K * chunks / 8) single-wave workgroups; XCD x takes the x-th eighth of
// the item list in chunk-pair-major order (quad kernel, kOrder 1: the two 16-channel chunks of
// a 128-B line, adjacent, on one XCD).
// kChunks 2: one wave per (RoI, chunk pair) -- both 16-channel chunks of a 128-B line, one after
// the other on the SAME RoI fetch and setup (the record's first load and pair_setup were ~half of a
// small item's life); the grid is then 8 * ceil(K * ceil(chunks / 2) / 8).
template <int kStAux = kCpolNT, bool kStamp = false, int kSlabCells = 208, bool kSpan = false, int kWpe = 3,
          int kRot = 1, int kHybrid = 0, int kHybridHi = 0, int kIlv = 0, int kChunks = 1, int kOrder = 1, int kOpt = 0>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kWpe)))
roi_align_fwd_band_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out) {
  const int64_t t_start = (kStamp || kSpan) ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  // whole 1-KB DMA rounds: an LDS-DMA instruction writes 64 lanes x 16 B wherever its last cells
  // fall, so the interleaved and band stages (up to ceil(cells / 32 or / 16) rounds from the
  // slab start) write whole KB; the slab is rounded up to whole KB (the product's 240 cells:
  // exactly 15 KB, 10 workgroups per CU by LDS)
  __shared__ __attribute__((aligned(16))) float slab[(kSlabCells * 16 + 255) / 256 * 256];
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)slab);
  const uint32_t G = (uint32_t)(c.C + kQuadChunk - 1) / (uint32_t)kQuadChunk, K32 = (uint32_t)c.K;
  const int lane = threadIdx.x & (kWave - 1);
  if constexpr (kChunks == 2) {
    const uint32_t NP = (G + 1u) / 2u, total = K32 * NP, per = (total + 7u) / 8u;
    const uint32_t w = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
    const uint32_t wend = min((blockIdx.x & 7u) * per + per, total);
    if (w >= wend) return;
    const uint32_t p = w / K32, k = w - p * K32;
    PairGeom Gm;
    PairLane P;
    const RoiRaw raw = roi_fetch(c, (int64_t)k);
    pair_setup<(kHybrid || kIlv) ? 16 : 64>(lv, c, raw, lane, Gm, P);
    const bool two = 2u * p + 1u < G;
    const int64_t item0 = (int64_t)p * 2 * K32 + (two ? 2 * k : k);
    band_body<kStAux, kStamp, kSlabCells, kRot, kHybrid, kHybridHi, kIlv, kOpt>(c, out, (int64_t)k, (int)(2u * p),
                                                                                item0, sbase, t_start, lane, Gm, P);
    if (two) {
      // the first chunk's tap reads are complete (its evaluation waited on them) before the
      // second chunk's DMA overwrites the slab
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      band_body<kStAux, kStamp, kSlabCells, kRot, kHybrid, kHybridHi, kIlv, kOpt>(c, out, (int64_t)k,
                                                                                  (int)(2u * p + 1u), item0 + 1, sbase,
                                                                                  t_start, lane, Gm, P);
    }
    if (kSpan && threadIdx.x == 0) record_span(c, t_start);
    return;
  }
  const uint32_t total = K32 * G, per = (total + 7u) / 8u;
  const uint32_t w = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  const uint32_t wend = min((blockIdx.x & 7u) * per + per, total);
  if (w >= wend) return;
  const uint32_t p = w / (2u * K32), r = w - p * 2u * K32;
  int ch0;
  int64_t k0;
  if (kOrder == 0) {  // chunk-major: XCD x walks its eighth of the (chunk, RoI) list
    ch0 = (int)(w / K32);
    k0 = (int64_t)(w - (uint32_t)ch0 * K32);
  } else if (2u * p + 1u < G) {
    ch0 = (int)(2u * p + (r & 1u));
    k0 = (int64_t)(r >> 1);
  } else {  // odd chunk count: the last chunk alone
    ch0 = (int)(2u * p);
    k0 = (int64_t)r;
  }
  band_item<kStAux, kStamp, kSlabCells, kRot, kHybrid, kHybridHi, kIlv, kOpt>(lv, c, out, k0, ch0, w, sbase, t_start,
                                                                              lane);
  if (kSpan && threadIdx.x == 0) record_span(c, t_start);
}

// the band kernel's shape limits: a bin's rows (sampling 2: its two y samples' taps, <= 5
// rows -- dense windows of <= 4 ph rows space the 2 ph samples <= (4 ph - 1) / (2 ph - 1) <= 3
// rows apart, tap lists give 4) fit a band of the widest window row (4 pw entries, odd stride)
constexpr bool band_fits(int ph, int pw, int slab_cells) { return 5 * ((4 * pw) | 1) <= slab_cells; }

// ---------------------------------------------------------------------------
// Channel-group forward (round 6) for channels-last features: ONE workgroup of kNW waves per
// (RoI, 64 channels).  The RoI's tap window is staged once for the whole workgroup as
// [cell][64 channels] (256 B per cell, row stride = the window width): one LDS-DMA
// instruction moves 4 whole cells, the 16 lanes of a cell reading its 256 contiguous bytes
// (2 full 128-B lines; the 16-channel items issue 4 requests of 64 B or 16 of 16 B for the
// same cell), and the 4 (or 8) waves of the workgroup share the window instead of each
// staging its own copy.  Evaluation: lane = (bin b4 = lane / 16 of the step's 4 bins,
// channel quad q = lane % 16), every tap ONE ds_read_b128 at cell * 256 + q * 16.  The lanes
// of a ds_read_b128 bank group (MI355X_MICROARCH §LDS: {0-3,12-15,20-27}, ...) are the 8
// quads of each of two bins (or the 16 of one): since a cell spans all 64 banks, they hit 16
// distinct 16-B bank slots whatever the two cells are -- no bank conflicts by construction
// (the 16-channel layouts conflict on 43-61 % of their LDS cycles).  The bin's sample taps come
// from two tables in LDS (per y / x sample: slab row / column, tap delta, l, 1 - l), read
// once per bin and step (the 16 lanes of a bin read one address: a broadcast).  Windows
// above the slab are staged in bands of whole bin rows (a bin row whose dense rows alone
// exceed the slab: its 4 tap-list rows).  The results leave through the slab (after the last band) as the item's
// contiguous [64][ph * pw] output block in 16-B stores.  Operation order as every other
// forward kernel (((w1 v1 + w2 v2) + w3 v3) + w4 v4 per sample, samples summed (iy, ix) in
// order, then / 4): bit-identical.
constexpr int kCgChan = 64;  // channels per item

// kLd2: both sample rows' 16 tap reads in flight together (else the second row's 8 after the
// first row's sums: 32 VGPRs fewer)
// kOrder 0: XCD x walks the x-th eighth of the group-major (group, RoI) list (each XCD's L2 holds
// one 64-channel slice); 1: RoI-major (RoI, group) -- the 4 groups of a RoI adjacent.
// kStamp (tools-only timing builds): thread 0 writes 16 int64 per item after the output --
// s_memrealtime at start / setup done / first band landed / end, bands, window cells, RoI record
// landed, evaluation done, taps made, window extents, tables written.
template <int kNW, int kSlabCells, int kStAux = kCpolNT, bool kSpan = false, int kWpe = 0, bool kLd2 = true,
          int kOrder = 0, bool kStamp = false>
__global__ void __launch_bounds__(kNW * kWave) __attribute__((amdgpu_waves_per_eu(kWpe > 0 ? kWpe : 1)))
roi_align_fwd_cg_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out) {
  constexpr int SR = 2;
  constexpr int kJ = 16 / kNW;  // 4-bin steps per wave (<= 64 bins)
  static_assert(kNW == 2 || kNW == 4 || kNW == 8, "waves per workgroup");
  static_assert(kSlabCells >= 64 && kSlabCells % 4 == 0, "the output block [64][<= 64 bins] leaves through the slab");
  static_assert((kSlabCells + 3) / 4 <= 63 * kNW, "vmcnt is 6 bits");
  const int64_t t_start = (kSpan || kStamp) ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  int64_t t_rec = 0, t_setup = 0, t_land = 0, t_eval = 0, t_tap = 0, t_ext = 0, t_tab = 0;
  int n_bands = 0;
  __shared__ __attribute__((aligned(16))) float slab[kSlabCells * kCgChan];
  __shared__ __attribute__((aligned(16))) float4 tab[32];  // y samples [0, 16), x samples [16, 32)
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)slab);
  const uint32_t tbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float4*)tab);
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  // XCD x (= workgroup id mod 8) walks the x-th eighth of the group-major (group, RoI) list
  const uint32_t NG = (uint32_t)c.C / kCgChan, K32 = (uint32_t)c.K;
  const uint32_t total = K32 * NG, per = (total + 7u) / 8u;
  const uint32_t w = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  if (w >= min((blockIdx.x & 7u) * per + per, total)) return;
  const uint32_t grp = kOrder == 0 ? w / K32 : w % NG;
  const int64_t k = kOrder == 0 ? (int64_t)(w - grp * K32) : (int64_t)(w / NG);
  const int nbins = c.ph * c.pw;
  const int nq = nbins * kCgChan / 4;  // 16-B units of the item's output block
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + (k * c.C + (int64_t)grp * kCgChan) * nbins, (int64_t)nq * 16);
  // levels 0-3's parameters at constant offsets: loaded with the kernel's other arguments, in
  // flight together with the RoI record, then picked by the RoI's level (a uniform select) --
  // indexed by the level, they were a second scalar round trip after the record's
  float sc4[4];
  int h4[4], w4[4], sy4[4], sx4[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    sc4[q] = lv.scale[q], h4[q] = lv.h[q], w4[q] = lv.w[q], sy4[q] = (int)lv.sy[q], sx4[q] = (int)lv.sx[q];
  const RoiRaw raw = roi_fetch(c, k);
  if (kStamp) t_rec = (int64_t)__builtin_amdgcn_s_memrealtime();
  const int l = roi_level(lv, raw.lvl);
  float scl;
  int H, W, sy, sx;
  if (l < 4) {
    auto pk = [&](const auto (&a)[4]) { return l == 0 ? a[0] : l == 1 ? a[1] : l == 2 ? a[2] : a[3]; };
    scl = pk(sc4), H = pk(h4), W = pk(w4), sy = pk(sy4), sx = pk(sx4);
  } else {
    scl = lv.scale[l], H = lv.h[l], W = lv.w[l], sy = (int)lv.sy[l], sx = (int)lv.sx[l];
  }
  const RoiGeom g = roi_geom_scaled(c, lv, raw, l, scl);
  // tap-list entries: lanes [0, 32) along y, [32, 64) along x; entry e = tap (e & 1 ? hi : lo) of sample e / 2
  const bool isx = lane >= 32;
  const int e = lane & 31;
  const int nl = isx ? 2 * SR * c.pw : 2 * SR * c.ph;
  int trow = -1, tlo = 0x7fffffff, thi = -1;
  float tl = 0.f, th = 0.f;
  if (e < nl) {
    const int s = e >> 1, p = s >> 1, i = s & 1;
    const float v = isx ? g.start_w + (float)p * g.bin_w + ((float)i + 0.5f) * g.bin_w * 0.5f
                        : g.start_h + (float)p * g.bin_h + ((float)i + 0.5f) * g.bin_h * 0.5f;
    const Tap t = make_tap(v, isx ? W : H);
    if (t.valid) trow = (e & 1) ? t.hi : t.lo, tlo = t.lo, thi = t.hi, tl = t.l, th = t.h;
  }
  // the window: the sample positions increase along each axis (start + p bin + (i + 0.5) bin / 2,
  // bin >= 1 / ph) and make_tap is monotonic, so the valid samples are one run of lanes whose first
  // lo and last hi bound it: a ballot and two readlanes per axis (round 5's DPP min / max chains
  // were ~0.4 us of the item's setup latency)
  if (kStamp) t_tap = (int64_t)__builtin_amdgcn_s_memrealtime();
  const uint64_t vm = __ballot(trow >= 0);
  const uint32_t vy = (uint32_t)vm, vx = (uint32_t)(vm >> 32);
  if (!vy || !vx) {  // no valid sample: every bin 0
    for (int u = (int)threadIdx.x; u < nq; u += kNW * kWave)
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, orr, u * 16, 0, kStAux);
    if (kSpan && threadIdx.x == 0) record_span(c, t_start);
    return;
  }
  const int y0 = __builtin_amdgcn_readlane(tlo, __builtin_ctz(vy));
  const int y1 = __builtin_amdgcn_readlane(thi, 31 - __builtin_clz(vy));
  const int x0 = __builtin_amdgcn_readlane(tlo, 32 + __builtin_ctz(vx));
  const int x1 = __builtin_amdgcn_readlane(thi, 63 - __builtin_clz(vx));
  if (kStamp) t_ext = (int64_t)__builtin_amdgcn_s_memrealtime();
  const int nly = 2 * SR * c.ph, nlx = 2 * SR * c.pw;
  const bool dy = y1 - y0 + 1 <= nly, dx = x1 - x0 + 1 <= nlx;  // dense window, else the tap-list entries
  const int R = dy ? y1 - y0 + 1 : nly, Cs = dx ? x1 - x0 + 1 : nlx;
  const bool dax = isx ? dx : dy;
  const int org = isx ? x0 : y0;
  // source byte offset of slab row e (y lanes) / slab column e (x lanes)
  const int src = (dax ? org + min(e, (isx ? Cs : R) - 1) : (trow >= 0 ? trow : org)) * (isx ? sx : sy) * 4;
  // y lanes: the tap-list entry's row (list bands of a dense window, below)
  const int srcl = (trow >= 0 ? trow : org) * sy * 4;
  // sample tables (lane 2 s of each half): slab row / column of the lo tap, hi - lo, l, h (0 when invalid)
  const bool tv = e < nl && trow >= 0 && (e & 1) == 0;
  const int r0 = tv ? (dax ? tlo - org : e) : 0, dr = tv ? (dax ? thi - tlo : 1) : 0;
  if (wave == 0 && (e & 1) == 0 && e < 32)
    tab[(isx ? 16 : 0) + (e >> 1)] = float4{__int_as_float(r0), __int_as_float(dr), tv ? tl : 0.f, tv ? th : 0.f};
  // windows above the slab: bin row p's slab rows [lo, hi] of its valid samples 2 p, 2 p + 1 (y lanes
  // 4 p, 4 p + 2), held by lane p; rows_cap = slab rows of the window's width
  if (kStamp) t_tab = (int64_t)__builtin_amdgcn_s_memrealtime();
  const bool multi = R * Cs > kSlabCells;
  const float rcs = __builtin_amdgcn_rcpf((float)Cs);  // (e + 0.5) * rcs: e / Cs within 3e-4 of a value
                                                       // >= 0.5 / Cs from an integer, for e < 1100
  int brl = 0, brh = -1, rows_cap = kSlabCells;
  if (multi) {
    const int rl = tv ? r0 : 0x7fffffff, rh = tv ? r0 + dr : -1;
    const int pr = min(lane, 15);
    brl = min(__shfl(rl, 4 * pr, kWave), __shfl(rl, 4 * pr + 2, kWave));
    brh = max(__shfl(rh, 4 * pr, kWave), __shfl(rh, 4 * pr + 2, kWave));
    rows_cap = (int)(((float)kSlabCells + 0.5f) * rcs);
  }
  const __amdgpu_buffer_rsrc_t fr =
      uniform_rsrc(lv.feat[l] + (int64_t)g.b * lv.sb[l],
                   ((int64_t)(c.C - 1) + (int64_t)(H - 1) * sy + (int64_t)(W - 1) * sx + 1) * 4);
  const int soff = (int)grp * kCgChan * 4;
  const int q = lane & 15, b4 = lane >> 4;
  f32x4 res[kJ];
#pragma unroll
  for (int j = 0; j < kJ; ++j) res[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int pb = 0;
  while (pb < c.ph) {
    // the band: bin rows [pb, pe) whose valid samples' rows fit rows_cap slab rows
    int rs = 0x7fffffff, re = -1, pe = pb;
    if (!multi) {
      rs = 0, re = R - 1, pe = c.ph;
    } else {
      while (pe < c.ph) {
        const int lo = __builtin_amdgcn_readlane(brl, pe), hi = __builtin_amdgcn_readlane(brh, pe);
        if (hi >= 0) {
          const int nrs = min(rs, lo), nre = max(re, hi);
          if (pe > pb && nre - nrs + 1 > rows_cap) break;
          rs = nrs, re = nre;
        }
        ++pe;
      }
      if (re < 0) rs = re = 0;  // bin rows without a valid sample: any one row (zero weights)
    }
    // a dense window whose single bin row spans more rows than the slab holds (samples far apart
    // with the rows between them clamped or outside: a RoI much larger than its level) is staged
    // as that bin row's 4 tap-list entries instead (cg_ok: 4 rows of the widest window fit)
    const bool lst = multi && dy && re - rs + 1 > rows_cap;
    if (lst) rs = 4 * pb, re = 4 * pb + 3, pe = pb + 1;
    const int nb = (re - rs + 1) * Cs;
    const int nj = (nb + 3) >> 2;
    if (kStamp && n_bands == 0) t_setup = (int64_t)__builtin_amdgcn_s_memrealtime();
    // stage: instruction J (waves take J = wave, wave + kNW, ...): cells 4 J .. 4 J + 3, 16 lanes per cell
    for (int J = wave; J < nj; J += kNW) {
      int cell = 4 * J + b4;
      const bool in = cell < nb;
      cell = in ? cell : 0;
      const int r = (int)(((float)cell + 0.5f) * rcs), cc = cell - r * Cs;
      const int voff = __shfl(lst ? srcl : src, rs + r, kWave) + __shfl(src, 32 + cc, kWave) + q * 16;
      lds_dma_at<16, 0>(fr, sbase + 1024u * (uint32_t)J, in ? voff : 0x40000000, soff);
    }
    wait_vmcnt<0>();
    __syncthreads();  // every wave's DMA (and wave 0's tables) landed
    if (kStamp && n_bands == 0) t_land = (int64_t)__builtin_amdgcn_s_memrealtime();
    ++n_bands;
    // evaluate the 4-bin steps holding bins of bin rows [pb, pe)
    const int bin_lo = pb * c.pw, bin_hi = min(pe * c.pw, nbins);
    const int rsb = rs;
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      const int t = wave + kNW * j;
      if (4 * t + 3 < bin_lo || 4 * t >= bin_hi) continue;  // wave-uniform
      int b4o = b4;
      asm volatile("" : "+v"(b4o));  // per-step bin indices computed here, not hoisted into live registers
      const int bin = 4 * t + b4o;
      const bool act = bin >= bin_lo && bin < bin_hi;
      const int bq = act ? bin : bin_lo;
      const int py = (int)(((uint32_t)bq * ((65536u + (uint32_t)c.pw - 1u) / (uint32_t)c.pw)) >> 16), px = bq - py * c.pw;
      f32x4 Y[2], X[2];
      Y[0] = lds_read_b128<0>(tbase + 32u * (uint32_t)py);
      Y[1] = lds_read_b128<16>(tbase + 32u * (uint32_t)py);
      X[0] = lds_read_b128<256>(tbase + 32u * (uint32_t)px);
      X[1] = lds_read_b128<272>(tbase + 32u * (uint32_t)px);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(Y[0]), "+v"(Y[1]), "+v"(X[0]), "+v"(X[1]) : : "memory");
      uint32_t ra[SR], rd[SR], ca[SR], cd[SR];
#pragma unroll
      for (int i = 0; i < SR; ++i) {
        // list band: sample 2 py + i's lo / hi taps are entries 4 py + 2 i, + 1 (dense tables: rows - rs)
        const int ry = lst ? 4 * py + 2 * i - rsb : max(__float_as_int(Y[i].x) - rsb, 0);
        ra[i] = (uint32_t)(ry * Cs) * 256u;
        rd[i] = (uint32_t)((lst ? 1 : __float_as_int(Y[i].y)) * Cs) * 256u;
        ca[i] = (uint32_t)__float_as_int(X[i].x) * 256u;
        cd[i] = (uint32_t)__float_as_int(X[i].y) * 256u;
      }
      const uint32_t qb = sbase + 16u * (uint32_t)q;
      f32x4 v[2][8];
      auto load = [&](auto hh) {
        constexpr int iy = decltype(hh)::value;
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) {
          const uint32_t a = qb + ra[iy] + ca[ix];
          v[iy][ix * 4 + 0] = lds_read_b128<0>(a);
          v[iy][ix * 4 + 1] = lds_read_b128<0>(a + cd[ix]);
          v[iy][ix * 4 + 2] = lds_read_b128<0>(a + rd[iy]);
          v[iy][ix * 4 + 3] = lds_read_b128<0>(a + rd[iy] + cd[ix]);
        }
      };
      load(std::integral_constant<int, 0>{});
      if constexpr (kLd2) load(std::integral_constant<int, 1>{});
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
      if constexpr (kLd2) lds_wait4<8>(v[0]);
      else lds_wait4<0>(v[0]);
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        const float wq[4] = {Y[0].w * X[ix].w, Y[0].w * X[ix].z, Y[0].z * X[ix].w, Y[0].z * X[ix].z};
        acc = acc + quad_val(wq, &v[0][ix * 4]);
      }
      if constexpr (!kLd2) {
        asm volatile("" : "+v"(acc));  // the first row's sums before the second row's reads: v[0] dies here
        load(std::integral_constant<int, 1>{});
      }
      lds_wait4<0>(v[1]);
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        const float wq[4] = {Y[1].w * X[ix].w, Y[1].w * X[ix].z, Y[1].z * X[ix].w, Y[1].z * X[ix].z};
        acc = acc + quad_val(wq, &v[1][ix * 4]);
      }
      if (act) res[j] = acc * 0.25f;  // count 4: / 4 == * 0.25
    }
    __syncthreads();  // the band's tap reads are done before the next band (or the outputs) overwrite the slab
    pb = pe;
  }
  if (kStamp) t_eval = (int64_t)__builtin_amdgcn_s_memrealtime();
  // outputs: [channel][bin] through the slab, then the contiguous block in 16-B stores
  float* ob = slab;
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const int bin = 4 * (wave + kNW * j) + b4;
    if (bin < nbins) {
      ob[(4 * q + 0) * nbins + bin] = res[j].x;
      ob[(4 * q + 1) * nbins + bin] = res[j].y;
      ob[(4 * q + 2) * nbins + bin] = res[j].z;
      ob[(4 * q + 3) * nbins + bin] = res[j].w;
    }
  }
  __syncthreads();
  const float4* o4 = reinterpret_cast<const float4*>(slab);
  for (int u = (int)threadIdx.x; u < nq; u += kNW * kWave) {
    const float4 v4 = o4[u];
    __builtin_amdgcn_raw_buffer_store_b128(
        u32x4{__float_as_uint(v4.x), __float_as_uint(v4.y), __float_as_uint(v4.z), __float_as_uint(v4.w)}, orr,
        u * 16, 0, kStAux);
  }
  if (kSpan && threadIdx.x == 0) record_span(c, t_start);
  if (kStamp && threadIdx.x == 0) {
    int64_t* st = reinterpret_cast<int64_t*>(out + c.K * c.C * nbins) + (int64_t)w * 16;  // 16 per item
    st[0] = t_start;
    st[1] = t_setup;
    st[2] = t_land;
    st[3] = (int64_t)__builtin_amdgcn_s_memrealtime();
    st[4] = n_bands;
    st[5] = R * Cs;
    st[6] = t_rec;
    st[7] = t_eval;
    st[8] = t_tap;
    st[9] = t_ext;
    st[10] = t_tab;
  }
}

// ---------------------------------------------------------------------------
// The channel-group forward with kItems items per workgroup, software-pipelined (round 6): the
// next item's RoI record, window and sample tables (the ~1.5-2 us setup chain: scalar loads, tap
// math, tables) are computed while the current item's window DMA is in flight, and the slab is
// never idle during a setup.  Tables double-buffered; barriers wait for LDS only (the output
// stores drain in the background).  Item j of workgroup r of XCD x: x * per + r + j * nwx (per
// items per XCD, nwx workgroups per XCD), so the resident workgroups of an XCD stay on nearby
// RoIs of one channel group.  Same evaluation as roi_align_fwd_cg_kernel: bit-identical.
__device__ __forceinline__ void lds_only_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

struct CgItem {  // wave-uniform (SGPRs); the per-lane tables live in LDS (CgTab)
  const float* base;  // image b of the RoI's level
  uint32_t extent;    // feature bytes addressable from base
  int k, grp, state;  // state 0: none, 1: no valid sample (zeros), 2: staged and evaluated
  int R, Cs, dy, multi, rows_cap;
  float rcs;
};

// An item's LDS tables (written by wave 0 in cg_setup): the sample tables (y samples [0, 16), x
// [16, 32): slab row / column of the lo tap, hi - lo, l, h), the source byte offsets of the window
// rows (dense or tap-list) and columns, the tap-list rows (list bands), bin-row row spans.
struct CgTab {
  float4 smp[32];
  int rsrc[32], rsrcl[32], csrc[32];
  int brl[8], brh[8];
};

template <int kSlabCells>
__device__ __forceinline__ void cg_setup(const RoiLevels& lv, const RoiCfg& c, uint32_t w, uint32_t wend, CgTab* tb,
                                         int lane, int wave, CgItem& it) {
  constexpr int SR = 2;
  if (w >= wend) {
    it.state = 0;
    return;
  }
  const uint32_t K32 = (uint32_t)c.K;
  it.grp = (int)(w / K32);
  it.k = (int)(w - (uint32_t)it.grp * K32);
  const RoiRaw raw = roi_fetch(c, (int64_t)it.k);
  const RoiGeom g = roi_geom_raw(c, lv, raw);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int sy = (int)lv.sy[l], sx = (int)lv.sx[l];
  const bool isx = lane >= 32;
  const int e = lane & 31;
  const int nl = isx ? 2 * SR * c.pw : 2 * SR * c.ph;
  int trow = -1, tlo = 0x7fffffff, thi = -1;
  float tl = 0.f, th = 0.f;
  if (e < nl) {
    const int s = e >> 1, p = s >> 1, i = s & 1;
    const float v = isx ? g.start_w + (float)p * g.bin_w + ((float)i + 0.5f) * g.bin_w * 0.5f
                        : g.start_h + (float)p * g.bin_h + ((float)i + 0.5f) * g.bin_h * 0.5f;
    const Tap t = make_tap(v, isx ? W : H);
    if (t.valid) trow = (e & 1) ? t.hi : t.lo, tlo = t.lo, thi = t.hi, tl = t.l, th = t.h;
  }
  const uint64_t vm = __ballot(trow >= 0);
  const uint32_t vy = (uint32_t)vm, vx = (uint32_t)(vm >> 32);
  if (!vy || !vx) {
    it.state = 1;
    return;
  }
  it.state = 2;
  const int y0 = __builtin_amdgcn_readlane(tlo, __builtin_ctz(vy));
  const int y1 = __builtin_amdgcn_readlane(thi, 31 - __builtin_clz(vy));
  const int x0 = __builtin_amdgcn_readlane(tlo, 32 + __builtin_ctz(vx));
  const int x1 = __builtin_amdgcn_readlane(thi, 63 - __builtin_clz(vx));
  const int nly = 2 * SR * c.ph, nlx = 2 * SR * c.pw;
  const bool dy = y1 - y0 + 1 <= nly, dx = x1 - x0 + 1 <= nlx;
  it.dy = dy;
  it.R = dy ? y1 - y0 + 1 : nly;
  it.Cs = dx ? x1 - x0 + 1 : nlx;
  it.multi = it.R * it.Cs > kSlabCells;
  it.rcs = __builtin_amdgcn_rcpf((float)it.Cs);
  it.rows_cap = it.multi ? (int)(((float)kSlabCells + 0.5f) * it.rcs) : kSlabCells;
  it.base = lv.feat[l] + (int64_t)g.b * lv.sb[l];
  it.extent = (uint32_t)(((int64_t)(c.C - 1) + (int64_t)(H - 1) * sy + (int64_t)(W - 1) * sx + 1) * 4);
  if (wave == 0) {
    const bool dax = isx ? dx : dy;
    const int org = isx ? x0 : y0;
    const int src = (dax ? org + min(e, (isx ? it.Cs : it.R) - 1) : (trow >= 0 ? trow : org)) * (isx ? sx : sy) * 4;
    if (isx) {
      tb->csrc[e] = src;
    } else {
      tb->rsrc[e] = src;
      tb->rsrcl[e] = (trow >= 0 ? trow : org) * sy * 4;
    }
    const bool tv = e < nl && trow >= 0 && (e & 1) == 0;
    const int r0 = tv ? (dax ? tlo - org : e) : 0, dr = tv ? (dax ? thi - tlo : 1) : 0;
    if ((e & 1) == 0)
      tb->smp[(isx ? 16 : 0) + (e >> 1)] = float4{__int_as_float(r0), __int_as_float(dr), tv ? tl : 0.f, tv ? th : 0.f};
    if (it.multi) {
      const int rl = tv ? r0 : 0x7fffffff, rh = tv ? r0 + dr : -1;
      const int pr = min(lane, 15);
      const int a = min(__shfl(rl, 4 * pr, kWave), __shfl(rl, 4 * pr + 2, kWave));
      const int b = max(__shfl(rh, 4 * pr, kWave), __shfl(rh, 4 * pr + 2, kWave));
      if (lane < 8) tb->brl[lane] = a, tb->brh[lane] = b;
    }
  }
}

// one item: its bands (staging, evaluation), the output block; hook() runs once, right after
// the first band's DMA is issued (or at once for an item without a valid sample)
template <int kNW, int kSlabCells, int kStAux, bool kLd2, typename Hook>
__device__ __forceinline__ void cg_body(const RoiCfg& c, const CgItem& it, float* __restrict__ out, float* slab,
                                        uint32_t sbase, const CgTab* tb, int lane, int wave, Hook&& hook) {
  const uint32_t tbase = (uint32_t)reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) const float4*)reinterpret_cast<const float4*>(tb->smp));
  constexpr int SR = 2;
  constexpr int kJ = 16 / kNW;
  const int nbins = c.ph * c.pw;
  const int nq = nbins * kCgChan / 4;
  if (it.state == 1) {
    const __amdgpu_buffer_rsrc_t orr =
        uniform_rsrc(out + ((int64_t)it.k * c.C + (int64_t)it.grp * kCgChan) * nbins, (int64_t)nq * 16);
    for (int u = (int)threadIdx.x; u < nq; u += kNW * kWave)
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, orr, u * 16, 0, kStAux);
    hook();
    return;
  }
  const int R = it.R, Cs = it.Cs;
  const float rcs = it.rcs;
  const int soff = it.grp * kCgChan * 4;
  const int q = lane & 15, b4 = lane >> 4;
  f32x4 res[kJ];
#pragma unroll
  for (int j = 0; j < kJ; ++j) res[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int pb = 0;
  bool first = true;
  while (pb < c.ph) {
    int rs = 0x7fffffff, re = -1, pe = pb;
    if (!it.multi) {
      rs = 0, re = R - 1, pe = c.ph;
    } else {
      while (pe < c.ph) {
        const int lo = __builtin_amdgcn_readfirstlane(tb->brl[pe]), hi = __builtin_amdgcn_readfirstlane(tb->brh[pe]);
        if (hi >= 0) {
          const int nrs = min(rs, lo), nre = max(re, hi);
          if (pe > pb && nre - nrs + 1 > it.rows_cap) break;
          rs = nrs, re = nre;
        }
        ++pe;
      }
      if (re < 0) rs = re = 0;
    }
    const bool lst = it.multi && it.dy && re - rs + 1 > it.rows_cap;
    if (lst) rs = 4 * pb, re = 4 * pb + 3, pe = pb + 1;
    const int nb = (re - rs + 1) * Cs;
    const int nj = (nb + 3) >> 2;
    for (int J = wave; J < nj; J += kNW) {
      int cell = 4 * J + b4;
      const bool in = cell < nb;
      cell = in ? cell : 0;
      const int r = (int)(((float)cell + 0.5f) * rcs), cc = cell - r * Cs;
      const int voff = (lst ? tb->rsrcl[rs + r] : tb->rsrc[rs + r]) + tb->csrc[cc] + q * 16;
      lds_dma_at<16, 0>(uniform_rsrc(it.base, (int64_t)it.extent), sbase + 1024u * (uint32_t)J,
                        in ? voff : 0x40000000, soff);
    }
    if (first) {
      hook();  // the next item's setup while this DMA is in flight
      first = false;
    }
    wait_vmcnt<0>();
    lds_only_barrier();  // every wave's DMA (and the tables) landed
    const int bin_lo = pb * c.pw, bin_hi = min(pe * c.pw, nbins);
    const int rsb = rs;
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      const int t = wave + kNW * j;
      if (4 * t + 3 < bin_lo || 4 * t >= bin_hi) continue;
      int b4o = b4;
      asm volatile("" : "+v"(b4o));
      const int bin = 4 * t + b4o;
      const bool act = bin >= bin_lo && bin < bin_hi;
      const int bq = act ? bin : bin_lo;
      const int py = (int)(((uint32_t)bq * ((65536u + (uint32_t)c.pw - 1u) / (uint32_t)c.pw)) >> 16), px = bq - py * c.pw;
      f32x4 Y[2], X[2];
      Y[0] = lds_read_b128<0>(tbase + 32u * (uint32_t)py);
      Y[1] = lds_read_b128<16>(tbase + 32u * (uint32_t)py);
      X[0] = lds_read_b128<256>(tbase + 32u * (uint32_t)px);
      X[1] = lds_read_b128<272>(tbase + 32u * (uint32_t)px);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(Y[0]), "+v"(Y[1]), "+v"(X[0]), "+v"(X[1]) : : "memory");
      uint32_t ra[SR], rd[SR], ca[SR], cd[SR];
#pragma unroll
      for (int i = 0; i < SR; ++i) {
        const int ry = lst ? 4 * py + 2 * i - rsb : max(__float_as_int(Y[i].x) - rsb, 0);
        ra[i] = (uint32_t)(ry * Cs) * 256u;
        rd[i] = (uint32_t)((lst ? 1 : __float_as_int(Y[i].y)) * Cs) * 256u;
        ca[i] = (uint32_t)__float_as_int(X[i].x) * 256u;
        cd[i] = (uint32_t)__float_as_int(X[i].y) * 256u;
      }
      const uint32_t qb = sbase + 16u * (uint32_t)q;
      f32x4 v[2][8];
      auto load = [&](auto hh) {
        constexpr int iy = decltype(hh)::value;
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) {
          const uint32_t a = qb + ra[iy] + ca[ix];
          v[iy][ix * 4 + 0] = lds_read_b128<0>(a);
          v[iy][ix * 4 + 1] = lds_read_b128<0>(a + cd[ix]);
          v[iy][ix * 4 + 2] = lds_read_b128<0>(a + rd[iy]);
          v[iy][ix * 4 + 3] = lds_read_b128<0>(a + rd[iy] + cd[ix]);
        }
      };
      load(std::integral_constant<int, 0>{});
      if constexpr (kLd2) load(std::integral_constant<int, 1>{});
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
      if constexpr (kLd2) lds_wait4<8>(v[0]);
      else lds_wait4<0>(v[0]);
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        const float wq[4] = {Y[0].w * X[ix].w, Y[0].w * X[ix].z, Y[0].z * X[ix].w, Y[0].z * X[ix].z};
        acc = acc + quad_val(wq, &v[0][ix * 4]);
      }
      if constexpr (!kLd2) {
        asm volatile("" : "+v"(acc));
        load(std::integral_constant<int, 1>{});
      }
      lds_wait4<0>(v[1]);
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        const float wq[4] = {Y[1].w * X[ix].w, Y[1].w * X[ix].z, Y[1].z * X[ix].w, Y[1].z * X[ix].z};
        acc = acc + quad_val(wq, &v[1][ix * 4]);
      }
      if (act) res[j] = acc * 0.25f;
    }
    lds_only_barrier();  // the band's tap reads are done before the next band (or the outputs) overwrite the slab
    pb = pe;
  }
  float* ob = slab;
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const int bin = 4 * (wave + kNW * j) + b4;
    if (bin < nbins) {
      ob[(4 * q + 0) * nbins + bin] = res[j].x;
      ob[(4 * q + 1) * nbins + bin] = res[j].y;
      ob[(4 * q + 2) * nbins + bin] = res[j].z;
      ob[(4 * q + 3) * nbins + bin] = res[j].w;
    }
  }
  lds_only_barrier();
  const __amdgpu_buffer_rsrc_t orr =
      uniform_rsrc(out + ((int64_t)it.k * c.C + (int64_t)it.grp * kCgChan) * nbins, (int64_t)nq * 16);
  const float4* o4 = reinterpret_cast<const float4*>(slab);
  for (int u = (int)threadIdx.x; u < nq; u += kNW * kWave) {
    const float4 v4 = o4[u];
    __builtin_amdgcn_raw_buffer_store_b128(
        u32x4{__float_as_uint(v4.x), __float_as_uint(v4.y), __float_as_uint(v4.z), __float_as_uint(v4.w)}, orr,
        u * 16, 0, kStAux);
  }
  lds_only_barrier();  // the output block's reads are done before the next item's DMA overwrites the slab
}

template <int kNW, int kSlabCells, int kItems, int kStAux = kCpolNT, bool kSpan = false, int kWpe = 0,
          bool kLd2 = false>
__global__ void __launch_bounds__(kNW * kWave) __attribute__((amdgpu_waves_per_eu(kWpe > 0 ? kWpe : 1)))
roi_align_fwd_cgp_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out) {
  static_assert(kNW == 2 || kNW == 4 || kNW == 8, "waves per workgroup");
  static_assert(kSlabCells >= 64 && kSlabCells % 4 == 0, "the output block [64][<= 64 bins] leaves through the slab");
  static_assert((kSlabCells + 3) / 4 <= 63 * kNW, "vmcnt is 6 bits");
  const int64_t t_start = kSpan ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  __shared__ __attribute__((aligned(16))) float slab[kSlabCells * kCgChan];
  __shared__ CgTab tab[2];  // double-buffered item tables
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)slab);
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  const uint32_t total = (uint32_t)c.K * ((uint32_t)c.C / kCgChan), per = (total + 7u) / 8u;
  const uint32_t nwx = (per + kItems - 1u) / kItems;  // workgroups per XCD
  const uint32_t x = blockIdx.x & 7u, r = blockIdx.x >> 3;
  const uint32_t wend = min(x * per + per, total);
  uint32_t w = x * per + r;
  CgItem cur, nxt;
  cg_setup<kSlabCells>(lv, c, w, wend, &tab[0], lane, wave, cur);
  lds_only_barrier();  // the first item's tables
  int b = 0;
  for (int j = 0; j < kItems && cur.state; ++j) {
    const uint32_t wn = j + 1 < kItems ? w + nwx : wend;
    nxt.state = 0;
    cg_body<kNW, kSlabCells, kStAux, kLd2>(c, cur, out, slab, sbase, &tab[b], lane, wave, [&] {
      cg_setup<kSlabCells>(lv, c, wn, wend, &tab[b ^ 1], lane, wave, nxt);
    });
    cur = nxt;
    w = wn;
    b ^= 1;
  }
  if (kSpan && threadIdx.x == 0) record_span(c, t_start);
}

// shapes the channel-group kernel takes: channels-last (quad_ok), C % 64 == 0, sampling 2, tap
// lists of <= 32 entries, <= 64 bins, a bin row's 4 tap-list rows of the widest window in the slab
static inline bool cg_ok(int32_t channels, int32_t ph, int32_t pw, int slab_cells) {
  return channels % kCgChan == 0 && 4 * ph <= 32 && 4 * pw <= 32 && ph * pw <= 64 && 4 * 4 * pw <= slab_cells;
}

static __global__ void __launch_bounds__(kRoiThreads) roi_align_bwd_kernel(RoiLevels lv, RoiCfg c,
                                                                    const float* __restrict__ gout) {
  __shared__ Tap ty[kMaxSamplesPerDim], tx[kMaxSamplesPerDim];
  const int64_t k = blockIdx.x;
  const int c0 = blockIdx.y * kRoiChanChunk;
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  fill_taps(g, c, H, W, ty, tx);
  __syncthreads();
  const int nbins = c.ph * c.pw;
  const int nch = min(kRoiChanChunk, c.C - c0);
  const bool tab = taps_fit(g, c);
  float* base = lv.grad[l] + (int64_t)g.b * lv.sb[l];
  const int64_t sy = lv.sy[l], sx = lv.sx[l], scs = lv.sc[l];
  const float* go = gout + (k * c.C + c0) * nbins;
  for (int item = threadIdx.x; item < nch * nbins; item += blockDim.x) {
    const int cl = item / nbins, bin = item - cl * nbins;
    const int py = bin / c.pw, px = bin - py * c.pw;
    float* f = base + (int64_t)(c0 + cl) * scs;
    const float gv = go[item];
    for (int iy = 0; iy < g.gh; ++iy) {
      const Tap a = tab ? ty[py * g.gh + iy] : make_tap(sample_y(g, py, iy), H);
      if (!a.valid) continue;
      for (int ix = 0; ix < g.gw; ++ix) {
        const Tap bx = tab ? tx[px * g.gw + ix] : make_tap(sample_x(g, px, ix), W);
        if (!bx.valid) continue;
        float g1 = gv * (a.h * bx.h) / g.count, g2 = gv * (a.h * bx.l) / g.count;
        float g3 = gv * (a.l * bx.h) / g.count, g4 = gv * (a.l * bx.l) / g.count;
        atomicAdd(&f[a.lo * sy + bx.lo * sx], g1);
        atomicAdd(&f[a.lo * sy + bx.hi * sx], g2);
        atomicAdd(&f[a.hi * sy + bx.lo * sx], g3);
        atomicAdd(&f[a.hi * sy + bx.hi * sx], g4);
      }
    }
  }
}

// Backward, window-accumulated (sampling 2, ph*pw <= 64): the default.  The
// per-tap form above issues 16 scattered global float atomics per (bin, channel)
// -- 205 M for a cfg2 batch, executed at the memory side at a small fraction of
// the coalesced atomic rate (MI355X_MICROARCH.md, global float atomics): 7.7 ms
// per train step.  Here each wave owns 16 channels of one RoI: per channel it
// sums the 16 weighted taps of every bin into an LDS copy of the RoI's tap window
// (ds_add_f32), then adds the window to the feature gradient with one global
// atomic per non-zero cell, lanes along window rows (count = 4 at sampling 2:
// (g * w) / 4 == (g * w) * 0.25 exactly, without the division sequence).  Windows above kBwdSlab
// floats keep the per-tap atomics.  Contributions are the reference's
// grad * w / count; float atomics make the summation order (and the last bits)
// run-dependent, as in torchvision's own CUDA backward.
constexpr int kBwdSlab = 1024;  // floats per wave

static __global__ void __launch_bounds__(kRoiThreads) roi_align_bwd_lds_kernel(RoiLevels lv, RoiCfg c,
                                                                        const float* __restrict__ gout) {
  constexpr int SR = 2, kCh = kRoiChanChunk / (kRoiThreads / kWave);
  __shared__ float slab_all[kRoiThreads / kWave][kBwdSlab];
  const int64_t k = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
  const int cw0 = blockIdx.y * kRoiChanChunk + wave * kCh;
  const int nch = min(kCh, c.C - cw0);
  if (nch <= 0) return;
  float* slab = slab_all[wave];
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw;
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
  if (y1 < y0 || x1 < x0) return;  // no valid tap: no gradient
  const int WW = x1 - x0 + 1, n = (y1 - y0 + 1) * WW;
  const int64_t sy = lv.sy[l], sx = lv.sx[l], scs = lv.sc[l];
  float* gbase = lv.grad[l] + (int64_t)g.b * lv.sb[l] + (int64_t)cw0 * scs;
  const float* go = gout + (k * c.C + cw0) * nbins;
  bool ok[SR][SR];
  float wt[SR][SR][4];
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
    }
  if (n > kBwdSlab) {  // window larger than the slab: per-tap global atomics
    for (int ch = 0; ch < nch; ++ch) {
      const float gv = active ? go[ch * nbins + bin] : 0.0f;
      float* f = gbase + (int64_t)ch * scs;
#pragma unroll
      for (int iy = 0; iy < SR; ++iy)
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) {
          if (!ok[iy][ix]) continue;
          const Tap a = ty[iy], b = tx[ix];
          atomicAdd(&f[a.lo * sy + b.lo * sx], gv * wt[iy][ix][0] / g.count);
          atomicAdd(&f[a.lo * sy + b.hi * sx], gv * wt[iy][ix][1] / g.count);
          atomicAdd(&f[a.hi * sy + b.lo * sx], gv * wt[iy][ix][2] / g.count);
          atomicAdd(&f[a.hi * sy + b.hi * sx], gv * wt[iy][ix][3] / g.count);
        }
    }
    return;
  }
  int cell[SR][SR][4];
#pragma unroll
  for (int iy = 0; iy < SR; ++iy)
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap a = ty[iy], b = tx[ix];
      const int rl = (a.lo - y0) * WW, rh = (a.hi - y0) * WW, cl = b.lo - x0, chh = b.hi - x0;
      cell[iy][ix][0] = rl + cl;
      cell[iy][ix][1] = rl + chh;
      cell[iy][ix][2] = rh + cl;
      cell[iy][ix][3] = rh + chh;
    }
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  const int r0 = lane / WW, col0 = lane - r0 * WW, dr = kWave / WW, dc = kWave - dr * WW;
  for (int ch = 0; ch < nch; ++ch) {
    for (int e = lane; e < n; e += kWave) slab[e] = 0.0f;
    wave_sync();
    const float gv = active ? go[ch * nbins + bin] : 0.0f;
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix)
        if (ok[iy][ix])
#pragma unroll
          for (int q = 0; q < 4; ++q) atomicAdd(&slab[cell[iy][ix][q]], gv * wt[iy][ix][q] * 0.25f);
    wave_sync();
    float* f = gbase + (int64_t)ch * scs;
    int r = r0, col = col0;
    for (int e = lane; e < n; e += kWave) {
      const float v = slab[e];
      if (v != 0.0f) atomicAdd(&f[(int64_t)(y0 + r) * sy + (int64_t)(x0 + col) * sx], v);
      r += dr;
      col += dc;
      if (col >= WW) col -= WW, ++r;
    }
    wave_sync();  // the window is re-zeroed for the next channel only after every lane read it
  }
}

// ---------------------------------------------------------------------------
// Backward, separable tap sums (sampling 2, 4*ph and 4*pw <= 32): the default.
// LDS float atomics (ds_add_f32) run several times slower than plain LDS
// traffic on gfx950 (tools/probe/probe_bwd.py: the same accumulation took 7x
// longer with ds_add_f32 than with a racy read-modify-write), and degenerate
// RoIs (the random-init proposals clamped to the image border: half the cfg2
// RoIs are < 1 px tall) pile all their taps on a few cells, which serialises
// any per-cell scheme.  The taps are separable: cell (y, x) receives
// (g[py][px] * (wy * wx)) * 0.25 for every y tap entry (py, iy, lo|hi) on row y
// and every x tap entry (px, ix, lo|hi) on column x; wy * wx is exactly the
// reference's w1..w4 (hy*hx, hy*lx, ly*hx, ly*lx), so every contribution is the
// reference's grad * w / count.  A wave sorts its RoI's <= 4*ph y entries by
// row and <= 4*pw x entries by column once.  Per channel pair, lane (half h,
// j) owns x entry j of channel h and walks the y entries in row order (a
// uniform loop): it accumulates its contributions, and at the end of each row
// a segmented sum over the lanes of equal column leaves each (row, column)
// cell's total in one lane, which adds it to the feature gradient with one
// global atomic.  No LDS atomics, no divergence; the order of the float sums
// differs from the reference's (float atomics already make it run-dependent,
// as in torchvision's CUDA backward).
constexpr int kSepEnt = 32;  // tap entries per axis and wave half: 4 * ph, 4 * pw <= 32

// kFixed (deterministic backward, frh_roi_align_bwd_fixed): lv.grad[l] points at int64
// accumulators with the gradient's element strides; each (RoI, row, column) sum is added as
// rint(sum * scale) by an integer atomic -- integer adds are associative, so the total is the
// same whatever order the RoIs arrive in (the float-atomic form's order is the scheduler's).
// scale = 2^(62 - hb - E), max|grad_out| < 2^E (the call's own max pass), hb = ceil(log2(K *
// bins)): a cell receives at most max|grad_out| * K * bins, so |total * scale| < 2^62.  A
// non-finite max gives scale -1: no atomics, and the conversion writes NaN.
__device__ __forceinline__ double bwd_fixed_scale(const uint32_t* fix_max, int hb) {
  const uint32_t m = __hip_atomic_load(const_cast<uint32_t*>(fix_max), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (m >= 0x7f800000u) return -1.0;
  const int E = (int)(m >> 23) - 126;  // exponent field 0 (zero / subnormal): < 2^-126
  return ldexp(1.0, 62 - hb - E);
}

// max |g| over n floats as the bits of |g| (monotonic for non-negative floats; NaN above inf):
// a wave max, then a workgroup max in LDS, then ONE atomicMax per workgroup into *out (zeroed by
// the caller's memset).  The grid is small (kAbsmaxBlocks): every atomic lands on one word and
// such atomics serialise at the L2 (a wave-level atomic from 8192 waves cost ~80 us).
constexpr int kAbsmaxBlocks = 256, kAbsmaxThreads = 256;
static __global__ void __launch_bounds__(kAbsmaxThreads) roi_bwd_absmax_kernel(const float* __restrict__ g, int64_t n,
                                                                               uint32_t* out) {
  __shared__ uint32_t wm[kAbsmaxThreads / kWave];
  uint32_t m = 0u;
  const int64_t n4 = (reinterpret_cast<uintptr_t>(g) & 15) == 0 ? n / 4 : 0;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = g4[q];
    m = max(m, max(max(__float_as_uint(v.x) & 0x7fffffffu, __float_as_uint(v.y) & 0x7fffffffu),
                   max(__float_as_uint(v.z) & 0x7fffffffu, __float_as_uint(v.w) & 0x7fffffffu)));
  }
  for (int64_t q = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x)
    m = max(m, __float_as_uint(g[q]) & 0x7fffffffu);
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, kWave));
  if ((threadIdx.x & (kWave - 1)) == 0) wm[threadIdx.x / kWave] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t b = 0u;
    for (int i = 0; i < kAbsmaxThreads / kWave; ++i) b = max(b, wm[i]);
    if (b) atomicMax(out, b);
  }
}

template <bool kFixed = false>
__global__ void __launch_bounds__(kRoiThreads) roi_align_bwd_sep_kernel(RoiLevels lv, RoiCfg c,
                                                                         const float* __restrict__ gout) {
  constexpr int kCh = kRoiChanChunk / (kRoiThreads / kWave);  // channels per wave (even)
  __shared__ int yent_all[kRoiThreads / kWave][kSepEnt];      // row << 16 | py, sorted by (row, entry)
  __shared__ float yw_all[kRoiThreads / kWave][kSepEnt];
  __shared__ int xpos_all[kRoiThreads / kWave][kSepEnt];      // position of each x entry, unsorted
  __shared__ float gv_all[kRoiThreads / kWave][2 * kWave];
  const int64_t k = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
  const int cw0 = blockIdx.y * kRoiChanChunk + wave * kCh;
  const int nch = min(kCh, c.C - cw0);
  if (nch <= 0) return;
  int* yent = yent_all[wave];
  float* yw = yw_all[wave];
  int* xpos = xpos_all[wave];
  float* gv = gv_all[wave];
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int ph = c.ph, pw = c.pw, nbins = ph * pw;
  const int nye = 4 * ph, nxe = 4 * pw;
  const int h = lane >> 5, j = lane & 31;
  // tap entry e of an axis: sample e / 2 (bin e / 4, sub-sample (e / 2) & 1), lo (e even) or hi
  auto entry = [&](int e, float start, float bin, int size, int* pos, float* w) {
    const Tap t = make_tap(start + (float)(e >> 2) * bin + ((float)((e >> 1) & 1) + 0.5f) * bin * 0.5f, size);
    *pos = t.valid ? ((e & 1) ? t.hi : t.lo) : -1;
    *w = (e & 1) ? t.l : t.h;
  };
  int yp, xp;
  float ywv, xwv;
  entry(j, g.start_h, g.bin_h, H, &yp, &ywv);
  entry(j, g.start_w, g.bin_w, W, &xp, &xwv);
  if (j >= nye) yp = -1;
  if (j >= nxe) xp = -1;
  if (h == 0) xpos[j] = xp < 0 ? (1 << 20) : xp;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // x entries: rank by (col, entry); lane (h, j) takes the j-th in column order
  int xrank = 0;
  for (int e = 0; e < nxe; ++e) {
    const int pe = xpos[e], pm = xpos[j];
    xrank += (pe < pm || (pe == pm && e < j)) ? 1 : 0;
  }
  // y entries: rank by (row, entry), written sorted
  {
    int yrank = 0;
    const int pm = yp < 0 ? (1 << 20) : yp;
    for (int e = 0; e < nye; ++e) {
      const int pe = __shfl(yp < 0 ? (1 << 20) : yp, e, kWave);
      yrank += (pe < pm || (pe == pm && e < j)) ? 1 : 0;
    }
    if (h == 0 && j < nye && yp >= 0) {
      yent[yrank] = (yp << 16) | (j >> 2);
      yw[yrank] = ywv;
    }
  }
  int nyv = 0, nxv = 0;  // valid entries (uniform)
  {
    const uint64_t my = __ballot(h == 0 && yp >= 0), mx = __ballot(h == 0 && xp >= 0);
    nyv = __popcll(my);
    nxv = __popcll(mx);
  }
  if (nyv == 0 || nxv == 0) return;  // no valid tap: no gradient
  // this lane's x entry (column order) and the segment of lanes sharing its column
  int my_col = -1, my_px = 0;
  float my_wx = 0.0f;
  // scatter the x entries into column order through LDS
  __shared__ int xs_all[kRoiThreads / kWave][kSepEnt];
  __shared__ float xw_all[kRoiThreads / kWave][kSepEnt];
  int* xs = xs_all[wave];
  float* xw = xw_all[wave];
  if (h == 0 && xp >= 0) {
    xs[xrank] = (xp << 16) | (j >> 2);
    xw[xrank] = xwv;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const bool xv = j < nxv;
  if (xv) {
    my_col = xs[j] >> 16;
    my_px = xs[j] & 0xffff;
    my_wx = xw[j];
  }
  // segment of equal columns within the half: [j - lead, j + trail]
  int trail = 0;
  for (int d = 1; d < kSepEnt; ++d) {
    const int jj = j + d;
    if (jj < nxv && (xs[jj] >> 16) == my_col) trail = d;
  }
  const bool head = xv && (j == 0 || (xs[j - 1] >> 16) != my_col);
  const int64_t sy = lv.sy[l], sx = lv.sx[l], scs = lv.sc[l];
  const int64_t goff0 = (int64_t)g.b * lv.sb[l] + (int64_t)cw0 * scs;
  const float* go = gout + (k * c.C + cw0) * nbins;
  const double fscale = kFixed ? bwd_fixed_scale(c.fix_max, c.fix_hb) : 0.0;
  if (kFixed && fscale < 0.0) return;  // non-finite gradient: the conversion writes NaN
  for (int ch = 0; ch < nch; ch += 2) {
    // grad_out of channels ch, ch + 1 (a missing odd last channel reads 0 and is not written)
    for (int e = lane; e < 2 * nbins; e += kWave) {
      const int hh = e >= nbins ? 1 : 0;
      gv[hh * kWave + (e - hh * nbins)] = (ch + hh < nch) ? go[(ch + hh) * nbins + (e - hh * nbins)] : 0.0f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int64_t fo = goff0 + (int64_t)(ch + h) * scs;
    const bool live = xv && ch + h < nch;
    float acc = 0.0f;
    for (int i = 0; i < nyv; ++i) {
      const int ye = yent[i];
      const int row = ye >> 16, py = ye & 0xffff;
      const float wy = yw[i];
      const float gvv = gv[h * kWave + py * pw + my_px];
      acc = acc + (live ? gvv * (wy * my_wx) * 0.25f : 0.0f);  // (g * w) / count, count = 4
      if (i + 1 == nyv || (yent[i + 1] >> 16) != row) {  // end of this row's entries (uniform)
        float sum = acc;
#pragma unroll
        for (int d = 1; d < kSepEnt; d <<= 1) {
          const float t = __shfl_down(sum, d, 32);
          if (d <= trail) sum = sum + t;
        }
        if (head && live && sum != 0.0f) {
          const int64_t e = fo + (int64_t)row * sy + (int64_t)my_col * sx;
          if constexpr (kFixed)
            atomicAdd(reinterpret_cast<unsigned long long*>(lv.grad[l]) + e,
                      (unsigned long long)(long long)rint((double)sum * fscale));
          else
            atomicAdd(lv.grad[l] + e, sum);
        }
        acc = 0.0f;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ---------------------------------------------------------------------------
// Backward for channels-last gradients (unit channel stride: the product trunk's FPN
// levels), sampling 2, ph, pw <= 8 (round 5).  The separable sums of roi_align_bwd_sep_kernel
// with the lanes turned: one wave per (RoI, 64 channels), lane = channel, so every gradient
// atomic is one coalesced 256-B run (512 B in fixed point) of a cell's channels instead of
// one 4-B add per line (the sep kernel's lanes are the window's columns, C * 4 bytes apart in
// NHWC: 0.7-2.7 ms per cfg2 backward).  The RoI's 4 ph y and 4 pw x tap entries are sorted by
// row / column once (wave-uniform lists in LDS); per row, R[px] = sum of wy * g[py][px] over
// the row's y entries, then per column cell = 0.25 * sum of wx * R[px] over the column's x
// entries -- mathematically the reference's sum of g * (wy * wx) / count, in another order
// (float atomics are run-order dependent anyway; the fixed-point form is order-independent).
// kNW (round 6): a workgroup of kNW waves per (RoI, 64 channels) sharing the staged grad_out and
// the sorted tap lists; wave w takes the RoI's distinct tap rows w, w + kNW, ... (the row loop was
// one wave's serial chain -- 28 rows x 28 column entries on VOC-sized windows).  Each cell's sum
// is the same as with one wave (same entries, same order): bit-identical per cell.
template <bool kFixed = false, int kNW = 1>
__global__ void __launch_bounds__(kNW * kWave) roi_align_bwd_nhwc_kernel(RoiLevels lv, RoiCfg c,
                                                                       const float* __restrict__ gout) {
  constexpr int kMaxP = 8;
  __shared__ __attribute__((aligned(16))) float gs[kMaxP * kMaxP * kWave];  // grad_out of the 64 channels, [lane][bin]
  __shared__ float rs_all[kNW][kMaxP * kWave];  // each wave's current row sums, [px][lane]
  __shared__ int ye[kSepEnt], xe[kSepEnt];      // sorted tap entries: position << 16 | bin index
  __shared__ float yws[kSepEnt], xws[kSepEnt];
  const int64_t k = blockIdx.x;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = kNW == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  float* rs = rs_all[wave];
  const int c0 = blockIdx.y * kWave, ch = c0 + lane;
  const bool live = ch < c.C;
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl, H = lv.h[l], W = lv.w[l];
  const int ph = c.ph, pw = c.pw, nbins = ph * pw, nye = 4 * ph, nxe = 4 * pw;
  {  // [K][C][bins]: the 64 channels are one contiguous run, staged as it lies ([lane][bin]) by
     // LDS-DMA, 256 B per instruction, every instruction in flight together (round 6: a load ->
     // LDS-store loop left one global round trip per bin in series); channels past C read 0
    const float* go = gout + (k * c.C + c0) * nbins;
    const int nvalid = min(kWave, c.C - c0) * nbins;
    const __amdgpu_buffer_rsrc_t gr = uniform_rsrc(go, (int64_t)nvalid * 4);
    const uint32_t gsb = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)gs);
    for (int i0 = wave; i0 < nbins; i0 += 32 * kNW) {
      for (int i = i0; i < min(nbins, i0 + 32 * kNW); i += kNW)
        lds_dma_at<4, 0>(gr, gsb + 256u * (uint32_t)i, lane * 4, i * 256);
      wait_vmcnt<0>();
    }
  }
  // tap entry e of an axis: sample e / 2 (bin e / 4, sub-sample (e / 2) & 1), lo (e even) or hi
  auto entry = [&](int e, float start, float bin, int size, int* pos, float* w) {
    const Tap t = make_tap(start + (float)(e >> 2) * bin + ((float)((e >> 1) & 1) + 0.5f) * bin * 0.5f, size);
    *pos = t.valid ? ((e & 1) ? t.hi : t.lo) : -1;
    *w = (e & 1) ? t.l : t.h;
  };
  int yp = -1, xp = -1;
  float ywv = 0.0f, xwv = 0.0f;
  if (lane < nye) entry(lane, g.start_h, g.bin_h, H, &yp, &ywv);
  if (lane < nxe) entry(lane, g.start_w, g.bin_w, W, &xp, &xwv);
  if (lane >= nye) yp = -1;
  if (lane >= nxe) xp = -1;
  const int nyv = __popcll(__ballot(yp >= 0)), nxv = __popcll(__ballot(xp >= 0));
  if (wave == 0) {
    const int ypm = yp < 0 ? (1 << 20) : yp, xpm = xp < 0 ? (1 << 20) : xp;
    int yr = 0, xr = 0;  // rank by (position, entry)
    for (int e = 0; e < nye; ++e) {
      const int pe = __shfl(ypm, e, kWave);
      yr += (pe < ypm || (pe == ypm && e < lane)) ? 1 : 0;
    }
    for (int e = 0; e < nxe; ++e) {
      const int pe = __shfl(xpm, e, kWave);
      xr += (pe < xpm || (pe == xpm && e < lane)) ? 1 : 0;
    }
    if (yp >= 0) ye[yr] = (yp << 16) | (lane >> 2), yws[yr] = ywv;
    if (xp >= 0) xe[xr] = (xp << 16) | (lane >> 2), xws[xr] = xwv;
  }
  if constexpr (kNW > 1) {
    __syncthreads();  // the staged grad_out (every wave's DMA) and wave 0's sorted lists
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (nyv == 0 || nxv == 0) return;  // no valid tap: no gradient (uniform over the workgroup)
  const int64_t base = (int64_t)g.b * lv.sb[l] + ch, sy = lv.sy[l], sx = lv.sx[l];
  const double fscale = kFixed ? bwd_fixed_scale(c.fix_max, c.fix_hb) : 0.0;
  if (kFixed && fscale < 0.0) return;  // non-finite gradient: the conversion writes NaN
  float R[kMaxP];
#pragma unroll
  for (int px = 0; px < kMaxP; ++px) R[px] = 0.0f;
  int ro = 0;  // ordinal of the current distinct row: this wave's rows are ro % kNW == wave
  for (int i = 0; i < nyv; ++i) {
    const int yv = ye[i], row = yv >> 16, py = yv & 0xffff;
    const bool mine = kNW == 1 || ro % kNW == wave;
    if (mine) {
      const float wy = yws[i];
#pragma unroll
      for (int px = 0; px < kMaxP; ++px)
        if (px < pw) R[px] = R[px] + wy * gs[lane * nbins + py * pw + px];
    }
    if (i + 1 < nyv && (ye[i + 1] >> 16) == row) continue;  // the row continues (uniform)
    ++ro;
    if (!mine) continue;
#pragma unroll
    for (int px = 0; px < kMaxP; ++px)  // the lane's own slots: no wave sync needed
      if (px < pw) rs[px * kWave + lane] = R[px], R[px] = 0.0f;
    float acc = 0.0f;
    for (int jx = 0; jx < nxv; ++jx) {
      const int xv = xe[jx], col = xv >> 16, px = xv & 0xffff;
      acc = acc + xws[jx] * rs[px * kWave + lane];
      if (jx + 1 < nxv && (xe[jx + 1] >> 16) == col) continue;
      const float v = acc * 0.25f;  // / count (4 samples)
      acc = 0.0f;
      if (!live || v == 0.0f) continue;
      const int64_t e = base + (int64_t)row * sy + (int64_t)col * sx;
      if constexpr (kFixed)
        atomicAdd(reinterpret_cast<unsigned long long*>(lv.grad[l]) + e,
                  (unsigned long long)(long long)rint((double)v * fscale));
      else
        atomicAdd(lv.grad[l] + e, v);
    }
  }
}

// The channels-last backward with the tap lists in registers (round 6): the sorted y / x tap
// entries sit one per lane and are read by v_readlane with the wave-uniform loop index (a
// scalar, no LDS round trip), the row sums R[px] stay in registers and the column loop picks
// R[px] by a uniform select -- the round-5 kernel read each x entry, its weight and R[px]
// from LDS in a dependent chain (two LDS round trips per (row, column) pair: ~50 us of serial
// latency per wave on VOC-sized windows).  Same sums in the same order: each cell's
// contribution is bit-identical to roi_align_bwd_nhwc_kernel's.
// kStore (tools-only diagnostic): plain stores instead of the atomics (wrong sums): the kernel's
// time without the atomic traffic; kDiag (tools-only): 1 = no column loop (the row sums stored),
// 2 = return after the tap-entry setup
template <bool kFixed = false, bool kStore = false, int kDiag = 0>
__global__ void __launch_bounds__(kWave) roi_align_bwd_nhwc2_kernel(RoiLevels lv, RoiCfg c,
                                                                  const float* __restrict__ gout) {
  constexpr int kMaxP = 8;
  __shared__ __attribute__((aligned(16))) float gs[kMaxP * kMaxP * kWave];  // grad_out, [lane][bin]
  __shared__ int ye[kSepEnt], xe[kSepEnt];     // sorted tap entries: position << 16 | bin index
  __shared__ float yws[kSepEnt], xws[kSepEnt];
  const int64_t k = blockIdx.x;
  const int lane = threadIdx.x;
  const int c0 = blockIdx.y * kWave, ch = c0 + lane;
  const bool live = ch < c.C;
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl, H = lv.h[l], W = lv.w[l];
  const int ph = c.ph, pw = c.pw, nbins = ph * pw, nye = 4 * ph, nxe = 4 * pw;
  {  // the wave's contiguous [64][bins] grad_out block by LDS-DMA (as roi_align_bwd_nhwc_kernel)
    const float* go = gout + (k * c.C + c0) * nbins;
    const int nvalid = min(kWave, c.C - c0) * nbins;
    const __amdgpu_buffer_rsrc_t gr = uniform_rsrc(go, (int64_t)nvalid * 4);
    const uint32_t gsb = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)gs);
    for (int i0 = 0; i0 < nbins; i0 += 32) {
      const int i1 = min(nbins, i0 + 32);
      for (int i = i0; i < i1; ++i) lds_dma_at<4, 0>(gr, gsb + 256u * (uint32_t)i, lane * 4, i * 256);
      wait_vmcnt<0>();
    }
  }
  auto entry = [&](int e, float start, float bin, int size, int* pos, float* w) {
    const Tap t = make_tap(start + (float)(e >> 2) * bin + ((float)((e >> 1) & 1) + 0.5f) * bin * 0.5f, size);
    *pos = t.valid ? ((e & 1) ? t.hi : t.lo) : -1;
    *w = (e & 1) ? t.l : t.h;
  };
  int yp = -1, xp = -1;
  float ywv = 0.0f, xwv = 0.0f;
  if (lane < nye) entry(lane, g.start_h, g.bin_h, H, &yp, &ywv);
  if (lane < nxe) entry(lane, g.start_w, g.bin_w, W, &xp, &xwv);
  if (lane >= nye) yp = -1;
  if (lane >= nxe) xp = -1;
  const int ypm = yp < 0 ? (1 << 20) : yp, xpm = xp < 0 ? (1 << 20) : xp;
  int yr = 0, xr = 0;  // rank by (position, entry)
  for (int e = 0; e < nye; ++e) {
    const int pe = __shfl(ypm, e, kWave);
    yr += (pe < ypm || (pe == ypm && e < lane)) ? 1 : 0;
  }
  for (int e = 0; e < nxe; ++e) {
    const int pe = __shfl(xpm, e, kWave);
    xr += (pe < xpm || (pe == xpm && e < lane)) ? 1 : 0;
  }
  if (yp >= 0) ye[yr] = (yp << 16) | (lane >> 2), yws[yr] = ywv;
  if (xp >= 0) xe[xr] = (xp << 16) | (lane >> 2), xws[xr] = xwv;
  const int nyv = __popcll(__ballot(yp >= 0)), nxv = __popcll(__ballot(xp >= 0));
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (nyv == 0 || nxv == 0) return;  // no valid tap: no gradient
  if (kDiag == 2) {
    if (ye[0] == 0x7fffffff) lv.grad[l][lane] = 1.0f;  // keep the setup alive
    return;
  }
  // lane i holds sorted entry i of each axis (read by v_readlane below)
  const int ye_l = lane < kSepEnt ? ye[lane] : 0, xe_l = lane < kSepEnt ? xe[lane] : 0;
  const float yw_l = lane < kSepEnt ? yws[lane] : 0.0f, xw_l = lane < kSepEnt ? xws[lane] : 0.0f;
  const int64_t base = (int64_t)g.b * lv.sb[l] + ch, sy = lv.sy[l], sx = lv.sx[l];
  const double fscale = kFixed ? bwd_fixed_scale(c.fix_max, c.fix_hb) : 0.0;
  if (kFixed && fscale < 0.0) return;  // non-finite gradient: the conversion writes NaN
  float R[kMaxP];
#pragma unroll
  for (int px = 0; px < kMaxP; ++px) R[px] = 0.0f;
  for (int i = 0; i < nyv; ++i) {
    const int yv = __builtin_amdgcn_readlane(ye_l, i), row = yv >> 16, py = yv & 0xffff;
    const float wy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(yw_l), i));
    const float* gr = gs + lane * nbins + py * pw;
#pragma unroll
    for (int px = 0; px < kMaxP; ++px)
      if (px < pw) R[px] = R[px] + wy * gr[px];
    if (i + 1 < nyv && (__builtin_amdgcn_readlane(ye_l, i + 1) >> 16) == row) continue;  // the row continues
    if (kDiag == 1) {
      float t = 0.0f;
#pragma unroll
      for (int px = 0; px < kMaxP; ++px) t = t + R[px], R[px] = 0.0f;
      if (live) __builtin_nontemporal_store(t, lv.grad[l] + base + (int64_t)row * sy);
      continue;
    }
    float acc = 0.0f;
    for (int jx = 0; jx < nxv; ++jx) {
      const int xv = __builtin_amdgcn_readlane(xe_l, jx), col = xv >> 16, px = xv & 0xffff;
      const float wx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xw_l), jx));
      float r = R[0];
#pragma unroll
      for (int q = 1; q < kMaxP; ++q) r = px == q ? R[q] : r;  // uniform select
      acc = acc + wx * r;
      if (jx + 1 < nxv && (__builtin_amdgcn_readlane(xe_l, jx + 1) >> 16) == col) continue;
      const float v = acc * 0.25f;  // / count (4 samples)
      acc = 0.0f;
      if (!live || v == 0.0f) continue;
      const int64_t e = base + (int64_t)row * sy + (int64_t)col * sx;
      if constexpr (kStore)
        __builtin_nontemporal_store(v, lv.grad[l] + e);
      else if constexpr (kFixed)
        atomicAdd(reinterpret_cast<unsigned long long*>(lv.grad[l]) + e,
                  (unsigned long long)(long long)rint((double)v * fscale));
      else
        atomicAdd(lv.grad[l] + e, v);
    }
#pragma unroll
    for (int px = 0; px < kMaxP; ++px) R[px] = 0.0f;
  }
}

// the fixed-point accumulators to the f32 gradient, element by element (dense buffers)
static __global__ void roi_bwd_fixed_to_f32_kernel(const long long* __restrict__ acc, float* __restrict__ grad, int64_t n,
                                                   const uint32_t* fix_max, int hb) {
  const double s = bwd_fixed_scale(fix_max, hb);
  const double inv = s > 0.0 ? 1.0 / s : (double)NAN;  // 1 / 2^k is exact
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x)
    grad[q] = (float)((double)acc[q] * inv);
}

// ---------------------------------------------------------------------------
// Channels-last forward (features with unit channel stride: the FPN's NHWC outputs).
// One wave per (RoI, 64 channels), lane = channel: every tap is wave-uniform, so the
// sample geometry is computed once per wave (14 y- and 14 x-samples, one lane each,
// broadcast by v_readlane) and every feature access is a 256-B run of one cell's
// channels.  The RoI's tap cells (the dense window [y0, y1] x [x0, x1], or per axis the
// 2 * 2 * P (lo, hi) tap list when the window is wider -- as the pair kernel) are staged
// into the wave's LDS slab by 16-B LDS-DMA, one 1-KB instruction per 4 cells (full
// 128-B lines); a window with more than kCells cells is staged in bands of slab rows,
// each band holding whole sample rows.  Each sample's four taps are ds_read_b32 of
// consecutive channels (conflict-free); the bilinear sums run per lane in torchvision's
// operation order, so the result is bit-identical to the other kernels.  The 7 x 7
// outputs of the lane's channel collect in VGPRs and leave through the slab, transposed
// to [channel][bin], as 16-B stores of one contiguous 12.5-KB block.
constexpr int kNhwcGroup = 64;  // channels per wave

// kRegOut: the outputs stay in VGPRs until the end (LDS = the slab only) instead of a
// separate [channel][bin] LDS buffer.  kStamp (tools-only timing builds): lane 0 writes 8
// int64 per item after the output -- s_memrealtime at start / prologue done / first band
// landed / eval done / end, bands staged, cells of the first band, XCD.
template <int PH, int PW, int kCells, int kStAux, bool kRegOut = true, bool kStamp = false>
__global__ void __launch_bounds__(kWave) roi_align_fwd_nhwc_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out) {
  const int64_t t_start = kStamp ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  int64_t t_pro = 0, t_land = 0, t_eval = 0;
  int n_bands = 0, first_cells = 0;
  static_assert(2 * PH <= 32 && 2 * PW <= 32 && kCells % 4 == 0 && kCells >= 2 * 4 * PW, "tap lanes / DMA rounds");
  static_assert(!kRegOut || kCells >= PH * PW, "the outputs leave through the slab");
  constexpr int NLY = 4 * PH, NLX = 4 * PW;  // tap-list lengths
  constexpr int NB = PH * PW;
  __shared__ __attribute__((aligned(16))) float slab[kCells * kNhwcGroup];
  __shared__ __attribute__((aligned(16))) float obuf[kRegOut ? 4 : kNhwcGroup * NB];  // [channel][bin]
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)slab);
  const int lane = threadIdx.x;
  // XCD x (= workgroup id mod 8) walks the x-th eighth of the group-major (group, RoI) list
  const uint32_t G = (uint32_t)c.C / kNhwcGroup, K32 = (uint32_t)c.K;
  const uint32_t total = K32 * G, per = (total + 7u) / 8u;
  const uint32_t w = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  if (w >= min((blockIdx.x & 7u) * per + per, total)) return;
  const int grp = (int)(w / K32);
  const int64_t k = (int64_t)(w - (uint32_t)grp * K32);
  const RoiRaw raw = roi_fetch(c, k);
  const RoiGeom g = roi_geom_raw(c, lv, raw);
  const int l = g.lvl, H = lv.h[l], W = lv.w[l];
  // lane s < 2 PH: y sample s (bin s / 2, sub-sample s % 2); lane 32 + s < 32 + 2 PW: x sample s
  const bool isy = lane < 2 * PH, isx = lane >= 32 && lane < 32 + 2 * PW;
  const int s = isy ? lane : lane - 32;
  Tap t{0, 0, 0.f, 0.f, 0};
  if (isy || isx) {
    const float st = isy ? g.start_h : g.start_w, bn = isy ? g.bin_h : g.bin_w;
    t = make_tap(st + (float)(s >> 1) * bn + ((float)(s & 1) + 0.5f) * bn * 0.5f, isy ? H : W);
  }
  const bool tv = (isy || isx) && t.valid;
  const int y0 = __builtin_amdgcn_readfirstlane(wave_min_i32(isy && tv ? t.lo : 1 << 30));
  const int y1 = __builtin_amdgcn_readfirstlane(wave_max_i32(isy && tv ? t.hi : -1));
  const int x0 = __builtin_amdgcn_readfirstlane(wave_min_i32(isx && tv ? t.lo : 1 << 30));
  const int x1 = __builtin_amdgcn_readfirstlane(wave_max_i32(isx && tv ? t.hi : -1));
  float* o = out + (k * c.C + (int64_t)grp * kNhwcGroup) * NB;  // [64][NB], contiguous
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(o, (int64_t)kNhwcGroup * NB * 4);
  if (!(y1 >= y0 && x1 >= x0)) {  // no valid sample: every bin is 0
    for (int e = lane; e < kNhwcGroup * NB / 4; e += kWave)
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, orr, e * 16, 0, kStAux);
    return;
  }
  const bool dy = y1 - y0 + 1 <= NLY, dx = x1 - x0 + 1 <= NLX;
  const int R = dy ? y1 - y0 + 1 : NLY, Cs = dx ? x1 - x0 + 1 : NLX;
  // per-lane sample data: slab indices (row of y sample / column of x sample) and factors,
  // zeroed (and pointed at index 0) for invalid samples
  const int i0 = !tv ? 0 : (isy ? (dy ? t.lo - y0 : 2 * s) : (dx ? t.lo - x0 : 2 * s));
  const int i1 = !tv ? 0 : (isy ? (dy ? t.hi - y0 : 2 * s + 1) : (dx ? t.hi - x0 : 2 * s + 1));
  const float fl = tv ? t.l : 0.f, fh = tv ? t.h : 0.f;
  // tap-list source rows / columns: list entry e of an axis is tap (e & 1 ? hi : lo) of sample e / 2
  // (the source lane supplies both taps; the destination picks by its own parity)
  const int ysrc_e = (lane < NLY) ? lane : 0, xsrc_e = (lane < NLX) ? lane : 0;
  const int ylo_s = __shfl(tv ? t.lo : y0, ysrc_e >> 1, kWave), yhi_s = __shfl(tv ? t.hi : y0, ysrc_e >> 1, kWave);
  const int xlo_s = __shfl(tv ? t.lo : x0, 32 + (xsrc_e >> 1), kWave);
  const int xhi_s = __shfl(tv ? t.hi : x0, 32 + (xsrc_e >> 1), kWave);
  const int ysrc = (ysrc_e & 1) ? yhi_s : ylo_s, xsrc = (xsrc_e & 1) ? xhi_s : xlo_s;
  const int64_t sy = lv.sy[l], sx = lv.sx[l];
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l];
  const __amdgpu_buffer_rsrc_t fr =
      uniform_rsrc(base, ((int64_t)(H - 1) * sy + (int64_t)(W - 1) * sx + c.C) * 4);
  const int rows_cap = kCells / Cs;  // >= 2: Cs <= NLX
  const uint32_t inv = (65536u + (uint32_t)Cs - 1u) / (uint32_t)Cs;  // e / Cs for e < 1024
  const int quad = (lane & 15) * 16, soff = grp * kNhwcGroup * 4;
  int band_lo = 0, band_hi = 0;
  if (kStamp) t_pro = (int64_t)__builtin_amdgcn_s_memrealtime();
  // sample row sr (in order): stage its band if needed, then acc[px] += its two samples of each bin column
  auto row = [&](int sr, float (&acc)[PW]) {
    // opaque copies: the broadcasts are re-read per row, not hoisted into ~60 live SGPRs
    int a0 = i0, a1 = i1, av = tv;
    float al = fl, ah = fh;
    asm volatile("" : "+v"(a0), "+v"(a1), "+v"(av), "+v"(al), "+v"(ah));
    int r0 = __builtin_amdgcn_readlane(a0, sr), r1 = __builtin_amdgcn_readlane(a1, sr);
    const float ly = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(al), sr));
    const float hy = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(ah), sr));
    if (!__builtin_amdgcn_readlane(av, sr) && band_hi > band_lo) r0 = r1 = band_lo;  // zero weights: any cell
    if (r0 < band_lo || r1 >= band_hi) {  // stage the band of slab rows [r0, r0 + rows_cap)
      band_lo = r0;
      band_hi = min(r0 + rows_cap, R);
      const int ncell = (band_hi - band_lo) * Cs;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the previous band's tap reads are done
      __builtin_amdgcn_wave_barrier();
      for (int i = 0; 4 * i < ncell; ++i) {
        int e = 4 * i + (lane >> 4);
        e = e < ncell ? e : ncell - 1;
        const int rr = (int)(((uint32_t)e * inv) >> 16), cc = e - rr * Cs;
        const int yy = dy ? y0 + band_lo + rr : __shfl(ysrc, band_lo + rr, kWave);
        const int xx = dx ? x0 + cc : __shfl(xsrc, cc, kWave);
        lds_dma_at<16, 0>(fr, sbase + 1024u * (uint32_t)i, (int)(((int64_t)yy * sy + (int64_t)xx * sx) * 4) + quad,
                          soff);
      }
      wait_vmcnt<0>();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (kStamp) {
        if (n_bands == 0) t_land = (int64_t)__builtin_amdgcn_s_memrealtime(), first_cells = ncell;
        ++n_bands;
      }
    }
    const float* row0 = slab + (r0 - band_lo) * Cs * kNhwcGroup + lane;
    const float* row1 = slab + (r1 - band_lo) * Cs * kNhwcGroup + lane;
#pragma unroll
    for (int ix = 0; ix < 2 * PW; ++ix) {
      const int q0 = __builtin_amdgcn_readlane(a0, 32 + ix) * kNhwcGroup;
      const int q1 = __builtin_amdgcn_readlane(a1, 32 + ix) * kNhwcGroup;
      const float lx = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(al), 32 + ix));
      const float hx = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(ah), 32 + ix));
      const float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
      const float val = ((w1 * row0[q0] + w2 * row0[q1]) + w3 * row1[q0]) + w4 * row1[q1];
      acc[ix >> 1] = acc[ix >> 1] + val;
    }
  };
  float* ob = kRegOut ? slab : obuf;  // [channel][bin]
  if constexpr (kRegOut) {
    // the 7 x 7 outputs of this lane's channel in VGPRs: a dynamic bin-row loop shifts each
    // row's results into the tail of outv (static indices only), then out through the slab
    float outv[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) outv[j] = 0.0f;
    for (int py = 0; py < PH; ++py) {
      float acc[PW];
#pragma unroll
      for (int px = 0; px < PW; ++px) acc[px] = 0.0f;
      row(2 * py, acc);
      row(2 * py + 1, acc);
#pragma unroll
      for (int j = 0; j < NB - PW; ++j) outv[j] = outv[j + PW];
#pragma unroll
      for (int px = 0; px < PW; ++px) outv[NB - PW + px] = acc[px] * 0.25f;  // count 4: / 4 == * 0.25
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < NB; ++j) ob[lane * NB + j] = outv[j];  // stride NB (odd): no bank conflicts
  } else {
    for (int py = 0; py < PH; ++py) {
      float acc[PW];
#pragma unroll
      for (int px = 0; px < PW; ++px) acc[px] = 0.0f;
      row(2 * py, acc);
      row(2 * py + 1, acc);
#pragma unroll
      for (int px = 0; px < PW; ++px) ob[lane * NB + py * PW + px] = acc[px] * 0.25f;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (kStamp) t_eval = (int64_t)__builtin_amdgcn_s_memrealtime();
  const float4* s4 = reinterpret_cast<const float4*>(ob);
  for (int e = lane; e < kNhwcGroup * NB / 4; e += kWave) {
    const float4 q = s4[e];
    __builtin_amdgcn_raw_buffer_store_b128(
        u32x4{__float_as_uint(q.x), __float_as_uint(q.y), __float_as_uint(q.z), __float_as_uint(q.w)}, orr, e * 16, 0,
        kStAux);
  }
  if (kStamp && lane == 0) {
    int64_t* st = reinterpret_cast<int64_t*>(out + c.K * c.C * NB) + (int64_t)w * 8;
    st[0] = t_start;
    st[1] = t_pro;
    st[2] = t_land;
    st[3] = t_eval;
    st[4] = (int64_t)__builtin_amdgcn_s_memrealtime();
    st[5] = n_bands;
    st[6] = first_cells;
    st[7] = blockIdx.x & 7;
  }
}

static inline int32_t make_levels(int32_t L, const float* const* feats, float* const* grads, const int32_t* feat_hw,
                           const int64_t* strides, const float* scales, RoiLevels* lv) {
  FRH_REQUIRE(L >= 1 && L <= FRH_MAX_LEVELS, "num_levels %d out of range", L);
  FRH_REQUIRE(feat_hw && scales && strides, "null pointer argument");
  lv->L = L;
  lv->B = 0x7fffffff;  // the entry points set the batch size (roi_image)
  for (int l = 0; l < L; ++l) {
    lv->feat[l] = feats ? feats[l] : nullptr;
    lv->grad[l] = grads ? grads[l] : nullptr;
    lv->h[l] = feat_hw[2 * l];
    lv->w[l] = feat_hw[2 * l + 1];
    FRH_REQUIRE(lv->h[l] > 0 && lv->w[l] > 0, "level %d has an empty feature map", l);
    lv->sb[l] = strides[4 * l];
    lv->sc[l] = strides[4 * l + 1];
    lv->sy[l] = strides[4 * l + 2];
    lv->sx[l] = strides[4 * l + 3];
    lv->scale[l] = scales[l];
  }
  return FRH_OK;
}


static inline int32_t roi_common_checks(int32_t batch, int32_t channels, int64_t num_rois, int32_t ph, int32_t pw,
                                 const float* rois) {
  FRH_REQUIRE(batch >= 1 && channels >= 1 && num_rois >= 0 && ph >= 1 && pw >= 1, "bad sizes");
  FRH_REQUIRE(num_rois == 0 || rois, "null rois");
  FRH_REQUIRE(num_rois < (int64_t)0x7fffffff, "too many rois");
  return FRH_OK;
}

// shape classes of the forward kernels
struct FwdCaps {
  bool buf;    // 32-bit byte offsets within every (image, level) slice, sampling 2, ph*pw <= 256
  bool lds;    // + ph*pw <= 64 and 2*ph, 2*pw <= 64
  bool x4;     // + unit x stride, 16-B aligned rows / channel planes / bases (16-B LDS-DMA)
};

static inline FwdCaps fwd_caps(const RoiLevels& lv, int32_t channels, int32_t ph, int32_t pw, int32_t sr) {
  FwdCaps f;
  f.buf = sr == 2 && ph * pw <= kRoiThreads;
  for (int l = 0; l < lv.L; ++l) {
    const int64_t ext = ((int64_t)(channels - 1) * lv.sc[l] + (int64_t)(lv.h[l] - 1) * lv.sy[l] +
                         (int64_t)(lv.w[l] - 1) * lv.sx[l] + 1) * 4;
    f.buf = f.buf && lv.sc[l] >= 0 && lv.sy[l] >= 0 && lv.sx[l] >= 0 && ext < ((int64_t)1 << 31);
  }
  f.lds = f.buf && ph * pw <= 64 && 2 * ph <= 64 && 2 * pw <= 64;
  f.x4 = f.lds;
  for (int l = 0; l < lv.L; ++l)
    f.x4 = f.x4 && lv.sx[l] == 1 && lv.sy[l] % 4 == 0 && lv.sc[l] % 4 == 0 && lv.sb[l] % 4 == 0 &&
           (reinterpret_cast<uintptr_t>(lv.feat[l]) & 15) == 0;
  return f;
}


// kernels of the product's forward, chosen by shape class
constexpr int kNhwcCells = 56;  // slab cells of the channels-last kernel (14 KB + 12.25 KB of outputs per wave)

// channels-last features: unit channel stride, 16-B aligned cells, 64-channel groups
static inline bool nhwc_ok(const RoiLevels& lv, int32_t channels, int32_t ph, int32_t pw, int32_t sr) {
  if (sr != 2 || ph != 7 || pw != 7 || channels % kNhwcGroup != 0) return false;
  for (int l = 0; l < lv.L; ++l) {
    const int64_t ext = ((int64_t)(lv.h[l] - 1) * lv.sy[l] + (int64_t)(lv.w[l] - 1) * lv.sx[l] + channels) * 4;
    if (lv.sc[l] != 1 || lv.sx[l] < channels || lv.sy[l] < lv.sx[l] || lv.sx[l] % 4 || lv.sy[l] % 4 ||
        lv.sb[l] % 4 || (reinterpret_cast<uintptr_t>(lv.feat[l]) & 15) || ext >= ((int64_t)1 << 31))
      return false;
  }
  return true;
}

// channels-last features for the quad kernel: unit channel stride, C % 4 == 0, 16-B aligned
static inline bool quad_ok(const FwdCaps& f, const RoiLevels& lv, int32_t channels, int32_t ph, int32_t pw,
                           int slab_cells = QuadLayout<1>::kCells) {
  if (!f.buf || channels % 4 != 0 || 4 * ph > kWave || 4 * pw > kWave || ph * pw > kWave ||
      quad_max_cells(ph, pw) > slab_cells)
    return false;
  for (int l = 0; l < lv.L; ++l)
    if (lv.sc[l] != 1 || lv.sx[l] % 4 || lv.sy[l] % 4 || lv.sb[l] % 4 || (reinterpret_cast<uintptr_t>(lv.feat[l]) & 15))
      return false;
  return true;
}

static inline bool pair_ok(const FwdCaps& f, int32_t channels, int32_t ph, int32_t pw) {
  return f.lds && channels % 2 == 0 && 4 * ph <= kWave && 4 * pw <= kWave &&
         4 * ph * (4 * pw + 1) <= PairLayout<1>::kCells;
}

}  // namespace frh
