// TOOLS-ONLY RoIAlign forward candidates built on the product's quad-kernel pieces
// (roi_kernels.h), measured and not adopted: roi_lab variants 19/20 (RoI setup
// shared by a 4-wave workgroup) and 23 (software-pipelined persistent waves).
#pragma once
#include "roi_kernels.h"

namespace frh {

// The quad kernel with the RoI setup shared by a workgroup: 4 waves per (RoI, 64 channels),
// wave 0 computes the RoI's tap state (pair_setup) and hands it to the other three through
// LDS (18 dwords per lane), so the ~480-instruction setup runs once per 64 channels, not
// once per 16; each wave then stages and evaluates its own 16 channels.  Tools-only
// candidate (roi_lab variant 19).  Grid: 8 * ceil(K * groups / 8) workgroups of 256.
template <int kStAux = kCpolNT, int kOut = 0>
__global__ void __launch_bounds__(4 * kWave) roi_align_fwd_quad4_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float slab[4][kQuadSlab];
  __shared__ __attribute__((aligned(16))) float obuf[4][kOut == 1 ? 4 * kQuadWave * kWave : 4];
  __shared__ PairLane sp[kWave];
  __shared__ PairGeom sg;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave)), lane = threadIdx.x & (kWave - 1);
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)slab[wave]);
  const uint32_t NG = (uint32_t)(c.C + 16 * kQuadWave - 1) / (uint32_t)(16 * kQuadWave), K32 = (uint32_t)c.K;
  const uint32_t total = K32 * NG, per = (total + 7u) / 8u;
  const uint32_t w = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  const uint32_t wend = min((blockIdx.x & 7u) * per + per, total);
  if (w >= wend) return;
  const int grp = (int)(w / K32);
  const int64_t k0 = (int64_t)(w - (uint32_t)grp * K32);
  PairGeom G;
  PairLane P;
  if (wave == 0) {
    const RoiRaw raw = roi_fetch(c, k0);
    pair_setup<16>(lv, c, raw, lane, G, P);
    sp[lane] = P;
    if (lane == 0) sg = G;
  }
  __syncthreads();
  if (wave != 0) {
    P = sp[lane];
    G.empty = __builtin_amdgcn_readfirstlane(sg.empty);
    G.y0 = __builtin_amdgcn_readfirstlane(sg.y0), G.x0 = __builtin_amdgcn_readfirstlane(sg.x0);
    G.R = __builtin_amdgcn_readfirstlane(sg.R), G.Cs = __builtin_amdgcn_readfirstlane(sg.Cs);
    G.Cs2 = __builtin_amdgcn_readfirstlane(sg.Cs2);
    G.dy = __builtin_amdgcn_readfirstlane(sg.dy), G.dx = __builtin_amdgcn_readfirstlane(sg.dx);
    G.sy = __builtin_amdgcn_readfirstlane(sg.sy), G.sx = __builtin_amdgcn_readfirstlane(sg.sx);
    G.scs = __builtin_amdgcn_readfirstlane(sg.scs);
    G.inv = (uint32_t)__builtin_amdgcn_readfirstlane((int)sg.inv);
    G.extent = (uint32_t)__builtin_amdgcn_readfirstlane((int)sg.extent);
    const uint64_t b = reinterpret_cast<uint64_t>(sg.base);
    G.base = reinterpret_cast<const float*>(
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32) |
        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b));
  }
  const int chunk = grp * 4 + wave;
  if (chunk * 4 * kQuadWave >= c.C) return;
  quad_body<kStAux, false, kQuadWave, kOut>(G, P, c, out, k0, chunk, w, sbase, 0, lane, obuf[wave]);
}

// ---------------------------------------------------------------------------
// Software-pipelined persistent quad kernel (tools-only candidate, roi_lab variant 23):
// each wave walks its XCD's items (RoI, 16 channels) as units of one channel quad, two
// 8-KB slabs: unit u+1's window DMA is in flight while unit u is evaluated, and the next
// item's setup runs while the current unit's DMA lands.  Same slab layout (D = 1: up to 512
// cells), operation order and outputs as the quad kernel; windows of more cells take the
// global gather per quad, empty RoIs store zeros.
struct QpItem {
  PairGeom G;
  PairLane P;
  int64_t k;
  int cw0, nq;
  int D;    // quads per stage (4, 2, 1: the quad kernel's slab layouts); 0: global gather
  int nst;  // stages
};

__device__ __forceinline__ void qp_load(const RoiLevels& lv, const RoiCfg& c, uint32_t w, uint32_t K32, int lane,
                                        QpItem& it) {
  const int ch = (int)(w / K32);
  it.k = (int64_t)(w - (uint32_t)ch * K32);
  it.cw0 = ch * 4 * kQuadWave;
  it.nq = min(kQuadWave, (c.C - it.cw0) / 4);
  const RoiRaw raw = roi_fetch(c, it.k);
  pair_setup<16>(lv, c, raw, lane, it.G, it.P);
  const int ncell = it.G.R * it.G.Cs2;
  it.D = it.G.empty ? 4 : ncell <= QuadLayout<4>::kCells ? 4 : ncell <= QuadLayout<2>::kCells ? 2
                                                     : ncell <= QuadLayout<1>::kCells ? 1 : 0;
  it.nst = it.D ? (it.nq + it.D - 1) / it.D : it.nq;
}

__device__ __forceinline__ bool qp_staged(const QpItem& it) { return !it.G.empty && it.D > 0; }

// stage s of a staged item: region d (RS(D) dwords) <- quad s * D + d of every window cell
__device__ __forceinline__ void qp_issue(const QpItem& it, int s, uint32_t sb, int lane) {
  const PairGeom& G = it.G;
  const int ncell = G.R * G.Cs2;
  const int nr = (ncell + kWave - 1) / kWave;
  const int RSb = 4 * ((kQuadSlab / it.D) / 256 * 256);  // region bytes
  const __amdgpu_buffer_rsrc_t fr = uniform_rsrc(G.base, (int64_t)G.extent);
  for (int d = 0; d < it.D; ++d) {
    const int soff = (it.cw0 + 4 * min(s * it.D + d, it.nq - 1)) * 4;
    for (int j = 0; j < nr; ++j) {
      int e = j * kWave + lane;
      e = e < ncell ? e : 0;
      const int r = (int)(((uint32_t)e * G.inv) >> 16), col = min(e - r * G.Cs2, G.Cs - 1);
      const int goff = (G.dy && G.dx) ? ((G.y0 + r) * G.sy + (G.x0 + col) * G.sx) * 4
                                      : __shfl(it.P.rsrc, r, kWave) + __shfl(it.P.csrc, col, kWave);
      lds_dma_at<16, 0>(fr, sb + (uint32_t)(d * RSb) + 1024u * (uint32_t)j, goff, soff);
    }
  }
}

// one quad of a staged item from its slab region at rb (byte address): the quad kernel's evaluation
__device__ __forceinline__ f32x4 qp_eval(const PairLane& P, uint32_t rb) {
  constexpr int SR = 2;
  f32x4 v[2][8];
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  float ly_h[SR], ly_l[SR], lx_h[SR], lx_l[SR];
  uint32_t lb[SR][SR], ldq[SR], ldr[SR];
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    ly_h[i] = P.fyh[i], ly_l[i] = P.fyl[i], lx_h[i] = P.fxh[i], lx_l[i] = P.fxl[i], ldq[i] = P.tdq[i], ldr[i] = P.tdr[i];
#pragma unroll
    for (int j = 0; j < SR; ++j) lb[i][j] = rb + P.tb0[i][j];
  }
  auto tap = [&](int iy, int ix, int q) -> uint32_t {
    return lb[iy][ix] + ((q & 1) ? ldq[ix] : 0u) + ((q & 2) ? ldr[iy] : 0u);
  };
#pragma unroll
  for (int ix = 0; ix < SR; ++ix)
#pragma unroll
    for (int q = 0; q < 4; ++q) v[0][ix * 4 + q] = lds_read_b128<0>(tap(0, ix, q));
#pragma unroll
  for (int ix = 0; ix < SR; ++ix)
#pragma unroll
    for (int q = 0; q < 4; ++q) v[1][ix * 4 + q] = lds_read_b128<0>(tap(1, ix, q));
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
  return acc * 0.25f;
}

// quad q of an item whose window does not fit the slab: taps gathered from global memory
__device__ __forceinline__ f32x4 qp_global(const QpItem& it, int q) {
  constexpr int SR = 2;
  const PairGeom& G = it.G;
  const PairLane& P = it.P;
  const __amdgpu_buffer_rsrc_t fr = uniform_rsrc(G.base, (int64_t)G.extent);
  const int soff = (it.cw0 + 4 * q) * 4;
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int iy = 0; iy < SR; ++iy)
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const uint32_t t0 = P.tb0[iy][ix] / 16u;
      const int r0 = (int)(t0 / (uint32_t)G.Cs2), c0 = (int)(t0 - (uint32_t)r0 * (uint32_t)G.Cs2);
      const int r1 = r0 + (int)(P.tdr[iy] / 16u / (uint32_t)G.Cs2), c1 = c0 + (int)(P.tdq[ix] / 16u);
      const int ro0 = __shfl(P.rsrc, r0, kWave), ro1 = __shfl(P.rsrc, r1, kWave);
      const int co0 = __shfl(P.csrc, c0, kWave), co1 = __shfl(P.csrc, c1, kWave);
      f32x4 x[4];
      const int offs[4] = {ro0 + co0, ro0 + co1, ro1 + co0, ro1 + co1};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(fr, offs[t], soff, 0);
        x[t] = f32x4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
      }
      const float w[4] = {P.fyh[iy] * P.fxh[ix], P.fyh[iy] * P.fxl[ix], P.fyl[iy] * P.fxh[ix], P.fyl[iy] * P.fxl[ix]};
      acc = acc + quad_val(w, x);
    }
  return acc * 0.25f;
}

// s_waitcnt vmcnt(n) for n in {0, 4, 8, 12, 16} (the previous unit's store count)
__device__ __forceinline__ void qp_wait(int n) {
  if (n >= 16) wait_vmcnt<16>();
  else if (n >= 12) wait_vmcnt<12>();
  else if (n >= 8) wait_vmcnt<8>();
  else if (n >= 4) wait_vmcnt<4>();
  else wait_vmcnt<0>();
}

template <int kStAux = kCpolNT>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(2))) roi_align_fwd_quadp_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float slab[2][kQuadSlab];
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t sb0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)slab[0]);
  const uint32_t sbs[2] = {sb0, sb0 + 4u * kQuadSlab};
  const uint32_t G = (uint32_t)(c.C + 4 * kQuadWave - 1) / (uint32_t)(4 * kQuadWave), K32 = (uint32_t)c.K;
  const uint32_t total = K32 * G, per = (total + 7u) / 8u;
  const uint32_t xcd = blockIdx.x & 7u, nw = gridDim.x >> 3;
  const uint32_t lo = xcd * per, hi = min(lo + per, total);
  uint32_t w = lo + (blockIdx.x >> 3);
  if (w >= hi) return;
  const int nbins = c.ph * c.pw;
  const int ovoff = lane < nbins ? lane * 4 : 0x40000000;
  const int ostep = nbins * 4;
  QpItem A, B;
  qp_load(lv, c, w, K32, lane, A);
  int s = 0, cur = 0, prev_stores = 0;
  if (qp_staged(A)) qp_issue(A, 0, sbs[0], lane);
  for (;;) {
    // the next unit: the next stage of this item, or stage 0 of the wave's next item
    const bool same = s + 1 < A.nst;
    const uint32_t wn = w + nw;
    const bool more = same || wn < hi;
    if (!same && more) qp_load(lv, c, wn, K32, lane, B);  // overlaps the current unit's DMA
    // this unit's DMA landed; the previous unit's output stores (younger: vector memory
    // operations complete in issue order) may still be in flight
    qp_wait(prev_stores);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (more) {
      if (same) {
        if (qp_staged(A)) qp_issue(A, s + 1, sbs[cur ^ 1], lane);
      } else if (qp_staged(B)) {
        qp_issue(B, 0, sbs[cur ^ 1], lane);
      }
    }
    const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + (A.k * c.C + A.cw0) * nbins, (int64_t)4 * A.nq * nbins * 4);
    const int D = A.D ? A.D : 1;
    const int RSb = 4 * ((kQuadSlab / D) / 256 * 256);
    prev_stores = 0;
    for (int d = 0; d < D; ++d) {
      const int q = s * D + d;
      if (q >= A.nq) break;
      f32x4 r = {0.0f, 0.0f, 0.0f, 0.0f};
      if (A.G.empty) {
      } else if (A.D) {
        r = qp_eval(A.P, sbs[cur] + (uint32_t)(d * RSb));
      } else {
        r = qp_global(A, q);
      }
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.x), orr, ovoff, (4 * q) * ostep, kStAux);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.y), orr, ovoff, (4 * q + 1) * ostep, kStAux);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.z), orr, ovoff, (4 * q + 2) * ostep, kStAux);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.w), orr, ovoff, (4 * q + 3) * ostep, kStAux);
      prev_stores += 4;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!more) break;
    cur ^= 1;
    if (same) {
      ++s;
    } else {
      A = B;
      s = 0;
      w = wn;
    }
  }
}

// ---------------------------------------------------------------------------
// Processing order for the forward (kFwdSorted): the RoIs' records grouped by (image, level,
// 8 x 8-cell tile of the RoI centre, tiles row-major), so the waves a XCD runs together stage
// overlapping windows while they are still in its L2.  One 1024-thread workgroup: a counting sort
// over at most kSortBins bins (more tiles fold modulo kSortBins: still grouped), records written
// 8 words each (the RoI's 5 words as given, its level, its index, 0).  Order inside a bin is
// arbitrary: every output row is its own RoI's, whatever the order.
constexpr int kSortThreads = 1024, kSortBins = 4096, kSortTile = 8;
__device__ __forceinline__ int roi_sort_bin(const RoiLevels& lv, const RoiCfg& c, int64_t k) {
  const float* r = c.rois + k * 5;
  const int b = (int)r[0];
  const int l = c.levels ? (int)c.levels[k] : 0;
  int tb = 0, T = 0;
  for (int i = 0; i < lv.L; ++i) {
    const int n = ((lv.h[i] + kSortTile - 1) / kSortTile) * ((lv.w[i] + kSortTile - 1) / kSortTile);
    tb += i < l ? n : 0;
    T += n;
  }
  const int th = (lv.h[l] + kSortTile - 1) / kSortTile, tw = (lv.w[l] + kSortTile - 1) / kSortTile;
  const float sc = lv.scale[l];
  const int ty = min(max((int)(0.5f * (r[2] + r[4]) * sc) / kSortTile, 0), th - 1);
  const int tx = min(max((int)(0.5f * (r[1] + r[3]) * sc) / kSortTile, 0), tw - 1);
  return (int)(((int64_t)max(b, 0) * T + tb + ty * tw + tx) % kSortBins);
}

static __global__ void __launch_bounds__(kSortThreads) roi_sort_kernel(RoiLevels lv, RoiCfg c, int32_t* rec) {
  __shared__ uint32_t h[kSortBins];
  __shared__ uint32_t part[kSortThreads / kWave];
  const int t = threadIdx.x;
  for (int i = t; i < kSortBins; i += kSortThreads) h[i] = 0u;
  __syncthreads();
  for (int64_t k = t; k < c.K; k += kSortThreads) atomicAdd(&h[roi_sort_bin(lv, c, k)], 1u);
  __syncthreads();
  // exclusive scan of the bins: thread t owns bins 4t .. 4t + 3
  constexpr int kPer = kSortBins / kSortThreads;
  uint32_t v[kPer], sum = 0u;
#pragma unroll
  for (int i = 0; i < kPer; ++i) sum += (v[i] = h[kPer * t + i]);
  uint32_t incl = sum;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t x = __shfl_up(incl, o, kWave);
    if (lane_id() >= o) incl += x;
  }
  if (lane_id() == kWave - 1) part[t / kWave] = incl;
  __syncthreads();
  uint32_t pre = 0u;
  for (int i = 0; i < t / kWave; ++i) pre += part[i];
  uint32_t run = pre + incl - sum;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    h[kPer * t + i] = run;
    run += v[i];
  }
  __syncthreads();
  for (int64_t k = t; k < c.K; k += kSortThreads) {
    const uint32_t pos = atomicAdd(&h[roi_sort_bin(lv, c, k)], 1u);
    const int32_t* r = reinterpret_cast<const int32_t*>(c.rois + k * 5);
    int4* o = reinterpret_cast<int4*>(rec + (int64_t)pos * 8);
    o[0] = make_int4(r[0], r[1], r[2], r[3]);
    o[1] = make_int4(r[4], c.levels ? (int)c.levels[k] : 0, (int)k, 0);
  }
}

// Round-6 experiment (tools only; measured slower: the backward is bound by its atomics, not by
// the 8 waves per CU its LDS staging allows -- DESIGN §4).  The channels-last backward with 7 x 7 bins and the wave's grad_out held in registers (49 per lane:
// its channel's bins) instead of LDS: the kernel's LDS is the four tap-entry tables (< 0.5 KB),
// so residency is set by registers (~20 waves per CU against 8 with the 18.9-KB LDS staging).
// The bin row and column of a tap entry are wave-uniform, so the register operand is chosen by a
// uniform switch (static indices).  Same operation order as roi_align_bwd_nhwc_kernel: the same
// per-(RoI, row, column) sums, bit for bit.
template <bool kFixed = false>
__global__ void __launch_bounds__(kWave) roi_align_bwd_nhwc_reg_kernel(RoiLevels lv, RoiCfg c,
                                                                     const float* __restrict__ gout) {
  constexpr int P = 7, NB = P * P;
  __shared__ int ye[kSepEnt], xe[kSepEnt];  // sorted tap entries: position << 16 | bin index
  __shared__ float yws[kSepEnt], xws[kSepEnt];
  const int64_t k = blockIdx.x;
  const int lane = threadIdx.x;
  const int c0 = blockIdx.y * kWave, ch = c0 + lane;
  const bool live = ch < c.C;
  float gr[NB];  // grad_out of this lane's channel, bin py * 7 + px
  {
    const float* go = gout + (k * c.C + (live ? ch : c0)) * NB;
#pragma unroll
    for (int b = 0; b < NB; ++b) gr[b] = live ? go[b] : 0.0f;
  }
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl, H = lv.h[l], W = lv.w[l];
  constexpr int nye = 4 * P, nxe = 4 * P;
  auto entry = [&](int e, float start, float bin, int size, int* pos, float* w) {
    const Tap t = make_tap(start + (float)(e >> 2) * bin + ((float)((e >> 1) & 1) + 0.5f) * bin * 0.5f, size);
    *pos = t.valid ? ((e & 1) ? t.hi : t.lo) : -1;
    *w = (e & 1) ? t.l : t.h;
  };
  int yp = -1, xp = -1;
  float ywv = 0.0f, xwv = 0.0f;
  if (lane < nye) entry(lane, g.start_h, g.bin_h, H, &yp, &ywv);
  if (lane < nxe) entry(lane, g.start_w, g.bin_w, W, &xp, &xwv);
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
  const int64_t base = (int64_t)g.b * lv.sb[l] + ch, sy = lv.sy[l], sx = lv.sx[l];
  const double fscale = kFixed ? bwd_fixed_scale(c.fix_max, c.fix_hb) : 0.0;
  if (kFixed && fscale < 0.0) return;  // non-finite gradient: the conversion writes NaN
  float R[P];
#pragma unroll
  for (int px = 0; px < P; ++px) R[px] = 0.0f;
  for (int i = 0; i < nyv; ++i) {
    const int yv = __builtin_amdgcn_readfirstlane(ye[i]), row = yv >> 16, py = yv & 0xffff;
    const float wy = yws[i];
    switch (py) {  // wave-uniform: static register operands
#define FRH_ROW_CASE(Q)                                                       \
  case Q:                                                                     \
    _Pragma("unroll") for (int px = 0; px < P; ++px) R[px] = R[px] + wy * gr[Q * P + px]; \
    break;
      FRH_ROW_CASE(0) FRH_ROW_CASE(1) FRH_ROW_CASE(2) FRH_ROW_CASE(3) FRH_ROW_CASE(4) FRH_ROW_CASE(5) FRH_ROW_CASE(6)
#undef FRH_ROW_CASE
      default: break;
    }
    if (i + 1 < nyv && (ye[i + 1] >> 16) == row) continue;  // the row continues (uniform)
    float acc = 0.0f;
    for (int jx = 0; jx < nxv; ++jx) {
      const int xv = __builtin_amdgcn_readfirstlane(xe[jx]), col = xv >> 16, px = xv & 0xffff;
      const float rv = px == 0 ? R[0] : px == 1 ? R[1] : px == 2 ? R[2] : px == 3 ? R[3] : px == 4 ? R[4]
                                                                                             : px == 5 ? R[5] : R[6];
      acc = acc + xws[jx] * rv;
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
#pragma unroll
    for (int px = 0; px < P; ++px) R[px] = 0.0f;
  }
}

}  // namespace frh
