// a14: RoIAlign forward as a row sweep over whole feature planes.
// Reference: lib/region.py:243-306 (BasicRoIExtractor: map_rois_to_levels, then
// per level torchvision RoIAlign(output_size, 1/stride, sampling_ratio=2),
// legacy aligned=False semantics; one call per image and level in the reference).
//
// Why a sweep.  A per-RoI kernel stages every RoI's tap window of every
// channel on its own.  In NCHW a window row of a few cells is a partial 128-B
// line, and overlapping RoIs fetch the same lines again: on the cfg2 RoIs that
// is 4.8 M line fetches (609 MB) for 106 MB of feature planes, and the kernel
// ends up bound by on-chip line traffic and per-wave latency.  Here one
// workgroup owns one (level, image, channel pair) and streams that plane pair
// top to bottom through an LDS ring of kSwRing rows, exactly once, with full
// 256-B LDS-DMA rows.  Every RoI is cut into "items" = (RoI, bin row py): an
// item's 2 sample rows span at most bin_h / 2 + 2 feature rows (13 at cfg2),
// so it is evaluated as soon as the sweep has landed its last row, while its
// first row is still in the ring.  Items are bucketed by that last row (step
// = 2 rows) in LDS by the workgroup itself; a tiny plan launch precomputes
// each item's y taps and each (RoI, px)'s x taps once, for all channels.
//
// Workgroup: 2 loader waves (one row of each step each, 4-B LDS-DMA with the
// two channels interleaved [x][2], kSwLook steps in flight, counted vmcnt) and
// 6 compute waves (lane = one bin of one item; 16 ds_read_b64 taps, both
// channels with packed f32 math).  One barrier per pass (384 bins).
// Items whose row span exceeds kSwSpan (never at sampling ratio 2 unless a RoI
// is > 20 x 7 rows tall on its level) are evaluated after the sweep straight
// from global memory.  Same operation order as torchvision's CPU kernel:
// bit-identical to every other forward kernel and the oracle.
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "roi_common.h"

namespace frh {

constexpr int kSwRing = 64;   // LDS ring rows (power of two)
constexpr int kSwStep = 8;    // rows per sweep step (one per loader wave)
constexpr int kSwLook = 4;    // steps of DMA in flight ahead of the one evaluated
constexpr int kSwSpan = 17;   // largest item row span the ring serves (see the assert)
constexpr int kSwLoad = kSwStep;
constexpr int kSwComp = 8;
constexpr int kSwThreads = (kSwLoad + kSwComp) * kWave;
constexpr int kSwLanes = kSwComp * kWave;
constexpr int kSwDepth = 4;   // passes of tap records prefetched ahead by the compute lanes
constexpr uint32_t kSwBig = 0xffffu;
// One barrier per step.  The DMA of step s + 1 + kSwLook is issued while step s may
// still be evaluated: the rows it overwrites (up to kStep (s + 1 + kSwLook) + kStep - 1
// - kSwRing) must be older than the first row an item of step s can need (kStep s -
// kSwSpan + 1).
static_assert(kSwSpan < kSwRing - kSwStep * (kSwLook + 2) + 2, "ring too small for the span");

struct SwPlan {
  uint32_t* key;  // [K*ph] (image * L + level) << 16 | step of the item's last row (kSwBig: span > kSwSpan)
  int4* item;     // [K*ph] {lo0 | hi0 << 16, lo1 | hi1 << 16, l0, l1}: the bin row's 2 y samples (lo = -1: invalid)
  int4* xtap;     // [K*pw] the same for the 2 x samples of (RoI, px)
};

struct SwArgs {
  int B, np;       // images, channel pairs
  int max_slots;   // sum over levels of ceil(H / kSwStep) + 1
  int nitems;      // K * ph
  int max_pass;    // capacity of the LDS pass table
};

// roi_geom (same order of operations) with the image index and level clamped into range
__device__ __forceinline__ RoiGeom sweep_geom(const RoiCfg& c, const RoiLevels& lv, int64_t k, int B) {
  RoiGeom g;
  const float* r = c.rois + k * 5;
  g.b = (int)r[0];
  g.b = g.b < 0 ? 0 : (g.b >= B ? B - 1 : g.b);
  g.lvl = c.levels ? (int)c.levels[k] : 0;
  g.lvl = g.lvl < 0 ? 0 : (g.lvl >= lv.L ? lv.L - 1 : g.lvl);
  const float sc = lv.scale[g.lvl];
  const float off = c.aligned ? 0.5f : 0.0f;
  float sw = r[1] * sc - off, sh = r[2] * sc - off;
  float ew = r[3] * sc - off, eh = r[4] * sc - off;
  float rw = ew - sw, rh = eh - sh;
  if (!c.aligned) {
    rw = fmaxf(rw, 1.0f);
    rh = fmaxf(rh, 1.0f);
  }
  g.start_w = sw;
  g.start_h = sh;
  g.bin_h = rh / (float)c.ph;
  g.bin_w = rw / (float)c.pw;
  g.gh = c.sampling;
  g.gw = c.sampling;
  g.count = (float)(c.sampling * c.sampling);
  return g;
}

__device__ __forceinline__ int pack_tap(const Tap& t) { return t.valid ? ((t.lo & 0xffff) | (t.hi << 16)) : -1; }

__global__ void __launch_bounds__(256) roi_sweep_plan_kernel(RoiLevels lv, RoiCfg c, int B, SwPlan P) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t ni = c.K * c.ph, nx = c.K * c.pw;
  if (t < ni) {
    const int64_t k = t / c.ph;
    const int py = (int)(t - k * c.ph);
    const RoiGeom g = sweep_geom(c, lv, k, B);
    const int H = lv.h[g.lvl];
    const Tap a = make_tap(sample_y(g, py, 0), H), d = make_tap(sample_y(g, py, 1), H);
    uint32_t step = 0;
    if (a.valid || d.valid) {
      const int yf = a.valid ? (d.valid ? min(a.lo, d.lo) : a.lo) : d.lo;
      const int yl = a.valid ? (d.valid ? max(a.hi, d.hi) : a.hi) : d.hi;
      step = yl - yf + 1 > kSwSpan ? kSwBig : (uint32_t)(yl / kSwStep);
    }
    P.key[t] = ((uint32_t)(g.b * lv.L + g.lvl) << 16) | step;
    P.item[t] = make_int4(pack_tap(a), pack_tap(d), __float_as_int(a.l), __float_as_int(d.l));
  }
  if (t < nx) {
    const int64_t k = t / c.pw;
    const int px = (int)(t - k * c.pw);
    const RoiGeom g = sweep_geom(c, lv, k, B);
    const int W = lv.w[g.lvl];
    const Tap a = make_tap(sample_x(g, px, 0), W), d = make_tap(sample_x(g, px, 1), W);
    P.xtap[t] = make_int4(pack_tap(a), pack_tap(d), __float_as_int(a.l), __float_as_int(d.l));
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// One lane's bin: id and taps (prefetched kSwDepth passes ahead).
struct SwBin {
  int id;  // item id (-1: idle lane)
  int4 item, xtap;
};

// Per-level feature slice of this task's channel pair.
struct SwLevel {
  __amdgpu_buffer_rsrc_t fr;
  int sy4, sc4, W, H;
};

__device__ __forceinline__ SwLevel sweep_level(const RoiLevels& lv, int l, int b, int cp) {
  SwLevel q;
  q.H = lv.h[l];
  q.W = lv.w[l];
  q.sy4 = (int)lv.sy[l] * 4;
  q.sc4 = (int)lv.sc[l] * 4;
  const float* base = lv.feat[l] + (int64_t)b * lv.sb[l] + (int64_t)(2 * cp) * lv.sc[l];
  q.fr = uniform_rsrc(base, ((int64_t)lv.sc[l] + (int64_t)(q.H - 1) * lv.sy[l] + q.W) * 4);
  return q;
}

// LDS carve-up shared by the forward and backward sweeps (dynamic LDS only: no static
// __shared__ in front, so the ring stays 16-B aligned).
struct SwLds {
  int* sc;         // [0] total items, [1] passes, [2] global steps
  int* lvi;        // per level: last swept step, gbase (global step of its step 0), slot base
  char* ring;      // kSwRing rows x RS bytes
  int2* pass;      // [max_pass] {i0, n | level << 16 | first << 31}
  int* cnt;        // [max_slots] counts -> item offsets
  int* cur;        // [max_slots] pass bases, then scatter cursors
  uint16_t* list;  // [nitems] item ids by (level, step)
  uint8_t* glev;   // [max_slots] level of global step g
};

__device__ __forceinline__ SwLds sweep_lds(char* smem, const SwArgs& A, int RS) {
  SwLds d;
  d.sc = reinterpret_cast<int*>(smem);
  d.lvi = d.sc + 4;
  d.ring = smem + 128;
  d.pass = reinterpret_cast<int2*>(d.ring + kSwRing * RS);
  d.cnt = reinterpret_cast<int*>(d.pass + A.max_pass);
  d.cur = d.cnt + A.max_slots;
  d.list = reinterpret_cast<uint16_t*>(d.cur + A.max_slots);
  d.glev = reinterpret_cast<uint8_t*>(d.list + A.nitems);
  return d;
}

__device__ __forceinline__ int sweep_nst(const RoiLevels& lv, int l) { return (lv.h[l] + kSwStep - 1) / kSwStep; }
__device__ __forceinline__ int sweep_sbase(const RoiLevels& lv, int l) {  // a level's steps, then its long-span slot
  int s0 = 0;
  for (int m = 0; m < l; ++m) s0 += sweep_nst(lv, m) + 1;
  return s0;
}

// Buckets the items of image b by (level, step) in LDS and builds the pass table.
// kAll: sweep every step of every level (backward: every gradient row is written);
// else each level up to its last step with items (levels without items: skipped).
template <bool kAll>
__device__ void sweep_prologue(const RoiLevels& lv, const RoiCfg& c, const SwArgs& A, const SwPlan& P, const SwLds& d,
                               int b) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int L = lv.L;
  const int nslots = sweep_sbase(lv, L);
  for (int i = tid; i < nslots; i += kSwThreads) d.cnt[i] = 0;
  __syncthreads();
  // thread t takes a contiguous run of RoIs: the lanes of a wave hit different steps (little LDS contention)
  const int K = (int)c.K, ph = c.ph, pw = c.pw;
  const int per_t = (K + kSwThreads - 1) / kSwThreads;
  const int kb = tid * per_t, ke = min(K, kb + per_t);
  for (int k = kb; k < ke; ++k) {
    const uint32_t k0 = P.key[k * ph];
    const int bl = (int)(k0 >> 16), kbimg = bl / L;
    if (kbimg != b) continue;
    const int l = bl - kbimg * L, s0 = sweep_sbase(lv, l), big = s0 + sweep_nst(lv, l);
    for (int py = 0; py < ph; ++py) {
      const uint32_t st = P.key[k * ph + py] & 0xffffu;
      atomicAdd(&d.cnt[st == kSwBig ? big : s0 + (int)st], 1);
    }
  }
  __syncthreads();
  const int ipp = kSwLanes / pw;  // items per pass
  if (wave == 0) {
    int g = 0;
    for (int l = 0; l < L; ++l) {
      const int s0 = sweep_sbase(lv, l), n = sweep_nst(lv, l);
      int hi = n - 1;
      if (!kAll) {
        hi = -1;
        for (int b0 = 0; b0 < n; b0 += kWave) {
          const uint64_t m = __ballot(b0 + lane < n && d.cnt[s0 + b0 + lane] > 0);
          if (m) hi = b0 + 63 - __clzll(m);
        }
      }
      if (lane == 0) {
        d.lvi[3 * l] = hi;
        d.lvi[3 * l + 1] = g;
        d.lvi[3 * l + 2] = s0;
      }
      for (int j = lane; j <= hi; j += kWave) d.glev[g + j] = (uint8_t)l;
      g += hi + 1;
    }
    int run = 0, prun = 0;
    for (int l = 0; l < L; ++l) {
      const int s0 = sweep_sbase(lv, l), n = sweep_nst(lv, l), hi = d.lvi[3 * l];
      for (int b0 = 0; b0 <= n; b0 += kWave) {  // steps 0 .. n - 1 and the long-span slot n
        const int j = b0 + lane;
        const int v = j <= n ? d.cnt[s0 + j] : 0;
        const int np = j <= hi ? max(1, (v + ipp - 1) / ipp) : 0;
        int inc = v, pinc = np;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
          const int u = __shfl_up(inc, o, kWave), pu = __shfl_up(pinc, o, kWave);
          if (lane >= o) inc += u, pinc += pu;
        }
        if (j <= n) {
          d.cnt[s0 + j] = run + inc - v;
          d.cur[s0 + j] = prun + pinc - np;
        }
        run += __shfl(inc, kWave - 1, kWave);
        prun += __shfl(pinc, kWave - 1, kWave);
      }
    }
    if (lane == 0) {
      d.sc[0] = run;
      d.sc[1] = prun;
      d.sc[2] = g;
    }
  }
  __syncthreads();
  // pass table (at least one pass per swept step), then the scatter cursors
  for (int f = tid; f < nslots; f += kSwThreads) {
    int l = 0;
    while (l + 1 < L && sweep_sbase(lv, l + 1) <= f) ++l;
    const int s = f - sweep_sbase(lv, l);
    if (s > d.lvi[3 * l]) continue;  // past the level's last swept step, or its long-span slot
    const int i0 = d.cnt[f], n = d.cnt[f + 1] - i0, pb = d.cur[f];
    const int np = max(1, (n + ipp - 1) / ipp);
    for (int j = 0; j < np; ++j)
      d.pass[pb + j] = make_int2(i0 + j * ipp, min(ipp, n - j * ipp) | (l << 16) | (j == 0 ? (int)0x80000000 : 0));
  }
  __syncthreads();
  for (int f = tid; f < nslots; f += kSwThreads) d.cur[f] = d.cnt[f];
  __syncthreads();
  for (int k = kb; k < ke; ++k) {
    const uint32_t k0 = P.key[k * ph];
    const int bl = (int)(k0 >> 16), kbimg = bl / L;
    if (kbimg != b) continue;
    const int l = bl - kbimg * L, s0 = sweep_sbase(lv, l), big = s0 + sweep_nst(lv, l);
    for (int py = 0; py < ph; ++py) {
      const uint32_t st = P.key[k * ph + py] & 0xffffu;
      d.list[atomicAdd(&d.cur[st == kSwBig ? big : s0 + (int)st], 1)] = (uint16_t)(k * ph + py);
    }
  }
  __syncthreads();
}

// Unpacked taps of one bin (sampling ratio 2): rows / columns of the 2 x 2 samples.
struct SwTaps {
  int ylo[2], yhi[2], xlo[2], xhi[2];
  float ly[2], lx[2];
};

__device__ __forceinline__ SwTaps sweep_taps(const int4& item, const int4& xtap) {
  SwTaps t;
  t.ylo[0] = (int)(short)(item.x & 0xffff), t.yhi[0] = item.x >> 16;
  t.ylo[1] = (int)(short)(item.y & 0xffff), t.yhi[1] = item.y >> 16;
  t.xlo[0] = (int)(short)(xtap.x & 0xffff), t.xhi[0] = xtap.x >> 16;
  t.xlo[1] = (int)(short)(xtap.y & 0xffff), t.xhi[1] = xtap.y >> 16;
  t.ly[0] = __int_as_float(item.z), t.ly[1] = __int_as_float(item.w);
  t.lx[0] = __int_as_float(xtap.z), t.lx[1] = __int_as_float(xtap.w);
  return t;
}

// Workgroup = (image b, channel pair cp): sweeps every level that has RoIs of
// image b, finest first, as one continuous row stream through the ring.
template <int NI>
__global__ void __launch_bounds__(kSwThreads) roi_sweep_fwd_kernel(RoiLevels lv, RoiCfg c, SwArgs A, SwPlan P,
                                                                   float* __restrict__ out, int64_t* dbg) {
  // dbg (diagnostics only; nullptr in product runs): per workgroup 8 x int64 s_memrealtime stamps
  const int64_t t_start = dbg ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  constexpr int RS = (32 * NI + 1) * 8;  // ring row: 32 NI cells x 2 channels (+1 cell: bank spread)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const SwLds D = sweep_lds(smem, A, RS);
  char* ring = D.ring;
  const int2* pass = D.pass;
  const int* cnt = D.cnt;
  const uint16_t* list = D.list;
  const uint8_t* glev = D.glev;
  const int* lvi = D.lvi;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int b = blockIdx.x / A.np, cp = blockIdx.x - b * A.np;
  const int L = lv.L;
  const int ph = c.ph, pw = c.pw, nbins = ph * pw;
  const int nslots = sweep_sbase(lv, L);
  auto nst_of = [&](int l) { return sweep_nst(lv, l); };
  sweep_prologue<false>(lv, c, A, P, D, b);
  const int total = D.sc[0], npass = D.sc[1], G = D.sc[2];
  if (total == 0) return;  // image without RoIs: uniform exit (nothing in flight yet)
  const int64_t t_list = dbg ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;

  if (wave < kSwLoad) {
    // ---- loader: row kSwStep s + wave of global step g = (level, s); ring slot = global row & (kSwRing - 1)
    int cl = -1;
    SwLevel q{};
    int vo[NI];
    auto issue = [&](int g) {
      const int gg = g < G ? g : G - 1;  // past the end: harmless re-loads of the last step's rows
      const int l = glev[gg];
      if (l != cl) {
        cl = l;
        q = sweep_level(lv, l, b, cp);
#pragma unroll
        for (int j = 0; j < NI; ++j) vo[j] = min(32 * j + (lane >> 1), q.W - 1) * 4 + (lane & 1) * q.sc4;
      }
      const int s = gg - lvi[3 * l + 1];
      const int row = s * kSwStep + wave, y = row < q.H ? row : q.H - 1;
      char* dst = ring + ((g * kSwStep + wave) & (kSwRing - 1)) * RS;
#pragma unroll
      for (int j = 0; j < NI; ++j) lds_dma<4>(q.fr, reinterpret_cast<float*>(dst + j * 256), vo[j], y * q.sy4);
    };
    if (G > 0) {
#pragma unroll
      for (int g = 0; g < kSwLook; ++g) issue(g);
      for (int g = 0; g < G; ++g) {
        issue(g + kSwLook);
        wait_vmcnt<kSwLook * NI>();  // this wave's row of step g has landed (the barrier publishes it)
        __syncthreads();
      }
      wait_vmcnt<0>();
    }
    if (dbg && wave == 0 && lane == 0) {
      int64_t* d = dbg + (int64_t)blockIdx.x * 8;
      d[0] = t_start;
      d[1] = t_list;
      d[2] = (int64_t)__builtin_amdgcn_s_memrealtime();
      d[3] = G;
      d[4] = npass;
      d[5] = total;
    }
    return;
  }

  // ---- compute waves: lane = (item slot qi, px) of a pass, one bin per pass
  const int q = (wave - kSwLoad) * kWave + lane;
  const int qi = q / pw, qx = q - qi * pw;
  auto fetch = [&](int p) {
    SwBin r;
    const int2 d = pass[p];
    const int n = d.y & 0xffff;
    r.id = qi < n ? (int)list[d.x + qi] : -1;
    const int id = r.id >= 0 ? r.id : 0;
    r.item = P.item[id];
    r.xtap = P.xtap[(int64_t)(id / ph) * pw + qx];
    return r;
  };
  // taps of one bin; kRing: from the ring (level row y -> slot (row0 + y) & mask), else from global memory
  auto eval_store = [&](const SwBin& r, int px, int row0, const SwLevel& gq, auto from_ring) {
    constexpr bool kRing = decltype(from_ring)::value;
    if (r.id < 0) return;
    const int k = r.id / ph, py = r.id - k * ph;
    int ylo[2], yhi[2], xlo[2], xhi[2];
    float ly[2], lx[2];
    ylo[0] = (int)(short)(r.item.x & 0xffff), yhi[0] = r.item.x >> 16;
    ylo[1] = (int)(short)(r.item.y & 0xffff), yhi[1] = r.item.y >> 16;
    xlo[0] = (int)(short)(r.xtap.x & 0xffff), xhi[0] = r.xtap.x >> 16;
    xlo[1] = (int)(short)(r.xtap.y & 0xffff), xhi[1] = r.xtap.y >> 16;
    ly[0] = __int_as_float(r.item.z), ly[1] = __int_as_float(r.item.w);
    lx[0] = __int_as_float(r.xtap.z), lx[1] = __int_as_float(r.xtap.w);
    f32x2 v[2][2][4];
    bool ok[2][2];
#pragma unroll
    for (int iy = 0; iy < 2; ++iy)
#pragma unroll
      for (int ix = 0; ix < 2; ++ix) {
        ok[iy][ix] = ylo[iy] >= 0 && xlo[ix] >= 0;
        const int y0 = ok[iy][ix] ? ylo[iy] : 0, y1 = ok[iy][ix] ? yhi[iy] : 0;
        const int x0 = ok[iy][ix] ? xlo[ix] : 0, x1 = ok[iy][ix] ? xhi[ix] : 0;
        if constexpr (kRing) {
          const f32x2* r0 = reinterpret_cast<const f32x2*>(ring + ((row0 + y0) & (kSwRing - 1)) * RS);
          const f32x2* r1 = reinterpret_cast<const f32x2*>(ring + ((row0 + y1) & (kSwRing - 1)) * RS);
          v[iy][ix][0] = r0[x0];
          v[iy][ix][1] = r0[x1];
          v[iy][ix][2] = r1[x0];
          v[iy][ix][3] = r1[x1];
        } else {
          const int o[4] = {y0 * gq.sy4 + x0 * 4, y0 * gq.sy4 + x1 * 4, y1 * gq.sy4 + x0 * 4, y1 * gq.sy4 + x1 * 4};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[iy][ix][e] = f32x2{__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gq.fr, o[e], 0, 0)),
                                 __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gq.fr, o[e], gq.sc4, 0))};
        }
      }
    f32x2 acc = {0.0f, 0.0f};
#pragma unroll
    for (int iy = 0; iy < 2; ++iy) {
      const float hy = 1.0f - ly[iy];
#pragma unroll
      for (int ix = 0; ix < 2; ++ix) {
        const float hx = 1.0f - lx[ix];
        const float w1 = hy * hx, w2 = hy * lx[ix], w3 = ly[iy] * hx, w4 = ly[iy] * lx[ix];
        const f32x2* x = v[iy][ix];
        const f32x2 val = ((f32x2(w1) * x[0] + f32x2(w2) * x[1]) + f32x2(w3) * x[2]) + f32x2(w4) * x[3];
        acc = acc + (ok[iy][ix] ? val : f32x2{0.0f, 0.0f});
      }
    }
    const f32x2 res = acc * 0.25f;  // count = 2 x 2 samples: an exact power of two
    float* o = out + ((int64_t)k * c.C + 2 * cp) * nbins + py * pw + px;
    o[0] = res.x;
    o[nbins] = res.y;
  };

  // kSwDepth passes of records in flight (static register slots: the loop is unrolled by kSwDepth);
  // one barrier per global step, before its first pass
  const SwLevel none{};
  SwBin qb[kSwDepth];
#pragma unroll
  for (int u = 0; u < kSwDepth; ++u)
    if (u < npass) qb[u] = fetch(u);
  for (int p0 = 0; p0 < npass; p0 += kSwDepth) {
#pragma unroll
    for (int u = 0; u < kSwDepth; ++u) {
      const int p = p0 + u;
      if (p < npass) {
        const int d = pass[p].y;
        if (d < 0) __syncthreads();  // first pass of a step (uniform)
        const int l = (d >> 16) & 0x7fff;
        const SwBin cu = qb[u];
        if (p + kSwDepth < npass) qb[u] = fetch(p + kSwDepth);
        eval_store(cu, qx, lvi[3 * l + 1] * kSwStep, none, std::true_type{});
      }
    }
  }
  if (dbg && wave == kSwLoad && lane == 0) dbg[(int64_t)gridDim.x * 8 + blockIdx.x] = (int64_t)__builtin_amdgcn_s_memrealtime();

  // ---- long-span items of every level, straight from global memory (rare)
  for (int l = 0; l < L; ++l) {
    const int s0 = lvi[3 * l + 2], bs = s0 + nst_of(l);
    const int nbig = cnt[bs + 1 < nslots ? bs + 1 : bs] - cnt[bs];
    const int nb = (bs + 1 < nslots ? nbig : total - cnt[bs]);
    if (nb <= 0) continue;
    const SwLevel gq = sweep_level(lv, l, b, cp);
    for (int f = q; f < nb * pw; f += kSwLanes) {
      SwBin r;
      const int fi = f / pw, px = f - fi * pw;
      r.id = (int)list[cnt[bs] + fi];
      r.item = P.item[r.id];
      r.xtap = P.xtap[(int64_t)(r.id / ph) * pw + px];
      eval_store(r, px, 0, gq, std::false_type{});
    }
  }
}

// Backward as the same sweep, run in reverse roles.  The ring holds the gradient
// rows of this (image, channel pair) being accumulated: a step's rows enter the
// ring zeroed, every item adds its bins' weighted grad_out into them with LDS
// float atomics (the reference's grad * w / count per tap), and a row is written
// to the gradient tensor with plain stores once no later item can touch it
// (3 steps later: an item of step s reaches back kSwSpan - 1 rows).  Every
// gradient element of every level is written exactly once (rows without
// contributions as zeros), so the gradient needs no clearing and no global
// atomics.  Long-span items add with global atomics after the sweep.  Like
// torchvision's CUDA backward, the summation order (and the last bits) depends
// on the order of the LDS atomics.
template <int NI, int kMode = 0>  // kMode (diagnostics): 1 = plain LDS read-modify-write, 2 = no LDS update
__global__ void __launch_bounds__(kSwThreads) roi_sweep_bwd_kernel(RoiLevels lv, RoiCfg c, SwArgs A, SwPlan P,
                                                                   const float* __restrict__ gout) {
  constexpr int RS = (32 * NI + 1) * 8;
  static_assert(kSwSpan <= 2 * kSwStep + 1, "rows are flushed 3 steps after they enter the ring");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const SwLds D = sweep_lds(smem, A, RS);
  char* ring = D.ring;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int b = blockIdx.x / A.np, cp = blockIdx.x - b * A.np;
  const int L = lv.L;
  const int ph = c.ph, pw = c.pw, nbins = ph * pw;
  sweep_prologue<true>(lv, c, A, P, D, b);
  const int total = D.sc[0], npass = D.sc[1], G = D.sc[2];
  const int* lvi = D.lvi;

  if (wave < kSwLoad) {
    // ---- flushers: row kSwStep s + wave of each step: zero it on entry, write it out 3 steps later
    auto slot = [&](int g) { return ring + ((g * kSwStep + wave) & (kSwRing - 1)) * RS; };
    auto zero = [&](int g) {
      float4* r = reinterpret_cast<float4*>(slot(g));
      for (int e = lane; e < 16 * NI; e += kWave) r[e] = make_float4(0.f, 0.f, 0.f, 0.f);
    };
    auto flush = [&](int g) {
      if (g < 0 || g >= G) return;
      const int l = D.glev[g];
      const int y = (g - lvi[3 * l + 1]) * kSwStep + wave, H = lv.h[l], W = lv.w[l];
      if (y >= H) return;
      const f32x2* r = reinterpret_cast<const f32x2*>(slot(g));
      float* g0 = lv.grad[l] + (int64_t)b * lv.sb[l] + (int64_t)(2 * cp) * lv.sc[l] + (int64_t)y * lv.sy[l];
      float* g1 = g0 + lv.sc[l];
      for (int x = lane; x < W; x += kWave) {
        const f32x2 v = r[x];
        g0[x] = v.x;
        g1[x] = v.y;
      }
    };
    zero(0);
    for (int g = 0; g < G; ++g) {
      __syncthreads();  // step g is being evaluated; steps <= g - 1 are done
      flush(g - 3);
      zero(g + 1);
    }
    __syncthreads();  // the last step is done
    flush(G - 3);
    flush(G - 2);
    flush(G - 1);
    __threadfence();  // the rows are visible before the long-span atomics add on top
    __syncthreads();
    return;
  }

  // ---- compute waves: lane = (item slot qi, px) of a pass, one bin per pass
  const int q = (wave - kSwLoad) * kWave + lane;
  const int qi = q / pw, qx = q - qi * pw;
  struct SwGBin {
    int id;
    int4 item, xtap;
    float g0, g1;
  };
  auto load_bin = [&](int id, int px) {
    SwGBin r;
    r.id = id;
    const int i = id >= 0 ? id : 0;
    const int k = i / ph, py = i - k * ph;
    r.item = P.item[i];
    r.xtap = P.xtap[(int64_t)k * pw + px];
    const float* go = gout + ((int64_t)k * c.C + 2 * cp) * nbins + py * pw + px;
    r.g0 = go[0];
    r.g1 = go[nbins];
    return r;
  };
  auto fetch = [&](int p) {
    const int2 d = D.pass[p];
    return load_bin(qi < (d.y & 0xffff) ? (int)D.list[d.x + qi] : -1, qx);
  };
  // kRing: add into the ring (level row y -> slot (row0 + y) & mask), else global atomics
  auto scatter = [&](const SwGBin& r, int row0, float* g0, int64_t sy, int64_t sc, auto to_ring) {
    constexpr bool kRing = decltype(to_ring)::value;
    if (r.id < 0) return;
    const SwTaps t = sweep_taps(r.item, r.xtap);
#pragma unroll
    for (int iy = 0; iy < 2; ++iy) {
      if (t.ylo[iy] < 0) continue;
      const float hy = 1.0f - t.ly[iy];
#pragma unroll
      for (int ix = 0; ix < 2; ++ix) {
        if (t.xlo[ix] < 0) continue;
        const float hx = 1.0f - t.lx[ix];
        const float w[4] = {hy * hx, hy * t.lx[ix], t.ly[iy] * hx, t.ly[iy] * t.lx[ix]};
        const int ys[4] = {t.ylo[iy], t.ylo[iy], t.yhi[iy], t.yhi[iy]};
        const int xs[4] = {t.xlo[ix], t.xhi[ix], t.xlo[ix], t.xhi[ix]};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a0 = r.g0 * w[e] * 0.25f, a1 = r.g1 * w[e] * 0.25f;  // (g * w) / count, count = 4
          if constexpr (kRing) {
            float* cell = reinterpret_cast<float*>(ring + ((row0 + ys[e]) & (kSwRing - 1)) * RS) + 2 * xs[e];
            if (kMode == 0) {
              atomicAdd(cell, a0);
              atomicAdd(cell + 1, a1);
            } else if (kMode == 1) {
              cell[0] += a0;
              cell[1] += a1;
            } else if (a0 == 1234.5f) {
              cell[0] = a1;
            }
          } else {
            float* cell = g0 + ys[e] * sy + xs[e];
            atomicAdd(cell, a0);
            atomicAdd(cell + sc, a1);
          }
        }
      }
    }
  };
  SwGBin qb[kSwDepth];
#pragma unroll
  for (int u = 0; u < kSwDepth; ++u)
    if (u < npass) qb[u] = fetch(u);
  for (int p0 = 0; p0 < npass; p0 += kSwDepth) {
#pragma unroll
    for (int u = 0; u < kSwDepth; ++u) {
      const int p = p0 + u;
      if (p < npass) {
        const int d = D.pass[p].y;
        if (d < 0) __syncthreads();  // first pass of a step (uniform)
        const int l = (d >> 16) & 0x7fff;
        const SwGBin cu = qb[u];
        if (p + kSwDepth < npass) qb[u] = fetch(p + kSwDepth);
        scatter(cu, lvi[3 * l + 1] * kSwStep, nullptr, 0, 0, std::true_type{});
      }
    }
  }
  __syncthreads();  // the last step is done (the flushers write the last rows)
  __syncthreads();  // ... and have written them
  // ---- long-span items of every level: global atomics on top of the written rows (rare)
  for (int l = 0; l < L; ++l) {
    const int s0 = lvi[3 * l + 2], bs = s0 + sweep_nst(lv, l);
    const int nb = (l + 1 < L ? D.cnt[bs + 1] : total) - D.cnt[bs];
    if (nb <= 0) continue;
    float* g0 = lv.grad[l] + (int64_t)b * lv.sb[l] + (int64_t)(2 * cp) * lv.sc[l];
    for (int f = q; f < nb * pw; f += kSwLanes) {
      const int fi = f / pw, px = f - fi * pw;
      scatter(load_bin((int)D.list[D.cnt[bs] + fi], px), 0, g0, lv.sy[l], lv.sc[l], std::false_type{});
    }
  }
}

struct SwLayout {
  size_t key, item, xtap, total;
};

static SwLayout sweep_layout(int64_t K, int ph, int pw) {
  auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
  SwLayout z;
  z.key = 0;
  z.item = al((size_t)K * ph * 4);
  z.xtap = z.item + al((size_t)K * ph * 16);
  z.total = z.xtap + al((size_t)K * pw * 16);
  return z;
}

}  // namespace frh

using namespace frh;

extern "C" size_t frh_roi_align_sweep_workspace(int64_t num_rois, int32_t pooled_h, int32_t pooled_w) {
  if (num_rois < 0 || pooled_h < 1 || pooled_w < 1) return 0;
  return sweep_layout(num_rois, pooled_h, pooled_w).total;
}

// Shape / layout requirements of the sweep kernel; anything else takes the per-RoI kernels.
static bool sweep_supported(const RoiLevels& lv, int32_t batch, int32_t channels, int64_t K, int32_t ph, int32_t pw,
                            int32_t sr, int* ni, int* max_slots, int* max_pass, size_t* lds) {
  if (sr != 2 || channels % 2 != 0 || pw > kWave || K * ph > 65535 || K * ph < 1) return false;
  if ((int64_t)batch * lv.L > 65535) return false;
  int maxw = 0, slots = 0;
  for (int l = 0; l < lv.L; ++l) {
    if (lv.sx[l] != 1 || lv.sc[l] < 0 || lv.sy[l] < 0 || lv.sb[l] < 0) return false;
    const int64_t ext = ((int64_t)lv.sc[l] + (int64_t)(lv.h[l] - 1) * lv.sy[l] + lv.w[l]) * 4;
    if (ext >= ((int64_t)1 << 31)) return false;
    maxw = std::max(maxw, (int)lv.w[l]);
    slots += (lv.h[l] + kSwStep - 1) / kSwStep + 1;
  }
  if (maxw > 256) return false;
  *ni = maxw <= 32 ? 1 : (maxw <= 64 ? 2 : (maxw <= 128 ? 4 : 8));
  *max_slots = slots;
  const int ipp = kSwLanes / pw;
  *max_pass = (int)(slots + (K * ph + ipp - 1) / ipp + 1);
  *lds = 128 + (size_t)kSwRing * (32 * *ni + 1) * 8 + (size_t)*max_pass * 8 + (size_t)2 * slots * 4 +
         (size_t)K * ph * 2 + (size_t)slots;
  *lds = (*lds + 15) & ~(size_t)15;
  return *lds <= 160 * 1024;
}

extern "C" int32_t frh_roi_align_fwd_sweep(int32_t num_levels, const float* const* feats, const int32_t* feat_hw,
                                           const int64_t* strides, const float* scales, int32_t batch,
                                           int32_t channels, const float* rois, const int64_t* roi_levels,
                                           int64_t num_rois, int32_t pooled_h, int32_t pooled_w,
                                           int32_t sampling_ratio, int32_t aligned, float* out, void* workspace,
                                           size_t ws_bytes, void* stream) {
  FRH_REQUIRE(batch >= 1 && channels >= 1 && num_rois >= 0 && pooled_h >= 1 && pooled_w >= 1, "bad sizes");
  FRH_REQUIRE(num_levels >= 1 && num_levels <= FRH_MAX_LEVELS && feat_hw && strides && scales, "bad levels");
  if (num_rois == 0) return FRH_OK;
  FRH_REQUIRE(feats && rois && out, "null pointer argument");
  RoiLevels lv;
  lv.L = num_levels;
  for (int l = 0; l < num_levels; ++l) {
    lv.feat[l] = feats[l];
    lv.grad[l] = nullptr;
    lv.h[l] = feat_hw[2 * l];
    lv.w[l] = feat_hw[2 * l + 1];
    FRH_REQUIRE(lv.h[l] > 0 && lv.w[l] > 0, "level %d has an empty feature map", l);
    lv.sb[l] = strides[4 * l];
    lv.sc[l] = strides[4 * l + 1];
    lv.sy[l] = strides[4 * l + 2];
    lv.sx[l] = strides[4 * l + 3];
    lv.scale[l] = scales[l];
  }
  int ni = 0, max_slots = 0, max_pass = 0;
  size_t lds = 0;
  const SwLayout z = sweep_layout(num_rois, pooled_h, pooled_w);
  if (!sweep_supported(lv, batch, channels, num_rois, pooled_h, pooled_w, sampling_ratio, &ni, &max_slots, &max_pass, &lds) ||
      !workspace || ws_bytes < z.total)
    return frh_roi_align_fwd_strided(num_levels, feats, feat_hw, strides, scales, batch, channels, rois, roi_levels,
                                     num_rois, pooled_h, pooled_w, sampling_ratio, aligned, out, stream);
  char* ws = static_cast<char*>(workspace);
  static int dbg_on = -1;
  if (dbg_on < 0) dbg_on = getenv("FRH_SWEEP_DBG") ? 1 : 0;
  const size_t ntask = (size_t)batch * (channels / 2);
  int64_t* dbg = (dbg_on && ws_bytes >= z.total + ntask * 9 * 8) ? reinterpret_cast<int64_t*>(ws + z.total) : nullptr;
  SwPlan P{reinterpret_cast<uint32_t*>(ws + z.key), reinterpret_cast<int4*>(ws + z.item),
           reinterpret_cast<int4*>(ws + z.xtap)};
  RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned};
  hipStream_t st = as_stream(stream);
  const int64_t nplan = num_rois * std::max(pooled_h, pooled_w);
  hipLaunchKernelGGL(roi_sweep_plan_kernel, dim3((unsigned)((nplan + 255) / 256)), dim3(256), 0, st, lv, c, batch, P);
  SwArgs A{batch, channels / 2, max_slots, (int)(num_rois * pooled_h), max_pass};
  const dim3 grid((unsigned)(batch * (channels / 2)));
  static bool attr_done[4] = {false, false, false, false};
  const void* fn = ni == 1 ? (const void*)roi_sweep_fwd_kernel<1> : ni == 2 ? (const void*)roi_sweep_fwd_kernel<2>
                 : ni == 4 ? (const void*)roi_sweep_fwd_kernel<4> : (const void*)roi_sweep_fwd_kernel<8>;
  const int ai = ni == 1 ? 0 : (ni == 2 ? 1 : (ni == 4 ? 2 : 3));
  if (!attr_done[ai]) {
    FRH_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_done[ai] = true;
  }
  if (ni == 1)
    hipLaunchKernelGGL(roi_sweep_fwd_kernel<1>, grid, dim3(kSwThreads), lds, st, lv, c, A, P, out, dbg);
  else if (ni == 2)
    hipLaunchKernelGGL(roi_sweep_fwd_kernel<2>, grid, dim3(kSwThreads), lds, st, lv, c, A, P, out, dbg);
  else if (ni == 4)
    hipLaunchKernelGGL(roi_sweep_fwd_kernel<4>, grid, dim3(kSwThreads), lds, st, lv, c, A, P, out, dbg);
  else
    hipLaunchKernelGGL(roi_sweep_fwd_kernel<8>, grid, dim3(kSwThreads), lds, st, lv, c, A, P, out, dbg);
  return check_launch("frh_roi_align_fwd_sweep");
}

extern "C" int32_t frh_roi_align_bwd_sweep(int32_t num_levels, float* const* grad_feats, const int32_t* feat_hw,
                                           const int64_t* strides, const float* scales, int32_t batch,
                                           int32_t channels, const float* rois, const int64_t* roi_levels,
                                           int64_t num_rois, int32_t pooled_h, int32_t pooled_w,
                                           int32_t sampling_ratio, int32_t aligned, const float* grad_out,
                                           void* workspace, size_t ws_bytes, void* stream) {
  FRH_REQUIRE(batch >= 1 && channels >= 1 && num_rois >= 0 && pooled_h >= 1 && pooled_w >= 1, "bad sizes");
  FRH_REQUIRE(num_levels >= 1 && num_levels <= FRH_MAX_LEVELS && feat_hw && strides && scales, "bad levels");
  FRH_REQUIRE(grad_feats, "null pointer argument");
  RoiLevels lv;
  lv.L = num_levels;
  for (int l = 0; l < num_levels; ++l) {
    lv.feat[l] = nullptr;
    lv.grad[l] = grad_feats[l];
    lv.h[l] = feat_hw[2 * l];
    lv.w[l] = feat_hw[2 * l + 1];
    FRH_REQUIRE(lv.h[l] > 0 && lv.w[l] > 0, "level %d has an empty feature map", l);
    lv.sb[l] = strides[4 * l];
    lv.sc[l] = strides[4 * l + 1];
    lv.sy[l] = strides[4 * l + 2];
    lv.sx[l] = strides[4 * l + 3];
    lv.scale[l] = scales[l];
  }
  int ni = 0, max_slots = 0, max_pass = 0;
  size_t lds = 0;
  const SwLayout z = sweep_layout(num_rois, pooled_h, pooled_w);
  hipStream_t st = as_stream(stream);
  const bool ok = num_rois > 0 && rois && grad_out && workspace && ws_bytes >= z.total &&
                  sweep_supported(lv, batch, channels, num_rois, pooled_h, pooled_w, sampling_ratio, &ni, &max_slots,
                                  &max_pass, &lds);
  if (!ok) {  // the caller clears the gradient and takes frh_roi_align_bwd_strided
    set_error("frh_roi_align_bwd_sweep: shape / layout / workspace outside the sweep kernel");
    return FRH_EUNSUPPORTED;
  }
  char* ws = static_cast<char*>(workspace);
  SwPlan P{reinterpret_cast<uint32_t*>(ws + z.key), reinterpret_cast<int4*>(ws + z.item),
           reinterpret_cast<int4*>(ws + z.xtap)};
  RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned};
  const int64_t nplan = num_rois * std::max(pooled_h, pooled_w);
  hipLaunchKernelGGL(roi_sweep_plan_kernel, dim3((unsigned)((nplan + 255) / 256)), dim3(256), 0, st, lv, c, batch, P);
  SwArgs A{batch, channels / 2, max_slots, (int)(num_rois * pooled_h), max_pass};
  const dim3 grid((unsigned)(batch * (channels / 2)));
  static bool attr_done[4] = {false, false, false, false};
  const void* fn = ni == 1 ? (const void*)roi_sweep_bwd_kernel<1, 0> : ni == 2 ? (const void*)roi_sweep_bwd_kernel<2, 0>
                 : ni == 4 ? (const void*)roi_sweep_bwd_kernel<4, 0> : (const void*)roi_sweep_bwd_kernel<8, 0>;
  const int ai = ni == 1 ? 0 : (ni == 2 ? 1 : (ni == 4 ? 2 : 3));
  if (!attr_done[ai]) {
    FRH_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_done[ai] = true;
  }
  static int bwd_mode = -1;
  if (bwd_mode < 0) bwd_mode = getenv("FRH_SWEEP_BWD_MODE") ? atoi(getenv("FRH_SWEEP_BWD_MODE")) : 0;
  if (ni == 8 && bwd_mode == 1) {
    FRH_HIP(hipFuncSetAttribute((const void*)roi_sweep_bwd_kernel<8, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipLaunchKernelGGL((roi_sweep_bwd_kernel<8, 1>), grid, dim3(kSwThreads), lds, st, lv, c, A, P, grad_out);
  } else if (ni == 8 && bwd_mode == 2) {
    FRH_HIP(hipFuncSetAttribute((const void*)roi_sweep_bwd_kernel<8, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipLaunchKernelGGL((roi_sweep_bwd_kernel<8, 2>), grid, dim3(kSwThreads), lds, st, lv, c, A, P, grad_out);
  } else if (ni == 1)
    hipLaunchKernelGGL(roi_sweep_bwd_kernel<1>, grid, dim3(kSwThreads), lds, st, lv, c, A, P, grad_out);
  else if (ni == 2)
    hipLaunchKernelGGL(roi_sweep_bwd_kernel<2>, grid, dim3(kSwThreads), lds, st, lv, c, A, P, grad_out);
  else if (ni == 4)
    hipLaunchKernelGGL(roi_sweep_bwd_kernel<4>, grid, dim3(kSwThreads), lds, st, lv, c, A, P, grad_out);
  else
    hipLaunchKernelGGL(roi_sweep_bwd_kernel<8>, grid, dim3(kSwThreads), lds, st, lv, c, A, P, grad_out);
  return check_launch("frh_roi_align_bwd_sweep");
}
