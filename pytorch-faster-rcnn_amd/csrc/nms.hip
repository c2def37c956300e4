// a10: greedy NMS with torchvision.ops.nms semantics on pre-sorted segments
// (call sites lib/heads/rpn_head.py:103, lib/utils.py:220).
//
// Two launches:
//  mask: one wave per (segment, 64-row block, 64-col block >= row block);
//        lane i sets bit j when IoU(row i, col j) > thr (j after i), the
//        64 column boxes staged in LDS.  Rows are 64-bit words per col block.
//  scan: one workgroup per segment walks the row blocks in score order.
//        Wave 0 resolves the block's 64 candidates sequentially with
//        readlane'd diagonal words (pure register/SALU work), then all
//        waves OR the kept rows' words into the LDS suppression bitmap with
//        8 independent loads per lane in flight.
#include <stdlib.h>
#include <string.h>

#include <math.h>

#include <type_traits>

#include "block_ops.h"

namespace frh {

constexpr int kMaxNmsWords = 256;  // n <= 16384 boxes per segment

// The suppression test IoU > thr without the division.  v = RN(inter / union) is
// a float, so v > thr (double) <=> v >= t_up, the smallest float above thr, <=>
// inter / union > mid = (t_dn + t_up) / 2 (ties: round-half-even picks t_up iff its
// significand is even).  mid has 25 significant bits and union 24, so mid * union
// is exact in double and the comparison below decides exactly what the reference's
// float division + double compare decides.  union <= 0 / NaN take the division.
struct NmsThr {
  double thr, mid;
  int tie_up, fast;
};

static NmsThr nms_thr(double thr) {
  NmsThr t{thr, 0.0, 0, 0};
  if (!(thr > 0.0 && thr < 1.0)) return t;
  float up = (float)thr;
  if ((double)up <= thr) up = nextafterf(up, 2.0f);
  const float dn = nextafterf(up, 0.0f);
  t.mid = 0.5 * ((double)dn + (double)up);
  uint32_t bits;
  memcpy(&bits, &up, 4);
  t.tie_up = (bits & 1u) == 0;
  t.fast = 1;
  return t;
}

// kFast (0 < thr < 1): IoU <= 0 or NaN whenever union <= 0 or NaN, never above thr
template <bool kFast>
__device__ __forceinline__ bool iou_above(float4 a, float area_a, float4 b, float area_b, const NmsThr& T) {
  const float w = fmaxf(0.0f, fminf(a.z, b.z) - fmaxf(a.x, b.x));
  const float h = fmaxf(0.0f, fminf(a.w, b.w) - fmaxf(a.y, b.y));
  const float inter = w * h;
  const float uni = (area_a + area_b) - inter;
  if (kFast) {  // bitwise, not short-circuit: no branches in the unrolled column loop
    const double lhs = (double)inter, rhs = T.mid * (double)uni;
    return (uni > 0.0f) & ((lhs > rhs) | ((lhs == rhs) & (T.tie_up != 0)));
  }
  return (double)(inter / uni) > T.thr;
}

// one wave per (segment, 64-row block, 64-col block >= row block); four column
// blocks per 256-thread workgroup, each wave staging its own column boxes
template <int kMode = 0>  // timing diagnostics only (tools/bench_nms.py): 1 = no IoU loop, 2 = no store
__global__ void __launch_bounds__(256) nms_mask_kernel(const float* __restrict__ boxes, int64_t seg_stride,
                                                       const int32_t* __restrict__ counts, int64_t n_max, int nbw,
                                                       NmsThr T, uint64_t* __restrict__ mask) {
  __shared__ float4 cb_box_all[4][64];
  __shared__ float cb_area_all[4][64];
  const int wv = threadIdx.x >> 6, t = threadIdx.x & 63;
  const int s = blockIdx.z, rb = blockIdx.y, cb = blockIdx.x * 4 + wv;
  if (cb < rb || cb >= nbw) return;
  const int n = counts[s];
  if (rb * 64 >= n || cb * 64 >= n) return;
  float4* cb_box = cb_box_all[wv];
  float* cb_area = cb_area_all[wv];
  const float4* bx = reinterpret_cast<const float4*>(boxes + (int64_t)s * seg_stride);
  const int col = cb * 64 + t;
  if (col < n) {
    float4 c = bx[col];
    cb_box[t] = c;
    cb_area[t] = (c.z - c.x) * (c.w - c.y);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int row = rb * 64 + t;
  if (row >= n) return;
  const float4 a = bx[row];
  const float aa = (a.z - a.x) * (a.w - a.y);
  const int ncols = min(64, n - cb * 64);
  const int start = (cb == rb) ? t + 1 : 0;
  uint64_t bits = 0;
  // uniform trip count, unrolled: the LDS broadcast reads of 8 column boxes issue together
  // (columns outside [start, ncols) are masked, their LDS slots may hold stale boxes)
  if (kMode != 1) {
    auto sweep = [&](auto fast) {
      constexpr bool F = decltype(fast)::value;
      for (int j0 = 0; j0 < 64; j0 += 8) {
        float4 cbx[8];
        float cba[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          cbx[u] = cb_box[j0 + u];
          cba[u] = cb_area[j0 + u];
        }
        uint32_t hit = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) hit |= (uint32_t)iou_above<F>(a, aa, cbx[u], cba[u], T) << u;
        bits |= (uint64_t)hit << j0;
      }
    };
    if (T.fast)
      sweep(std::true_type{});
    else
      sweep(std::false_type{});
    // columns outside [start, ncols) (stale LDS slots, the diagonal and below)
    const uint64_t hi = ncols >= 64 ? ~0ull : ((1ull << ncols) - 1ull);
    const uint64_t lo = start >= 64 ? ~0ull : ((1ull << start) - 1ull);
    bits &= hi & ~lo;
  }
  if (kMode != 2 || bits == 12345ull) mask[((int64_t)s * n_max + row) * nbw + cb] = bits;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readfirstlane64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

__global__ void __launch_bounds__(256) nms_scan_kernel(const uint64_t* __restrict__ mask,
                                                       const int32_t* __restrict__ counts, int64_t n_max, int nbw,
                                                       int max_keep, int32_t* __restrict__ keep, int64_t kstride,
                                                       int32_t* __restrict__ kcounts) {
  __shared__ uint64_t remv[kMaxNmsWords];
  __shared__ uint64_t s_kb;
  __shared__ int s_nkeep;
  const int s = blockIdx.x, tid = threadIdx.x;
  const int n = counts[s];
  const int nb = (n + 63) >> 6;
  for (int w = tid; w < nb; w += blockDim.x) remv[w] = 0;
  if (tid == 0) s_nkeep = 0;
  __syncthreads();
  const uint64_t* M = mask + (int64_t)s * n_max * nbw;
  int32_t* K = keep + (int64_t)s * kstride;
  const int q = tid & 31, rg = tid >> 5;  // word offset / row group of 8 for the OR phase
  for (int b = 0; b < nb; ++b) {
    const int nk = s_nkeep;
    if (max_keep >= 0 && nk >= max_keep) break;
    if (tid < 64) {
      const int row = b * 64 + tid;
      const uint64_t diag = row < n ? M[(int64_t)row * nbw + b] : 0ull;
      uint64_t r = remv[b];
      const int valid = n - b * 64;
      if (valid < 64) r |= (~0ull) << valid;
      uint64_t kb = 0;
      for (int i = 0; i < 64; ++i) {
        uint64_t di = readlane64(diag, i);
        if (!((r >> i) & 1ull)) {
          kb |= 1ull << i;
          r |= di;
        }
      }
      if (max_keep >= 0) {
        int room = max_keep - nk;
        while (__popcll(kb) > room) kb &= ~(1ull << (63 - __clzll(kb)));  // drop lowest-score extras
      }
      if ((kb >> tid) & 1ull) K[nk + __popcll(kb & lanemask_lt())] = row;
      if (tid == 0) {
        s_kb = kb;
        s_nkeep = nk + __popcll(kb);
      }
    }
    __syncthreads();
    const uint64_t kb = s_kb;
    if (kb) {
      for (int w0 = b + 1; w0 < nb; w0 += 32) {
        const int w = w0 + q;
        if (w < nb) {
          uint64_t v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            int row = b * 64 + rg * 8 + j;
            row = row < n ? row : n - 1;
            v[j] = M[(int64_t)row * nbw + w];
          }
          uint64_t acc = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc |= ((kb >> (rg * 8 + j)) & 1ull) ? v[j] : 0ull;
          if (acc) atomicOr((unsigned long long*)&remv[w], (unsigned long long)acc);
        }
      }
    }
    __syncthreads();
  }
  if (tid == 0) kcounts[s] = s_nkeep;
}

// Pipelined scan: the resolve chain of one segment never waits on memory.
//  wave 0 (resolver), per 64-row block b: suppression word remv[b] | own,
//    resolve the 64 candidates by visiting only unsuppressed ones (lowest set
//    bit of the complement, readlane of the diagonal word), publish the kept
//    bits, and OR the kept rows' word b+1 itself (wave-wide OR) -> `own` for
//    the next block.  Its diagonal / next-word tiles come from an LDS ring.
//  wave 1 (loader): stages the diagonal and next-word tiles of blocks ahead
//    of the resolver into a kNmsRing-deep LDS ring.
//  waves 2..3 (helpers), per block j: prefetch rows of block j for words
//    >= j+2 BEFORE its kept bits exist, then OR the kept rows into remv with
//    LDS atomics and publish their own progress (one counter per wave).  The resolver needs block j's
//    helpers only at block j+2: one block of slack.
// Wave hand-off is through LDS counters (release/acquire, workgroup scope).
constexpr int kNmsHelpers = 2;
constexpr int kNmsRing = 8;
constexpr int kNmsRowGroups = kNmsHelpers * kWave / 32;  // 4 row groups x 32 word lanes
constexpr int kNmsRowsPer = 64 / kNmsRowGroups;

// OR over the 64 lanes with DPP row ops (no LDS round trip); uniform result.
__device__ __forceinline__ uint32_t wave_or_u32_dpp(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false);  // row_half_mirror
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false);  // row_mirror
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast15
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint64_t wave_or_u64_dpp(uint64_t v) {
  return ((uint64_t)wave_or_u32_dpp((uint32_t)(v >> 32)) << 32) | wave_or_u32_dpp((uint32_t)v);
}

__device__ __forceinline__ int lds_acquire(int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ uint64_t wave_or_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t w = ((uint64_t)(uint32_t)__shfl_xor((int)(v >> 32), o, kWave) << 32) |
                       (uint32_t)__shfl_xor((int)(uint32_t)v, o, kWave);
    v |= w;
  }
  return v;
}

template <int kParallel>
__global__ void __launch_bounds__(256) nms_scan_pipe_kernel(const uint64_t* __restrict__ mask,
                                                            const int32_t* __restrict__ counts, int64_t n_max,
                                                            int nbw, int max_keep, int32_t* __restrict__ keep,
                                                            int64_t kstride, int32_t* __restrict__ kcounts,
                                                            uint64_t* __restrict__ dbg) {
  __shared__ uint64_t remv[kMaxNmsWords];
  __shared__ uint64_t kbs[kMaxNmsWords];
  __shared__ uint64_t ring_diag[kNmsRing][kWave], ring_next[kNmsRing][kWave];
  __shared__ int s_resolved, s_tiles, s_stop;
  __shared__ int s_applied[kNmsHelpers];  // per helper wave: blocks applied (a shared count could hide a laggard)
  const int s = blockIdx.x, tid = threadIdx.x, wave = tid / kWave, lane = tid & (kWave - 1);
  const int n = counts[s];
  const int nb = (n + 63) >> 6;
  for (int w = tid; w < nb; w += blockDim.x) remv[w] = 0;
  if (tid < kNmsHelpers) s_applied[tid] = 0;
  if (tid == 0) {
    s_resolved = 0;
    s_tiles = 0;
    s_stop = nb;
  }
  __syncthreads();
  const uint64_t* M = mask + (int64_t)s * n_max * nbw;
  if (wave == 0) {
    int32_t* K = keep + (int64_t)s * kstride;
    int nk = 0;
    uint64_t own = 0;
    for (int b = 0; b < nb; ++b) {
      if (dbg && lane == 0) dbg[(int64_t)s * 4 * kMaxNmsWords + 4 * b] = wall_clock64();
      while (lds_acquire(&s_tiles) < b + 1) __builtin_amdgcn_s_sleep(1);
      if (dbg && lane == 0) dbg[(int64_t)s * 4 * kMaxNmsWords + 4 * b + 1] = wall_clock64();
      if (b >= 2)
        for (int hw = 0; hw < kNmsHelpers; ++hw)
          while (lds_acquire(&s_applied[hw]) < b - 1) __builtin_amdgcn_s_sleep(1);
      if (dbg && lane == 0) dbg[(int64_t)s * 4 * kMaxNmsWords + 4 * b + 2] = wall_clock64();
      const uint64_t diag = ring_diag[b % kNmsRing][lane], nxt = ring_next[b % kNmsRing][lane];
      // r / kb / todo are wave-uniform: readfirstlane makes that provable, so the
      // visit loop runs on the scalar unit (s_ff1, s_or) with one readlane pair each
      uint64_t r = readfirstlane64(remv[b] | own);
      const int valid = n - b * 64;
      if (valid < 64) r |= (~0ull) << valid;
      // Bit-parallel greedy: an undecided candidate with no undecided suppressor
      // before it is kept; the victims of the newly kept are dropped; repeat.
      // Same keep set as the one-by-one greedy (the lowest undecided index is
      // always decided, so it terminates), in rounds = suppression-chain depth.
      uint64_t kb = 0, und = ~r;
      if (kParallel == 1) {
        while (und) {
          const uint64_t sup = wave_or_u64_dpp(((und >> lane) & 1ull) ? diag : 0ull);
          const uint64_t nk = und & ~sup;
          kb |= nk;
          const uint64_t vic = wave_or_u64_dpp(((nk >> lane) & 1ull) ? diag : 0ull);
          und &= ~(nk | vic);
        }
      } else if (kParallel == 2) {
        while (und) {
          const uint64_t sup = readfirstlane64(wave_or_u64(((und >> lane) & 1ull) ? diag : 0ull));
          const uint64_t nk = und & ~sup;
          kb |= nk;
          const uint64_t vic = readfirstlane64(wave_or_u64(((nk >> lane) & 1ull) ? diag : 0ull));
          und &= ~(nk | vic);
        }
      } else {
        while (und) {
          const int i = __builtin_ctzll(und);
          kb |= 1ull << i;
          r |= readlane64(diag, i);
          und = ~r & ((i == 63) ? 0ull : (~0ull << (i + 1)));
        }
      }
      bool stop = false;
      if (max_keep >= 0) {
        const int room = max_keep - nk;
        while (__popcll(kb) > room) kb &= ~(1ull << (63 - __clzll(kb)));  // drop lowest-score extras
        stop = nk + __popcll(kb) >= max_keep;
      }
      if ((kb >> lane) & 1ull) K[nk + __popcll(kb & lanemask_lt())] = b * 64 + lane;
      nk += __popcll(kb);
      own = wave_or_u64_dpp(((kb >> lane) & 1ull) ? nxt : 0ull);
      if (dbg && lane == 0) dbg[(int64_t)s * 4 * kMaxNmsWords + 4 * b + 3] = wall_clock64();
      if (lane == 0) {
        kbs[b] = kb;
        if (stop) s_stop = b;
        lds_release(&s_resolved, stop ? nb + kNmsRing + 1 : b + 1);
      }
      if (stop) break;
    }
    if (lane == 0) kcounts[s] = nk;
  } else if (wave == 1) {
    for (int j = 0; j < nb; ++j) {
      const int row = j * 64 + lane, rc = row < n ? row : n - 1;
      const uint64_t d = M[(int64_t)rc * nbw + j];
      const uint64_t x = M[(int64_t)rc * nbw + (j + 1 < nbw ? j + 1 : j)];
      while (lds_acquire(&s_resolved) < j - kNmsRing + 1) __builtin_amdgcn_s_sleep(1);
      if (s_stop < j) break;
      ring_diag[j % kNmsRing][lane] = row < n ? d : 0ull;
      ring_next[j % kNmsRing][lane] = (row < n && j + 1 < nb) ? x : 0ull;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) lds_release(&s_tiles, j + 1);
    }
  } else {
    const int h = tid - 2 * kWave;   // 0 .. 127
    const int q = h & 31, rg = h >> 5;  // word lane, row group
    // rows of block j, first word chunk (word j + 2 + q), loaded one block ahead
    auto load = [&](int j, uint64_t (&v)[kNmsRowsPer]) {
      const int wq = j + 2 + q, wc = wq < nbw ? wq : nbw - 1;
#pragma unroll
      for (int t = 0; t < kNmsRowsPer; ++t) {
        const int rowj = j * 64 + rg + kNmsRowGroups * t;
        v[t] = M[(int64_t)(rowj < n ? rowj : n - 1) * nbw + wc];
      }
    };
    uint64_t v[kNmsRowsPer], vn[kNmsRowsPer];
    load(0, v);
    for (int j = 0; j < nb; ++j) {
      const int wq = j + 2 + q;
      load(j + 1 < nb ? j + 1 : j, vn);  // unconditional: keeps the vmcnt accounting exact
      while (lds_acquire(&s_resolved) < j + 1) __builtin_amdgcn_s_sleep(1);
      if (s_stop < j) break;
      const uint64_t kb = kbs[j];
      for (int w = wq; w < nb; w += 32) {
        uint64_t acc = 0;
#pragma unroll
        for (int t = 0; t < kNmsRowsPer; ++t) {
          const int rr = rg + kNmsRowGroups * t, rowj = j * 64 + rr;
          if (((kb >> rr) & 1ull) && rowj < n) acc |= (w == wq) ? v[t] : M[(int64_t)rowj * nbw + w];
        }
        if (acc) atomicOr((unsigned long long*)&remv[w], (unsigned long long)acc);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) lds_release(&s_applied[wave - 2], j + 1);
#pragma unroll
      for (int t = 0; t < kNmsRowsPer; ++t) v[t] = vn[t];
    }
  }
}

// tools/bench_nms.py hooks (not part of the public header): scan variant 0 = legacy
// block-synchronous scan, 1 = pipelined; optional per-block resolver timestamps.
static int g_nms_scan_variant = -1;
static int g_nms_mask_mode = 0;
static uint64_t* g_nms_dbg = nullptr;

int32_t launch_nms_sorted(int32_t S, const float* boxes, int64_t seg_stride, const int32_t* counts, int32_t n_max,
                          double thr, int32_t max_keep, int32_t* keep, int64_t kstride, int32_t* kcounts,
                          uint64_t* mask, hipStream_t st) {
  const int nbw = (n_max + 63) / 64;
  dim3 g((nbw + 3) / 4, nbw, S);
  if (g_nms_mask_mode == 1)
    hipLaunchKernelGGL(nms_mask_kernel<1>, g, dim3(256), 0, st, boxes, seg_stride, counts, (int64_t)n_max, nbw,
                       nms_thr(thr), mask);
  else if (g_nms_mask_mode == 2)
    hipLaunchKernelGGL(nms_mask_kernel<2>, g, dim3(256), 0, st, boxes, seg_stride, counts, (int64_t)n_max, nbw,
                       nms_thr(thr), mask);
  else
    hipLaunchKernelGGL(nms_mask_kernel<0>, g, dim3(256), 0, st, boxes, seg_stride, counts, (int64_t)n_max, nbw,
                       nms_thr(thr), mask);
  if (g_nms_scan_variant < 0) g_nms_scan_variant = getenv("FRH_NMS_SCAN_LEGACY") ? 0 : 1;
  if (g_nms_scan_variant == 0)
    hipLaunchKernelGGL(nms_scan_kernel, dim3(S), dim3(256), 0, st, mask, counts, (int64_t)n_max, nbw, max_keep, keep,
                       kstride, kcounts);
  else if (g_nms_scan_variant == 3)
    hipLaunchKernelGGL(nms_scan_pipe_kernel<2>, dim3(S), dim3(256), 0, st, mask, counts, (int64_t)n_max, nbw,
                       max_keep, keep, kstride, kcounts, g_nms_dbg);
  else if (g_nms_scan_variant == 2)
    hipLaunchKernelGGL(nms_scan_pipe_kernel<0>, dim3(S), dim3(256), 0, st, mask, counts, (int64_t)n_max, nbw,
                       max_keep, keep, kstride, kcounts, g_nms_dbg);
  else
    hipLaunchKernelGGL(nms_scan_pipe_kernel<1>, dim3(S), dim3(256), 0, st, mask, counts, (int64_t)n_max, nbw,
                       max_keep, keep, kstride, kcounts, g_nms_dbg);
  return check_launch("nms");
}

size_t nms_mask_bytes(int32_t S, int32_t n_max) {
  const size_t nbw = (size_t)((n_max + 63) / 64);
  return (size_t)S * (size_t)n_max * nbw * sizeof(uint64_t);
}

}  // namespace frh

using namespace frh;

extern "C" void frh_nms_mask_debug(int32_t mode) { g_nms_mask_mode = mode; }

extern "C" void frh_nms_scan_debug(int32_t variant, void* timestamps) {
  g_nms_scan_variant = variant;
  g_nms_dbg = reinterpret_cast<uint64_t*>(timestamps);
}

extern "C" size_t frh_nms_workspace(int32_t num_segs, int32_t n_max) {
  return nms_mask_bytes(num_segs, n_max > 0 ? n_max : 1);
}

extern "C" int32_t frh_nms_sorted(int32_t num_segs, const float* boxes, int64_t seg_stride, const int32_t* counts,
                                  int32_t n_max, double iou_thr, int32_t max_keep, int32_t* keep,
                                  int64_t keep_seg_stride, int32_t* keep_counts, void* workspace, size_t ws_bytes,
                                  void* stream) {
  FRH_REQUIRE(num_segs >= 0 && n_max >= 0, "negative sizes");
  if (num_segs == 0) return FRH_OK;
  FRH_REQUIRE(n_max <= 64 * kMaxNmsWords, "n_max %d exceeds %d", n_max, 64 * kMaxNmsWords);
  FRH_REQUIRE(boxes && counts && keep && keep_counts, "null pointer argument");
  FRH_REQUIRE(workspace && ws_bytes >= frh_nms_workspace(num_segs, n_max), "workspace too small");
  if (n_max == 0) {
    FRH_HIP(hipMemsetAsync(keep_counts, 0, sizeof(int32_t) * num_segs, as_stream(stream)));
    return FRH_OK;
  }
  return launch_nms_sorted(num_segs, boxes, seg_stride, counts, n_max, iou_thr, max_keep, keep, keep_seg_stride,
                           keep_counts, reinterpret_cast<uint64_t*>(workspace), as_stream(stream));
}
