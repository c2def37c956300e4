// a10: greedy NMS with torchvision.ops.nms semantics on pre-sorted segments
// (call sites lib/heads/rpn_head.py:103, lib/utils.py:220).
//
// Two launches:
//  mask: one wave per (segment, 64-row block rb, 64-col block cb >= rb) -- the
//        grid covers the upper triangle only.  The suppression relation is
//        stored as COLUMN words: for column j of the tile, the 64-bit set of
//        rows of block rb whose box suppresses box j (row < column, IoU > thr).
//        Layout: per segment the upper triangle, column-block-major (tile
//        (rb, cb) at cb (cb + 1) / 2 + rb, 64 words each), so the tiles of one
//        column block are contiguous; a segment's tiles start at seg_base[s]
//        (caller-computed, e.g. sized by each segment's own count) or at
//        s * tri(nbw) when seg_base is null.
//  scan: one workgroup per segment walks the blocks in score order (the
//        resolve chain of a segment is inherently sequential).  For block b the
//        column span of tiles (0..b, b) is staged in LDS by LDS-DMA ahead of
//        time; the suppression of b's candidates by all earlier kept rows is
//        one per-lane AND/OR pass over the span plus one ballot, and the
//        bit-parallel greedy over the 64 candidates is two ballots per round.
// The RPN proposals run the same mask and scan as ONE launch (nms_fused_kernel, below
// nms_scan_kernel): mask tiles and per-segment scans together, tile flags between them.
#include <stdlib.h>
#include <string.h>

#include <math.h>

#include <algorithm>
#include <atomic>
#include <type_traits>

#include "cdna.h"
#include "seg_topk.h"

namespace frh {

// n <= 184 320 boxes per segment: the scan's kept sets (23 KB of static LDS) beside its
// 128-KB staging ring fit a CU's 160 KB, and a segment's mask triangle (tri(nbw) x 512 B)
// stays below the 2 GB its buffer descriptor's 32-bit offsets address
constexpr int kMaxNmsWords = 2880;

// The suppression test IoU > thr without the division.  v = RN(inter / union) is
// a float, so v > thr (double) <=> v >= t_up, the smallest float above thr, <=>
// inter / union > mid = (t_dn + t_up) / 2 (ties: round-half-even picks t_up iff its
// significand is even).  mid has 25 significant bits and union 24, so mid * union
// is exact in double and the comparison below decides exactly what the reference's
// float division + double compare decides.  union <= 0 / NaN take the division.
// (This is torchvision's CPU rule; its CUDA kernel compares against float(thr) and
// differs exactly at IoU == float(thr) when float(thr) > thr, e.g. thr = 0.3:
// DESIGN.md §5, tests/test_hand_derived.py.)
struct NmsThr {
  double thr, mid;
  int tie_up, fast;
  float hi, lo;  // float bounds around mid (nms_thr): inter > RN(hi * union) => above, < RN(lo * union) => not
};

static NmsThr nms_thr(double thr) {
  NmsThr t{thr, 0.0, 0, 0, 0.0f, 0.0f};
  if (!(thr > 0.0 && thr < 1.0)) return t;
  float up = (float)thr;
  if ((double)up <= thr) up = nextafterf(up, 2.0f);
  const float dn = nextafterf(up, 0.0f);
  t.mid = 0.5 * ((double)dn + (double)up);
  uint32_t bits;
  memcpy(&bits, &up, 4);
  t.tie_up = (bits & 1u) == 0;
  t.fast = 1;
  // hi >= mid (1 + 2^-20), lo <= mid (1 - 2^-20): a float product RN(hi * u) is within a
  // factor (1 +- 2^-24) of hi * u, so for u >= 2^-100 (no underflow) inter > RN(hi * u)
  // implies inter > mid * u and inter < RN(lo * u) implies inter < mid * u.  Everything
  // else (IoU within ~1e-6 of thr, unions in (0, 2^-100]) takes the exact test; unions <= 0
  // or NaN are decided (not above) without it -- degenerate boxes are common in RPN output.
  t.hi = nextafterf((float)(t.mid * (1.0 + 0x1p-20)), 2.0f);
  t.lo = nextafterf((float)(t.mid * (1.0 - 0x1p-20)), 0.0f);
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

// min / max of finite non-negative floats as integer min / max of their bits (the same
// order; no IEEE-mode NaN quieting of memory operands, which doubles fminf / fmaxf)
__device__ __forceinline__ float nn_min(float x, float y) { return __int_as_float(min(__float_as_int(x), __float_as_int(y))); }
__device__ __forceinline__ float nn_max(float x, float y) { return __int_as_float(max(__float_as_int(x), __float_as_int(y))); }
__device__ __forceinline__ bool nn_finite(float4 v) {  // every coordinate in [+0, inf)
  return ((uint32_t)__float_as_int(v.x) < 0x7f800000u) & ((uint32_t)__float_as_int(v.y) < 0x7f800000u) &
         ((uint32_t)__float_as_int(v.z) < 0x7f800000u) & ((uint32_t)__float_as_int(v.w) < 0x7f800000u);
}

// The float filter of the exact test (0 < thr < 1): sets *amb when it cannot decide.
// kNN: both boxes' coordinates are finite and >= +0 (nn_finite).
template <bool kNN>
__device__ __forceinline__ bool iou_above_filter(float4 a, float area_a, float4 b, float area_b, const NmsThr& T,
                                                 bool* amb) {
  const float w = kNN ? fmaxf(0.0f, nn_min(a.z, b.z) - nn_max(a.x, b.x)) : fmaxf(0.0f, fminf(a.z, b.z) - fmaxf(a.x, b.x));
  const float h = kNN ? fmaxf(0.0f, nn_min(a.w, b.w) - nn_max(a.y, b.y)) : fmaxf(0.0f, fminf(a.w, b.w) - fmaxf(a.y, b.y));
  const float inter = w * h;
  const float uni = (area_a + area_b) - inter;
  // union <= 0 or NaN: decided (the exact test needs union > 0); 0 < union <= 2^-100 (the
  // products could underflow): undecided
  const bool pos = uni > 0x1p-100f;
  const bool above = pos & (inter > T.hi * uni);
  const bool below = !(uni > 0.0f) | (pos & (inter < T.lo * uni));
  *amb = !(above | below);
  return above;
}

__host__ __device__ __forceinline__ int64_t tri_tiles(int64_t nbw) { return nbw * (nbw + 1) / 2; }

// tile t of a segment's upper triangle, column-block-major: column blocks before cb
// hold cb (cb + 1) / 2 tiles; cb = max{c : c (c + 1) / 2 <= t}
__device__ __forceinline__ void tri_tile(int t, int* rb, int* cb) {
  int c = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
  c = max(c, 0);
  while (c > 0 && c * (c + 1) / 2 > t) --c;
  while ((c + 1) * (c + 2) / 2 <= t) ++c;
  *cb = c;
  *rb = t - c * (c + 1) / 2;
}

// first word of tile (rb, cb) of the segment whose tiles start at tile `base`
__device__ __forceinline__ int64_t tile_word(int64_t base, int rb, int cb) {
  return (base + (int64_t)cb * (cb + 1) / 2 + rb) * 64;
}

__device__ __forceinline__ int64_t seg_tile_base(const int64_t* seg_base, int s, int nbw) {
  return seg_base ? seg_base[s] : (int64_t)s * tri_tiles(nbw);
}

// One wave's tile (rb, cb) of a segment of n boxes: r = row box rb * 64 + t, a = column box
// cb * 64 + t (lane t); returns lane t's column word (0 past the count).  rb_box / rb_area:
// the wave's own 64-slot LDS staging.
__device__ __forceinline__ uint64_t mask_tile_word(float4 r, float4 a, int n, int rb, int cb, int t, const NmsThr& T,
                                                   float4* rb_box, float* rb_area) {
  const int row = rb * 64 + t, col = cb * 64 + t;
  const bool row_nn = row >= n || nn_finite(r);
  rb_box[t] = r;
  rb_area[t] = (r.z - r.x) * (r.w - r.y);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const bool cvalid = col < n;
  const float aa = (a.z - a.x) * (a.w - a.y);
  uint64_t colw = 0;
  // uniform trip count, unrolled: the LDS broadcast reads of 8 row boxes issue together
  // (rows past n are masked below, their LDS slots may hold stale boxes)
  auto sweep = [&](auto fast) {
    constexpr bool F = decltype(fast)::value;
#pragma nounroll
    for (int i0 = 0; i0 < 64; i0 += 8) {
      float4 rbx[8];
      float rba[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        rbx[u] = rb_box[i0 + u];
        rba[u] = rb_area[i0 + u];
      }
      uint32_t hit = 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) hit |= (uint32_t)iou_above<F>(rbx[u], rba[u], a, aa, T) << u;
      colw |= (uint64_t)hit << i0;
    }
  };
  // rows and column all finite and >= +0 (proposals clipped to the image): integer min / max
  const bool nn = !__builtin_amdgcn_ballot_w64(!(row_nn & (!cvalid || nn_finite(a))));
  auto filtered = [&](auto knn) {
    constexpr bool NN = decltype(knn)::value;
    // float filter; an 8-row batch with any undecided pair in the wave is redone exactly
#pragma nounroll
    for (int i0 = 0; i0 < 64; i0 += 8) {
      float4 rbx[8];
      float rba[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        rbx[u] = rb_box[i0 + u];
        rba[u] = rb_area[i0 + u];
      }
      uint32_t hit = 0;
      uint64_t amb = 0;  // wave masks (SALU): no per-lane bool materialisation
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        bool au;
        hit |= (uint32_t)iou_above_filter<NN>(rbx[u], rba[u], a, aa, T, &au) << u;
        amb |= __builtin_amdgcn_ballot_w64(au);
      }
      if (amb) {
        hit = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) hit |= (uint32_t)iou_above<true>(rbx[u], rba[u], a, aa, T) << u;
      }
      colw |= (uint64_t)hit << i0;
    }
  };
  if (T.fast && nn)
    filtered(std::true_type{});
  else if (T.fast)
    filtered(std::false_type{});
  else
    sweep(std::false_type{});
  const int nrows = min(64, n - rb * 64);
  if (nrows < 64) colw &= (1ull << nrows) - 1ull;
  if (cb == rb) colw &= t == 0 ? 0ull : (~0ull >> (64 - t));  // rows before the column only
  return cvalid ? colw : 0ull;
}

// Four tiles per 256-thread workgroup, each wave staging its tile's 64 ROW boxes in
// LDS; lane = column.  Lane j sweeps the rows and sets bit i of its column word when
// row i suppresses box j.  IoU is symmetric bit for bit (min / max and the area sum
// (area_i + area_j) - inter commute exactly), so this is the reference's test of the
// kept box i against candidate j.
__global__ void __launch_bounds__(256) nms_mask_kernel(const float* __restrict__ boxes, int64_t seg_stride,
                                                       const int32_t* __restrict__ counts, int n_max, int nbw,
                                                       NmsThr T, uint64_t* __restrict__ mask,
                                                       const int64_t* __restrict__ seg_base) {
  __shared__ float4 rb_box_all[4][64];
  __shared__ float rb_area_all[4][64];
  const int wv = threadIdx.x >> 6, t = threadIdx.x & 63;
  const int s = blockIdx.y, tile = blockIdx.x * 4 + wv;
  if (tile >= nbw * (nbw + 1) / 2) return;
  int rb, cb;
  tri_tile(__builtin_amdgcn_readfirstlane(tile), &rb, &cb);
  rb = __builtin_amdgcn_readfirstlane(rb);
  cb = __builtin_amdgcn_readfirstlane(cb);
  // the count, the row box and the column box in flight together (indices clamped to
  // the buffer: slots past the count are read, never used)
  const float4* bx = reinterpret_cast<const float4*>(boxes + (int64_t)s * seg_stride);
  const int n = counts[s];
  const float4 r = bx[min(rb * 64 + t, n_max - 1)];
  const float4 a = bx[min(cb * 64 + t, n_max - 1)];
  if (rb * 64 >= n || cb * 64 >= n) return;
  mask[tile_word(seg_tile_base(seg_base, s, nbw), rb, cb) + t] =
      mask_tile_word(r, a, n, rb, cb, t, T, rb_box_all[wv], rb_area_all[wv]);
}

__device__ __forceinline__ uint64_t readfirstlane64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// LDS flag poll by hand: ds_read_b32 + lgkmcnt(0) in one asm statement ("memory": later
// LDS reads stay behind it).  One CU serves a wave's LDS operations in order, so reads
// issued after the flag was seen observe what its writer stored before setting it.  The
// atomic-acquire form makes the compiler wait for the wave's in-flight LDS-DMA copies
// (s_waitcnt vmcnt(0)) before every poll.
__device__ __forceinline__ int lds_poll(int* p) {
  int v;
  const uint32_t a = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) int*)p);
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return __builtin_amdgcn_readfirstlane(v);
}
// The resolver's reads for one block in ONE asm statement: the block's ready flag first,
// then its partial word and three staged tiles, one wait.  One CU serves LDS requests in
// order, so if the flag read returns the block as ready, the reads issued after it see
// the data its loader stored (or whose LDS-DMA it waited for) before publishing.
__device__ __forceinline__ int lds_block_reads(const int* flag, const uint64_t* pa, const uint64_t* t1a,
                                               const uint64_t* t2a, const uint64_t* da, uint64_t& pw, uint64_t& t1,
                                               uint64_t& t2, uint64_t& d) {
  auto la = [](const void* q) {
    return (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)q);
  };
  int f;
  asm volatile(
      "ds_read_b32 %0, %5\n\t"
      "ds_read_b64 %1, %6\n\t"
      "ds_read_b64 %2, %7\n\t"
      "ds_read_b64 %3, %8\n\t"
      "ds_read_b64 %4, %9\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(f), "=&v"(pw), "=&v"(t1), "=&v"(t2), "=&v"(d)
      : "v"(la(flag)), "v"(la(pa)), "v"(la(t1a)), "v"(la(t2a)), "v"(la(da))
      : "memory");
  return __builtin_amdgcn_readfirstlane(f);
}

__device__ __forceinline__ int lds_acquire(int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// s_waitcnt vmcnt(N') for the largest supported N' <= n (waiting for fewer
// outstanding operations than needed is always safe)
__device__ __forceinline__ void wait_vmcnt_atmost(int n) {
  if (n >= 32) wait_vmcnt<32>();
  else if (n >= 16) wait_vmcnt<16>();
  else if (n >= 8) wait_vmcnt<8>();
  else if (n >= 4) wait_vmcnt<4>();
  else if (n >= 2) wait_vmcnt<2>();
  else if (n >= 1) wait_vmcnt<1>();
  else wait_vmcnt<0>();
}

// Scan, one 256-thread workgroup per segment: wave 0 resolves, waves 1..3 stage.
//
//  Loader (wave 1 + (b % 3) owns block b):
//   (1) once the ring slot b % kNmsRing is free (the resolver has finished block
//       b - kNmsRing), copies the column span of tiles (j, b), j in [j0, b],
//       j0 = max(0, b - kNmsSpan + 1) (contiguous in the mask) into the slot by
//       16-B LDS-DMA;
//   (2) one block later (after issuing its next block's copies, so the copies
//       overlap), waits for these copies (counted vmcnt) and for the resolver to
//       have finished block b - 3, and folds the kept rows of blocks j <= b - 3
//       into the slot's partial word: lane c = OR_j (tile(j, b)[c] & kept[j])
//       (LDS; tiles j < j0 from global memory);
//   (3) publishes ready[slot] = b + 1.
//  Resolver, block b: waits ready[b % kNmsRing] == b + 1, then
//    acc = partial | (tile(b-2, b) & kept[b-2]) | (tile(b-1, b) & kept[b-1])
//  -- the last two blocks' kept sets are in its own scalar registers --,
//    suppressed = ballot(acc != 0) | past-the-end columns,
//  resolves the 64 candidates with the diagonal tile (b, b) in bit-parallel
//  rounds (an undecided candidate with no undecided suppressor before it is kept,
//  its victims dropped; same keep set as the one-by-one greedy, rounds =
//  suppression-chain depth), stores the kept indices and kept[b] (LDS), then
//  publishes s_resolved = b + 1.
// Ordering.  All flags and shared data are in LDS, which one CU serves in order:
//  a flag store issued after a wave's LDS writes (or after the counted vmcnt wait
//  that shows its LDS-DMA copies landed) is observed after them, so plain
//  (relaxed) flag stores behind an `s_waitcnt lgkmcnt(0)` / vmcnt wait suffice, and
//  no release fence waits for the keep-list stores to global memory.
// Progress.  The resolver waits on ready[b], which needs the resolver at b - 3
//  (two blocks of slack for the loader's fold) and the slot at b - kNmsRing; a
//  loader waits only on s_resolved.  Every counter advances unconditionally, and a
//  max_keep stop sets s_stop and pushes s_resolved past the end so every loader exits.
constexpr int kNmsRing = 8;
constexpr int kNmsSpan = 32;     // tiles per staged span (segments up to 2048 boxes fully staged)
constexpr int kNmsLoaders = 3;

__device__ __forceinline__ void lds_flag(int* p, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// kStamp (tools-only timing build): per (segment, block) 8 int64 of s_memrealtime at
// stamps + (s * nbw + b) * 8: [0] resolver starts waiting, [1] block ready seen, [2]
// resolved and published, [3] loader published the fold, [4] loader issued the copies.
template <bool kStamp>
__global__ void __launch_bounds__(256) nms_scan_kernel(const uint64_t* __restrict__ mask,
                                                       const int32_t* __restrict__ counts, int nbw, int span,
                                                       int max_keep, int32_t* __restrict__ keep, int64_t kstride,
                                                       int32_t* __restrict__ kcounts,
                                                       const int64_t* __restrict__ seg_base, int64_t* stamps) {
  extern __shared__ __attribute__((aligned(16))) uint64_t nms_lds[];
  __shared__ uint64_t kept[kMaxNmsWords];
  __shared__ uint64_t partial[kNmsRing][kWave];
  __shared__ int ready[kNmsRing];
  __shared__ int s_resolved, s_stop;
  const int s = blockIdx.x, tid = threadIdx.x, lane = tid & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);  // uniform: the copies' offsets stay scalar
  const int n = counts[s];
  const int nb = (n + 63) >> 6;
  if (tid < kNmsRing) ready[tid] = 0;
  if (tid == 0) {
    s_resolved = 0;
    s_stop = nb;
  }
  __syncthreads();
  const int slot_words = ((span + 1) & ~1) * 64;  // whole 1 KB copies: an even number of tiles
  const int64_t base = seg_tile_base(seg_base, s, nbw);
  if (wave == 0) {
    int32_t* K = keep + (int64_t)s * kstride;
    int nk = 0;
    uint64_t kb1 = 0, kb2 = 0;  // kept sets of blocks b-1, b-2
    auto stamp = [&](int b, int i) {
      if (kStamp && lane == 0) stamps[((int64_t)s * nbw + b) * 8 + i] = (int64_t)__builtin_amdgcn_s_memrealtime();
    };
    for (int b = 0; b < nb; ++b) {
      stamp(b, 0);
      const uint64_t* slot = nms_lds + (b % kNmsRing) * slot_words;
      const int j0 = max(0, b - span + 1);
      // tiles b-1 and b-2 are always staged (span >= min(nbw, 3)); before block 2 the reads
      // are clamped into the slot and masked by the empty kept sets kb1 / kb2.  The block's
      // data is read together with its ready flag (the loaders are normally ahead); if it
      // was not ready, poll, then read again.
      const uint64_t* pa = &partial[b % kNmsRing][lane];
      const uint64_t* t1a = slot + max(b - 1 - j0, 0) * 64 + lane;
      const uint64_t* t2a = slot + max(b - 2 - j0, 0) * 64 + lane;
      const uint64_t* da = slot + (b - j0) * 64 + lane;
      uint64_t pw, t1, t2, d;
      if (lds_block_reads(&ready[b % kNmsRing], pa, t1a, t2a, da, pw, t1, t2, d) != b + 1) {
        while (lds_poll(&ready[b % kNmsRing]) != b + 1) __builtin_amdgcn_s_sleep(1);
        lds_block_reads(&ready[b % kNmsRing], pa, t1a, t2a, da, pw, t1, t2, d);
      }
      stamp(b, 1);
      const uint64_t acc = pw | (t1 & kb1) | (t2 & kb2);
      uint64_t r = __ballot(acc != 0ull);
      const int valid = n - b * 64;
      if (valid < 64) r |= (~0ull) << valid;
      uint64_t kb = 0, und = ~r;
      while (und) {
        const uint64_t sup = __ballot((d & und) != 0ull);
        const uint64_t nkp = und & ~sup;
        kb |= nkp;
        const uint64_t vic = __ballot((d & nkp) != 0ull);
        und &= ~(nkp | vic);
      }
      bool stop = false;
      if (max_keep >= 0) {
        const int room = max_keep - nk;
        while (__popcll(kb) > room) kb &= ~(1ull << (63 - __clzll(kb)));  // drop lowest-score extras
        stop = nk + __popcll(kb) >= max_keep;
      }
      if ((kb >> lane) & 1ull) K[nk + __popcll(kb & lanemask_lt())] = b * 64 + lane;
      nk += __popcll(kb);
      kb2 = kb1;
      kb1 = kb;
      if (lane == 0) {  // in-order LDS: the loaders see kept[b] / s_stop once they see the flag
        kept[b] = kb;
        if (stop) s_stop = b;
        asm volatile("" ::: "memory");
        __hip_atomic_store(&s_resolved, stop ? nb + kNmsRing + 1 : b + 1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      stamp(b, 2);
      if (stop) break;
    }
    if (lane == 0) kcounts[s] = nk;
  } else {
    // descriptor over this segment's tiles (its own count's triangle; a span copy that runs
    // one tile past the last column block reads zeros from the range check)
    const int64_t seg_words = tri_tiles(nb) * 64;
    const __amdgpu_buffer_rsrc_t mr = uniform_rsrc(mask + base * 64, seg_words * 8);
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint64_t*)nms_lds);
    auto finish = [&](int p) {  // fold the kept rows of blocks <= p - 3 into p's partial word, publish p
      while (lds_poll(&s_resolved) < p - 2) __builtin_amdgcn_s_sleep(1);
      if (s_stop < p) return;
      const uint64_t* slot = nms_lds + (p % kNmsRing) * slot_words;
      const int j0 = max(0, p - span + 1);
      uint64_t acc = 0;
      int j = 0;
      for (; j < j0 && j + 2 < p; ++j) acc |= mask[tile_word(base, j, p) + lane] & kept[j];
      for (; j + 8 <= p - 2; j += 8) {  // eight words per batch: their LDS reads overlap
        uint64_t t[8], k[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          t[u] = slot[(j + u - j0) * 64 + lane];
          k[u] = kept[j + u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc |= t[u] & k[u];
      }
      for (; j < p - 2; ++j) acc |= slot[(j - j0) * 64 + lane] & kept[j];
      partial[p % kNmsRing][lane] = acc;
      if (lane == 0) lds_flag(&ready[p % kNmsRing], p + 1);
      if (kStamp && lane == 0) stamps[((int64_t)s * nbw + p) * 8 + 3] = (int64_t)__builtin_amdgcn_s_memrealtime();
    };
    int prev = -1;
    for (int b = wave - 1; b < nb; b += kNmsLoaders) {
      while (lds_poll(&s_resolved) < b - kNmsRing + 1) __builtin_amdgcn_s_sleep(1);
      if (s_stop < b) break;
      const int j0 = max(0, b - span + 1);
      const int ninst = (b - j0 + 2) >> 1;  // 1 KB (two tiles) per wave-instruction
      const uint32_t dst = lds0 + (uint32_t)((b % kNmsRing) * slot_words * 8);
      const int src = (int)((tile_word(0, j0, b)) * 8);
      for (int k = 0; k < ninst; ++k) lds_dma_at<16>(mr, dst + (uint32_t)k * 1024u, lane * 16, src + k * 1024);
      if (kStamp && lane == 0) stamps[((int64_t)s * nbw + b) * 8 + 4] = (int64_t)__builtin_amdgcn_s_memrealtime();
      if (prev >= 0) {
        wait_vmcnt_atmost(ninst);  // prev's copies are older than these ninst
        asm volatile("" ::: "memory");
        finish(prev);
      }
      prev = b;
    }
    wait_vmcnt<0>();
    asm volatile("" ::: "memory");
    if (prev >= 0 && !(s_stop < prev)) finish(prev);
  }
}

// ---------------------------------------------------------------- one-launch NMS
// The RPN proposals' NMS (rpn_proposals_impl): mask and scan of every segment in ONE
// launch, so a segment's scan resolves its early blocks while the mask of its later
// columns is still being computed (the two-launch form above runs them back to back).
//  Grid (1-D, 512 threads): S scan workgroups first (blockIdx < S, dispatched first), then
//  mask workgroups of 8 tiles (one per wave) in COLUMN order across segments: global tile g
//  is column cb, segment s, row block rb with g = S cb (cb + 1) / 2 + s (cb + 1) + rb, so the
//  columns every scan needs first are dispatched first; mask waves of the first columns also
//  issue at a higher s_setprio than those of the last ones, and the scan waves at the top.
//  Hand-off (hand-off table row 1): a mask wave writes its 64 column words with sc1 stores,
//  waits vmcnt(0), then sets its tile's flag word (sc1 store); a loader polls a column's
//  flags and reads its tiles with sc1 loads.  Flags are zero on entry (the caller's
//  memset).  Mask workgroups wait for nothing; a scan workgroup waits only for mask
//  workgroups, but workgroups are dispatched in order, so no mask workgroup starts before
//  all S scan workgroups have: the S scan workgroups must be resident together with room
//  left for mask workgroups.  The host admits S <= a quarter of the device's resident
//  capacity of this kernel (nms_fused_fits: CU count x occupancy; 256 on a whole MI355X).
//  Every global wait is bounded (kSpinTicks): a wait that runs out ORs
//  FRH_DEVERR_NMS_COLUMN into the caller's status word and ends the scan workgroup's work
//  (the loader sets s_stop = -1 and wakes the resolver, which then stops and releases the
//  other loaders) -- never a hang, never a keep list from tiles that were not published.
//  Scan workgroup: wave 0 resolves as nms_scan_kernel's resolver, but ORs in FOUR near
//  tiles itself (p-1 .. p-4: the loaders' fold then waits for the resolver four blocks back,
//  not two -- with two, the fold hand-off chain, about 0.9 us per round, bounded the scan to
//  0.3 us per block); waves 1..7 stage block p (p = wave - 1 mod 7): once the ring slot is
//  free and column p is complete, the near tiles (p-i, p) and the diagonal (p, p) go to the
//  slot, and the fold of the kept rows of blocks <= p - 5 (tiles read into registers, 16
//  per batch) into the slot's partial word; then ready = p + 1.
constexpr int kFzThreads = 512;
constexpr int kFzWaves = kFzThreads / kWave;
constexpr int kFzLoaders = kFzWaves - 1;
constexpr int kFzRing = 8;
constexpr int kFzNear = 4;  // near tiles (p - i, p), i = 1..kFzNear, ORed in by the resolver
constexpr int kFzSlotWords = (kFzNear + 2) * kWave;  // [partial | tile (p-1, p) .. (p-4, p) | tile (p, p)] x 64 lanes

// The resolver's reads for one block of the one-launch scan in ONE asm statement: the
// ready flag, then the slot's partial word, its kFzNear near tiles and the diagonal tile
// (consecutive 512-byte rows of the slot), one wait -- as lds_block_reads.
__device__ __forceinline__ int fz_block_reads(const int* flag, const uint64_t* slot, uint64_t& pw, uint64_t (&nr)[4],
                                              uint64_t& d) {
  static_assert(kFzNear == 4, "fz_block_reads reads four near tiles");
  auto la = [](const void* q) {
    return (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)q);
  };
  int f;
  asm volatile(
      "ds_read_b32 %0, %7\n\t"
      "ds_read_b64 %1, %8\n\t"
      "ds_read_b64 %2, %8 offset:512\n\t"
      "ds_read_b64 %3, %8 offset:1024\n\t"
      "ds_read_b64 %4, %8 offset:1536\n\t"
      "ds_read_b64 %5, %8 offset:2048\n\t"
      "ds_read_b64 %6, %8 offset:2560\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(f), "=&v"(pw), "=&v"(nr[0]), "=&v"(nr[1]), "=&v"(nr[2]), "=&v"(nr[3]), "=&v"(d)
      : "v"(la(flag)), "v"(la(slot))
      : "memory");
  return __builtin_amdgcn_readfirstlane(f);
}
constexpr int kFzMaxSegs = 256;
constexpr int kFzMaxBlocks = 1024;  // kept sets in LDS: segments of up to 65 536 boxes

__device__ __forceinline__ void fz_setprio(int q) {  // s_setprio takes an immediate
  if (q >= 3) __builtin_amdgcn_s_setprio(3);
  else if (q == 2) __builtin_amdgcn_s_setprio(2);
  else if (q == 1) __builtin_amdgcn_s_setprio(1);
}

// a staged tile word, read sc1 like every hand-off word (a plain load measured no faster:
// the words come from other XCDs' write-through stores either way)
__device__ __forceinline__ uint64_t fz_tile(const uint64_t* p) { return xwg_load(p); }

// wait until the flags of tiles (0..p, p) -- contiguous from col_flags -- are all set;
// false when the wait ran out (status flagged) or the workgroup is stopping (s_stop < 0)
__device__ __forceinline__ bool fz_wait_column(const uint32_t* col_flags, int p, int lane, int32_t* status,
                                               int* s_stop) {
  for (int j0 = 0; j0 <= p; j0 += kWave) {
    const int cnt = min(kWave, p + 1 - j0);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (true) {
      const uint32_t v = lane < cnt ? xwg_load(col_flags + j0 + lane) : 1u;
      if (!__ballot(v == 0u)) break;
      __builtin_amdgcn_s_sleep(1);
      if (lds_poll(s_stop) < 0) return false;
      if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
        if (lane == 0) atomicOr(status, FRH_DEVERR_NMS_COLUMN);
        return false;
      }
    }
  }
  return true;
}

// kscore (RPN proposals, else null): the kept rows' scores, compact beside the keep list
// ([s * n_max + j] = score of keep[j]), for the cross-level merge launch (proposals.hip
// rpn_merge_wide_kernel: one round trip to gather them instead of keep index -> score).  The
// loaders stage block p's 64 row scores in the LDS ring beside its tiles; the resolver stores
// the kept ones.
//
// kStamp (tools-only timing build): s_memrealtime per (segment, block) at stamps +
// (s * nbw + b) * 8: [0] loader starts b (slot free), [1] column b seen complete, [2] b
// published, [3] b resolved, [4] / [5] the fold's last batch waits for / got the kept sets;
// then per tile at stamps + S * nbw * 8 + s * tri + tile: its flag set.
template <bool kStamp>
__global__ void __launch_bounds__(kFzThreads) __attribute__((amdgpu_waves_per_eu(8))) nms_fused_kernel(int S, const float* __restrict__ boxes,
                                                               int64_t seg_stride, const int32_t* __restrict__ counts,
                                                               int n_max, int nbw, NmsThr T, uint64_t* mask,
                                                               uint32_t* flags, int max_keep,
                                                               int32_t* __restrict__ keep, int64_t kstride,
                                                               int32_t* __restrict__ kcounts, int32_t* status,
                                                               int64_t* stamps, const float* __restrict__ row_scores,
                                                               uint32_t* __restrict__ kscore) {
  // scan: ring [kFzRing][kFzSlotWords] then kept[kFzMaxBlocks]; mask: per wave 64 row boxes + areas
  __shared__ __attribute__((aligned(16))) uint64_t fz_lds[kFzRing * kFzSlotWords + kFzMaxBlocks];
  __shared__ int ready[kFzRing];
  __shared__ int s_resolved, s_stop;
  __shared__ float ring_sc[kFzRing * kWave];  // kscore: block p's 64 row scores beside its tiles
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int64_t tri = tri_tiles(nbw);
  if ((int)blockIdx.x >= S) {
    // ---------------- mask: one tile per wave
    const int64_t g = ((int64_t)blockIdx.x - S) * kFzWaves + wave;
    if (g >= (int64_t)S * tri) return;
    int cb = (int)((sqrtf(8.0f * (float)g / (float)S + 1.0f) - 1.0f) * 0.5f);
    cb = max(cb, 0);
    while (cb > 0 && (int64_t)S * cb * (cb + 1) / 2 > g) --cb;
    while ((int64_t)S * (cb + 1) * (cb + 2) / 2 <= g) ++cb;
    const int rem = (int)(g - (int64_t)S * cb * (cb + 1) / 2);
    const int s = __builtin_amdgcn_readfirstlane(rem / (cb + 1));
    const int rb = __builtin_amdgcn_readfirstlane(rem - s * (cb + 1));
    cb = __builtin_amdgcn_readfirstlane(cb);
    fz_setprio(2 - min(2, (3 * cb) / nbw));
    const float4* bx = reinterpret_cast<const float4*>(boxes + (int64_t)s * seg_stride);
    const int n = min(max(counts[s], 0), n_max);  // clamped: memory-safe after a flagged upstream abort
    const float4 r = bx[min(rb * 64 + lane, n_max - 1)];
    const float4 a = bx[min(cb * 64 + lane, n_max - 1)];
    if (rb * 64 >= n || cb * 64 >= n) return;
    float4* rows = reinterpret_cast<float4*>(fz_lds) + wave * kWave;
    float* areas = reinterpret_cast<float*>(reinterpret_cast<float4*>(fz_lds) + kFzWaves * kWave) + wave * kWave;
    const uint64_t w = mask_tile_word(r, a, n, rb, cb, lane, T, rows, areas);
    xwg_store(mask + tile_word((int64_t)s * tri, rb, cb) + lane, w);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) xwg_store(flags + (int64_t)s * tri + (int64_t)cb * (cb + 1) / 2 + rb, 1u);
    if (kStamp && lane == 0)
      stamps[(int64_t)S * nbw * 8 + (int64_t)s * tri + (int64_t)cb * (cb + 1) / 2 + rb] =
          (int64_t)__builtin_amdgcn_s_memrealtime();
    return;
  }
  // ---------------- scan of segment s
  const int s = blockIdx.x;
  const int n = min(max(counts[s], 0), n_max);
  const int nb = (n + 63) >> 6;
  uint64_t* ring = fz_lds;
  uint64_t* kept = fz_lds + kFzRing * kFzSlotWords;
  if (tid < kFzRing) ready[tid] = 0;
  if (tid == 0) {
    s_resolved = 0;
    s_stop = nb;
  }
  __syncthreads();
  __builtin_amdgcn_s_setprio(3);
  if (wave == 0) {
    int32_t* K = keep + (int64_t)s * kstride;
    int nk = 0;
    uint64_t kbh[kFzNear] = {};  // kept sets of blocks b-1 .. b-kFzNear
    for (int b = 0; b < nb; ++b) {
      const uint64_t* slot = ring + (b % kFzRing) * kFzSlotWords + lane;
      uint64_t pw, nr[kFzNear], d;
      if (fz_block_reads(&ready[b % kFzRing], slot, pw, nr, d) != b + 1) {
        while (lds_poll(&ready[b % kFzRing]) != b + 1) __builtin_amdgcn_s_sleep(1);
        fz_block_reads(&ready[b % kFzRing], slot, pw, nr, d);
      }
      if (lds_poll(&s_stop) < 0) {  // a loader's wait ran out (status flagged): stop, release the loaders
        if (lane == 0)
          __hip_atomic_store(&s_resolved, nb + kFzRing + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
      uint64_t acc = pw;
#pragma unroll
      for (int i = 0; i < kFzNear; ++i) acc |= nr[i] & kbh[i];
      uint64_t r = __ballot(acc != 0ull);
      const int valid = n - b * 64;
      if (valid < 64) r |= (~0ull) << valid;
      uint64_t kb = 0, und = ~r;
      while (und) {
        const uint64_t sup = __ballot((d & und) != 0ull);
        const uint64_t nkp = und & ~sup;
        kb |= nkp;
        const uint64_t vic = __ballot((d & nkp) != 0ull);
        und &= ~(nkp | vic);
      }
      bool stop = false;
      if (max_keep >= 0) {
        const int room = max_keep - nk;
        while (__popcll(kb) > room) kb &= ~(1ull << (63 - __clzll(kb)));  // drop lowest-score extras
        stop = nk + __popcll(kb) >= max_keep;
      }
      if ((kb >> lane) & 1ull) {
        const int at = nk + __popcll(kb & lanemask_lt());
        K[at] = b * 64 + lane;
        if (kscore) kscore[(int64_t)s * n_max + at] = __float_as_uint(ring_sc[(b % kFzRing) * kWave + lane]);
      }
      nk += __popcll(kb);
#pragma unroll
      for (int i = kFzNear - 1; i > 0; --i) kbh[i] = kbh[i - 1];
      kbh[0] = kb;
      if (lane == 0) {  // in-order LDS: the loaders see kept[b] / s_stop once they see the count
        kept[b] = kb;
        if (stop) s_stop = b;
        asm volatile("" ::: "memory");
        __hip_atomic_store(&s_resolved, stop ? nb + kFzRing + 1 : b + 1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
        if (kStamp) stamps[((int64_t)s * nbw + b) * 8 + 3] = (int64_t)__builtin_amdgcn_s_memrealtime();
      }
      if (stop) break;
    }
    if (lane == 0) kcounts[s] = nk;
  } else {  // loaders
    const uint32_t* sflags = flags + (int64_t)s * tri;
    const uint64_t* smask = mask + (int64_t)s * tri * 64;
    for (int p = wave - 1; p < nb; p += kFzLoaders) {
      while (lds_poll(&s_resolved) < p - kFzRing + 1) __builtin_amdgcn_s_sleep(1);  // slot of p - kFzRing free
      if (s_stop < p) break;
      const int64_t c0 = (int64_t)p * (p + 1) / 2;  // tile (j, p) is tile c0 + j of the segment
      // kscore: the block's row scores (the previous launch's output), in flight over the wait
      const float rsc = kscore ? row_scores[(int64_t)s * n_max + min(p * 64 + lane, n_max - 1)] : 0.0f;
      if (kStamp && lane == 0) stamps[((int64_t)s * nbw + p) * 8] = (int64_t)__builtin_amdgcn_s_memrealtime();
      if (!fz_wait_column(sflags + c0, p, lane, status, &s_stop)) {
        // stop the workgroup: s_stop < 0 first, then wake the resolver on this block's flag (LDS is
        // served in order: the resolver sees s_stop once it sees the flag)
        if (lane == 0) {
          __hip_atomic_store(&s_stop, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          asm volatile("" ::: "memory");
          lds_flag(&ready[p % kFzRing], p + 1);
        }
        break;
      }
      if (kStamp && lane == 0) stamps[((int64_t)s * nbw + p) * 8 + 1] = (int64_t)__builtin_amdgcn_s_memrealtime();
      const uint64_t* col = smask + c0 * 64 + lane;
      const uint64_t d = fz_tile(col + (int64_t)p * 64);
      uint64_t nr[kFzNear];
  #pragma unroll
      for (int i = 0; i < kFzNear; ++i) nr[i] = p > i ? fz_tile(col + (int64_t)(p - 1 - i) * 64) : 0ull;
      // fold blocks j < jf = p - kFzNear (their kept sets appear as the resolver passes them)
      // Batches of 16 tile words, branch-free (indices clamped to the last fold tile, extra
      // words masked out): one memory round trip per 16 tiles.  (Eight per batch with the next
      // batch prefetched needs 16 more VGPRs than the 64 that 8 waves per SIMD allow, so the
      // compiler reused the registers and waited for each batch before issuing the next.)
      const int jf = p - kFzNear;
      uint64_t acc = 0;
      if (jf > 0) {
        const int jl = jf - 1;
        for (int j0 = 0; j0 < jf; j0 += 16) {
          uint64_t t[16];
  #pragma unroll
          for (int u = 0; u < 16; ++u) t[u] = fz_tile(col + (int64_t)min(j0 + u, jl) * 64);
          const int need = min(j0 + 16, jf);
          if (kStamp && lane == 0 && j0 + 16 >= jf) stamps[((int64_t)s * nbw + p) * 8 + 4] = (int64_t)__builtin_amdgcn_s_memrealtime();
          while (lds_poll(&s_resolved) < need) __builtin_amdgcn_s_sleep(1);
          if (kStamp && lane == 0 && j0 + 16 >= jf) stamps[((int64_t)s * nbw + p) * 8 + 5] = (int64_t)__builtin_amdgcn_s_memrealtime();
  #pragma unroll
          for (int u = 0; u < 16; ++u) {
            const uint64_t k = kept[min(j0 + u, jl)];
            acc |= (j0 + u < jf) ? (t[u] & k) : 0ull;
          }
        }
      }
      uint64_t* slot = ring + (p % kFzRing) * kFzSlotWords + lane;
      slot[0] = acc;
  #pragma unroll
      for (int i = 0; i < kFzNear; ++i) slot[(1 + i) * kWave] = nr[i];
      slot[(1 + kFzNear) * kWave] = d;
      ring_sc[(p % kFzRing) * kWave + lane] = rsc;
      if (lane == 0) lds_flag(&ready[p % kFzRing], p + 1);
      if (kStamp && lane == 0) stamps[((int64_t)s * nbw + p) * 8 + 2] = (int64_t)__builtin_amdgcn_s_memrealtime();
    }
  }
}

// The scan's dynamic LDS (up to 128 KB) needs the per-device function attribute; it is
// set for every device the first time a launch runs on it (one bit per device id;
// setting it twice from racing threads is harmless).
static std::atomic<uint64_t> g_scan_attr_devices{0};

static int32_t nms_scan_attr() {
  int dev = 0;
  FRH_HIP(hipGetDevice(&dev));
  const uint64_t bit = dev < 64 ? (1ull << dev) : 0ull;
  if (bit && (g_scan_attr_devices.load(std::memory_order_acquire) & bit)) return FRH_OK;
  FRH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(nms_scan_kernel<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kNmsRing * kNmsSpan * 64 * 8));
  FRH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(nms_scan_kernel<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kNmsRing * kNmsSpan * 64 * 8));
  g_scan_attr_devices.fetch_or(bit, std::memory_order_acq_rel);
  return FRH_OK;
}

int32_t launch_nms_sorted(int32_t S, const float* boxes, int64_t seg_stride, const int32_t* counts, int32_t n_max,
                          double thr, int32_t max_keep, int32_t* keep, int64_t kstride, int32_t* kcounts,
                          uint64_t* mask, const int64_t* seg_base, hipStream_t st, int64_t* stamps) {
  const int nbw = (n_max + 63) / 64;
  FRH_REQUIRE(nbw <= kMaxNmsWords, "n_max %d exceeds %d", n_max, 64 * kMaxNmsWords);
  const int32_t r = nms_scan_attr();
  if (r) return r;
  dim3 g((unsigned)((tri_tiles(nbw) + 3) / 4), S);
  hipLaunchKernelGGL(nms_mask_kernel, g, dim3(256), 0, st, boxes, seg_stride, counts, n_max, nbw, nms_thr(thr), mask,
                     seg_base);
  const int span = std::min(nbw, kNmsSpan);
  const size_t lds = (size_t)kNmsRing * ((span + 1) & ~1) * 64 * sizeof(uint64_t);
  if (stamps)
    hipLaunchKernelGGL(nms_scan_kernel<true>, dim3(S), dim3(256), lds, st, mask, counts, nbw, span, max_keep, keep,
                       kstride, kcounts, seg_base, stamps);
  else
    hipLaunchKernelGGL(nms_scan_kernel<false>, dim3(S), dim3(256), lds, st, mask, counts, nbw, span, max_keep, keep,
                       kstride, kcounts, seg_base, nullptr);
  return check_launch("nms");
}

// One-launch NMS (nms_fused_kernel) of S segments at most n_max boxes each, tiles at
// s * tri(nbw) (no seg_base); flags: nms_fused_flag_bytes(S, n_max) bytes, zero on entry
// (left set: the caller zeroes them again before the next call).  S scan workgroups must be
// resident beside mask workgroups: at most a quarter of the device's capacity of the kernel.
bool nms_fused_fits(int32_t S, int32_t n_max) {
  return S >= 1 && S <= kFzMaxSegs && n_max >= 1 && (n_max + 63) / 64 <= kFzMaxBlocks &&
         S <= resident_capacity(reinterpret_cast<const void*>(nms_fused_kernel<false>), kFzThreads) / 4;
}

size_t nms_fused_flag_bytes(int32_t S, int32_t n_max) {  // one word per tile (+ one spare)
  return ((size_t)S * (size_t)tri_tiles((n_max + 63) / 64) + 1) * sizeof(uint32_t);
}

int32_t launch_nms_fused(int32_t S, const float* boxes, int64_t seg_stride, const int32_t* counts, int32_t n_max,
                         double thr, int32_t max_keep, int32_t* keep, int64_t kstride, int32_t* kcounts,
                         uint64_t* mask, uint32_t* flags, int32_t* status, hipStream_t st, int64_t* stamps = nullptr,
                         const float* row_scores = nullptr, uint32_t* kscore = nullptr) {
  FRH_REQUIRE(nms_fused_fits(S, n_max), "one-launch NMS: %d segments of %d boxes out of range", S, n_max);
  FRH_REQUIRE(status, "null status word");
  FRH_REQUIRE(!kscore || row_scores, "kept scores need the row scores");
  const int nbw = (n_max + 63) / 64;
  const int64_t grid = S + ((int64_t)S * tri_tiles(nbw) + kFzWaves - 1) / kFzWaves;
  FRH_REQUIRE(grid < ((int64_t)1 << 31), "too many mask tiles");
  if (stamps)
    hipLaunchKernelGGL(nms_fused_kernel<true>, dim3((unsigned)grid), dim3(kFzThreads), 0, st, (int)S, boxes,
                       seg_stride, counts, n_max, nbw, nms_thr(thr), mask, flags, max_keep, keep, kstride, kcounts,
                       status, stamps, row_scores, kscore);
  else
    hipLaunchKernelGGL(nms_fused_kernel<false>, dim3((unsigned)grid), dim3(kFzThreads), 0, st, (int)S, boxes,
                       seg_stride, counts, n_max, nbw, nms_thr(thr), mask, flags, max_keep, keep, kstride, kcounts,
                       status, nullptr, row_scores, kscore);
  return check_launch("nms_fused");
}

size_t nms_mask_bytes(int32_t S, int32_t n_max) {  // S triangles of the n_max segment, 64 column words per tile
  return (size_t)S * (size_t)tri_tiles((n_max + 63) / 64) * 64 * sizeof(uint64_t);
}

}  // namespace frh

using namespace frh;

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
                           keep_counts, reinterpret_cast<uint64_t*>(workspace), nullptr, as_stream(stream), nullptr);
}
