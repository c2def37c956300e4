// Segmented top-k over u32 keys, spread over the chip: one 256-thread
// workgroup per 4096-key chunk of every segment.
//
// Used by the RPN score selection (pre_nms of up to ~117k anchors per (image,
// level); rpn_head.py:84-90) and the device sampler (k of up to ~155k
// candidates; region.py:43-57).  After one memset, three launches:
//   keys    : the caller's key kernel writes the keys and, per chunk, an LDS
//             histogram of their top hb bits (hb <= 12), flushed into the
//             segment's global histogram with atomics (tk_hist1_*).
//   refine  : every chunk workgroup finds bucket b1 and the slots k1 left in it
//             ("take every nonzero key" when there are at most k) from that
//             histogram and counts its b1 keys into a histogram of the next 12
//             bits; the segment's last workgroup (done counter) finds bucket b2
//             and the slots k2 left in the prefix P = b1:b2 and publishes them.
//   collect : every chunk workgroup selects its keys above P and lists its
//             keys equal to P (candidates); the last workgroup sorts the
//             candidates by (key desc, index asc) in LDS, selects the first k2
//             and runs the caller's finish.
// When the first-level buckets are small (uniform keys: the device sampler)
// the refine launch is skipped and P = b1 (tk_plan_direct).
// Every workgroup loads its 16 keys per thread at once and reserves list slots
// with one atomic per workgroup, so a launch costs a handful of memory round
// trips.  Data handed between workgroups inside a launch (second histogram,
// candidate and selection lists) is written with atomics and read by the last
// workgroup with atomic read-modify-writes -- both execute at the memory side,
// no XCD L2 state is involved -- after each writer's vmcnt(0) and its
// workgroup's done-counter add.
// Result: k_v = min(k, #nonzero keys) selections -- the k_v largest keys, ties
// broken by lowest index -- handed to the caller's policy (no order).  Key 0
// means "not a candidate".
#pragma once
#include "block_ops.h"

namespace frh {

constexpr int kTkThreads = 256;
constexpr int kTkPerThread = 16;
constexpr int kTkChunk = kTkThreads * kTkPerThread;  // keys per workgroup
constexpr int kTkBins2 = 4096;                       // second level: 12 bits
constexpr int kTkCandCap = 4096;                     // prefix ties sorted in LDS

// per-segment state words (zeroed by the caller's memset; TK_N / TK_K may be
// seeded by the key kernel)
enum { TK_N = 0, TK_K = 1, TK_OUT = 2, TK_CAND = 3, TK_DONE1 = 4, TK_DONE2 = 5, TK_CNT = 6,
       TK_ALL = 7, TK_KV = 8, TK_P = 9, TK_K2 = 10, TK_BAR1 = 11, TK_BAR2 = 12, TK_BAR3 = 13,
       TK_BAR4 = 14, TK_ERR = 15, TK_WORDS = 16 };

struct TkBufs {
  const uint32_t* keys;  // [V][ld]
  int64_t ld;
  uint32_t* hist1;       // [V][1 << hb]
  int hb;                // first-level bits (<= 12)
  uint32_t* hist2;       // [V][kTkBins2]
  int32_t* state;        // [V][TK_WORDS]
  uint64_t* cand;        // [V][ld] candidate list: key << 32 | ~index
};


// The one-launch kernels' barrier counters: 32 words (one 128-B line) per segment after the
// state words, so the lanes polling a barrier never share a line with the list reservations'
// atomics.  bars = state + tk_bars_offset(V) words.
__host__ __device__ inline int tk_bars_offset(int V) { return (V * TK_WORDS + 31) & ~31; }
constexpr int kBarWords = 32;

inline size_t tk_zero_bytes(int V, int hb) {  // hist1 + hist2 + state + barrier lines, contiguous
  return (size_t)V * (((size_t)1 << hb) + kTkBins2) * sizeof(uint32_t) +
         ((size_t)tk_bars_offset(V) + (size_t)V * kBarWords) * sizeof(int32_t);
}

// ------------------------------------------- cross-workgroup hand-off words
// Payload handed from the chunk workgroups of a launch to its last workgroup:
// written with agent-scope relaxed stores (sc1: write-through, the line leaves
// the writer's L2) or memory-side atomics, read with agent-scope relaxed loads
// (sc1: L1 bypassed) after every writer's vmcnt(0) wait and its workgroup's
// done-counter add has been seen (MI355X_MICROARCH.md, hand-off table row 1).
__device__ __forceinline__ void xwg_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void xwg_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t xwg_load(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t xwg_load(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t xwg_load(const int32_t* p) {
  return __hip_atomic_load(const_cast<int32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------ wave helpers
// histogram add aggregated over the wave's most common bin (the first active
// lane's): a concentrated key set costs one LDS atomic per wave, not 64
// conflicting ones.  Wave-uniform call.  (A second aggregation round -- for key sets
// straddling two bins -- measured slower on both the RPN and the sampler keys: round 4.)
__device__ __forceinline__ void tk_hist_add(uint32_t* h, bool act, uint32_t bin) {
  const uint64_t am = __ballot(act);
  if (!am) return;
  const int l0 = __builtin_ctzll(am);
  const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bin, l0);
  const uint64_t same = __ballot(act && bin == b0);
  if (lane_id() == l0) atomicAdd(&h[b0], (uint32_t)__popcll(same));
  if (act && bin != b0) atomicAdd(&h[bin], 1u);
}

// Workgroup-aggregated reservation of `cnt` slots per thread in the list
// behind the global `counter` (one atomic per workgroup): returns this
// thread's first slot.  Block-uniform call; part / sh[2]: LDS scratch (sh[0] /
// sh[1] = the workgroup's first slot / count, valid until the next call).
__device__ __forceinline__ int block_reserve(int cnt, int* counter, int* part, int* sh) {
  const int t = threadIdx.x, w = t / kWave;
  __syncthreads();  // part / sh free
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int x = __shfl_up(incl, o, kWave);
    if (lane_id() >= o) incl += x;
  }
  if (lane_id() == kWave - 1) part[w] = incl;
  __syncthreads();
  int pre = 0, tot = 0;
  for (int i = 0; i < (int)blockDim.x / kWave; ++i) {
    const int c = part[i];
    pre += i < w ? c : 0;
    tot += c;
  }
  if (t == 0) {
    sh[0] = tot ? atomicAdd(counter, tot) : 0;
    sh[1] = tot;
  }
  __syncthreads();
  return sh[0] + pre + incl - cnt;  // sh[0] = the workgroup's first slot, sh[1] = its count
}

// The same for two lists whose counters are adjacent words (c[0]: selections,
// c[1]: candidates; 8-byte aligned): one packed scan and ONE 64-bit atomic.  Per
// workgroup each count is < 65536.  Returns this thread's first (selection,
// candidate) slots; sh[0] / sh[1] = the workgroup's first selection slot /
// selection count, *cb = its first candidate slot.
__device__ __forceinline__ int2 block_reserve2(int nsel, int ncand, int* c, int* part, int* sh, int* cb) {
  const int t = threadIdx.x, w = t / kWave;
  __syncthreads();  // part / sh free
  const int cnt = nsel | (ncand << 16);
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int x = __shfl_up(incl, o, kWave);
    if (lane_id() >= o) incl += x;
  }
  if (lane_id() == kWave - 1) part[w] = incl;
  __syncthreads();
  int pre = 0, tot = 0;
  for (int i = 0; i < (int)blockDim.x / kWave; ++i) {
    const int v = part[i];
    pre += i < w ? v : 0;
    tot += v;
  }
  if (t == 0) {
    const uint32_t ts = (uint32_t)tot & 0xffffu, tc = (uint32_t)tot >> 16;
    const unsigned long long old =
        tot ? atomicAdd(reinterpret_cast<unsigned long long*>(c), ((unsigned long long)tc << 32) | ts) : 0ull;
    sh[0] = (int)(uint32_t)old;
    sh[1] = (int)ts;
    *cb = (int)(uint32_t)(old >> 32);
  }
  __syncthreads();
  const int ex = pre + incl - cnt;
  return make_int2(sh[0] + (ex & 0xffff), *cb + (ex >> 16));
}

// Two block_reserve2 reservations (counter pairs c0 and c1, each 8-byte aligned) in one
// round trip: both 64-bit atomics issued by thread 0 before either result is used.  Returns
// the first (selection, candidate) slots of this thread in list 0 (.x, .y) and list 1 (.z, .w).
__device__ __forceinline__ int4 block_reserve4(int nsel0, int ncand0, int nsel1, int ncand1, int* c0, int* c1,
                                               int* part, int* sh) {
  const int t = threadIdx.x, w = t / kWave, nw = (int)blockDim.x / kWave;
  __syncthreads();  // part / sh free
  int a = nsel0 | (ncand0 << 16), b = nsel1 | (ncand1 << 16);
  int ia = a, ib = b;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int xa = __shfl_up(ia, o, kWave), xb = __shfl_up(ib, o, kWave);
    if (lane_id() >= o) ia += xa, ib += xb;
  }
  if (lane_id() == kWave - 1) part[w] = ia, part[nw + w] = ib;
  __syncthreads();
  int pa = 0, ta = 0, pb = 0, tb = 0;
  for (int i = 0; i < nw; ++i) {
    const int va = part[i], vb = part[nw + i];
    pa += i < w ? va : 0;
    ta += va;
    pb += i < w ? vb : 0;
    tb += vb;
  }
  if (t == 0) {
    auto pack = [](int tot) { return ((unsigned long long)((uint32_t)tot >> 16) << 32) | ((uint32_t)tot & 0xffffu); };
    const unsigned long long oa = ta ? atomicAdd(reinterpret_cast<unsigned long long*>(c0), pack(ta)) : 0ull;
    const unsigned long long ob = tb ? atomicAdd(reinterpret_cast<unsigned long long*>(c1), pack(tb)) : 0ull;
    sh[0] = (int)(uint32_t)oa, sh[1] = (int)(uint32_t)(oa >> 32);
    sh[2] = (int)(uint32_t)ob, sh[3] = (int)(uint32_t)(ob >> 32);
  }
  __syncthreads();
  const int ea = pa + ia - a, eb = pb + ib - b;
  return make_int4(sh[0] + (ea & 0xffff), sh[1] + (ea >> 16), sh[2] + (eb & 0xffff), sh[3] + (eb >> 16));
}

// --------------------------------------------- first-level histogram (keys)
// The key kernels build it per chunk: clear, add, flush (block-uniform calls).
__device__ __forceinline__ void tk_hist1_clear(uint32_t* h, int bins) {
  for (int i = threadIdx.x; i < bins; i += blockDim.x) h[i] = 0u;
  __syncthreads();
}
__device__ __forceinline__ void tk_hist1_flush(const uint32_t* h, int bins, uint32_t* gh) {
  __syncthreads();
  for (int i = threadIdx.x; i < bins; i += blockDim.x) {
    const uint32_t c = h[i];
    if (c) atomicAdd(&gh[i], c);
  }
}

// ------------------------------------------------------------ select state
struct alignas(16) TkSmem {  // 16-B aligned: the fused selection reads record pairs with ds_read_b128
  union {
    struct {
      uint32_t h1[4096];
      uint32_t h2[kTkBins2];
    };
    uint64_t cand[kTkCandCap];
  };
  TopkSmem fb;
  int part[2 * kTkThreads / kWave];
  int last, bin, above, tot, ncand;
  int base, tot_sel;  // block_reserve's (first slot, count); adjacent
  int cbase;          // block_reserve2's first candidate slot
  int res4[4];        // block_reserve4's first slots
};

// Suffix search over 2^hb bins (highest first), 256 threads: sm.bin / sm.above
// such that above < krem <= above + h[bin]; sm.tot = the total (no bin written
// when krem > tot).  rd(i) reads bin i.
template <class Rd>
__device__ __forceinline__ void tk_find(TkSmem& sm, int bins, int krem, Rd rd) {
  const int t = threadIdx.x, w = t / kWave;
  const int per = bins / kTkThreads;  // 16 or 1 (hb = 12 or 8)
  const int hi = bins - per * t;      // thread t owns [hi - per, hi), descending
  int b[16], s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    b[i] = i < per ? (int)rd(hi - 1 - i) : 0;
    s += b[i];
  }
  int incl = s;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int x = __shfl_up(incl, o, kWave);
    if (lane_id() >= o) incl += x;
  }
  if (lane_id() == kWave - 1) sm.part[w] = incl;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kTkThreads / kWave; ++i) {
    const int c = sm.part[i];
    pre += i < w ? c : 0;
    tot += c;
  }
  incl += pre;
  int run = incl - s;
  if (run < krem && incl >= krem) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i < per && run + b[i] >= krem) {
        sm.bin = hi - 1 - i;
        sm.above = run;
        break;
      }
      run += b[i];
    }
  }
  if (t == 0) sm.tot = tot;
  __syncthreads();
}

// This workgroup's 16 keys per thread (key r of thread t = chunk index
// r * 256 + t), all loads in flight at once; index >= n reads as 0.
__device__ __forceinline__ void tk_load_chunk(const uint32_t* kk, int64_t base, int n, uint32_t (&key)[kTkPerThread]) {
#pragma unroll
  for (int r = 0; r < kTkPerThread; ++r) {
    const int64_t i = base + r * kTkThreads + threadIdx.x;
    key[r] = i < n ? kk[i] : 0u;
  }
}

// check in once this workgroup's atomics have completed: true in the last
// workgroup of the segment (block-uniform)
__device__ __forceinline__ bool tk_check_in(int* done, TkSmem& sm) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) sm.last = atomicAdd(done, 1) == (int)gridDim.x - 1;
  __syncthreads();
  return sm.last != 0;
}

// ------------------------------------------------------ in-launch segment barrier
// The fused selections (rpn_select_kernel, sampler_fused_kernel) keep a segment's
// workgroups in one launch across their phases: each arrives on a per-segment
// counter once its own stores and atomics have completed (vmcnt(0) in every wave,
// then one agent-scope atomic add behind a workgroup barrier) and lane 0 polls
// the counter with sc1 loads (hand-off table row 1: everything handed across is
// written sc1 or by memory-side atomics and read back sc1).  Residency: a
// segment's workgroups are contiguous in dispatch order and the host keeps the
// grid's live workgroups within a fraction of the device's resident capacity
// (resident_capacity: CU count x occupancy of the kernel, queried per device), so
// the polled workgroups are normally resident.  The spin is bounded (kSpinTicks of
// the 100 MHz clock): a wait that runs out ORs `bit` into the caller's device status
// word and returns false in every thread of the workgroup, which then ends its work
// (include/frcnn_amd.h FRH_DEVERR_*): a loud error, never a hang, never a selection
// from partial histograms.
#ifndef FRH_SPIN_TICKS
#define FRH_SPIN_TICKS 20000000ull  // 200 ms (tools: a build with 0 makes every unmet wait run out)
#endif
constexpr uint64_t kSpinTicks = FRH_SPIN_TICKS;

__device__ __forceinline__ bool seg_barrier(int32_t* counter, int target, int32_t* status, int32_t bit) {
  __shared__ int s_ok;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = 1;
    atomicAdd(counter, 1);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (xwg_load(counter) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
        atomicOr(status, bit);
        ok = 0;
        break;
      }
    }
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

// ------------------------------------------------- top-k of a small LDS list
// The k largest (1 <= k <= n) of n DISTINCT u64 values v[0..n) in LDS whose bits above
// `top` (<= 64) all equal those of P0: radix passes of 8 bits downwards from `top`, each an LDS
// histogram (sm.fb.hist) of the values still matching the prefix + tk_find, stopping as soon
// as the bin holding the k-th value is taken whole.  v is taken iff (v >> sh) >= (P >> sh).
// No sort: a few passes where a bitonic network over n takes log2(n)^2 / 2 barriers.
struct LdsCut {
  uint64_t P;
  int sh;
};

__device__ LdsCut lds_topk_cut(const uint64_t* v, int n, int k, int top, uint64_t P0, TkSmem& sm) {
  const int t = threadIdx.x, nt = blockDim.x;
  uint64_t P = P0;
  int krem = k;
  for (int sh = top - 8; sh >= 0; sh -= 8) {
    for (int i = t; i < 256; i += nt) sm.fb.hist[i] = 0u;
    __syncthreads();
    for (int j = t; j < n; j += nt) {
      const uint64_t x = v[j];
      if (sh + 8 >= 64 || (x >> (sh + 8)) == (P >> (sh + 8))) atomicAdd(&sm.fb.hist[(x >> sh) & 255u], 1u);
    }
    __syncthreads();
    tk_find(sm, 256, krem, [&](int i) { return sm.fb.hist[i]; });
    const int b = sm.bin, above = sm.above;
    const int cnt = (int)sm.fb.hist[b];
    __syncthreads();  // hist / bin read by every thread before the next pass
    P |= (uint64_t)b << sh;
    krem -= above;
    if (cnt == krem) return LdsCut{P, sh};
  }
  return LdsCut{P, 0};
}

// ------------------------------------------------------------- refine launch
// Chunk blockIdx.x of segment v.  k <= 0 selects nothing.
__device__ void tk_refine_chunk(const TkBufs& b, int v, int n, int k, TkSmem& sm) {
  const int t = threadIdx.x;
  const int bins1 = 1 << b.hb;
  const int sh1 = 32 - b.hb, sh2 = sh1 - 12;
  int32_t* st = b.state + v * TK_WORDS;
  for (int i = t; i < bins1; i += kTkThreads) sm.h1[i] = b.hist1[(int64_t)v * bins1 + i];
  for (int i = t; i < kTkBins2; i += kTkThreads) sm.h2[i] = 0u;
  __syncthreads();
  tk_find(sm, bins1, k > 0 ? k : 1, [&](int i) { return sm.h1[i]; });
  const bool all = k <= 0 || sm.tot <= k;
  const uint32_t b1 = (uint32_t)sm.bin;
  const int k1 = k - sm.above;
  const int64_t base = (int64_t)blockIdx.x * kTkChunk;
  uint32_t* gh2 = b.hist2 + (int64_t)v * kTkBins2;
  if (!all && base < n) {
    uint32_t key[kTkPerThread];
    tk_load_chunk(b.keys + (int64_t)v * b.ld, base, n, key);
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r)
      tk_hist_add(sm.h2, key[r] != 0u && (key[r] >> sh1) == b1, (key[r] >> sh2) & 0xfffu);
    __syncthreads();
    for (int i = t; i < kTkBins2; i += kTkThreads) {
      const uint32_t c = sm.h2[i];
      if (c) atomicAdd(&gh2[i], c);
    }
  }
  if (!tk_check_in(&st[TK_DONE1], sm)) return;
  // last workgroup: find 2 (atomic reads: memory-side values), publish
  int P = 0, k2 = 0;
  if (!all) {
    tk_find(sm, kTkBins2, k1, [&](int i) { return xwg_load(gh2 + i); });
    P = (int)((b1 << 12) | (uint32_t)sm.bin);
    k2 = k1 - sm.above;
  }
  if (t == 0) {
    st[TK_ALL] = all ? 1 : 0;
    st[TK_KV] = k <= 0 ? 0 : (all ? sm.tot : k);
    st[TK_P] = P;
    st[TK_K2] = k2;
  }
}

// ------------------------------------------------------------ collect launch
// What the collect launch selects: every nonzero key when `all` (kv of them);
// otherwise keys whose top bits (key >> sh) exceed P, plus the first k2 (by key
// desc, index asc) of the keys whose top bits equal P.
struct TkPlan {
  bool all;
  int kv;
  uint32_t P;
  int sh;
  int k2;
};

// the plan the refine launch published for segment v
__device__ __forceinline__ TkPlan tk_plan_refined(const TkBufs& b, int v) {
  const int32_t* st = b.state + v * TK_WORDS;
  return TkPlan{st[TK_ALL] != 0, st[TK_KV], (uint32_t)st[TK_P], 32 - b.hb - 12, st[TK_K2]};
}

// Two-level plan straight from a first-level histogram (no refine launch): the
// bucket b1 holding the k-th key is the prefix; rd(i) reads bin i (all threads).
template <class Rd>
__device__ __forceinline__ TkPlan tk_plan_direct(int hb, int k, TkSmem& sm, Rd rd) {
  tk_find(sm, 1 << hb, k > 0 ? k : 1, rd);
  const bool all = k <= 0 || sm.tot <= k;
  return TkPlan{all, k <= 0 ? 0 : (all ? sm.tot : k), (uint32_t)sm.bin, 32 - hb, k - sm.above};
}

// Chunk blockIdx.x of segment v.  Pol:
//   void select(int index, uint32_t key, int slot)  one selection; slot = its
//        position among the segment's k_v selections
//   void finish(int kv)   last workgroup, all threads, after every select
// The state words TK_OUT, TK_CAND, TK_DONE2 of v start at 0.
template <class Pol>
__device__ void tk_collect_chunk(const TkBufs& b, int v, int n, const TkPlan& plan, Pol& pol, TkSmem& sm) {
  const int t = threadIdx.x;
  int32_t* st = b.state + v * TK_WORDS;
  const bool all = plan.all;
  const int kv = plan.kv, k2 = plan.k2, sh = plan.sh;
  const uint32_t P = plan.P;
  const uint32_t* kk = b.keys + (int64_t)v * b.ld;
  uint64_t* cand = b.cand + (int64_t)v * b.ld;
  const int64_t base = (int64_t)blockIdx.x * kTkChunk;
  if (kv > 0 && base < n) {
    uint32_t key[kTkPerThread];
    tk_load_chunk(kk, base, n, key);
    uint32_t sel = 0u, eq = 0u;
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r) {
      const uint32_t pre = key[r] >> sh;
      sel |= (key[r] != 0u && (all || pre > P)) ? 1u << r : 0u;
      eq |= (key[r] != 0u && !all && pre == P) ? 1u << r : 0u;
    }
    // one reservation for both lists (TK_OUT, TK_CAND adjacent)
    static_assert(TK_CAND == TK_OUT + 1 && TK_OUT % 2 == 0, "adjacent, 8-byte aligned counters");
    const int2 slots = block_reserve2(__popc(sel), __popc(eq), &st[TK_OUT], sm.part, &sm.base, &sm.cbase);
    // candidates: straight to the segment's list (no dependent loads)
    int c = slots.y;
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r)
      if (eq & (1u << r))
        xwg_store(cand + c++, ((uint64_t)key[r] << 32) | (uint32_t)~(uint32_t)(base + r * kTkThreads + t));
    // selections: staged in LDS, then handed to the policy one per thread per
    // round, so the policy's loads for a round are in flight together
    int s = slots.x;
    const int gbase = sm.base, nsel = sm.tot_sel;
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r)
      if (sel & (1u << r)) sm.cand[s++ - gbase] = ((uint64_t)key[r] << 32) | (uint32_t)(base + r * kTkThreads + t);
    __syncthreads();
    for (int j0 = 0; j0 < nsel; j0 += kTkThreads) {
      const int j = j0 + t;
      if (j < nsel) {
        const uint64_t e = sm.cand[j];
        pol.select((int)(uint32_t)e, (uint32_t)(e >> 32), gbase + j);
      }
    }
  }
  if (!tk_check_in(&st[TK_DONE2], sm)) return;
  if (kv == 0 || all) {
    pol.finish(kv);
    return;
  }
  // last workgroup: order the prefix ties, take the first k2
  const int nabove = kv - k2;
  const int ncand = xwg_load(st + TK_CAND);
  if (ncand <= kTkCandCap) {
    const int P2 = next_pow2(ncand > 1 ? ncand : 1);
    for (int j = t; j < P2; j += kTkThreads)
      sm.cand[j] = j < ncand ? xwg_load(cand + j) : 0ull;
    __syncthreads();
    block_bitonic_sort_desc(sm.cand, P2);
    for (int j = t; j < k2; j += kTkThreads) {
      const uint64_t e = sm.cand[j];
      pol.select((int)~(uint32_t)e, (uint32_t)(e >> 32), nabove + j);
    }
  } else {
    // degenerate key set (> kTkCandCap keys share the prefix): exact
    // radix select restricted to the prefix, lowest index first among equal
    // keys; indices staged in the (consumed) candidate row, read back in-workgroup
    int32_t* idx = reinterpret_cast<int32_t*>(cand);
    auto key_of = [&](int i) -> uint32_t {
      const uint32_t key = kk[i];
      return (key >> sh) == P ? key : 0u;
    };
    block_topk_select(key_of, n, k2, idx, sm.fb);
    for (int j = t; j < k2; j += kTkThreads) pol.select(idx[j], kk[idx[j]], nabove + j);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  pol.finish(kv);
}

// ------------------------------------------- register bitonic sort (desc)
// kTkThreads threads x E elements (E = 2^LE), P = kTkThreads * E keys, pad with 0.
// Every compare-exchange happens in registers: before a stage whose partner
// distance 2^j is not among the element-index bits [r0, r0 + LE) a thread
// holds, the elements are re-dealt through `lds` (P entries) so that thread t's
// register e holds element g(t, e) = (t >> r0) << (r0 + LE) | e << r0 | t mod 2^r0
// with r0 = max(0, j - LE + 1) -- one re-deal per LE stages.  The network is
// unrolled at compile time.  In and out: x[e] = element t * E + e.
__device__ __forceinline__ int tk_gidx(int t, int e, int r0, int le) {
  return ((t >> r0) << (r0 + le)) | (e << r0) | (t & ((1 << r0) - 1));
}

template <int E>
__device__ __forceinline__ void reg_bitonic_sort_desc(uint64_t (&x)[E], uint64_t* lds) {
  constexpr int LE = E == 1 ? 0 : E == 2 ? 1 : E == 4 ? 2 : E == 8 ? 3 : 4;
  static_assert((1 << LE) == E && E >= 2, "E must be 2, 4, 8 or 16");
  constexpr int LP = 8 + LE;  // kTkThreads == 256
  const int t = threadIdx.x;
  int r0 = 0;
  auto redeal = [&](int nr0) {
#pragma unroll
    for (int e = 0; e < E; ++e) lds[tk_gidx(t, e, r0, LE)] = x[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = lds[tk_gidx(t, e, nr0, LE)];
    __syncthreads();
    r0 = nr0;
  };
#pragma unroll
  for (int ls = 1; ls <= LP; ++ls) {
#pragma unroll
    for (int j = ls - 1; j >= 0; --j) {
      if (j < r0 || j >= r0 + LE) redeal(j - LE + 1 < 0 ? 0 : j - LE + 1);
      const int eb = j - r0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if ((e >> eb) & 1) continue;
        const int e2 = e | (1 << eb);
        const bool desc = ((tk_gidx(t, e, r0, LE) >> ls) & 1) == 0;
        const uint64_t a = x[e], c = x[e2];
        const bool sw = desc ? (a < c) : (a > c);
        x[e] = sw ? c : a;
        x[e2] = sw ? a : c;
      }
    }
  }
  if (r0 != 0) redeal(0);
}

}  // namespace frh
