// Multi-workgroup segmented top-k over precomputed u32 keys.
//
// Used by the RPN score selection (pre_nms of ~117k anchors per (image,
// level)) and the device sampler (k of up to ~130k candidates).  A single
// workgroup per segment (block_topk_select) reads every key once per radix
// byte from one CU; here every pass is spread over the whole chip:
//   hist1   : 4096-bin histogram of key[31:20] per segment (LDS, flushed with
//             global atomics), all chunks of all segments in one grid; the
//             last workgroup of a segment to finish (done counter) then runs
//   find1   : a suffix scan of the histogram -> bucket b1, remaining slots k1
//             (also decides "take everything" when n <= k), and clears the
//             histogram for
//   hist2   : histogram of key[19:8] for keys in bucket b1, whose last
//             workgroup per segment runs
//   find2   : bucket b2, remaining slots k2  (prefix P = b1:b2, 24 bits)
//   collect : keys with key>>8 > P are selected, keys with key>>8 == P become
//             candidates (appends aggregated per wave: one atomic per wave)
//   final   : one workgroup per segment sorts the candidates by
//             (key desc, index asc) and appends the first k2.
// Four launches per selection.  The last-workgroup hand-off reads the histogram
// with atomic read-modify-writes (performed at the memory side, like the flush
// atomics it reads), after every wave's flush atomics have completed (vmcnt(0))
// and a barrier, so no cross-XCD cache state is involved.
// Result: out[v][0..k_v) = indices of the k_v largest keys, ties broken by
// lowest index, in no particular order.  Key 0 means "not a candidate".
#pragma once
#include "block_ops.h"

namespace frh {

constexpr int kTkBins = 4096;
constexpr int kTkThreads = 256;
constexpr int kTkPerThread = 16;
constexpr int kTkChunk = kTkThreads * kTkPerThread;
constexpr int kTkCandCap = 8192;  // candidates sorted in LDS; more -> radix fallback

// per-segment state words
enum { TK_N = 0, TK_K = 1, TK_ALL = 2, TK_B1 = 3, TK_K1 = 4, TK_B2 = 5, TK_K2 = 6, TK_OUT = 7, TK_CAND = 8,
       TK_DONE0 = 9, TK_DONE1 = 10, TK_WORDS = 16 };

struct TopkBuffers {
  const uint32_t* keys;  // [V][ld]
  int64_t ld;
  uint32_t* hist;        // [V][kTkBins]
  int32_t* state;        // [V][TK_WORDS]; TK_N and TK_K filled by the key generator
  int32_t* out;          // [V][out_ld]
  int64_t out_ld;
  int32_t* cand;         // [V][kTkCandCap]
  int V;
};

// kernels have internal linkage: every translation unit that includes this
// header gets its own copy (no cross-TU device symbols)
namespace {

// The find step of pass `pass` for segment v, run by one whole 256-thread workgroup:
// suffix scan of the histogram from the highest bin; bucket where the running count
// reaches the remaining slots.  `rd(i)` reads bin i.
template <class Rd>
__device__ __forceinline__ void tk_find(int32_t* st, int pass, Rd rd, int* part, int* sel_bin, int* sel_above) {
  const int t = threadIdx.x;
  int bins[16];
  const int hi = kTkBins - 16 * t;  // thread t owns bins [4096 - 16(t+1), 4096 - 16t) (descending order)
  int s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    bins[i] = rd(hi - 1 - i);
    s += bins[i];
  }
  if (pass == 0) {  // total candidates = sum of the histogram
    const int tot = block_sum(s, part);
    if (t == 0) {
      st[TK_ALL] = (tot <= st[TK_K]) ? 1 : 0;
      if (st[TK_K] > tot) st[TK_K] = tot;
      st[TK_OUT] = 0;
      st[TK_CAND] = 0;
    }
    __syncthreads();
    if (st[TK_ALL]) return;
  }
  const int krem = pass == 0 ? st[TK_K] : st[TK_K1];
  if (krem <= 0) {  // nothing (more) to select: a prefix no key can exceed, zero slots
    if (t == 0) {
      st[pass == 0 ? TK_B1 : TK_B2] = kTkBins - 1;
      st[pass == 0 ? TK_K1 : TK_K2] = 0;
      if (pass == 0) {
        st[TK_B2] = kTkBins - 1;
        st[TK_K2] = 0;
      }
    }
    return;
  }
  // inclusive prefix over threads (descending bin order): wave scans + wave totals
  int incl = s;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int x = __shfl_up(incl, o, kWave);
    if ((t & (kWave - 1)) >= o) incl += x;
  }
  const int w = t / kWave;
  if ((t & (kWave - 1)) == kWave - 1) part[w] = incl;
  __syncthreads();
  for (int i = 0; i < w; ++i) incl += part[i];
  int run = incl - s;  // count in bins above my range
  if (run < krem && incl >= krem) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (run + bins[i] >= krem) {
        *sel_bin = hi - 1 - i;
        *sel_above = run;
        break;
      }
      run += bins[i];
    }
  }
  __syncthreads();
  if (t == 0) {
    if (pass == 0) {
      st[TK_B1] = *sel_bin;
      st[TK_K1] = krem - *sel_above;
    } else {
      st[TK_B2] = *sel_bin;
      st[TK_K2] = krem - *sel_above;
    }
  }
}

// histogram pass + (last workgroup of the segment) the find step
__global__ void __launch_bounds__(kTkThreads) tk_hist_kernel(TopkBuffers b, int pass) {
  __shared__ uint32_t h[kTkBins];
  __shared__ int part[kTkThreads / kWave];
  __shared__ int last, sel_bin, sel_above;
  const int v = blockIdx.y;
  const int64_t base = (int64_t)blockIdx.x * kTkChunk;
  int32_t* st = b.state + v * TK_WORDS;
  const int n = st[TK_N];
  if (pass == 1 && st[TK_ALL]) return;  // uniform per segment: no find either
  uint32_t* gh = b.hist + (int64_t)v * kTkBins;
  if (base < n) {
    for (int i = threadIdx.x; i < kTkBins; i += kTkThreads) h[i] = 0;
    __syncthreads();
    const uint32_t* kk = b.keys + (int64_t)v * b.ld;
    const uint32_t b1 = (uint32_t)st[TK_B1];
#pragma unroll 4
    for (int r = 0; r < kTkPerThread; ++r) {
      int64_t i = base + r * kTkThreads + threadIdx.x;
      if (i < n) {
        uint32_t key = kk[i];
        if (key) {
          if (pass == 0)
            atomicAdd(&h[key >> 20], 1u);
          else if ((key >> 20) == b1)
            atomicAdd(&h[(key >> 8) & 0xfffu], 1u);
        }
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kTkBins; i += kTkThreads)
      if (h[i]) atomicAdd(&gh[i], h[i]);
  }
  // every workgroup of the segment checks in once its flush atomics have completed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(&st[pass == 0 ? TK_DONE0 : TK_DONE1], 1) == (int)gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  tk_find(st, pass, [&](int i) { return (int)atomicAdd(&gh[i], 0u); }, part, &sel_bin, &sel_above);
  if (pass == 0) {  // clear for pass 2 (read in the next launch)
    __syncthreads();
    for (int i = threadIdx.x; i < kTkBins; i += kTkThreads) gh[i] = 0;
  }
}

// wave-aggregated append: every lane with `take` gets a distinct slot of `list`
__device__ __forceinline__ int wave_append(bool take, int* counter) {
  const uint64_t m = __ballot(take);
  if (!m) return -1;
  const int leader = __builtin_ctzll(m);
  int base = 0;
  if ((int)(threadIdx.x & (kWave - 1)) == leader) base = atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader, kWave);
  return take ? base + __popcll(m & lanemask_lt()) : -1;
}

__global__ void __launch_bounds__(kTkThreads) tk_collect_kernel(TopkBuffers b) {
  const int v = blockIdx.y;
  const int64_t base = (int64_t)blockIdx.x * kTkChunk;
  int32_t* st = b.state + v * TK_WORDS;
  const int n = st[TK_N];
  if (base >= n) return;
  const bool all = st[TK_ALL] != 0;
  const uint32_t P = ((uint32_t)st[TK_B1] << 12) | (uint32_t)st[TK_B2];
  const uint32_t* kk = b.keys + (int64_t)v * b.ld;
  int32_t* out = b.out + (int64_t)v * b.out_ld;
  int32_t* cand = b.cand + (int64_t)v * kTkCandCap;
  for (int r = 0; r < kTkPerThread; ++r) {
    const int64_t i = base + r * kTkThreads + threadIdx.x;
    if (base + r * kTkThreads >= n) break;  // uniform
    const uint32_t key = i < n ? kk[i] : 0u;
    const uint32_t p = key >> 8;
    const bool sel = key && (all || p > P), cnd = key && !all && p == P;
    const int o = wave_append(sel, &st[TK_OUT]);
    if (o >= 0) out[o] = (int32_t)i;
    const int c = wave_append(cnd, &st[TK_CAND]);
    if (c >= 0 && c < kTkCandCap) cand[c] = (int32_t)i;
  }
}

// one 1024-thread block per segment: order candidates, append the best k2.
__global__ void __launch_bounds__(1024) tk_final_kernel(TopkBuffers b) {
  __shared__ uint64_t sk[kTkCandCap];
  __shared__ TopkSmem sm;
  const int v = blockIdx.x;
  int32_t* st = b.state + v * TK_WORDS;
  if (st[TK_ALL]) return;
  const int k2 = st[TK_K2];
  const int ncand = st[TK_CAND];
  const uint32_t* kk = b.keys + (int64_t)v * b.ld;
  int32_t* out = b.out + (int64_t)v * b.out_ld;
  const int base = st[TK_OUT];
  if (ncand <= kTkCandCap) {
    const int32_t* cand = b.cand + (int64_t)v * kTkCandCap;
    const int P2 = next_pow2(ncand > 1 ? ncand : 1);
    for (int j = threadIdx.x; j < P2; j += blockDim.x) {
      uint64_t key = 0;
      if (j < ncand) {
        int i = cand[j];
        key = ((uint64_t)kk[i] << 32) | (uint32_t)(~(uint32_t)i);
      }
      sk[j] = key;
    }
    __syncthreads();
    block_bitonic_sort_desc(sk, P2);
    for (int j = threadIdx.x; j < k2; j += blockDim.x) out[base + j] = (int)(~(uint32_t)sk[j]);
  } else {
    // degenerate key distribution (> kTkCandCap keys share 24 bits): exact
    // single-block radix select restricted to the prefix
    const uint32_t P = ((uint32_t)st[TK_B1] << 12) | (uint32_t)st[TK_B2];
    const int n = st[TK_N];
    auto key_of = [&](int i) -> uint32_t {
      uint32_t key = kk[i];
      return (key >> 8) == P ? key : 0u;
    };
    block_topk_select(key_of, n, k2, out + base, sm);
  }
  if (threadIdx.x == 0) st[TK_OUT] = base + k2;
}

}  // namespace

inline size_t tk_state_bytes(int V) { return (size_t)V * TK_WORDS * sizeof(int32_t); }
inline size_t tk_hist_bytes(int V) { return (size_t)V * kTkBins * sizeof(uint32_t); }
inline size_t tk_cand_bytes(int V) { return (size_t)V * kTkCandCap * sizeof(int32_t); }

// Runs hist+find (x2), collect, final.  The caller has written keys and the TK_N /
// TK_K words of state (state's other words and hist must be zero).
static inline void tk_launch(const TopkBuffers& b, int64_t n_max, hipStream_t st) {
  dim3 grid((unsigned)((n_max + kTkChunk - 1) / kTkChunk), (unsigned)b.V);
  hipLaunchKernelGGL(tk_hist_kernel, grid, dim3(kTkThreads), 0, st, b, 0);
  hipLaunchKernelGGL(tk_hist_kernel, grid, dim3(kTkThreads), 0, st, b, 1);
  hipLaunchKernelGGL(tk_collect_kernel, grid, dim3(kTkThreads), 0, st, b);
  hipLaunchKernelGGL(tk_final_kernel, dim3(b.V), dim3(1024), 0, st, b);
}

}  // namespace frh
