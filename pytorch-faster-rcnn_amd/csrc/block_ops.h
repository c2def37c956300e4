// Workgroup-level building blocks shared by the sampler, proposal and merge
// kernels: ordered scans over wave ballots, radix top-k selection and an LDS
// bitonic sort.  All of them assume blockDim.x is a multiple of 64.
#pragma once
#include "common.h"

namespace frh {

// Exclusive rank of this lane's flag within the block (in thread order) and
// the block total.  `wave_tot` is LDS scratch of blockDim.x/64 ints.
__device__ __forceinline__ int block_rank(bool flag, int* wave_tot, int* total) {
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint64_t bal = __ballot(flag);
  int lane_rank = __popcll(bal & lanemask_lt());
  if (lane_id() == 0) wave_tot[w] = __popcll(bal);
  __syncthreads();
  int off = 0, tot = 0;
  for (int i = 0; i < nw; ++i) {
    int c = wave_tot[i];
    off += (i < w) ? c : 0;
    tot += c;
  }
  __syncthreads();
  *total = tot;
  return off + lane_rank;
}

// Block-wide sum of an int (all threads get the result).  scratch: nw ints.
__device__ __forceinline__ int block_sum(int v, int* scratch) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane_id() == 0) scratch[w] = v;
  __syncthreads();
  int t = 0;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  __syncthreads();
  return t;
}

// predicate families over int64 labels (sampler candidates, chosen rows)
enum LabelPred { kPos = 0, kNeg = 1, kChosen = 2 };
__device__ __forceinline__ bool label_pred(int64_t v, int which) {
  return which == kPos ? v > 0 : (which == kNeg ? v == 0 : v >= 0);
}

struct TopkSmem {
  uint32_t hist[256];
  int scan[256];
  int wave_tot[16];
  int sel_digit, sel_above;
  int cnt_gt;
};

// The threshold of block_topk_select's selection (n > k > 0): T = the k-th largest key and
// krem = how many keys equal to T are taken (the lowest indices among them); every key > T
// is taken.  key_of(i) must be pure (one radix pass per byte).
template <class KeyF>
__device__ uint2 block_topk_threshold(KeyF key_of, int n, int k, TopkSmem& sm) {
  const int tid = threadIdx.x, nt = blockDim.x;
  uint32_t prefix = 0, pmask = 0;
  int krem = k;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256; i += nt) sm.hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += nt) {
      uint32_t kk = key_of(i);
      if ((kk & pmask) == prefix) atomicAdd(&sm.hist[(kk >> shift) & 255u], 1u);
    }
    __syncthreads();
    // inclusive scan over digits in descending order (digit 255 first)
    if (tid < 256) sm.scan[tid] = (int)sm.hist[255 - tid];
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      int v = 0;
      if (tid < 256 && tid >= o) v = sm.scan[tid - o];
      __syncthreads();
      if (tid < 256) sm.scan[tid] += v;
      __syncthreads();
    }
    if (tid < 256) {
      int incl = sm.scan[tid];
      int excl = incl - (int)sm.hist[255 - tid];
      if (incl >= krem && excl < krem) {
        sm.sel_digit = 255 - tid;
        sm.sel_above = excl;
      }
    }
    __syncthreads();
    krem -= sm.sel_above;
    prefix |= (uint32_t)sm.sel_digit << shift;
    pmask |= 255u << shift;
    __syncthreads();
  }
  return make_uint2(prefix, (uint32_t)krem);
}

// Select the k largest u32 keys among indices [0, n) (ties: lowest index
// first).  Writes the selected indices (unordered) to out_idx and returns
// min(n, k).  key_of(i) is evaluated several times per element (one radix
// pass per byte), so it must be pure.
template <class KeyF>
__device__ int block_topk_select(KeyF key_of, int n, int k, int* out_idx, TopkSmem& sm) {
  const int tid = threadIdx.x, nt = blockDim.x;
  if (k <= 0 || n <= 0) return 0;
  if (n <= k) {
    for (int i = tid; i < n; i += nt) out_idx[i] = i;
    __syncthreads();
    return n;
  }
  const uint2 th = block_topk_threshold(key_of, n, k, sm);
  const uint32_t T = th.x;
  const int krem = (int)th.y;
  const int n_gt = k - krem;  // keys strictly greater than T
  if (tid == 0) sm.cnt_gt = 0;
  __syncthreads();
  int eq_taken = 0;
  for (int base = 0; base < n; base += nt) {
    int i = base + tid;
    uint32_t kk = i < n ? key_of(i) : 0u;
    bool gt = i < n && kk > T;
    bool eq = i < n && kk == T;
    if (gt) out_idx[atomicAdd(&sm.cnt_gt, 1)] = i;
    int tot;
    int r = block_rank(eq, sm.wave_tot, &tot);
    if (eq && eq_taken + r < krem) out_idx[n_gt + eq_taken + r] = i;
    eq_taken += tot;
  }
  __syncthreads();
  return k;
}

// In-place descending bitonic sort of P (power of two) u64 keys in LDS.
__device__ __forceinline__ void block_bitonic_sort_desc(uint64_t* keys, int P) {
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < (P >> 1); t += nt) {
        int lo = 2 * t - (t & (stride - 1));
        int hi = lo + stride;
        bool desc = ((lo & size) == 0);
        uint64_t a = keys[lo], b = keys[hi];
        bool swap = desc ? (a < b) : (a > b);
        if (swap) {
          keys[lo] = b;
          keys[hi] = a;
        }
      }
      __syncthreads();
    }
  }
}

__host__ __device__ inline int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// 32-bit mix (splitmix-style finaliser) for the device sampler keys.
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint32_t a, uint32_t b) {
  uint64_t z = seed ^ ((uint64_t)a << 32 | b);
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

}  // namespace frh
