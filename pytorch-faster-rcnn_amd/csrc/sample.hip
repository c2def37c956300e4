// a5: RandomSampler (lib/region.py:43-57,112-126) and the ordered segmented
// compaction it and the target gathers are built on.
//
// Ordered compaction = two launches: per-chunk predicate counts, then each
// chunk block adds the counts of its preceding chunks and ranks its own
// elements with wave ballots (coalesced: round r of a chunk reads elements
// base + r*256 + tid).
#include "seg_topk.h"

namespace frh {

constexpr int kChunkThreads = 256;
constexpr int kChunkRounds = 16;
constexpr int kChunk = kChunkThreads * kChunkRounds;  // 4096 elements per block

__host__ __device__ inline int64_t n_chunks(int64_t n) { return (n + kChunk - 1) / kChunk; }


struct CompactArgs {
  const int64_t* labels;
  int64_t label_seg_stride;
  const int32_t* num;
  int64_t max_n;
  int npred;        // 1 or 2
  int pred[2];      // LabelPred per output list
  int32_t* chunk_counts;  // [S][nchunks][2]
  int64_t nchunks;
};

__global__ void __launch_bounds__(kChunkThreads) chunk_count_kernel(CompactArgs p) {
  __shared__ int scratch[kChunkThreads / kWave];
  const int s = blockIdx.y;
  const int64_t c = blockIdx.x;
  const int64_t n = p.num[s];
  const int64_t base = c * kChunk;
  int cnt[2] = {0, 0};
  if (base < n) {
    const int64_t* lab = p.labels + (int64_t)s * p.label_seg_stride;
    for (int r = 0; r < kChunkRounds; ++r) {
      int64_t i = base + r * kChunkThreads + threadIdx.x;
      if (i < n) {
        int64_t v = lab[i];
        cnt[0] += label_pred(v, p.pred[0]);
        if (p.npred > 1) cnt[1] += label_pred(v, p.pred[1]);
      }
    }
  }
  int t0 = block_sum(cnt[0], scratch);
  int t1 = block_sum(cnt[1], scratch);
  if (threadIdx.x == 0) {
    p.chunk_counts[((int64_t)s * p.nchunks + c) * 2 + 0] = t0;
    p.chunk_counts[((int64_t)s * p.nchunks + c) * 2 + 1] = t1;
  }
}

// Writes list[pred][s][pos] = index (int32) for every element satisfying the
// predicate, in ascending order; totals to counts[s*2+pred].
struct ListWriter {
  int32_t* list[2];
  int64_t list_seg_stride;
  int32_t* counts;
};

__global__ void __launch_bounds__(kChunkThreads) chunk_write_lists_kernel(CompactArgs p, ListWriter w) {
  __shared__ int scratch[kChunkThreads / kWave];
  const int s = blockIdx.y;
  const int64_t c = blockIdx.x;
  const int64_t n = p.num[s];
  const int64_t base = c * kChunk;
  const bool last = (n == 0) ? (c == 0) : (base <= n - 1 && n - 1 < base + kChunk);
  if (base >= n && !last) return;
  // prefix of preceding chunks
  int pre[2] = {0, 0};
  for (int64_t q = threadIdx.x; q < c; q += kChunkThreads) {
    pre[0] += p.chunk_counts[((int64_t)s * p.nchunks + q) * 2 + 0];
    pre[1] += p.chunk_counts[((int64_t)s * p.nchunks + q) * 2 + 1];
  }
  pre[0] = block_sum(pre[0], scratch);
  pre[1] = block_sum(pre[1], scratch);
  const int64_t* lab = p.labels + (int64_t)s * p.label_seg_stride;
  for (int r = 0; r < kChunkRounds; ++r) {
    int64_t i = base + r * kChunkThreads + threadIdx.x;
    int64_t v = i < n ? lab[i] : -1;
    for (int k = 0; k < p.npred; ++k) {
      bool f = i < n && label_pred(v, p.pred[k]);
      int tot;
      int rk = block_rank(f, scratch, &tot);
      if (f) w.list[k][(int64_t)s * w.list_seg_stride + pre[k] + rk] = (int32_t)i;
      pre[k] += tot;
    }
  }
  if (last && threadIdx.x == 0 && w.counts) {
    w.counts[s * 2 + 0] = pre[0];
    if (p.npred > 1) w.counts[s * 2 + 1] = pre[1];
  }
}

__global__ void fill_i64_kernel(int64_t* out, int64_t seg_stride, const int32_t* num, int64_t max_n,
                                int64_t v) {
  const int s = blockIdx.y;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < max_n && i < num[s]) out[(int64_t)s * seg_stride + i] = v;
}

// numpy-parity apply: keep the host-chosen list positions.
__global__ void sample_apply_kernel(const int64_t* lab_in, int64_t label_seg_stride,
                                    const int32_t* pos_list, const int32_t* neg_list,
                                    int64_t list_seg_stride, const int32_t* keep_pos,
                                    const int32_t* keep_neg, int64_t keep_ld,
                                    const int32_t* keep_counts, int64_t* lab_out) {
  const int s = blockIdx.y;
  const int which = blockIdx.z;  // 0 pos, 1 neg
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= keep_counts[s * 2 + which]) return;
  const int32_t* keep = (which == 0 ? keep_pos : keep_neg) + (int64_t)s * keep_ld;
  const int32_t* list = (which == 0 ? pos_list : neg_list) + (int64_t)s * list_seg_stride;
  int64_t box = list[keep[j]];
  lab_out[(int64_t)s * label_seg_stride + box] = lab_in[(int64_t)s * label_seg_stride + box];
}

// device-RNG sampler: virtual top-k segment v = 2s (positives) / 2s+1
// (negatives); key = candidate ? (~hash(seed, v, box) | 1) : 0, so the k
// largest keys are a uniform k-subset of the candidates.  Also resets
// labels_out to -1 and writes, per 4096-box chunk, the candidate counts and the
// histograms of the keys' top 8 bits (plain stores: the keys are uniform, so
// 256 buckets leave ~n/256 keys in the k-th one and no refine launch is
// needed); chunk 0 zeroes the collect launch's state words.  Grid (chunks,
// images); no memset.
constexpr int kSampHistBits = 8;
constexpr int kSampBins = 1 << kSampHistBits;

struct SampBufs {
  TkBufs tk;
  uint32_t* part_hist;   // [V][nchunk][kSampBins]
  int32_t* part_count;   // [V][nchunk]
  int nchunk;
  int32_t* sel;          // nullable: [V][sel_ld] the selected indices (any order)
  int64_t sel_ld;
  int32_t* sel_cnt;      // [V] how many
};

// 1024 threads x 4 boxes per 4096-box chunk (the collect launch's chunk): four times
// the waves of a 256-thread chunk for the same histogram layout.
constexpr int kSkThreads = 1024;
constexpr int kSkPer = kTkChunk / kSkThreads;

static __global__ void __launch_bounds__(kSkThreads) sampler_keys_kernel(const int64_t* lab_in, int64_t lstride,
                                                                         const int32_t* num, uint64_t seed,
                                                                         SampBufs sb, int64_t* lab_out) {
  __shared__ uint32_t h[2][kSampBins];
  __shared__ int scratch[kSkThreads / kWave];
  const TkBufs& b = sb.tk;
  const int s = blockIdx.y, c = blockIdx.x;
  const int64_t n = num[s];
  const int64_t base = (int64_t)c * kTkChunk;
  if (c == 0 && threadIdx.x < 2 * TK_WORDS) b.state[2 * s * TK_WORDS + threadIdx.x] = 0;
  tk_hist1_clear(&h[0][0], 2 * kSampBins);
  uint32_t* kp = const_cast<uint32_t*>(b.keys) + (int64_t)(2 * s) * b.ld;
  uint32_t* kn = kp + b.ld;
  int cp = 0, cn = 0;
  int64_t lab[kSkPer];  // every label load in flight at once
#pragma unroll
  for (int r = 0; r < kSkPer; ++r) {
    const int64_t i = base + r * kSkThreads + threadIdx.x;
    lab[r] = i < n ? lab_in[(int64_t)s * lstride + i] : -1;
  }
#pragma unroll
  for (int r = 0; r < kSkPer; ++r) {
    const int64_t i = base + r * kSkThreads + threadIdx.x;
    const bool pos = lab[r] > 0, neg = lab[r] == 0;
    if (lab_out && i < n) lab_out[(int64_t)s * lstride + i] = -1;
    const uint32_t keyp = pos ? ((~hash_u32(seed, 2 * s, (uint32_t)i)) | 1u) : 0u;
    const uint32_t keyn = neg ? ((~hash_u32(seed, 2 * s + 1, (uint32_t)i)) | 1u) : 0u;
    if (i < b.ld) {
      kp[i] = keyp;
      kn[i] = keyn;
    }
    tk_hist_add(h[0], pos, keyp >> (32 - kSampHistBits));
    tk_hist_add(h[1], neg, keyn >> (32 - kSampHistBits));
    cp += pos;
    cn += neg;
  }
  cp = block_sum(cp, scratch);
  cn = block_sum(cn, scratch);
  if (threadIdx.x == 0) {
    sb.part_count[(int64_t)(2 * s) * sb.nchunk + c] = cp;
    sb.part_count[(int64_t)(2 * s + 1) * sb.nchunk + c] = cn;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * kSampBins; i += kSkThreads) {
    const int w = i / kSampBins;
    sb.part_hist[((int64_t)(2 * s + w) * sb.nchunk + c) * kSampBins + (i % kSampBins)] = h[w][i % kSampBins];
  }
}

// sampler policy of the segmented top-k: a selected box gets its input label
// back (labels_out was reset to -1 by the key kernel) and / or is listed at its
// selection slot (the target gathers order the lists themselves)
struct SampPol {
  const int64_t* li;
  int64_t* lo;      // nullable
  int32_t* sel;     // nullable: this virtual segment's list
  int32_t* sel_cnt;
  __device__ void select(int i, uint32_t, int slot) {
    if (lo) lo[i] = li[i];
    if (sel) sel[slot] = i;
  }
  __device__ void finish(int kv) {
    if (sel_cnt && threadIdx.x == 0) *sel_cnt = kv;
  }
};

// Collect launch: grid (chunks, 2 x images), 256 threads.  Every workgroup sums
// the chunk histograms and counts of its segment and of the image's positive
// segment, derives k -- kp = min(npos, pos_num), kn = min(nneg, max_num - kp)
// (region.py:43-57) -- and the two-level plan, then collects (seg_topk.h).
static __global__ void __launch_bounds__(kTkThreads) sampler_collect_kernel(const int64_t* lab_in, int64_t lstride,
                                                                            const int32_t* num, int max_num,
                                                                            int pos_num, SampBufs sb,
                                                                            int64_t* lab_out) {
  __shared__ TkSmem sm;
  const int v = blockIdx.y, s = v >> 1, t = threadIdx.x;
  const int n = num[s];
  const int nch = (int)((n + kTkChunk - 1) / kTkChunk);
  int cp = 0, cn = 0;
  for (int c = t; c < nch; c += kTkThreads) {
    cp += sb.part_count[(int64_t)(2 * s) * sb.nchunk + c];
    cn += sb.part_count[(int64_t)(2 * s + 1) * sb.nchunk + c];
  }
  const int npos = block_sum(cp, sm.part), nneg = block_sum(cn, sm.part);
  const int kp = npos < pos_num ? npos : pos_num;
  const int slots = max_num - kp;
  const int k = (v & 1) ? (nneg < slots ? nneg : slots) : kp;
  uint32_t hsum = 0u;  // bin t (kSampBins == kTkThreads); 32 chunk loads in flight per step
  const uint32_t* ph = sb.part_hist + (int64_t)v * sb.nchunk * kSampBins + t;
  for (int c0 = 0; c0 < nch; c0 += 32) {
    uint32_t x[32];
#pragma unroll
    for (int c = 0; c < 32; ++c) x[c] = c0 + c < nch ? ph[(int64_t)(c0 + c) * kSampBins] : 0u;
#pragma unroll
    for (int c = 0; c < 32; ++c) hsum += x[c];
  }
  sm.h1[t] = hsum;
  __syncthreads();
  const TkPlan plan = tk_plan_direct(kSampHistBits, k, sm, [&](int i) { return sm.h1[i]; });
  SampPol pol{lab_in + (int64_t)s * lstride, lab_out ? lab_out + (int64_t)s * lstride : nullptr,
              sb.sel ? sb.sel + (int64_t)v * sb.sel_ld : nullptr, sb.sel ? sb.sel_cnt + v : nullptr};
  tk_collect_chunk(sb.tk, v, n, plan, pol, sm);
}

// ---------------------------------------------------------------------------
// One-launch device sampler for large images (the RPN's anchors): the keys and
// collect launches above as the phases of ONE launch, separated by in-launch image
// barriers (seg_topk.h seg_barrier).  Workgroup x of image s owns boxes
// [4096x, 4096x + 4096) (16 per thread, labels and keys in registers throughout):
//   1. labels -> positive / negative keys (the same hashes), LDS histograms of
//      their top 8 bits and the class counts, stored per chunk;         barrier
//   2. every workgroup sums the image's chunk counts and histograms: kp, kn
//      (region.py:43-57) and both two-level plans (tk_plan_direct);
//   3. its boxes above each plan's prefix are taken: output label and list slot (round 6:
//      slots from the phase-2 loads -- what the chunks before it take, a block sum, plus its
//      own prefix in thread order; no atomics, lists in box order); its prefix ties go to
//      the class's candidate list (slots likewise); every other box gets label -1;  barrier
//      (only when a class has ties)
//   4. workgroup 0 (positives) / 1 (negatives) orders the class's ties by (key desc, box
//      asc) and takes the first k2 (labels of all tied boxes, list slots of the taken ones);
// then the last workgroup to leave zeroes the image's state words, which is the
// workspace contract (frh_sample_zero_bytes: zero before, zero after).
// The selected set is exactly the two-launch path's.
// The grid's live workgroups must be resident together: the host admits at most half the
// device's resident capacity of the kernel (CU count x occupancy, queried per device: 2 per CU
// by registers on a whole MI355X since round 6's 48-chunk batches, so 256 admitted), else the
// keys + collect launches.

// Block-wide sums of four ints (all threads get them).  scratch: 4 * nw ints.
__device__ __forceinline__ int4 block_sum4(int4 v, int* scratch) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v.x += __shfl_xor(v.x, o, kWave);
    v.y += __shfl_xor(v.y, o, kWave);
    v.z += __shfl_xor(v.z, o, kWave);
    v.w += __shfl_xor(v.w, o, kWave);
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane_id() == 0) scratch[4 * w] = v.x, scratch[4 * w + 1] = v.y, scratch[4 * w + 2] = v.z, scratch[4 * w + 3] = v.w;
  __syncthreads();
  int4 t = make_int4(0, 0, 0, 0);
  for (int i = 0; i < nw; ++i) t.x += scratch[4 * i], t.y += scratch[4 * i + 1], t.z += scratch[4 * i + 2], t.w += scratch[4 * i + 3];
  __syncthreads();
  return t;
}

// This thread's first (selection, candidate) slots in list 0 (.x, .y) and list 1 (.z, .w): the
// workgroup's bases plus the exclusive prefix of the counts in thread order (per workgroup each
// count < 65536: packed pairs, one scan per list).  Block-uniform call; part: 2 * nw ints.
__device__ __forceinline__ int4 block_offsets4(int nsel0, int ncand0, int nsel1, int ncand1, int4 base, int* part) {
  const int t = threadIdx.x, w = t / kWave, nw = (int)blockDim.x / kWave;
  __syncthreads();  // part free
  const int a = nsel0 | (ncand0 << 16), b = nsel1 | (ncand1 << 16);
  int ia = a, ib = b;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int xa = __shfl_up(ia, o, kWave), xb = __shfl_up(ib, o, kWave);
    if (lane_id() >= o) ia += xa, ib += xb;
  }
  if (lane_id() == kWave - 1) part[w] = ia, part[nw + w] = ib;
  __syncthreads();
  int pa = 0, pb = 0;
  for (int i = 0; i < w; ++i) pa += part[i], pb += part[nw + i];
  __syncthreads();  // part reused after
  const int ea = pa + ia - a, eb = pb + ib - b;
  return make_int4(base.x + (ea & 0xffff), base.y + (ea >> 16), base.z + (eb & 0xffff), base.w + (eb >> 16));
}

constexpr int kSampBatch = 48;  // chunk histograms per thread and class in flight (phase 2)

struct SampFused {
  uint32_t* part_hist;   // [S][2][nchunk][kSampBins] per-chunk histograms (sc1 stores, every call)
  int32_t* part_count;   // [S][2][nchunk] per-chunk class counts
  int nchunk;
  int32_t* state;    // [S][2][TK_WORDS]     zero before and after
  uint64_t* cand;    // [S][2][ld] prefix ties: key << 32 | ~box
  int64_t ld;
  int32_t* sel;      // nullable: [S][2][sel_ld]
  int64_t sel_ld;
  int32_t* sel_cnt;  // [S][2]
  int64_t* stamps;   // tools timing only (null in the product): 16 int64 per workgroup
  int32_t* status;   // the caller's device status word (FRH_DEVERR_SAMPLER_BARRIER)
  uint64_t* spec;      // [S][2][nchunk][kSpecCap] the chunk's window records: key << 32 | ~box
  int32_t* part_spec;  // [S][nchunk] the chunk's negatives in the key window
};

// Window records (round 6): every positive and every negative whose key has its top kSpecBits
// bits set (1/128 of the uniform keys) is written, per chunk, as (key << 32 | ~box) to the
// chunk's own record row.  After the first barrier, when the window holds the whole selection
// -- at least kn negatives in it (or all of them), every positive listed, no chunk row and no
// class above the LDS capacity -- the k largest records of each class are exactly the
// selection, and two workgroups finish the call from the records alone (fast path); otherwise
// every workgroup goes on with the histogram phases 2-4.
constexpr int kSpecBits = 7;
constexpr int kSpecCap = 256;  // records per chunk row and class

__device__ __forceinline__ uint32_t samp_key(uint64_t seed, int v, int i, bool cand) {
  return cand ? ((~hash_u32(seed, (uint32_t)v, (uint32_t)i)) | 1u) : 0u;
}

static __global__ void __launch_bounds__(kTkThreads) sampler_fused_kernel(const int64_t* lab_in, int64_t lstride,
                                                                          const int32_t* num, int max_num,
                                                                          int pos_num, uint64_t seed, SampFused f,
                                                                          int64_t* lab_out) {
  __shared__ TkSmem sm;
  __shared__ uint32_t hc[2 * kSampBins];
  const int s = blockIdx.y, x = blockIdx.x, t = threadIdx.x;
  const int n = num[s];
  const int G = n > kTkChunk ? (n + kTkChunk - 1) / kTkChunk : 1;
  if (x >= G) return;
  // A set status word means an earlier one-launch call (this kernel or the RPN's) ran out of a
  // wait: this workspace's zero region may hold its counters, so a barrier here could pass on
  // them early.  Do nothing; the word stays set (the loss entries turn it into NaN losses) until
  // the host's check clears it and replaces the workspace.  (Loaded here, tested before the
  // first zero-region access, so the load overlaps phase 1.)
  const int32_t status0 = __hip_atomic_load(f.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  auto stamp = [&](int q) {
    if (f.stamps && t == 0)
      f.stamps[((int64_t)s * gridDim.x + x) * 16 + q] = (int64_t)__builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  int32_t* st = f.state + (int64_t)(2 * s) * TK_WORDS;  // [2][TK_WORDS]: positives, negatives
  int32_t* bar = f.state + tk_bars_offset(2 * (int)gridDim.y) + s * kBarWords;  // its own line
  const int64_t* li = lab_in + (int64_t)s * lstride;
  int64_t* lo = lab_out ? lab_out + (int64_t)s * lstride : nullptr;
  const int base = x * kTkChunk;

  // ---- phase 1
  int32_t lab[kTkPerThread];  // box labels (-1, 0, g + 1) fit 32 bits: kept to the end
#pragma unroll
  for (int r = 0; r < kTkPerThread; ++r) {
    const int i = base + r * kTkThreads + t;
    lab[r] = i < n ? (int32_t)li[i] : -1;
  }
  for (int i = t; i < 2 * kSampBins; i += kTkThreads) hc[i] = 0u;
  __syncthreads();
  uint32_t key[kTkPerThread], posm = 0u, negm = 0u;
  int cp = 0, cn = 0;
#pragma unroll
  for (int r = 0; r < kTkPerThread; ++r) {
    const int i = base + r * kTkThreads + t;
    const bool pos = lab[r] > 0, neg = lab[r] == 0;
    posm |= pos ? 1u << r : 0u;
    negm |= neg ? 1u << r : 0u;
    key[r] = samp_key(seed, 2 * s + (neg ? 1 : 0), i, pos || neg);
    tk_hist_add(hc, pos, key[r] >> (32 - kSampHistBits));
    tk_hist_add(hc + kSampBins, neg, key[r] >> (32 - kSampHistBits));
    cp += pos;
    cn += neg;
  }
  stamp(1);
  uint32_t specm = posm;
#pragma unroll
  for (int r = 0; r < kTkPerThread; ++r)
    specm |= (((negm >> r) & 1u) && (key[r] >> (32 - kSpecBits)) == (1u << kSpecBits) - 1u) ? 1u << r : 0u;
  // one block scan gives the class counts and this thread's record slots: (positives | window
  // negatives << 16) and negatives per thread, packed (per workgroup each < 65536)
  int qp, qn, spec_n;
  {
    const int pa = cp | (__popc(specm & negm) << 16);
    int ia = pa, ib = cn;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int xa = __shfl_up(ia, o, kWave), xb = __shfl_up(ib, o, kWave);
      if (lane_id() >= o) ia += xa, ib += xb;
    }
    const int w = t / kWave;
    if (lane_id() == kWave - 1) sm.part[w] = ia, sm.part[kTkThreads / kWave + w] = ib;
    __syncthreads();
    int ea = 0, ta = 0, tb = 0;
#pragma unroll
    for (int i = 0; i < kTkThreads / kWave; ++i) {
      const int va = sm.part[i];
      ea += i < w ? va : 0;
      ta += va;
      tb += sm.part[kTkThreads / kWave + i];
    }
    ea += ia - pa;
    qp = ea & 0xffff, qn = ea >> 16;
    cp = ta & 0xffff, spec_n = ta >> 16, cn = tb;
  }
  {
    // this chunk's window records, in thread order (rows past kSpecCap are not written: such a
    // chunk sends the call to the histogram phases)
    uint64_t* rp = f.spec + ((int64_t)(2 * s) * f.nchunk + x) * kSpecCap;
    uint64_t* rn = rp + (int64_t)f.nchunk * kSpecCap;
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r) {
      if (!((specm >> r) & 1u)) continue;
      const int i = base + r * kTkThreads + t;
      const uint64_t rec = ((uint64_t)key[r] << 32) | (uint32_t)~(uint32_t)i;
      if ((posm >> r) & 1u) {
        if (qp < kSpecCap) xwg_store(rp + qp, rec);
        ++qp;
      } else {
        if (qn < kSpecCap) xwg_store(rn + qn, rec);
        ++qn;
      }
    }
    if (t == 0) xwg_store(reinterpret_cast<uint32_t*>(f.part_spec) + (int64_t)s * f.nchunk + x, (uint32_t)spec_n);
  }
  // this chunk's histograms and counts, write-through (one store per bin: no atomics on
  // the 256 hot bins of an image, which every chunk's uniform keys fill)
  uint32_t* ph = f.part_hist + (int64_t)(2 * s) * f.nchunk * kSampBins;  // [2][nchunk][bins]
  int32_t* pc = f.part_count + (int64_t)(2 * s) * f.nchunk;               // [2][nchunk]
  if (t == 0) {
    xwg_store(reinterpret_cast<uint32_t*>(pc) + x, (uint32_t)cp);
    xwg_store(reinterpret_cast<uint32_t*>(pc) + f.nchunk + x, (uint32_t)cn);
  }
  for (int i = t; i < 2 * kSampBins; i += kTkThreads)
    xwg_store(ph + ((int64_t)(i / kSampBins) * f.nchunk + x) * kSampBins + (i % kSampBins), hc[i]);
  stamp(2);
  // a call that cannot finish leaves defined (memory-safe) outputs all the same: the boxes of
  // `m` get label -1, and workgroup 0 lists nothing
  auto bail = [&](uint32_t m) {
    if (lo) {
#pragma unroll
      for (int r = 0; r < kTkPerThread; ++r) {
        const int i = base + r * kTkThreads + t;
        if (i < n && ((m >> r) & 1u)) lo[i] = -1;
      }
    }
    if (x == 0 && f.sel_cnt && t < 2) f.sel_cnt[2 * s + t] = 0;
  };
  if (status0 != 0) return bail(~0u);
  if (!seg_barrier(bar, G, f.status, FRH_DEVERR_SAMPLER_BARRIER)) return bail(~0u);
  stamp(3);
  // the last workgroup out leaves the image's zero region zero
  auto leave = [&]() {
    stamp(7);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) sm.last = atomicAdd(st + TK_DONE1, 1) == G - 1;
    __syncthreads();
    if (sm.last && t < 2 * TK_WORDS) xwg_store(reinterpret_cast<uint32_t*>(st) + t, 0u);
    if (sm.last && t < 2) xwg_store(reinterpret_cast<uint32_t*>(bar) + t, 0u);
    stamp(8);
  };

  // ---- fast path: the window records hold the selection (G <= kTkThreads: the host admits at
  // most 256 workgroups)
  {
    const int32_t* psn = f.part_spec + (int64_t)s * f.nchunk;
    const int cpv = t < G ? xwg_load(pc + t) : 0, cnv = t < G ? xwg_load(pc + f.nchunk + t) : 0;
    const int snv = t < G ? xwg_load(psn + t) : 0;
    const int4 tot = block_sum4(make_int4(cpv, cnv, snv, (cpv > kSpecCap || snv > kSpecCap) ? 1 : 0), sm.fb.wave_tot);
    const int npos = tot.x, nneg = tot.y, nspec = tot.z;
    const int kp = npos < pos_num ? npos : pos_num;
    const int kn = nneg < max_num - kp ? nneg : max_num - kp;
    const bool okp = npos <= kTkCandCap;
    const bool okn = kn <= 0 || (nspec <= kTkCandCap && (kn < nneg ? nspec >= kn : nspec == nneg));
    if (G <= kTkThreads && tot.w == 0 && okp && okn) {
      stamp(9);
      if (lo) {  // boxes outside the window: never selected
#pragma unroll
        for (int r = 0; r < kTkPerThread; ++r) {
          const int i = base + r * kTkThreads + t;
          if (i < n && !((specm >> r) & 1u)) lo[i] = -1;
        }
      }
      for (int c = 0; c < 2; ++c) {
        if (x != (c < G ? c : 0)) continue;
        const int v = 2 * s + c, kv = c ? kn : kp, nc = c ? nspec : npos;
        if (f.sel_cnt && t == 0) f.sel_cnt[v] = kv > 0 ? kv : 0;
        if (nc == 0) continue;
        // the class's records from every chunk row into LDS at the row's offset (an exclusive scan
        // of the row counts): wave w copies rows w, w + 4, ..., 64 records of 16 rows in flight
        stamp(4);
        const int rc = c ? snv : cpv;
        if (G <= kWave) {  // every row count is in wave 0: its own scan, one barrier
          if (t < kWave) {
            int inc = rc;
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
              const int y = __shfl_up(inc, o, kWave);
              if (lane_id() >= o) inc += y;
            }
            if (t < G) hc[t] = (uint32_t)(inc - rc), hc[kSampBins + t] = (uint32_t)rc;
          }
        } else {
          const int4 o = block_offsets4(rc, 0, 0, 0, make_int4(0, 0, 0, 0), sm.part);
          if (t < G) hc[t] = (uint32_t)o.x, hc[kSampBins + t] = (uint32_t)rc;
        }
        __syncthreads();
        const uint64_t* rows = f.spec + (int64_t)v * f.nchunk * kSpecCap;
        const int w = t / kWave, ln = lane_id();
        constexpr int kRowsPerWave = 16;
        uint64_t rec[kRowsPerWave];
#pragma unroll
        for (int u = 0; u < kRowsPerWave; ++u) {
          const int j = w + u * (kTkThreads / kWave);
          rec[u] = j < G && ln < (int)hc[kSampBins + j] ? xwg_load(rows + (int64_t)j * kSpecCap + ln) : 0ull;
        }
#pragma unroll
        for (int u = 0; u < kRowsPerWave; ++u) {
          const int j = w + u * (kTkThreads / kWave);
          if (j < G && ln < (int)hc[kSampBins + j]) sm.cand[hc[j] + ln] = rec[u];
        }
        // rows beyond 64 records, rows of chunks >= 64 (rare: one at a time)
        for (int j = w; j < G; j += kTkThreads / kWave)
          for (int l = (j < kRowsPerWave * (kTkThreads / kWave) ? kWave : 0) + ln; l < (int)hc[kSampBins + j]; l += kWave)
            sm.cand[hc[j] + l] = xwg_load(rows + (int64_t)j * kSpecCap + l);
        __syncthreads();
        stamp(5);
        const bool all = kv >= nc;
        LdsCut cut{0ull, 0};
        if (kv > 0 && !all)
          cut = c ? lds_topk_cut(sm.cand, nc, kv, 64 - kSpecBits, ((1ull << kSpecBits) - 1ull) << (64 - kSpecBits), sm)
                  : lds_topk_cut(sm.cand, nc, kv, 64, 0ull, sm);
        if (t == 0) sm.fb.cnt_gt = 0;
        __syncthreads();
        stamp(6);
        int32_t* sl = f.sel ? f.sel + (int64_t)v * f.sel_ld : nullptr;
        for (int q = t; q < nc; q += kTkThreads) {
          const uint64_t e = sm.cand[q];
          const int i = (int)~(uint32_t)e;
          const bool tk = kv > 0 && (all || (e >> cut.sh) >= (cut.P >> cut.sh));
          if (lo) lo[i] = tk ? (c ? (int64_t)0 : li[i]) : (int64_t)-1;
          if (sl && tk) sl[atomicAdd(&sm.fb.cnt_gt, 1)] = i;
        }
        __syncthreads();  // sm.cand, hc reused by the other class
      }
      leave();
      return;
    }
  }

  // ---- phase 2: the image's counts and histograms, summed over its chunks (bin t per thread)
  // the count loads (threads < G) and the first 2 x kSampBatch chunk-histogram loads are issued
  // together (48: one round trip for the cfg2 RPN's 38 chunks per image);
  // the sums over the chunks BEFORE this one (_lt) give this workgroup's list slots (phase 3)
  int sp0 = 0, sn0 = 0, sp_lt = 0, sn_lt = 0;
  uint32_t hp = 0u, hn = 0u, hp_lt = 0u, hn_lt = 0u;
  for (int c0 = 0; c0 < G; c0 += kSampBatch) {
    uint32_t a[kSampBatch], b[kSampBatch];
    const int cc = c0 + t;
    const int32_t cpv = cc < G && t < kSampBatch ? xwg_load(pc + cc) : 0, cnv = cc < G && t < kSampBatch ? xwg_load(pc + f.nchunk + cc) : 0;
#pragma unroll
    for (int c = 0; c < kSampBatch; ++c) {
      a[c] = c0 + c < G ? xwg_load(ph + (int64_t)(c0 + c) * kSampBins + t) : 0u;
      b[c] = c0 + c < G ? xwg_load(ph + ((int64_t)f.nchunk + c0 + c) * kSampBins + t) : 0u;
    }
    sp0 += cpv, sn0 += cnv;
    if (cc < x) sp_lt += cpv, sn_lt += cnv;
#pragma unroll
    for (int c = 0; c < kSampBatch; ++c) {
      hp += a[c], hn += b[c];
      if (c0 + c < x) hp_lt += a[c], hn_lt += b[c];
    }
  }
  const int npos = block_sum(sp0, sm.part), nneg = block_sum(sn0, sm.part);
  hc[t] = hp;
  hc[kSampBins + t] = hn;
  __syncthreads();
  const int kp = npos < pos_num ? npos : pos_num;
  const int kn = nneg < max_num - kp ? nneg : max_num - kp;
  TkPlan pl[2];
  pl[0] = tk_plan_direct(kSampHistBits, kp, sm, [&](int i) { return hc[i]; });
  pl[1] = tk_plan_direct(kSampHistBits, kn, sm, [&](int i) { return hc[kSampBins + i]; });
  stamp(4);

  // ---- phase 3 (the plans' fields by select, not by a per-box array index)
  uint32_t take = 0u, tie = 0u;
  const int sh = 32 - kSampHistBits;
#pragma unroll
  for (int r = 0; r < kTkPerThread; ++r) {
    const bool neg = (negm >> r) & 1u, cand = ((posm | negm) >> r) & 1u;
    const uint32_t pre = key[r] >> sh, P = neg ? pl[1].P : pl[0].P;
    const bool all = neg ? pl[1].all : pl[0].all;
    const bool live = cand && (neg ? pl[1].kv : pl[0].kv) > 0;
    take |= (live && (all || pre > P)) ? 1u << r : 0u;
    tie |= (live && !all && pre == P) ? 1u << r : 0u;
  }
  // both classes' (selection, candidate) slots without atomics: the chunks before this one take
  // their class count (plan `all`), or their keys in bins above P (and list their bin-P keys as
  // ties) -- sums of the phase-2 loads over t > P / t == P -- then this workgroup's own keys in
  // thread order.  (One contended atomic per workgroup on the image's counters, 38 workgroups
  // on one word at cfg2, cost more than these block sums.)  The lists come out in box order.
  int4 lbase;
  {
    const bool lp = pl[0].kv > 0, ln = pl[1].kv > 0;
    const int P0 = (int)pl[0].P, P1 = (int)pl[1].P;
    lbase = block_sum4(make_int4(!lp ? 0 : pl[0].all ? sp_lt : (t > P0 ? (int)hp_lt : 0),
                                (lp && !pl[0].all && t == P0) ? (int)hp_lt : 0,
                                !ln ? 0 : pl[1].all ? sn_lt : (t > P1 ? (int)hn_lt : 0),
                                (ln && !pl[1].all && t == P1) ? (int)hn_lt : 0),
                      sm.fb.wave_tot);
  }
  const int4 sl4 = block_offsets4(__popc(take & posm), __popc(tie & posm), __popc(take & negm), __popc(tie & negm),
                                  lbase, sm.part);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const uint32_t m = c ? negm : posm;
    int sp = c ? sl4.z : sl4.x, cq = c ? sl4.w : sl4.y;
    int32_t* sl = f.sel ? f.sel + (int64_t)(2 * s + c) * f.sel_ld : nullptr;
    uint64_t* cl = f.cand + (int64_t)(2 * s + c) * f.ld;
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r) {
      if (!((m >> r) & 1u)) continue;
      const int i = base + r * kTkThreads + t;
      if ((take >> r) & 1u) {
        if (sl) sl[sp] = i;
        ++sp;
      } else if ((tie >> r) & 1u) {
        xwg_store(cl + cq++, ((uint64_t)key[r] << 32) | (uint32_t)~(uint32_t)i);
      }
    }
  }
  if (lo) {
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r) {
      const int i = base + r * kTkThreads + t;
      if (i < n && !((tie >> r) & 1u)) lo[i] = ((take >> r) & 1u) ? (int64_t)lab[r] : (int64_t)-1;
    }
  }
  const bool ties = (pl[0].kv > 0 && !pl[0].all) || (pl[1].kv > 0 && !pl[1].all);
  stamp(5);
  if (ties && !seg_barrier(bar + 1, G, f.status, FRH_DEVERR_SAMPLER_BARRIER)) return bail(tie);
  stamp(6);

  // ---- phase 4: the prefix ties, positives by workgroup 0, negatives by workgroup 1 (0 if alone)
  for (int c = 0; c < 2; ++c) {
    if (x != (c < G ? c : 0)) continue;
    {
      const int v = 2 * s + c, kv = pl[c].kv;
      if (f.sel_cnt && t == 0) f.sel_cnt[v] = kv;
      if (kv == 0 || pl[c].all) continue;
      const int k2 = pl[c].k2, nabove = kv - k2;
      int32_t* sl = f.sel ? f.sel + (int64_t)v * f.sel_ld : nullptr;
      const uint64_t* cl = f.cand + (int64_t)v * f.ld;
      const int ncand = (int)hc[c * kSampBins + (int)pl[c].P];  // every key of the class in bin P
      if (ncand <= kTkCandCap) {
        // the k2 largest (key, ~box) of the prefix ties by radix passes over the key's
        // next bits (its top kSampHistBits are the plan's prefix): no sort
        for (int j = t; j < ncand; j += kTkThreads) sm.cand[j] = xwg_load(cl + j);
        if (t == 0) sm.fb.cnt_gt = 0;
        __syncthreads();
        const LdsCut cut = lds_topk_cut(sm.cand, ncand, k2, 64 - kSampHistBits,
                                        (uint64_t)pl[c].P << (64 - kSampHistBits), sm);
        for (int j = t; j < ncand; j += kTkThreads) {
          const uint64_t e = sm.cand[j];
          const int i = (int)~(uint32_t)e;
          const bool tk = (e >> cut.sh) >= (cut.P >> cut.sh);
          if (lo) lo[i] = tk ? li[i] : -1;
          if (sl && tk) sl[nabove + atomicAdd(&sm.fb.cnt_gt, 1)] = i;
        }
        __syncthreads();  // sm.cand reused by the other class
      } else {
        // more ties than the LDS sort holds: an exact radix threshold over the class's prefix
        // keys (recomputed from the labels), then one ordered pass labels every tied box
        const uint32_t P = pl[c].P;
        const int sh = pl[c].sh;
        auto key_of = [&](int i) -> uint32_t {
          const int64_t lb = li[i];
          const uint32_t kq = samp_key(seed, v, i, c ? lb == 0 : lb > 0);
          return (kq != 0u && (kq >> sh) == P) ? kq : 0u;
        };
        const uint2 th = block_topk_threshold(key_of, n, k2, sm.fb);
        const uint32_t T = th.x;
        const int krem = (int)th.y, n_gt = k2 - (int)th.y;
        if (t == 0) sm.fb.cnt_gt = 0;
        __syncthreads();
        int eq_taken = 0;
        for (int b0 = 0; b0 < n; b0 += kTkThreads) {
          const int i = b0 + t;
          const uint32_t kq = i < n ? key_of(i) : 0u;
          const bool gt = kq != 0u && kq > T, eq = kq != 0u && kq == T;
          int tot;
          const int rk = block_rank(eq, sm.fb.wave_tot, &tot);
          const bool tk = gt || (eq && eq_taken + rk < krem);
          if (kq != 0u && lo) lo[i] = tk ? li[i] : -1;
          if (sl && gt) sl[nabove + atomicAdd(&sm.fb.cnt_gt, 1)] = i;
          if (sl && eq && eq_taken + rk < krem) sl[nabove + n_gt + eq_taken + rk] = i;
          eq_taken += tot;
        }
        __syncthreads();
      }
    }
  }

  leave();
}

// Small images (num_boxes <= kSsMax, e.g. the RCNN stage's ~2000 proposal rows): the whole
// sampler of an image in ONE 1024-thread workgroup -- the same keys (hash of (seed, 2s or
// 2s + 1, box)), the same selection (the k largest keys, equal keys by ascending box), by
// an exact radix select over the keys held in registers: per 8-bit digit, an LDS
// histogram of the keys still tied with the threshold prefix, the digit holding the k-th
// key found by one wave, until the tied bucket is taken whole or the full key is fixed.
// No global round trips between the label loads and the outputs.
constexpr int kSsThreads = 1024;
constexpr int kSsPer = 16;
constexpr int kSsMax = kSsThreads * kSsPer;

struct SsPlan {
  uint32_t P;  // threshold prefix (pb bits)
  int pb;      // prefix bits fixed (0, 8, .., 32)
  int k;       // keys with prefix == P still to take
  int all;     // every key with prefix == P is taken
};

// Exact top-k plan over the nonzero keys key[r] of the workgroup (k >= 1, k < #nonzero).
// Block-uniform call.
__device__ SsPlan ss_plan(const uint32_t (&key)[kSsPer], int k, uint32_t* h, int* sh) {
  const int t = threadIdx.x;
  uint32_t P = 0u;
  int pb = 0;
  for (;;) {
    for (int i = t; i < 256; i += kSsThreads) h[i] = 0u;
    __syncthreads();
    const int sh_digit = 24 - pb;
#pragma unroll
    for (int r = 0; r < kSsPer; ++r) {
      const bool in = key[r] != 0u && (pb == 0 || (key[r] >> (32 - pb)) == P);
      if (in) atomicAdd(&h[(key[r] >> sh_digit) & 255u], 1u);
    }
    __syncthreads();
    if (t < kWave) {  // wave 0: lane l holds digits 255 - 4l .. 252 - 4l (descending)
      uint32_t c[4], sum = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) sum += (c[q] = h[255 - 4 * t - q]);
      uint32_t incl = sum;
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t x = __shfl_up(incl, o, kWave);
        if (t >= o) incl += x;
      }
      uint32_t run = incl - sum;  // keys with a larger digit than this lane's first
      if (run < (uint32_t)k && incl >= (uint32_t)k) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (run + c[q] >= (uint32_t)k) {
            sh[0] = 255 - 4 * t - q;  // the digit holding the k-th key
            sh[1] = (int)run;         // keys above it
            sh[2] = (int)c[q];        // keys in it
            break;
          }
          run += c[q];
        }
      }
    }
    __syncthreads();
    const uint32_t d = (uint32_t)sh[0];
    const int above = sh[1], inb = sh[2];
    __syncthreads();  // sh reused by the next level
    P = (P << 8) | d;
    pb += 8;
    k -= above;
    if (inb == k || pb == 32) return SsPlan{P, pb, k, inb == k};
  }
}

// grid (2, images): workgroup (w, s) selects image s's positives (w = 0) or negatives
// (w = 1), so only its own class's keys are hashed; both count both classes (kn depends on
// kp).  Box labels: the positives' workgroup writes positives and ignored boxes, the
// negatives' workgroup negatives.
__global__ void __launch_bounds__(kSsThreads) sampler_small_kernel(const int64_t* lab_in, int64_t lstride,
                                                                   const int32_t* num, int max_num, int pos_num,
                                                                   uint64_t seed, int64_t* lab_out, int32_t* sel,
                                                                   int64_t sel_ld, int32_t* sel_cnt) {
  __shared__ uint32_t h[256];
  __shared__ int scratch[kSsThreads / kWave];
  __shared__ int sh[4];
  __shared__ int slot;
  __shared__ int part[kSsThreads / kWave];
  const int w = blockIdx.x, s = blockIdx.y, t = threadIdx.x;
  const int v = 2 * s + w;
  const int n = num[s];
  int64_t lab[kSsPer];
  uint32_t key[kSsPer];
  int cnt[2] = {0, 0};
#pragma unroll
  for (int r = 0; r < kSsPer; ++r) {
    const int i = r * kSsThreads + t;
    lab[r] = i < n ? lab_in[(int64_t)s * lstride + i] : -1;
  }
#pragma unroll
  for (int r = 0; r < kSsPer; ++r) {
    const int i = r * kSsThreads + t;
    const bool pos = lab[r] > 0, neg = lab[r] == 0;
    cnt[0] += pos;
    cnt[1] += neg;
    key[r] = (w == 0 ? pos : neg) ? ((~hash_u32(seed, (uint32_t)v, (uint32_t)i)) | 1u) : 0u;
  }
  const int npos = block_sum(cnt[0], scratch), nneg = block_sum(cnt[1], scratch);
  const int kp = npos < pos_num ? npos : pos_num;
  const int kn = nneg < max_num - kp ? nneg : max_num - kp;
  const int k = w == 0 ? kp : kn, c = w == 0 ? npos : nneg;
  uint32_t take = 0u;  // bit r: element r taken
  if (k > 0 && k >= c) {  // every candidate
#pragma unroll
    for (int r = 0; r < kSsPer; ++r) take |= key[r] != 0u ? 1u << r : 0u;
  } else if (k > 0) {
    const SsPlan pl = ss_plan(key, k, h, sh);
    const int sh_p = 32 - pl.pb;
    uint32_t tie = 0u;
#pragma unroll
    for (int r = 0; r < kSsPer; ++r) {
      const uint32_t pre = key[r] >> sh_p;
      if (key[r] != 0u && pre > pl.P) take |= 1u << r;
      if (key[r] != 0u && pre == pl.P) tie |= 1u << r;
    }
    if (pl.all) {
      take |= tie;
    } else {  // the first pl.k tied keys by ascending box (box = r * kSsThreads + t)
      int before = 0;
      for (int r = 0; r < kSsPer; ++r) {
        if (r * kSsThreads >= n) break;  // uniform: rounds past the image's boxes hold no key
        int tot;
        const bool f = (tie >> r) & 1u;
        const int rk = block_rank(f, part, &tot);
        if (f && before + rk < pl.k) take |= 1u << r;
        before += tot;
      }
    }
  }
  if (t == 0) slot = 0;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kSsPer; ++r) {
    if (r * kSsThreads >= n) break;  // uniform (the RCNN stage's ~2000 rows: 2 of 16 rounds)
    const int i = r * kSsThreads + t;
    const bool tk = (take >> r) & 1u;
    const bool mine = w == 0 ? lab[r] != 0 : lab[r] == 0;  // positives + ignored, or negatives
    if (lab_out && i < n && mine) lab_out[(int64_t)s * lstride + i] = tk ? lab[r] : -1;
    if (sel) {
      const int sp = wave_append(tk, &slot);
      if (tk) sel[(int64_t)v * sel_ld + sp] = i;
    }
  }
  if (sel && t == 0) sel_cnt[v] = k > 0 ? k : 0;
}

int32_t launch_compact_lists(int32_t S, const int64_t* labels, int64_t label_seg_stride,
                             const int32_t* num, int64_t max_n, int npred, const int* preds,
                             int32_t** lists, int64_t list_seg_stride, int32_t* counts,
                             int32_t* chunk_counts, hipStream_t st) {
  CompactArgs p{labels, label_seg_stride, num, max_n, npred, {preds[0], npred > 1 ? preds[1] : preds[0]},
                chunk_counts, n_chunks(max_n > 0 ? max_n : 1)};
  dim3 grid((unsigned)p.nchunks, (unsigned)S);
  hipLaunchKernelGGL(chunk_count_kernel, grid, dim3(kChunkThreads), 0, st, p);
  ListWriter w{{lists[0], npred > 1 ? lists[1] : lists[0]}, list_seg_stride, counts};
  hipLaunchKernelGGL(chunk_write_lists_kernel, grid, dim3(kChunkThreads), 0, st, p, w);
  return check_launch("ordered compaction");
}

size_t compact_workspace(int32_t S, int64_t max_n) {
  return (size_t)S * (size_t)n_chunks(max_n > 0 ? max_n : 1) * 2 * sizeof(int32_t);
}

int32_t sample_random_impl(int32_t num_segs, const int64_t* labels_in, int64_t label_seg_stride,
                           const int32_t* num_boxes, int64_t max_boxes, int32_t max_num, int32_t pos_num,
                           uint64_t seed, int64_t* labels_out, int32_t* sel, int32_t* sel_counts, int32_t* status,
                           void* workspace, size_t ws_bytes, void* stream, bool two_launches,
                           int64_t* stamps = nullptr);

}  // namespace frh

using namespace frh;

static size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

struct SampLayout {
  size_t keys, cand, state, phist, pcount, spec, pspec, total;
  int64_t kld;
  int nchunk;
};

// The leading zero region (frh_sample_zero_bytes): the one-launch sampler's state words
// [V][TK_WORDS] and barrier lines, sized for the largest num_segs (kSampMaxSegs) whatever
// the call's, so that no other buffer of any call lies in it (a reused workspace stays
// zero there across calls of different num_segs and paths); the rest follows it.
constexpr int32_t kSampMaxSegs = 64;
static size_t samp_zero_bytes(int32_t S) {  // state words [2S][TK_WORDS] + a barrier line per image
  return al256(((size_t)tk_bars_offset(2 * S) + (size_t)S * kBarWords) * sizeof(int32_t));
}

static SampLayout samp_layout(int32_t S, int64_t max_boxes) {
  SampLayout z{};
  const size_t n = (size_t)(max_boxes > 0 ? max_boxes : 1);
  const int V = 2 * S;
  z.kld = (int64_t)n;
  z.nchunk = (int)((n + kTkChunk - 1) / kTkChunk);
  z.keys = samp_zero_bytes(kSampMaxSegs);
  z.cand = z.keys + al256((size_t)V * n * sizeof(uint32_t));
  z.state = z.cand + al256((size_t)V * n * sizeof(uint64_t));
  z.phist = z.state + al256((size_t)V * TK_WORDS * sizeof(int32_t));
  z.pcount = z.phist + al256((size_t)V * z.nchunk * kSampBins * sizeof(uint32_t));
  z.spec = z.pcount + al256((size_t)V * z.nchunk * sizeof(int32_t));
  z.pspec = z.spec + al256((size_t)V * z.nchunk * kSpecCap * sizeof(uint64_t));
  z.total = z.pspec + al256((size_t)S * z.nchunk * sizeof(int32_t));
  return z;
}

extern "C" size_t frh_sample_workspace(int32_t num_segs, int64_t max_boxes) {
  size_t a = al256(compact_workspace(num_segs, max_boxes));
  size_t b = samp_layout(num_segs, max_boxes).total;
  return a > b ? a : b;
}

extern "C" size_t frh_sample_zero_bytes(int32_t num_segs) {
  return num_segs > 0 ? samp_zero_bytes(kSampMaxSegs) : 0;
}

extern "C" int32_t frh_sample_candidates(int32_t num_segs, const int64_t* labels, int64_t label_seg_stride,
                                         const int32_t* num_boxes, int64_t max_boxes, int32_t* pos_list,
                                         int32_t* neg_list, int64_t list_seg_stride, int32_t* counts,
                                         void* workspace, size_t ws_bytes, void* stream) {
  FRH_REQUIRE(num_segs >= 0 && max_boxes >= 0, "negative sizes");
  if (num_segs == 0) return FRH_OK;
  FRH_REQUIRE(labels && num_boxes && pos_list && neg_list && counts, "null pointer argument");
  FRH_REQUIRE(workspace && ws_bytes >= compact_workspace(num_segs, max_boxes), "workspace too small");
  int preds[2] = {kPos, kNeg};
  int32_t* lists[2] = {pos_list, neg_list};
  return launch_compact_lists(num_segs, labels, label_seg_stride, num_boxes, max_boxes, 2, preds, lists,
                              list_seg_stride, counts, reinterpret_cast<int32_t*>(workspace),
                              as_stream(stream));
}

extern "C" int32_t frh_sample_apply(int32_t num_segs, const int64_t* labels_in, int64_t label_seg_stride,
                                    const int32_t* num_boxes, int64_t max_boxes, const int32_t* pos_list,
                                    const int32_t* neg_list, int64_t list_seg_stride,
                                    const int32_t* keep_pos, const int32_t* keep_neg, int64_t keep_ld,
                                    const int32_t* keep_counts, int64_t* labels_out, void* stream) {
  FRH_REQUIRE(num_segs >= 0 && max_boxes >= 0 && keep_ld >= 0, "negative sizes");
  if (num_segs == 0 || max_boxes == 0) return FRH_OK;
  FRH_REQUIRE(labels_in && labels_out && num_boxes && pos_list && neg_list && keep_counts,
              "null pointer argument");
  FRH_REQUIRE(labels_in != labels_out, "labels_out must not alias labels_in");
  hipStream_t st = as_stream(stream);
  dim3 g1((unsigned)((max_boxes + 255) / 256), (unsigned)num_segs);
  hipLaunchKernelGGL(fill_i64_kernel, g1, dim3(256), 0, st, labels_out, label_seg_stride, num_boxes,
                     max_boxes, (int64_t)-1);
  if (keep_ld > 0) {
    FRH_REQUIRE(keep_pos && keep_neg, "null keep lists");
    dim3 g2((unsigned)((keep_ld + 255) / 256), (unsigned)num_segs, 2);
    hipLaunchKernelGGL(sample_apply_kernel, g2, dim3(256), 0, st, labels_in, label_seg_stride, pos_list,
                       neg_list, list_seg_stride, keep_pos, keep_neg, keep_ld, keep_counts, labels_out);
  }
  return check_launch("frh_sample_apply");
}

extern "C" int32_t frh_sample_random(int32_t num_segs, const int64_t* labels_in, int64_t label_seg_stride,
                                     const int32_t* num_boxes, int64_t max_boxes, int32_t max_num,
                                     int32_t pos_num, uint64_t seed, int64_t* labels_out, int32_t* sel,
                                     int32_t* sel_counts, int32_t* status, void* workspace, size_t ws_bytes,
                                     void* stream) {
  return frh::sample_random_impl(num_segs, labels_in, label_seg_stride, num_boxes, max_boxes, max_num, pos_num, seed,
                                 labels_out, sel, sel_counts, status, workspace, ws_bytes, stream, false);
}

// two_launches: the keys + collect launches even where the one-launch sampler applies
// (tools: A/B timing and the equality test of the two)
int32_t frh::sample_random_impl(int32_t num_segs, const int64_t* labels_in, int64_t label_seg_stride,
                                const int32_t* num_boxes, int64_t max_boxes, int32_t max_num, int32_t pos_num,
                                uint64_t seed, int64_t* labels_out, int32_t* sel, int32_t* sel_counts,
                                int32_t* status, void* workspace, size_t ws_bytes, void* stream, bool two_launches,
                                int64_t* stamps) {
  FRH_REQUIRE(num_segs >= 0 && max_boxes >= 0, "negative sizes");
  FRH_REQUIRE(num_segs <= kSampMaxSegs, "num_segs %d exceeds %d", num_segs, kSampMaxSegs);
  FRH_REQUIRE(status, "null status word");
  FRH_REQUIRE(pos_num <= max_num && pos_num >= 0, "pos_num must be in [0, max_num]");
  if (num_segs == 0 || max_boxes == 0) return FRH_OK;
  FRH_REQUIRE(labels_in && num_boxes && (labels_out || sel), "null pointer argument");
  FRH_REQUIRE(!sel == !sel_counts, "sel and sel_counts go together");
  FRH_REQUIRE(labels_in != labels_out, "labels_out must not alias labels_in");
  FRH_REQUIRE(workspace && ws_bytes >= frh_sample_workspace(num_segs, max_boxes), "workspace too small");
  FRH_REQUIRE(max_boxes <= INT32_MAX, "max_boxes must fit in int32");
  static_assert(kSampBins == kTkThreads, "sampler_collect_kernel sums one bin per thread");
  hipStream_t st = as_stream(stream);
  if (max_boxes <= kSsMax) {  // one workgroup per image, one launch
    hipLaunchKernelGGL(sampler_small_kernel, dim3(2u, (unsigned)num_segs), dim3(kSsThreads), 0, st, labels_in,
                       label_seg_stride, num_boxes, max_num, pos_num, seed, labels_out, sel,
                       (int64_t)(max_num > 0 ? max_num : 1), sel_counts);
    return check_launch("frh_sample_random");
  }
  char* ws = reinterpret_cast<char*>(workspace);
  SampLayout z = samp_layout(num_segs, max_boxes);
  const int V = 2 * num_segs;
  if (!two_launches &&
      (int64_t)num_segs * z.nchunk <= resident_capacity(reinterpret_cast<const void*>(sampler_fused_kernel), kTkThreads) / 2) {
    SampFused f{reinterpret_cast<uint32_t*>(ws + z.phist), reinterpret_cast<int32_t*>(ws + z.pcount), z.nchunk,
                reinterpret_cast<int32_t*>(ws), reinterpret_cast<uint64_t*>(ws + z.cand), z.kld, sel,
                (int64_t)(max_num > 0 ? max_num : 1), sel_counts, stamps, status,
                reinterpret_cast<uint64_t*>(ws + z.spec), reinterpret_cast<int32_t*>(ws + z.pspec)};
    hipLaunchKernelGGL(sampler_fused_kernel, dim3((unsigned)z.nchunk, (unsigned)num_segs), dim3(kTkThreads), 0, st,
                       labels_in, label_seg_stride, num_boxes, max_num, pos_num, seed, f, labels_out);
    return check_launch("frh_sample_random");
  }
  SampBufs sb{TkBufs{reinterpret_cast<uint32_t*>(ws + z.keys), z.kld, nullptr, kSampHistBits, nullptr,
                     reinterpret_cast<int32_t*>(ws + z.state), reinterpret_cast<uint64_t*>(ws + z.cand)},
              reinterpret_cast<uint32_t*>(ws + z.phist), reinterpret_cast<int32_t*>(ws + z.pcount), z.nchunk,
              sel, (int64_t)(max_num > 0 ? max_num : 1), sel_counts};
  hipLaunchKernelGGL(sampler_keys_kernel, dim3((unsigned)z.nchunk, (unsigned)num_segs), dim3(kSkThreads), 0, st,
                     labels_in, label_seg_stride, num_boxes, seed, sb, labels_out);
  hipLaunchKernelGGL(sampler_collect_kernel, dim3((unsigned)z.nchunk, (unsigned)V), dim3(kTkThreads), 0, st,
                     labels_in, label_seg_stride, num_boxes, max_num, pos_num, sb, labels_out);
  return check_launch("frh_sample_random");
}
