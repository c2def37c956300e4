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
// labels_out to -1 and counts the candidates.
__global__ void sampler_keys_kernel(const int64_t* lab_in, int64_t lstride, const int32_t* num, uint64_t seed,
                                    uint32_t* keys, int64_t kld, int32_t* counts, int64_t* lab_out) {
  __shared__ int scratch[4];
  const int s = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = num[s];
  bool pos = false, neg = false;
  if (i < n) {
    int64_t l = lab_in[(int64_t)s * lstride + i];
    pos = l > 0;
    neg = l == 0;
    lab_out[(int64_t)s * lstride + i] = -1;
  }
  if (i < kld) {
    keys[(int64_t)(2 * s) * kld + i] = pos ? ((~hash_u32(seed, 2 * s, (uint32_t)i)) | 1u) : 0u;
    keys[(int64_t)(2 * s + 1) * kld + i] = neg ? ((~hash_u32(seed, 2 * s + 1, (uint32_t)i)) | 1u) : 0u;
  }
  int cp = block_sum(pos ? 1 : 0, scratch);
  int cn = block_sum(neg ? 1 : 0, scratch);
  if (threadIdx.x == 0) {
    if (cp) atomicAdd(&counts[2 * s], cp);
    if (cn) atomicAdd(&counts[2 * s + 1], cn);
  }
}

__global__ void sampler_k_kernel(const int32_t* num, const int32_t* counts, int S, int max_num, int pos_num,
                                 int32_t* state) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  int npos = counts[2 * s], nneg = counts[2 * s + 1];
  int kp = npos < pos_num ? npos : pos_num;
  int slots = max_num - kp;
  int kn = nneg < slots ? nneg : slots;
  state[(2 * s) * TK_WORDS + TK_N] = num[s];
  state[(2 * s) * TK_WORDS + TK_K] = kp;
  state[(2 * s + 1) * TK_WORDS + TK_N] = num[s];
  state[(2 * s + 1) * TK_WORDS + TK_K] = kn;
}

__global__ void sampler_apply_topk_kernel(const int64_t* lab_in, int64_t lstride, const int32_t* state,
                                          const int32_t* sel, int64_t sel_ld, int64_t* lab_out) {
  const int v = blockIdx.y, s = v >> 1;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= state[v * TK_WORDS + TK_K]) return;
  int64_t box = sel[(int64_t)v * sel_ld + j];
  lab_out[(int64_t)s * lstride + box] = lab_in[(int64_t)s * lstride + box];
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

}  // namespace frh

using namespace frh;

static size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

struct SampLayout {
  size_t keys, hist, state, counts, cand, sel, total;
};

static SampLayout samp_layout(int32_t S, int64_t max_boxes) {
  SampLayout z{};
  const size_t n = (size_t)(max_boxes > 0 ? max_boxes : 1);
  const int V = 2 * S;
  z.keys = 0;
  z.hist = z.keys + al256((size_t)V * n * sizeof(uint32_t));
  z.state = z.hist + al256(tk_hist_bytes(V));
  z.counts = z.state + al256(tk_state_bytes(V));
  z.cand = z.counts + al256((size_t)V * sizeof(int32_t));
  z.sel = z.cand + al256(tk_cand_bytes(V));
  z.total = z.sel + al256((size_t)V * n * sizeof(int32_t));
  return z;
}

extern "C" size_t frh_sample_workspace(int32_t num_segs, int64_t max_boxes) {
  size_t a = al256(compact_workspace(num_segs, max_boxes));
  size_t b = samp_layout(num_segs, max_boxes).total;
  return a > b ? a : b;
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
                                     int32_t pos_num, uint64_t seed, int64_t* labels_out,
                                     void* workspace, size_t ws_bytes, void* stream) {
  FRH_REQUIRE(num_segs >= 0 && max_boxes >= 0, "negative sizes");
  FRH_REQUIRE(pos_num <= max_num && pos_num >= 0, "pos_num must be in [0, max_num]");
  if (num_segs == 0 || max_boxes == 0) return FRH_OK;
  FRH_REQUIRE(labels_in && labels_out && num_boxes, "null pointer argument");
  FRH_REQUIRE(labels_in != labels_out, "labels_out must not alias labels_in");
  FRH_REQUIRE(workspace && ws_bytes >= frh_sample_workspace(num_segs, max_boxes), "workspace too small");
  hipStream_t st = as_stream(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  SampLayout z = samp_layout(num_segs, max_boxes);
  const int V = 2 * num_segs;
  uint32_t* keys = reinterpret_cast<uint32_t*>(ws + z.keys);
  int32_t* state = reinterpret_cast<int32_t*>(ws + z.state);
  int32_t* counts = reinterpret_cast<int32_t*>(ws + z.counts);
  int32_t* sel = reinterpret_cast<int32_t*>(ws + z.sel);
  FRH_HIP(hipMemsetAsync(ws + z.hist, 0, z.cand - z.hist, st));  // hist + state + counts
  dim3 g1((unsigned)((max_boxes + 255) / 256), (unsigned)num_segs);
  hipLaunchKernelGGL(sampler_keys_kernel, g1, dim3(256), 0, st, labels_in, label_seg_stride, num_boxes, seed, keys,
                     max_boxes, counts, labels_out);
  hipLaunchKernelGGL(sampler_k_kernel, dim3((unsigned)((num_segs + 63) / 64)), dim3(64), 0, st, num_boxes, counts,
                     num_segs, max_num, pos_num, state);
  TopkBuffers tb{keys, max_boxes, reinterpret_cast<uint32_t*>(ws + z.hist), state, sel, max_boxes,
                 reinterpret_cast<int32_t*>(ws + z.cand), V};
  tk_launch(tb, max_boxes, st);
  dim3 g2((unsigned)((max_num + 255) / 256), (unsigned)V);
  hipLaunchKernelGGL(sampler_apply_topk_kernel, g2, dim3(256), 0, st, labels_in, label_seg_stride, state, sel,
                     (int64_t)max_boxes, labels_out);
  return check_launch("frh_sample_random");
}
