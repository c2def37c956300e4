// a5: RandomSampler (lib/region.py:43-57,112-126) and the ordered segmented
// compaction it and the target gathers are built on.
//
// Ordered compaction = two launches: per-chunk predicate counts, then each
// chunk block adds the counts of its preceding chunks and ranks its own
// elements with wave ballots (coalesced: round r of a chunk reads elements
// base + r*256 + tid).
#include "block_ops.h"

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

// device-RNG sampler: one 1024-thread block per (segment, pos|neg)
constexpr int kSelThreads = 1024;
__global__ void __launch_bounds__(kSelThreads)
    sample_random_kernel(const int64_t* lab_in, int64_t label_seg_stride, const int32_t* pos_list,
                         const int32_t* neg_list, int64_t list_seg_stride, const int32_t* counts,
                         int max_num, int pos_num, uint64_t seed, int32_t* sel_scratch,
                         int64_t* lab_out) {
  __shared__ TopkSmem sm;
  const int s = blockIdx.x;
  const int which = blockIdx.y;
  const int npos = counts[s * 2 + 0], nneg = counts[s * 2 + 1];
  const int kpos = npos < pos_num ? npos : pos_num;
  const int nslots = max_num - kpos;
  const int k = which == 0 ? kpos : (nneg < nslots ? nneg : nslots);
  const int n = which == 0 ? npos : nneg;
  const int32_t* list = (which == 0 ? pos_list : neg_list) + (int64_t)s * list_seg_stride;
  int32_t* sel = sel_scratch + ((int64_t)s * 2 + which) * list_seg_stride;
  const uint32_t salt = (uint32_t)(s * 2 + which);
  auto key_of = [&](int i) -> uint32_t { return ~hash_u32(seed, salt, (uint32_t)list[i]); };
  int m = block_topk_select(key_of, n, k, sel, sm);
  for (int j = threadIdx.x; j < m; j += blockDim.x) {
    int64_t box = list[sel[j]];
    lab_out[(int64_t)s * label_seg_stride + box] = lab_in[(int64_t)s * label_seg_stride + box];
  }
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

extern "C" size_t frh_sample_workspace(int32_t num_segs, int64_t max_boxes) {
  size_t a = compact_workspace(num_segs, max_boxes);
  a = (a + 255) & ~(size_t)255;
  size_t lists = (size_t)num_segs * 2 * (size_t)(max_boxes > 0 ? max_boxes : 1) * sizeof(int32_t);  // pos/neg
  size_t sel = lists;
  size_t cnt = (size_t)num_segs * 2 * sizeof(int32_t);
  return a + ((lists + 255) & ~(size_t)255) + ((sel + 255) & ~(size_t)255) + cnt;
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
  size_t a = (compact_workspace(num_segs, max_boxes) + 255) & ~(size_t)255;
  int32_t* chunk_counts = reinterpret_cast<int32_t*>(ws);
  int32_t* lists = reinterpret_cast<int32_t*>(ws + a);
  size_t lists_b = ((size_t)num_segs * 2 * max_boxes * sizeof(int32_t) + 255) & ~(size_t)255;
  int32_t* sel = reinterpret_cast<int32_t*>(ws + a + lists_b);
  int32_t* counts = reinterpret_cast<int32_t*>(ws + a + 2 * lists_b);
  int32_t* pos_list = lists;
  int32_t* neg_list = lists + (int64_t)num_segs * max_boxes;
  int preds[2] = {kPos, kNeg};
  int32_t* lp[2] = {pos_list, neg_list};
  int32_t r = launch_compact_lists(num_segs, labels_in, label_seg_stride, num_boxes, max_boxes, 2, preds, lp,
                                   max_boxes, counts, chunk_counts, st);
  if (r) return r;
  dim3 g1((unsigned)((max_boxes + 255) / 256), (unsigned)num_segs);
  hipLaunchKernelGGL(fill_i64_kernel, g1, dim3(256), 0, st, labels_out, label_seg_stride, num_boxes,
                     max_boxes, (int64_t)-1);
  hipLaunchKernelGGL(sample_random_kernel, dim3((unsigned)num_segs, 2), dim3(kSelThreads), 0, st, labels_in,
                     label_seg_stride, pos_list, neg_list, (int64_t)max_boxes, counts, max_num, pos_num, seed,
                     sel, labels_out);
  return check_launch("frh_sample_random");
}
