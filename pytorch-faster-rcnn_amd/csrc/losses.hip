// Fused detection losses: classification (sigmoid focal,
// sigmoid BCE, softmax cross-entropy) and masked / class-selected smooth-L1,
// forward sums and backward gradients, straight from the head outputs.
//
// Reference: lib/losses.py:33-61 (sigmoid_focal_loss), :77-83
// (smooth_l1_loss_v2), :126-156 (CrossEntropyLoss), and their callers
// AnchorHead.calc_loss (lib/heads/anchor_head.py:113-139) and
// BBoxHead.calc_loss (lib/heads/bbox_head.py:56-87).  The reference builds a
// one-hot target, a sigmoid, pt, a focal weight, BCE-with-logits and a sum as
// separate tensors (about a dozen elementwise passes over [n, C] forward and
// as many backward), gathers the labelled class's deltas with an advanced
// index and masks negatives by boolean indexing (a host sync).  Here each loss
// is one streaming pass: the element (i, k) of the logits is read through
// explicit strides (so the channel-major [C, S] views the target gathers
// produce need no copy), the one-hot target is the comparison label[i] == k+1,
// and the per-block partial sums are finalised in a fixed order by the last
// workgroup (deterministic; no float atomics).  Backward recomputes the
// element's derivative and writes g * dL/dx, reading the upstream gradient
// from device memory (no host sync).
//
// The forward's finalisation rides in the same launch: every workgroup stores
// its partial write-through (agent-scope relaxed store), drains, and adds to an
// arrival counter; the workgroup whose add returns nb - 1 sums the nb partials
// (agent-scope loads) in the fixed order of the former separate finalise
// launch and resets the counter (MI355X_MICROARCH.md hand-off table, row 1:
// one signalling lane per workgroup, one unsharded counter, last adder told by
// its add's return value; grids capped at 256 workgroups).
//
// Bytes per element: forward 4 (logit) + 8/C (label); backward 4 + 4 + 8/C.
// Numerics follow torch's formulas (binary_cross_entropy_with_logits via
// log_sigmoid, pow backward, log_softmax backward); sums differ from torch's
// reduction order in the last bits, gradients agree to a few ulp.
#include "common.h"

#include <math.h>

#include <algorithm>

namespace frh {
namespace {

constexpr int kLossThreads = 256;
constexpr int kMaxPartials = 256;   // forward grid cap = partial slots
constexpr int kCounterBytes = 256;  // arrival counter block at the workspace start

enum ClsKind { kFocal = 0, kSigmoidBce = 1, kSoftmaxCe = 2 };

struct ClsArgs {
  const float* x;
  int64_t n, c, sr, sc;  // logit (i, k) at x[i*sr + k*sc]
  const void* target;    // int64 labels [n] (or float32 [n] for kSigmoidBce, C == 1)
  int32_t tfloat;
  float alpha, gamma;
  int32_t i_fast;        // element order: i fastest (channel-major views) or k fastest
};

__device__ __forceinline__ float target_at(const ClsArgs& a, int64_t i) {
  return a.tfloat ? static_cast<const float*>(a.target)[i]
                  : static_cast<float>(static_cast<const int64_t*>(a.target)[i]);
}

__device__ __forceinline__ int64_t label_at(const ClsArgs& a, int64_t i) {
  return static_cast<const int64_t*>(a.target)[i];
}

// rows labelled < 0 are padding rows of a fixed-capacity target buffer (frh_anchor_target /
// frh_bbox_target past their device count): they contribute nothing, forward or backward
// (the reference's sampled targets never carry such labels)
__device__ __forceinline__ bool ignored(const ClsArgs& a, int64_t i) { return !a.tfloat && label_at(a, i) < 0; }

// torch: binary_cross_entropy_with_logits = (1 - t) * x - log_sigmoid(x),
// log_sigmoid(x) = min(x, 0) - log1p(exp(-|x|)).
__device__ __forceinline__ float bce_logits(float x, float t) {
  float ls = fminf(x, 0.0f) - log1pf(expf(-fabsf(x)));
  return (1.0f - t) * x - ls;
}

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

// sigmoid_focal_loss element (losses.py:48-61) and its derivative.
__device__ __forceinline__ float focal_elem(float x, float t, float alpha, float gamma, float* dx) {
  float p = sigmoidf(x);
  float pt = p * t + (1.0f - p) * (1.0f - t);
  float at = alpha * t + (1.0f - alpha) * (1.0f - t);
  float q = 1.0f - pt;
  float qg = powf(q, gamma);
  float w = at * qg;
  float bce = bce_logits(x, t);
  if (dx) {
    // d/dx [bce * at * q^gamma] = (p - t) * w + bce * at * gamma * q^(gamma-1) * (-dpt/dx),
    // dpt/dx = p (1 - p) (2t - 1)
    float dq = gamma * powf(q, gamma - 1.0f);
    float dpt = p * (1.0f - p) * (2.0f * t - 1.0f);
    *dx = (p - t) * w - bce * at * dq * dpt;
  }
  return bce * w;
}

__device__ __forceinline__ void elem_index(const ClsArgs& a, int64_t e, int64_t* i, int64_t* k) {
  if (a.i_fast) {
    *k = e / a.n;
    *i = e - *k * a.n;
  } else {
    *i = e / a.c;
    *k = e - *i * a.c;
  }
}

// target of element (i, k): C == 1 sigmoid takes the label value itself
// (label.view(-1, 1).float(), losses.py:142), otherwise one-hot[:, 1:].
__device__ __forceinline__ float elem_target(const ClsArgs& a, int64_t i, int64_t k) {
  if (a.c == 1) return target_at(a, i);
  return label_at(a, i) == k + 1 ? 1.0f : 0.0f;
}

__device__ __forceinline__ float block_sum_f(float v, float* scratch) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) scratch[w] = v;
  __syncthreads();
  float t = 0.0f;
  if (threadIdx.x == 0)
    for (int j = 0; j < kLossThreads / kWave; ++j) t += scratch[j];
  return t;
}

struct FanIn {
  uint32_t* counter;      // zero between calls
  float* partial;         // [gridDim.x]
  float* out;
  const int32_t* status;  // nullable: the caller's device status word; nonzero -> NaN loss
};

// A nonzero device status word (an in-launch wait of an earlier one-launch kernel ran out,
// include/frcnn_amd.h FRH_DEVERR_*) makes the loss NaN: the outputs it was computed from are
// undefined, and the step's own loss read carries the failure without an extra host sync.
__device__ __forceinline__ bool status_set(const int32_t* status) {
  return status && __hip_atomic_load(const_cast<int32_t*>(status), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// Thread 0 holds the workgroup's partial sum.  The last workgroup to arrive sums
// all partials in a fixed order (double accumulation: one slot per thread, then
// a tree) and writes the loss.
__device__ void fan_in_finalize(float block_total, const FanIn& f) {
  __shared__ double s[kLossThreads];
  __shared__ int last;
  if (threadIdx.x == 0) {
    __hip_atomic_store(f.partial + blockIdx.x, block_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(f.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  double v = 0.0;
  for (int j = threadIdx.x; j < (int)gridDim.x; j += kLossThreads)
    v += (double)__hip_atomic_load(f.partial + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  s[threadIdx.x] = v;
  __syncthreads();
  for (int o = kLossThreads / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    f.out[0] = status_set(f.status) ? NAN : (float)s[0];
    __hip_atomic_store(f.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int kKind>
__global__ void __launch_bounds__(kLossThreads) cls_loss_fwd_kernel(ClsArgs a, FanIn f) {
  __shared__ float scratch[kLossThreads / kWave];
  float acc = 0.0f;
  if constexpr (kKind == kSoftmaxCe) {
    for (int64_t i = blockIdx.x * (int64_t)kLossThreads + threadIdx.x; i < a.n;
         i += (int64_t)gridDim.x * kLossThreads) {
      if (ignored(a, i)) continue;
      const float* row = a.x + i * a.sr;
      float m = -INFINITY;
      for (int64_t k = 0; k < a.c; ++k) m = fmaxf(m, row[k * a.sc]);
      float s = 0.0f;
      for (int64_t k = 0; k < a.c; ++k) s += expf(row[k * a.sc] - m);
      int64_t l = label_at(a, i);
      float xl = (l >= 0 && l < a.c) ? row[l * a.sc] : NAN;
      acc += (logf(s) + m) - xl;  // -log_softmax(x)[label]
    }
  } else {
    const int64_t total = a.n * a.c;
    for (int64_t e = blockIdx.x * (int64_t)kLossThreads + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * kLossThreads) {
      int64_t i, k;
      elem_index(a, e, &i, &k);
      if (ignored(a, i)) continue;
      float x = a.x[i * a.sr + k * a.sc];
      float t = elem_target(a, i, k);
      acc += kKind == kFocal ? focal_elem(x, t, a.alpha, a.gamma, nullptr) : bce_logits(x, t);
    }
  }
  fan_in_finalize(block_sum_f(acc, scratch), f);
}

template <int kKind>
__global__ void __launch_bounds__(kLossThreads) cls_loss_bwd_kernel(ClsArgs a, const float* gout, float* gx,
                                                                     int64_t gsr, int64_t gsc) {
  const float g = *gout;
  if constexpr (kKind == kSoftmaxCe) {
    for (int64_t i = blockIdx.x * (int64_t)kLossThreads + threadIdx.x; i < a.n;
         i += (int64_t)gridDim.x * kLossThreads) {
      if (ignored(a, i)) {
        for (int64_t k = 0; k < a.c; ++k) gx[i * gsr + k * gsc] = 0.0f;
        continue;
      }
      const float* row = a.x + i * a.sr;
      float m = -INFINITY;
      for (int64_t k = 0; k < a.c; ++k) m = fmaxf(m, row[k * a.sc]);
      float s = 0.0f;
      for (int64_t k = 0; k < a.c; ++k) s += expf(row[k * a.sc] - m);
      float ls = logf(s);
      int64_t l = label_at(a, i);
      // log_softmax backward: g_k - exp(logp_k) * sum(g), with g = -g at the label
      for (int64_t k = 0; k < a.c; ++k) {
        float sm = expf((row[k * a.sc] - m) - ls);
        gx[i * gsr + k * gsc] = (k == l ? -g : 0.0f) + sm * g;
      }
    }
  } else {
    const int64_t total = a.n * a.c;
    for (int64_t e = blockIdx.x * (int64_t)kLossThreads + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * kLossThreads) {
      int64_t i, k;
      elem_index(a, e, &i, &k);
      if (ignored(a, i)) {
        gx[i * gsr + k * gsc] = 0.0f;
        continue;
      }
      float x = a.x[i * a.sr + k * a.sc];
      float t = elem_target(a, i, k);
      float d;
      if (kKind == kFocal)
        focal_elem(x, t, a.alpha, a.gamma, &d);
      else
        d = sigmoidf(x) - t;
      gx[i * gsr + k * gsc] = g * d;
    }
  }
}

struct L1Args {
  const float* x;
  int64_t xs_i, xs_j, xs_l;  // x(i, j) at x[i*xs_i + j*xs_j + label[i]*xs_l]
  const float* y;
  int64_t ys_i, ys_j;
  const int64_t* label;      // optional: rows with label <= 0 contribute nothing
  int64_t n, m, n_sel;       // rows, columns per row, selectable classes (label < n_sel)
  float beta;
};

// smooth_l1_loss_v2 element (losses.py:77-83): d < beta ? d^2 / (2 beta) : d - beta / 2
__device__ __forceinline__ bool l1_row(const L1Args& a, int64_t i, int64_t* off) {
  int64_t l = a.label ? a.label[i] : 0;
  if (a.label && l <= 0) return false;
  *off = i * a.xs_i + (a.xs_l ? l * a.xs_l : 0);
  return true;
}

__global__ void __launch_bounds__(kLossThreads) smooth_l1_fwd_kernel(L1Args a, FanIn f) {
  __shared__ float scratch[kLossThreads / kWave];
  float acc = 0.0f;
  const int64_t total = a.n * a.m;
  for (int64_t e = blockIdx.x * (int64_t)kLossThreads + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * kLossThreads) {
    int64_t i = e / a.m, j = e - i * a.m, off;
    if (!l1_row(a, i, &off)) continue;
    if (a.xs_l && (a.label[i] >= a.n_sel)) {
      acc += NAN;
      continue;
    }
    float d = fabsf(a.x[off + j * a.xs_j] - a.y[i * a.ys_i + j * a.ys_j]);
    acc += d < a.beta ? (d * d) / (2.0f * a.beta) : d - 0.5f * a.beta;
  }
  fan_in_finalize(block_sum_f(acc, scratch), f);
}

// gx must be zero-filled by the caller: only the selected, unmasked elements are written.
__global__ void __launch_bounds__(kLossThreads) smooth_l1_bwd_kernel(L1Args a, const float* gout, float* gx,
                                                                     int64_t gs_i, int64_t gs_j, int64_t gs_l) {
  const float g = *gout;
  const int64_t total = a.n * a.m;
  for (int64_t e = blockIdx.x * (int64_t)kLossThreads + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * kLossThreads) {
    int64_t i = e / a.m, j = e - i * a.m, off;
    if (!l1_row(a, i, &off)) continue;
    int64_t l = a.xs_l ? a.label[i] : 0;
    if (l >= a.n_sel) continue;
    float diff = a.x[off + j * a.xs_j] - a.y[i * a.ys_i + j * a.ys_j];
    float d = fabsf(diff);
    float sgn = diff > 0.0f ? 1.0f : (diff < 0.0f ? -1.0f : 0.0f);
    float dd = d < a.beta ? (2.0f * d) / (2.0f * a.beta) : 1.0f;
    gx[i * gs_i + j * gs_j + l * gs_l] = g * dd * sgn;
  }
}

// Classification + regression loss of one head in ONE launch (AnchorHead / BBoxHead
// calc_loss with a sampler: anchor_head.py:113-139, bbox_head.py:56-87).  Workgroup b
// takes the cls elements of workgroup b of cls_loss_fwd_kernel's grid (b < nbc) and the
// smooth-L1 elements of workgroup b of smooth_l1_fwd_kernel's grid (b < nbr); the last
// workgroup to arrive sums each loss's partials in the fixed order of fan_in_finalize,
// so both sums equal the separate launches' bit for bit, and applies the heads' scaling
// as torch does it: loss = (sum * loss_weight) / avg_factor in f32.
struct DetScale {
  float wc, dc, wr, dr;
  float* out;             // [2]: cls, reg
  const int32_t* ndev;    // nullable: avg_factor = this device count for both (0 -> zero losses)
  const int32_t* status;  // nullable: device status word; nonzero -> NaN losses
};

__device__ void det_fan_in(float pc, float pr, uint32_t* counter, float* partial, int nbc, int nbr,
                           const DetScale& o) {
  __shared__ double s[kLossThreads];
  __shared__ int last;
  if (threadIdx.x == 0) {
    __hip_atomic_store(partial + blockIdx.x, pc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(partial + kMaxPartials + blockIdx.x, pr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  float res[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int nb = q ? nbr : nbc;
    const float* p = partial + q * kMaxPartials;
    double v = 0.0;
    for (int j = threadIdx.x; j < nb; j += kLossThreads)
      v += (double)__hip_atomic_load(const_cast<float*>(p + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s[threadIdx.x] = v;
    __syncthreads();
    for (int w = kLossThreads / 2; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
      __syncthreads();
    }
    res[q] = (float)s[0];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (o.ndev) {
      const int32_t nd = *o.ndev;
      const float d = (float)nd;
      o.out[0] = nd ? (res[0] * o.wc) / d : 0.0f;
      o.out[1] = nd ? (res[1] * o.wr) / d : 0.0f;
    } else {
      o.out[0] = (res[0] * o.wc) / o.dc;
      o.out[1] = (res[1] * o.wr) / o.dr;
    }
    if (status_set(o.status)) o.out[0] = o.out[1] = NAN;
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int kKind>
__global__ void __launch_bounds__(kLossThreads) det_loss_fwd_kernel(ClsArgs a, int nbc, L1Args r, int nbr,
                                                                    uint32_t* counter, float* partial, DetScale o) {
  __shared__ float scratch[kLossThreads / kWave];
  float acc = 0.0f;
  if ((int)blockIdx.x < nbc) {
    if constexpr (kKind == kSoftmaxCe) {
      for (int64_t i = blockIdx.x * (int64_t)kLossThreads + threadIdx.x; i < a.n; i += (int64_t)nbc * kLossThreads) {
        if (ignored(a, i)) continue;
        const float* row = a.x + i * a.sr;
        float m = -INFINITY;
        for (int64_t k = 0; k < a.c; ++k) m = fmaxf(m, row[k * a.sc]);
        float sm = 0.0f;
        for (int64_t k = 0; k < a.c; ++k) sm += expf(row[k * a.sc] - m);
        int64_t l = label_at(a, i);
        float xl = (l >= 0 && l < a.c) ? row[l * a.sc] : NAN;
        acc += (logf(sm) + m) - xl;
      }
    } else {
      const int64_t total = a.n * a.c;
      for (int64_t e = blockIdx.x * (int64_t)kLossThreads + threadIdx.x; e < total;
           e += (int64_t)nbc * kLossThreads) {
        int64_t i, k;
        elem_index(a, e, &i, &k);
        if (ignored(a, i)) continue;
        float x = a.x[i * a.sr + k * a.sc];
        float t = elem_target(a, i, k);
        acc += kKind == kFocal ? focal_elem(x, t, a.alpha, a.gamma, nullptr) : bce_logits(x, t);
      }
    }
  }
  float accr = 0.0f;
  if ((int)blockIdx.x < nbr) {
    const int64_t total = r.n * r.m;
    for (int64_t e = blockIdx.x * (int64_t)kLossThreads + threadIdx.x; e < total; e += (int64_t)nbr * kLossThreads) {
      int64_t i = e / r.m, j = e - i * r.m, off;
      if (!l1_row(r, i, &off)) continue;
      if (r.xs_l && (r.label[i] >= r.n_sel)) {
        accr += NAN;
        continue;
      }
      float d = fabsf(r.x[off + j * r.xs_j] - r.y[i * r.ys_i + j * r.ys_j]);
      accr += d < r.beta ? (d * d) / (2.0f * r.beta) : d - 0.5f * r.beta;
    }
  }
  const float pc = block_sum_f(acc, scratch);
  __syncthreads();
  const float pr = block_sum_f(accr, scratch);
  det_fan_in(pc, pr, counter, partial, nbc, nbr, o);
}


int grid_for(int64_t work) {
  int64_t b = (work + kLossThreads - 1) / kLossThreads;
  if (b < 1) b = 1;
  return (int)(b < kMaxPartials ? b : kMaxPartials);
}

int32_t check_cls(int32_t kind, const ClsArgs& a) {
  FRH_REQUIRE(kind >= kFocal && kind <= kSoftmaxCe, "cls loss: unknown kind %d", kind);
  FRH_REQUIRE(a.n >= 0 && a.c >= 1, "cls loss: bad shape [%lld, %lld]", (long long)a.n, (long long)a.c);
  FRH_REQUIRE(a.n * a.c < (int64_t(1) << 40), "cls loss: too many elements");
  FRH_REQUIRE(a.n == 0 || (a.x && a.target), "cls loss: null input");
  FRH_REQUIRE(!a.tfloat || (kind == kSigmoidBce && a.c == 1),
              "cls loss: float targets only for single-channel sigmoid BCE");
  return FRH_OK;
}

ClsArgs make_cls(const float* x, int64_t n, int64_t c, int64_t sr, int64_t sc, const void* target,
                 int32_t tfloat, float alpha, float gamma) {
  ClsArgs a;
  a.x = x;
  a.n = n;
  a.c = c;
  a.sr = sr;
  a.sc = sc;
  a.target = target;
  a.tfloat = tfloat;
  a.alpha = alpha;
  a.gamma = gamma;
  a.i_fast = (sr < sc) ? 1 : 0;
  return a;
}

int32_t check_l1(const L1Args& a) {
  FRH_REQUIRE(a.n >= 0 && a.m >= 1, "smooth l1: bad shape");
  FRH_REQUIRE(a.beta > 0.0f, "smooth l1: beta must be > 0");
  FRH_REQUIRE(a.n == 0 || (a.x && a.y), "smooth l1: null input");
  FRH_REQUIRE(a.xs_l == 0 || a.label, "smooth l1: class selection needs labels");
  FRH_REQUIRE(a.n_sel >= 1, "smooth l1: n_sel must be >= 1");
  return FRH_OK;
}

L1Args make_l1(const float* x, int64_t xs_i, int64_t xs_j, int64_t xs_l, const float* y, int64_t ys_i,
               int64_t ys_j, const int64_t* label, int64_t n, int64_t m, int64_t n_sel, float beta) {
  L1Args a;
  a.x = x;
  a.xs_i = xs_i;
  a.xs_j = xs_j;
  a.xs_l = xs_l;
  a.y = y;
  a.ys_i = ys_i;
  a.ys_j = ys_j;
  a.label = label;
  a.n = n;
  a.m = m;
  a.n_sel = n_sel;
  a.beta = beta;
  return a;
}

}  // namespace
}  // namespace frh

using namespace frh;

extern "C" {

size_t frh_loss_workspace(void) { return kCounterBytes + 2 * kMaxPartials * sizeof(float); }

static FanIn fan_in(void* workspace, float* out, const int32_t* status) {
  char* w = static_cast<char*>(workspace);
  return FanIn{reinterpret_cast<uint32_t*>(w), reinterpret_cast<float*>(w + kCounterBytes), out, status};
}

int32_t frh_cls_loss_fwd(int32_t kind, const float* x, int64_t n, int64_t c, int64_t sr, int64_t sc,
                         const void* target, int32_t target_is_float, float alpha, float gamma,
                         const int32_t* status, float* out, void* workspace, size_t ws_bytes, void* stream) {
  ClsArgs a = make_cls(x, n, c, sr, sc, target, target_is_float, alpha, gamma);
  int32_t st = check_cls(kind, a);
  if (st != FRH_OK) return st;
  FRH_REQUIRE(out, "cls loss: null output");
  FRH_REQUIRE(workspace && ws_bytes >= frh_loss_workspace(), "cls loss: workspace too small");
  const FanIn f = fan_in(workspace, out, status);
  int nb = grid_for(kind == kSoftmaxCe ? n : n * c);
  hipStream_t s = as_stream(stream);
  if (kind == kFocal)
    hipLaunchKernelGGL(cls_loss_fwd_kernel<kFocal>, dim3(nb), dim3(kLossThreads), 0, s, a, f);
  else if (kind == kSigmoidBce)
    hipLaunchKernelGGL(cls_loss_fwd_kernel<kSigmoidBce>, dim3(nb), dim3(kLossThreads), 0, s, a, f);
  else
    hipLaunchKernelGGL(cls_loss_fwd_kernel<kSoftmaxCe>, dim3(nb), dim3(kLossThreads), 0, s, a, f);
  return check_launch("frh_cls_loss_fwd");
}

int32_t frh_cls_loss_bwd(int32_t kind, const float* x, int64_t n, int64_t c, int64_t sr, int64_t sc,
                         const void* target, int32_t target_is_float, float alpha, float gamma,
                         const float* grad_out, float* grad_x, int64_t gsr, int64_t gsc, void* stream) {
  ClsArgs a = make_cls(x, n, c, sr, sc, target, target_is_float, alpha, gamma);
  int32_t st = check_cls(kind, a);
  if (st != FRH_OK) return st;
  FRH_REQUIRE(grad_out && (n == 0 || grad_x), "cls loss bwd: null gradient");
  if (n == 0) return FRH_OK;
  int nb = grid_for(kind == kSoftmaxCe ? n : n * c);
  hipStream_t s = as_stream(stream);
  if (kind == kFocal)
    hipLaunchKernelGGL(cls_loss_bwd_kernel<kFocal>, dim3(nb), dim3(kLossThreads), 0, s, a, grad_out, grad_x, gsr, gsc);
  else if (kind == kSigmoidBce)
    hipLaunchKernelGGL(cls_loss_bwd_kernel<kSigmoidBce>, dim3(nb), dim3(kLossThreads), 0, s, a, grad_out, grad_x, gsr,
                       gsc);
  else
    hipLaunchKernelGGL(cls_loss_bwd_kernel<kSoftmaxCe>, dim3(nb), dim3(kLossThreads), 0, s, a, grad_out, grad_x, gsr,
                       gsc);
  return check_launch("frh_cls_loss_bwd");
}

int32_t frh_smooth_l1_fwd(const float* x, int64_t xs_i, int64_t xs_j, int64_t xs_l, const float* y, int64_t ys_i,
                          int64_t ys_j, const int64_t* label, int64_t n, int64_t m, int64_t n_sel, float beta,
                          const int32_t* status, float* out, void* workspace, size_t ws_bytes, void* stream) {
  L1Args a = make_l1(x, xs_i, xs_j, xs_l, y, ys_i, ys_j, label, n, m, n_sel, beta);
  int32_t st = check_l1(a);
  if (st != FRH_OK) return st;
  FRH_REQUIRE(out, "smooth l1: null output");
  FRH_REQUIRE(workspace && ws_bytes >= frh_loss_workspace(), "smooth l1: workspace too small");
  int nb = grid_for(n * m);
  hipLaunchKernelGGL(smooth_l1_fwd_kernel, dim3(nb), dim3(kLossThreads), 0, as_stream(stream), a,
                     fan_in(workspace, out, status));
  return check_launch("frh_smooth_l1_fwd");
}

int32_t frh_det_loss_fwd(int32_t kind, const float* x, int64_t n, int64_t c, int64_t sr, int64_t sc,
                         const void* target, int32_t target_is_float, float alpha, float gamma, float cls_weight,
                         float cls_div, const float* rx, int64_t xs_i, int64_t xs_j, int64_t xs_l, const float* ry,
                         int64_t ys_i, int64_t ys_j, const int64_t* label, int64_t rn, int64_t rm, int64_t n_sel,
                         float beta, float reg_weight, float reg_div, const int32_t* div_count,
                         const int32_t* status, float* out, void* workspace, size_t ws_bytes, void* stream) {
  ClsArgs a = make_cls(x, n, c, sr, sc, target, target_is_float, alpha, gamma);
  int32_t st = check_cls(kind, a);
  if (st != FRH_OK) return st;
  L1Args r = make_l1(rx, xs_i, xs_j, xs_l, ry, ys_i, ys_j, label, rn, rm, n_sel, beta);
  st = check_l1(r);
  if (st != FRH_OK) return st;
  FRH_REQUIRE(out, "det loss: null output");
  FRH_REQUIRE(workspace && ws_bytes >= frh_loss_workspace(), "det loss: workspace too small");
  const int nbc = grid_for(kind == kSoftmaxCe ? n : n * c), nbr = grid_for(rn * rm);
  char* w = static_cast<char*>(workspace);
  uint32_t* counter = reinterpret_cast<uint32_t*>(w);
  float* partial = reinterpret_cast<float*>(w + kCounterBytes);
  const DetScale o{cls_weight, cls_div, reg_weight, reg_div, out, div_count, status};
  const dim3 g((unsigned)std::max(nbc, nbr));
  hipStream_t s = as_stream(stream);
  if (kind == kFocal)
    hipLaunchKernelGGL(det_loss_fwd_kernel<kFocal>, g, dim3(kLossThreads), 0, s, a, nbc, r, nbr, counter, partial, o);
  else if (kind == kSigmoidBce)
    hipLaunchKernelGGL(det_loss_fwd_kernel<kSigmoidBce>, g, dim3(kLossThreads), 0, s, a, nbc, r, nbr, counter, partial,
                       o);
  else
    hipLaunchKernelGGL(det_loss_fwd_kernel<kSoftmaxCe>, g, dim3(kLossThreads), 0, s, a, nbc, r, nbr, counter, partial,
                       o);
  return check_launch("frh_det_loss_fwd");
}

int32_t frh_smooth_l1_bwd(const float* x, int64_t xs_i, int64_t xs_j, int64_t xs_l, const float* y, int64_t ys_i,
                          int64_t ys_j, const int64_t* label, int64_t n, int64_t m, int64_t n_sel, float beta,
                          const float* grad_out, float* grad_x, int64_t gs_i, int64_t gs_j, int64_t gs_l,
                          void* stream) {
  L1Args a = make_l1(x, xs_i, xs_j, xs_l, y, ys_i, ys_j, label, n, m, n_sel, beta);
  int32_t st = check_l1(a);
  if (st != FRH_OK) return st;
  FRH_REQUIRE(grad_out && (n == 0 || grad_x), "smooth l1 bwd: null gradient");
  if (n == 0) return FRH_OK;
  hipLaunchKernelGGL(smooth_l1_bwd_kernel, dim3(grid_for(n * m)), dim3(kLossThreads), 0, as_stream(stream), a,
                     grad_out, grad_x, gs_i, gs_j, gs_l);
  return check_launch("frh_smooth_l1_bwd");
}

}  // extern "C"
