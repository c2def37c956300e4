/*
 * TEST INFRASTRUCTURE — CPU oracle for the frcnn_amd hot path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline.  The product
 * (pytorch-faster-rcnn_amd/) never links or calls it.
 *
 * Plain-C restatement of the reference's per-op arithmetic, scalar loops in
 * the reference's operation order (compile with -ffp-contract=off):
 *   calc_iou            lib/utils.py:151-172
 *   MaxIoUAssigner      lib/region.py:60-107
 *   AnchorCreator       lib/anchor.py:107-129
 *   inside masks        lib/region.py:10-29
 *   bbox2param          lib/utils.py:47-70
 *   param2bbox/clamp    lib/utils.py:83-144
 *   map_rois_to_levels  lib/region.py:256-264
 *   nms                 torchvision.ops.nms CPU kernel semantics (call sites
 *                       lib/heads/rpn_head.py:103, lib/utils.py:220)
 *   roi_align fwd/bwd   torchvision legacy RoIAlign (aligned=False) CPU
 *                       kernel semantics (lib/builder.py:9, lib/region.py:276)
 *   roi_pool            torchvision RoIPool semantics
 *   atss targets        lib/heads/fcos_head.py:51-116,283-368
 * torchvision is not vendored in the reference and not installed here: the
 * nms / roi_align / roi_pool rows are "parity unpinned" (SURVEY §8c).
 *
 * OpenMP (bench.py's host-core CPU baseline): the IoU table, the assignment,
 * the NMS suppression mask and RoIAlign run over the host's threads
 * (orc_set_threads); every output element is computed by one thread in the same
 * operation order, so results do not depend on the thread count.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* thread count of the parallel loops (1 = the scalar baseline); returns the previous */
int orc_set_threads(int n) {
#ifdef _OPENMP
  int prev = omp_get_max_threads();
  omp_set_num_threads(n > 0 ? n : 1);
  return prev;
#else
  (void)n;
  return 1;
#endif
}

/* Reusable scratch (the timed CPU baseline calls these functions repeatedly: a fresh
 * multi-MB malloc is an mmap whose pages are first-touched by every OpenMP thread at once,
 * serialising on the kernel's page-fault path -- the 16-thread assignment measured slower than
 * one thread).  Not reentrant: the oracle is called from one host thread. */
static void* scratch(int slot, size_t bytes) {
  static void* buf[4];
  static size_t cap[4];
  if (bytes > cap[slot]) {
    free(buf[slot]);
    buf[slot] = malloc(bytes);
    cap[slot] = buf[slot] ? bytes : 0;
  }
  return buf[slot];
}

static float iou_p1(const float* a, int64_t lda, int64_t i, const float* b, int64_t ldb, int64_t j) {
  float ax1 = a[i], ay1 = a[lda + i], ax2 = a[2 * lda + i], ay2 = a[3 * lda + i];
  float bx1 = b[j], by1 = b[ldb + j], bx2 = b[2 * ldb + j], by2 = b[3 * ldb + j];
  float tlx = ax1 > bx1 ? ax1 : bx1, tly = ay1 > by1 ? ay1 : by1;
  float brx = ax2 < bx2 ? ax2 : bx2, bry = ay2 < by2 ? ay2 : by2;
  float ai = ((brx - tlx) + 1.0f) * ((bry - tly) + 1.0f);
  ai = ai * ((tlx < brx && tly < bry) ? 1.0f : 0.0f);
  float aa = ((ax2 - ax1) + 1.0f) * ((ay2 - ay1) + 1.0f);
  float ab = ((bx2 - bx1) + 1.0f) * ((by2 - by1) + 1.0f);
  return ai / ((aa + ab) - ai);
}

/* calc_iou: out[n*k] row-major */
void orc_iou_table(const float* a, int64_t lda, int64_t n, const float* b, int64_t ldb, int64_t k, float* out) {
#pragma omp parallel for schedule(static) if (n * k > 65536)
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j < k; ++j) out[i * k + j] = iou_p1(a, lda, i, b, ldb, j);
}

/* torch.max(dim) semantics: first index of the max; NaN wins and stops */
static void row_max(const float* v, int64_t n, int64_t stride, float* m, int64_t* arg) {
  float mx = v[0];
  int64_t ai = 0;
  for (int64_t i = 0; i < n; ++i) {
    float x = v[i * stride];
    if (!(x <= mx)) {
      mx = x;
      ai = i;
      if (isnan(x)) break;
    }
  }
  *m = mx;
  *arg = ai;
}

/* MaxIoUAssigner.__call__ (region.py:75-107); labels int64, max_iou f32 */
int orc_maxiou_assign(const float* boxes, int64_t ld, int64_t n, const float* gts, int64_t gld, int64_t g,
                      float pos_iou, float neg_iou, float min_pos_iou, int64_t* labels, float* max_iou) {
  if (g <= 0) return -1;
  float* tab = (float*)scratch(0, sizeof(float) * (size_t)(n > 0 ? n : 1) * (size_t)g);
  float* colmax = (float*)malloc(sizeof(float) * (size_t)g);
  if (!tab || !colmax) return -2;
  orc_iou_table(boxes, ld, n, gts, gld, g, tab);
  /* per-gt max over the boxes (torch.max over dim 0: NaN wins): chunk maxima in
   * parallel, combined in chunk order with the same rule -- the same value */
  enum { kCh = 64 };
  float* part = (float*)malloc(sizeof(float) * (size_t)g * kCh);
  int64_t per = (n + kCh - 1) / kCh;
#pragma omp parallel for schedule(static) if (n > 65536)
  for (int q = 0; q < kCh; ++q) {
    int64_t lo = (int64_t)q * per, hi = lo + per < n ? lo + per : n;
    for (int64_t j = 0; j < g; ++j) {
      int64_t dummy;
      float m = NAN;
      if (hi > lo) row_max(tab + lo * g + j, hi - lo, g, &m, &dummy);
      part[(size_t)j * kCh + q] = hi > lo ? m : -INFINITY;
    }
  }
  for (int64_t j = 0; j < g; ++j) {
    float mx = part[(size_t)j * kCh];
    for (int q = 1; q < kCh && !isnan(mx); ++q) {
      float x = part[(size_t)j * kCh + q];
      if (!(x <= mx)) mx = x;
    }
    colmax[j] = mx;
  }
  free(part);
#pragma omp parallel for schedule(static) if (n > 65536)
  for (int64_t i = 0; i < n; ++i) {
    float m;
    int64_t arg;
    row_max(tab + i * g, g, 1, &m, &arg);
    int64_t lab = -1;
    if (m < neg_iou) lab = 0;
    if (m >= pos_iou) lab = 1;
    int64_t eq = -1;
    for (int64_t j = 0; j < g; ++j)
      if (tab[i * g + j] == colmax[j] && colmax[j] >= min_pos_iou) {
        eq = j;
        break;
      }
    if (eq >= 0) {
      arg = eq;
      lab = 1;
    }
    max_iou[i] = tab[i * g + arg];
    labels[i] = lab == 1 ? arg + 1 : lab;
  }
  free(colmax);
  return 0;
}

/* AnchorCreator.__call__ for one level: out [4, A*H*W] (row stride ld) */
void orc_anchor_grid(const float* ws, const float* hs, int a_n, int gh, int gw, float stride, int center_lt,
                     float* out, int64_t ld) {
  for (int a = 0; a < a_n; ++a)
    for (int y = 0; y < gh; ++y)
      for (int x = 0; x < gw; ++x) {
        int64_t i = ((int64_t)a * gh + y) * gw + x;
        float cx = (float)x * stride, cy = (float)y * stride;
        if (!center_lt) {
          cx = cx + stride / 2.0f;
          cy = cy + stride / 2.0f;
        }
        float hw = ws[a] / 2.0f, hh = hs[a] / 2.0f;
        out[i] = cx - hw;
        out[ld + i] = cy - hh;
        out[2 * ld + i] = cx + hw;
        out[3 * ld + i] = cy + hh;
      }
}

/* bbox2param + (p - mean) / std */
void orc_bbox2param(const float* base, int64_t ldb, const float* bbox, int64_t ldx, int64_t n, const float* means,
                    const float* stds, float* out, int64_t ldo) {
  for (int64_t i = 0; i < n; ++i) {
    float bx1 = base[i], by1 = base[ldb + i], bx2 = base[2 * ldb + i], by2 = base[3 * ldb + i];
    float gx1 = bbox[i], gy1 = bbox[ldx + i], gx2 = bbox[2 * ldx + i], gy2 = bbox[3 * ldx + i];
    float bw = (bx2 - bx1) + 1.0f, bh = (by2 - by1) + 1.0f;
    float gw = (gx2 - gx1) + 1.0f, gh = (gy2 - gy1) + 1.0f;
    float bcx = (bx2 + bx1) / 2.0f, bcy = (by2 + by1) / 2.0f;
    float gcx = (gx2 + gx1) / 2.0f, gcy = (gy2 + gy1) / 2.0f;
    float t[4] = {(gcx - bcx) / bw, (gcy - bcy) / bh, logf(gw / bw), logf(gh / bh)};
    for (int k = 0; k < 4; ++k) {
      float v = (t[k] - 0.0f) / 1.0f;
      out[k * ldo + i] = means ? (v - means[k]) / stds[k] : v;
    }
  }
}

static float clampf_t(float x, float lo, float hi) {
  float y = x < lo ? lo : x;
  return y > hi ? hi : y;
}

/* param2bbox over [4*ncls, n] coordinate-major classes, optional clamp */
void orc_param2bbox(const float* base, int64_t ldb, const float* param, int64_t ldp, int64_t n, int ncls,
                    const float* m, const float* sd, int clamp, float img_h, float img_w, float* out, int64_t ldo) {
  for (int c = 0; c < ncls; ++c)
    for (int64_t i = 0; i < n; ++i) {
      float ax1 = base[i], ay1 = base[ldb + i], ax2 = base[2 * ldb + i], ay2 = base[3 * ldb + i];
      float tx = param[(0 * ncls + c) * ldp + i] * sd[0] + m[0];
      float ty = param[(1 * ncls + c) * ldp + i] * sd[1] + m[1];
      float tw = param[(2 * ncls + c) * ldp + i] * sd[2] + m[2];
      float th = param[(3 * ncls + c) * ldp + i] * sd[3] + m[3];
      float bw = (ax2 - ax1) + 1.0f, bh = (ay2 - ay1) + 1.0f;
      float bcx = (ax2 + ax1) / 2.0f, bcy = (ay2 + ay1) / 2.0f;
      float cx = tx * bw + bcx, cy = ty * bh + bcy;
      float w = expf(tw) * bw, h = expf(th) * bh;
      float v[4] = {cx - w / 2.0f, cy - h / 2.0f, cx + w / 2.0f, cy + h / 2.0f};
      if (clamp) {
        v[0] = clampf_t(v[0], 0.0f, img_w - 1.0f);
        v[1] = clampf_t(v[1], 0.0f, img_h - 1.0f);
        v[2] = clampf_t(v[2], 0.0f, img_w - 1.0f);
        v[3] = clampf_t(v[3], 0.0f, img_h - 1.0f);
      }
      for (int k = 0; k < 4; ++k) out[(k * ncls + c) * ldo + i] = v[k];
    }
}

/* map_rois_to_levels on rois [K,5] */
void orc_roi_level_map(const float* rois, int64_t k, float finest, int L, int64_t* levels) {
  for (int64_t i = 0; i < k; ++i) {
    const float* r = rois + i * 5;
    float s = sqrtf(((r[3] - r[1]) + 1.0f) * ((r[4] - r[2]) + 1.0f));
    float v = s / finest + 1e-6f;
    float lg = (float)log2((double)v);
    float f = floorf(lg);
    if (f < 0.0f) f = 0.0f;
    if (f > (float)(L - 1)) f = (float)(L - 1);
    levels[i] = (int64_t)f;
  }
}

/* torchvision nms on boxes [n,4] already sorted by descending score;
 * keep = positions; returns count */
static int nms_above(const float* b, const float* area, int64_t i, int64_t j, double thr) {
  float xx1 = b[4 * i] > b[4 * j] ? b[4 * i] : b[4 * j];
  float yy1 = b[4 * i + 1] > b[4 * j + 1] ? b[4 * i + 1] : b[4 * j + 1];
  float xx2 = b[4 * i + 2] < b[4 * j + 2] ? b[4 * i + 2] : b[4 * j + 2];
  float yy2 = b[4 * i + 3] < b[4 * j + 3] ? b[4 * i + 3] : b[4 * j + 3];
  float w = xx2 - xx1, h = yy2 - yy1;
  w = w > 0.0f ? w : 0.0f;
  h = h > 0.0f ? h : 0.0f;
  float inter = w * h;
  float ovr = inter / ((area[i] + area[j]) - inter);
  return (double)ovr > thr;
}

/* torchvision nms on boxes [n,4] already sorted by descending score;
 * keep = positions; returns count.  Several threads: the upper-triangle
 * suppression bit mask in parallel (rows over threads), then the greedy scan
 * over it -- the same keep list as the sequential loop below. */
int64_t orc_nms_sorted(const float* b, int64_t n, double thr, int64_t max_keep, int64_t* keep) {
  float* area = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
  for (int64_t i = 0; i < n; ++i) area[i] = (b[4 * i + 2] - b[4 * i]) * (b[4 * i + 3] - b[4 * i + 1]);
  int64_t nk = 0;
  int threads = 1;
#ifdef _OPENMP
  threads = omp_get_max_threads();
#endif
  if (threads > 1 && n >= 512) {
    const int64_t nw = (n + 63) / 64;
    uint64_t* mask = (uint64_t*)scratch(1, (size_t)n * (size_t)nw * sizeof(uint64_t));
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < n; ++i) {
      for (int64_t w = 0; w < nw; ++w) mask[i * nw + w] = 0;
      for (int64_t j = i + 1; j < n; ++j)
        if (nms_above(b, area, i, j, thr)) mask[i * nw + j / 64] |= 1ull << (j % 64);
    }
    uint64_t* removed = (uint64_t*)calloc((size_t)nw, sizeof(uint64_t));
    for (int64_t i = 0; i < n; ++i) {
      if (removed[i / 64] >> (i % 64) & 1ull) continue;
      if (max_keep >= 0 && nk >= max_keep) break;
      keep[nk++] = i;
      for (int64_t w = i / 64; w < nw; ++w) removed[w] |= mask[i * nw + w];
    }
    free(removed);
    free(area);
    return nk;
  }
  unsigned char* sup = (unsigned char*)calloc((size_t)(n > 0 ? n : 1), 1);
  for (int64_t i = 0; i < n; ++i) {
    if (sup[i]) continue;
    if (max_keep >= 0 && nk >= max_keep) break;
    keep[nk++] = i;
    for (int64_t j = i + 1; j < n; ++j)
      if (!sup[j] && nms_above(b, area, i, j, thr)) sup[j] = 1;
  }
  free(sup);
  free(area);
  return nk;
}

typedef struct {
  int lo, hi, valid;
  float l, h;
} tap_t;

static tap_t mk_tap(float v, int size) {
  tap_t t;
  memset(&t, 0, sizeof(t));
  if (v < -1.0f || v > (float)size) return t;
  t.valid = 1;
  if (v <= 0.f) v = 0.f;
  int lo = (int)v, hi;
  if (lo >= size - 1) {
    hi = lo = size - 1;
    v = (float)lo;
  } else {
    hi = lo + 1;
  }
  t.lo = lo;
  t.hi = hi;
  t.l = v - (float)lo;
  t.h = 1.0f - t.l;
  return t;
}

/* torchvision RoIAlign forward over multi-level features.
 * feats[l]: pointer with element strides st[4l..] (b, c, y, x); rois [K,5];
 * levels [K] or NULL; out [K, C, ph, pw]. */
void orc_roi_align_fwd(int L, const float* const* feats, const int32_t* hw, const int64_t* st, const float* scales,
                       int C, const float* rois, const int64_t* levels, int64_t K, int ph, int pw, int sampling,
                       int aligned, float* out) {
  (void)L;
  /* torchvision's CPU kernel: the bilinear taps / weights of every sample of a RoI are
   * computed once (pre_calc) and reused by all channels; RoIs over the threads */
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t k = 0; k < K; ++k) {
    const float* r = rois + k * 5;
    int b = (int)r[0];
    int l = levels ? (int)levels[k] : 0;
    int H = hw[2 * l], W = hw[2 * l + 1];
    float sc = scales[l], off = aligned ? 0.5f : 0.0f;
    float sw = r[1] * sc - off, sh = r[2] * sc - off, ew = r[3] * sc - off, eh = r[4] * sc - off;
    float rw = ew - sw, rh = eh - sh;
    if (!aligned) {
      rw = rw > 1.0f ? rw : 1.0f;
      rh = rh > 1.0f ? rh : 1.0f;
    }
    float bh = rh / (float)ph, bw = rw / (float)pw;
    int gh = sampling > 0 ? sampling : (int)ceilf(rh / (float)ph);
    int gw = sampling > 0 ? sampling : (int)ceilf(rw / (float)pw);
    float cnt = (float)(gh * gw > 1 ? gh * gw : 1);
    int64_t sy = st[4 * l + 2], sx = st[4 * l + 3];
    const int ns = ph * pw * gh * gw;
    int64_t* pos = (int64_t*)malloc(sizeof(int64_t) * 4 * (size_t)ns);
    float* wt = (float*)malloc(sizeof(float) * 4 * (size_t)ns);
    unsigned char* ok = (unsigned char*)malloc((size_t)ns);
    int e = 0;
    for (int py = 0; py < ph; ++py)
      for (int px = 0; px < pw; ++px)
        for (int iy = 0; iy < gh; ++iy) {
          tap_t ty = mk_tap(sh + (float)py * bh + ((float)iy + 0.5f) * bh / (float)gh, H);
          for (int ix = 0; ix < gw; ++ix, ++e) {
            tap_t tx = mk_tap(sw + (float)px * bw + ((float)ix + 0.5f) * bw / (float)gw, W);
            ok[e] = (unsigned char)(ty.valid && tx.valid);
            wt[4 * e] = ty.h * tx.h, wt[4 * e + 1] = ty.h * tx.l, wt[4 * e + 2] = ty.l * tx.h, wt[4 * e + 3] = ty.l * tx.l;
            pos[4 * e] = ty.lo * sy + tx.lo * sx, pos[4 * e + 1] = ty.lo * sy + tx.hi * sx;
            pos[4 * e + 2] = ty.hi * sy + tx.lo * sx, pos[4 * e + 3] = ty.hi * sy + tx.hi * sx;
          }
        }
    for (int c = 0; c < C; ++c) {
      const float* f = feats[l] + b * st[4 * l] + c * st[4 * l + 1];
      const float* w4 = wt;
      const int64_t* p4 = pos;
      for (int bin = 0, q = 0; bin < ph * pw; ++bin) {
        float acc = 0.0f;
        for (int s = 0; s < gh * gw; ++s, ++q) {
          float val = 0.0f;
          if (ok[q]) {
            const float* w = w4 + 4 * q;
            const int64_t* p = p4 + 4 * q;
            val = ((w[0] * f[p[0]] + w[1] * f[p[1]]) + w[2] * f[p[2]]) + w[3] * f[p[3]];
          }
          acc = acc + val;
        }
        out[(k * C + c) * ph * pw + bin] = acc / cnt;
      }
    }
    free(pos);
    free(wt);
    free(ok);
  }
}

void orc_roi_align_bwd(int L, float* const* grads, const int32_t* hw, const int64_t* st, const float* scales, int C,
                       const float* rois, const int64_t* levels, int64_t K, int ph, int pw, int sampling, int aligned,
                       const float* gout) {
  for (int64_t k = 0; k < K; ++k) {
    const float* r = rois + k * 5;
    int b = (int)r[0];
    int l = levels ? (int)levels[k] : 0;
    int H = hw[2 * l], W = hw[2 * l + 1];
    float sc = scales[l], off = aligned ? 0.5f : 0.0f;
    float sw = r[1] * sc - off, sh = r[2] * sc - off, ew = r[3] * sc - off, eh = r[4] * sc - off;
    float rw = ew - sw, rh = eh - sh;
    if (!aligned) {
      rw = rw > 1.0f ? rw : 1.0f;
      rh = rh > 1.0f ? rh : 1.0f;
    }
    float bh = rh / (float)ph, bw = rw / (float)pw;
    int gh = sampling > 0 ? sampling : (int)ceilf(rh / (float)ph);
    int gw = sampling > 0 ? sampling : (int)ceilf(rw / (float)pw);
    float cnt = (float)(gh * gw > 1 ? gh * gw : 1);
    for (int c = 0; c < C; ++c) {
      float* f = grads[l] + b * st[4 * l] + c * st[4 * l + 1];
      int64_t sy = st[4 * l + 2], sx = st[4 * l + 3];
      for (int py = 0; py < ph; ++py)
        for (int px = 0; px < pw; ++px) {
          float g = gout[((k * C + c) * ph + py) * pw + px];
          for (int iy = 0; iy < gh; ++iy) {
            tap_t ty = mk_tap(sh + (float)py * bh + ((float)iy + 0.5f) * bh / (float)gh, H);
            if (!ty.valid) continue;
            for (int ix = 0; ix < gw; ++ix) {
              tap_t tx = mk_tap(sw + (float)px * bw + ((float)ix + 0.5f) * bw / (float)gw, W);
              if (!tx.valid) continue;
              f[ty.lo * sy + tx.lo * sx] += g * (ty.h * tx.h) / cnt;
              f[ty.lo * sy + tx.hi * sx] += g * (ty.h * tx.l) / cnt;
              f[ty.hi * sy + tx.lo * sx] += g * (ty.l * tx.h) / cnt;
              f[ty.hi * sy + tx.hi * sx] += g * (ty.l * tx.l) / cnt;
            }
          }
        }
    }
  }
}

/* torchvision RoIPool forward (argmax as flat y*W+x, -1 for empty bins) */
void orc_roi_pool_fwd(const float* feat, const int64_t* st, int H, int W, int C, float scale, const float* rois,
                      int64_t K, int ph, int pw, float* out, int32_t* argmax) {
  for (int64_t k = 0; k < K; ++k) {
    const float* r = rois + k * 5;
    int b = (int)r[0];
    int rsw = (int)roundf(r[1] * scale), rsh = (int)roundf(r[2] * scale);
    int rew = (int)roundf(r[3] * scale), reh = (int)roundf(r[4] * scale);
    int rw = rew - rsw + 1 > 1 ? rew - rsw + 1 : 1, rh = reh - rsh + 1 > 1 ? reh - rsh + 1 : 1;
    float bh = (float)rh / (float)ph, bw = (float)rw / (float)pw;
    for (int c = 0; c < C; ++c)
      for (int py = 0; py < ph; ++py)
        for (int px = 0; px < pw; ++px) {
          int hs = (int)floorf((float)py * bh) + rsh, he = (int)ceilf((float)(py + 1) * bh) + rsh;
          int ws = (int)floorf((float)px * bw) + rsw, we = (int)ceilf((float)(px + 1) * bw) + rsw;
          hs = hs < 0 ? 0 : (hs > H ? H : hs);
          he = he < 0 ? 0 : (he > H ? H : he);
          ws = ws < 0 ? 0 : (ws > W ? W : ws);
          we = we < 0 ? 0 : (we > W ? W : we);
          int empty = he <= hs || we <= ws;
          float m = empty ? 0.0f : -FLT_MAX;
          int mi = -1;
          for (int y = hs; y < he; ++y)
            for (int x = ws; x < we; ++x) {
              float v = feat[b * st[0] + c * st[1] + y * st[2] + x * st[3]];
              if (v > m) {
                m = v;
                mi = y * W + x;
              }
            }
          int64_t o = ((k * C + c) * ph + py) * pw + px;
          out[o] = m;
          argmax[o] = mi;
        }
  }
}

/* ATSS targets of one image: FCOSHead.single_image_targets_atss
 * (lib/heads/fcos_head.py:283-368) with its helpers topk_by_center (:106-116,
 * row index by floor division), bbox2ltrb (:78-87), positive_ltrb (:51-53),
 * centerness (:56-59), paint_value (:90-94), calc_iou (lib/utils.py:151-172).
 * Level l has a gh[l] x gw[l] grid, stride strides[l] and one anchor per cell
 * (anchors[l]: [4, gh*gw]).  Outputs cover the level-concatenated cells:
 * cls[N] (-1 outside the painted image area, 0 background, label), reg[N*4]
 * (ltrb, -1 where not positive), ctr[N] (-1 / 0 / centerness).
 * Top-k ties are broken by ascending cell index; the IoU mean / unbiased std
 * are accumulated in double and rounded to f32 (torch's f32 reduction order
 * can differ by an ulp: only an IoU within an ulp of mean+std could flip). */
static int cmp_dist(const void* a, const void* b) {
  const float* x = (const float*)a;
  const float* y = (const float*)b;
  if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
  return x[1] < y[1] ? -1 : (x[1] > y[1] ? 1 : 0);
}

void orc_atss_targets(int L, const int32_t* gh, const int32_t* gw, const float* strides,
                      const float* const* anchors, const float* gts, int64_t G, const int64_t* labels, int img_h,
                      int img_w, int topk, int64_t* cls, float* reg, float* ctr) {
  int64_t off[17], N = 0;
  for (int l = 0; l < L; ++l) {
    off[l] = N;
    N += (int64_t)gh[l] * gw[l];
  }
  float* maxiou = (float*)calloc((size_t)N, sizeof(float));
  for (int64_t i = 0; i < N; ++i) {
    cls[i] = -1;
    ctr[i] = -1.0f;
    reg[4 * i] = reg[4 * i + 1] = reg[4 * i + 2] = reg[4 * i + 3] = -1.0f;
  }
  for (int l = 0; l < L; ++l) {  /* paint_value([0, 0, img_w, img_h] * (1/stride)) */
    const float sc = (float)(1.0 / (double)strides[l]);
    const int x2 = (int)rintf((float)img_w * sc), y2 = (int)rintf((float)img_h * sc);
    for (int y = 0; y <= y2 && y < gh[l]; ++y)
      for (int x = 0; x <= x2 && x < gw[l]; ++x) {
        cls[off[l] + (int64_t)y * gw[l] + x] = 0;
        ctr[off[l] + (int64_t)y * gw[l] + x] = 0.0f;
      }
  }
  int64_t maxhw = 0;
  for (int l = 0; l < L; ++l) maxhw = (int64_t)gh[l] * gw[l] > maxhw ? (int64_t)gh[l] * gw[l] : maxhw;
  float* dist = (float*)malloc((size_t)maxhw * 2 * sizeof(float));
  int64_t* cidx = (int64_t*)malloc((size_t)L * topk * sizeof(int64_t));
  float* ciou = (float*)malloc((size_t)L * topk * sizeof(float));
  int* cnum = (int*)malloc((size_t)L * sizeof(int));
  for (int64_t g = 0; g < G; ++g) {
    const float b[4] = {gts[g], gts[G + g], gts[2 * G + g], gts[3 * G + g]};
    const float bcx = (b[2] + b[0]) / 2.0f, bcy = (b[3] + b[1]) / 2.0f;
    int tot = 0;
    for (int l = 0; l < L; ++l) {
      const int64_t hw = (int64_t)gh[l] * gw[l];
      const float* a = anchors[l];
      for (int64_t i = 0; i < hw; ++i) {
        const float acx = (a[2 * hw + i] + a[i]) / 2.0f, acy = (a[3 * hw + i] + a[hw + i]) / 2.0f;
        const float dx = acx - bcx, dy = acy - bcy;
        dist[2 * i] = sqrtf(dx * dx + dy * dy);
        dist[2 * i + 1] = (float)i;  /* exact: hw < 2^24 */
      }
      qsort(dist, (size_t)hw, 2 * sizeof(float), cmp_dist);
      const int k = (int64_t)topk < hw ? topk : (int)hw;
      for (int j = 0; j < k; ++j) {
        const int64_t i = (int64_t)dist[2 * j + 1];
        cidx[tot + j] = i;
        ciou[tot + j] = iou_p1(a, hw, i, b, 1, 0);
      }
      cnum[l] = k;
      tot += k;
    }
    double s = 0.0, ss = 0.0;
    for (int j = 0; j < tot; ++j) s += ciou[j];
    const double mean = s / tot;
    for (int j = 0; j < tot; ++j) ss += ((double)ciou[j] - mean) * ((double)ciou[j] - mean);
    const float thr = (float)mean + (float)sqrt(ss / (tot - 1));
    int j0 = 0;
    for (int l = 0; l < L; ++l) {
      for (int j = j0; j < j0 + cnum[l]; ++j) {
        const int64_t i = cidx[j];
        const int x = (int)(i % gw[l]), y = (int)(i / gw[l]);
        const float cx = (float)x * strides[l] + strides[l] / 2.0f, cy = (float)y * strides[l] + strides[l] / 2.0f;
        const float lt[4] = {cx - b[0], cy - b[1], b[2] - cx, b[3] - cy};
        const int pos_ltrb = lt[0] > 0 && lt[1] > 0 && lt[2] > 0 && lt[3] > 0;
        const int64_t c = off[l] + i;
        if (ciou[j] >= maxiou[c] && ciou[j] > thr && pos_ltrb) {
          cls[c] = labels[g];
          for (int q = 0; q < 4; ++q) reg[4 * c + q] = lt[q];
          maxiou[c] = ciou[j];
        }
      }
      j0 += cnum[l];
    }
  }
  for (int64_t c = 0; c < N; ++c)
    if (cls[c] > 0) {
      const float l = reg[4 * c] + 1e-6f, t = reg[4 * c + 1] + 1e-6f;
      const float r = reg[4 * c + 2] + 1e-6f, bb = reg[4 * c + 3] + 1e-6f;
      ctr[c] = sqrtf(((l < r ? l : r) / (l > r ? l : r)) * ((t < bb ? t : bb) / (t > bb ? t : bb)));
    }
  free(maxiou);
  free(dist);
  free(cidx);
  free(ciou);
  free(cnum);
}
