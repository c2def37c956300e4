// Memory-system probes for the RoIAlign forward design (tools only, not product).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void stream_read(const float4* __restrict__ p, int64_t n, float* sink) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = p[i];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) sink[0] = acc.x;
}

__global__ void stream_write(float4* __restrict__ q, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    q[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

// reads n_in float4 and writes n_out float4 in the same launch (interleaved per thread)
__global__ void stream_rw(const float4* __restrict__ p, int64_t n_in, float4* __restrict__ q, int64_t n_out,
                          float* sink) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int64_t T = (int64_t)gridDim.x * blockDim.x, t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = n_in > n_out ? n_in : n_out;
  for (int64_t i = t; i < n; i += T) {
    if (i < n_in) {
      float4 v = p[i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if (i < n_out) q[i] = acc;
  }
  if (acc.x == 1234.5f) sink[0] = acc.y;
}

extern "C" int probe_stream_read(const void* p, int64_t n4, void* sink, int grid, void* stream) {
  hipLaunchKernelGGL(stream_read, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float4*)p, n4, (float*)sink);
  return (int)hipGetLastError();
}
extern "C" int probe_stream_write(void* q, int64_t n4, int grid, void* stream) {
  hipLaunchKernelGGL(stream_write, dim3(grid), dim3(256), 0, (hipStream_t)stream, (float4*)q, n4);
  return (int)hipGetLastError();
}
extern "C" int probe_stream_rw(const void* p, int64_t n_in4, void* q, int64_t n_out4, void* sink, int grid,
                               void* stream) {
  hipLaunchKernelGGL(stream_rw, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float4*)p, n_in4, (float4*)q,
                     n_out4, (float*)sink);
  return (int)hipGetLastError();
}

// RoIAlign output store pattern: wave = (RoI, 16 channels), lane = bin (49 of 64),
// one 4-B store per lane per channel (196 B per store instruction).
__global__ void __launch_bounds__(256) store_pattern(float* __restrict__ out, int C, int nch_wave) {
  const int k = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c0 = (blockIdx.y * 4 + wave) * nch_wave;
  if (lane >= 49 || c0 >= C) return;
  float* o = out + ((int64_t)k * C + c0) * 49 + lane;
  for (int c = 0; c < nch_wave; ++c) o[c * 49] = (float)(c + lane);
}
// same bytes, each wave writes its contiguous 16*49 floats with lanes contiguous
__global__ void __launch_bounds__(256) store_contig(float* __restrict__ out, int C, int nch_wave) {
  const int k = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c0 = (blockIdx.y * 4 + wave) * nch_wave;
  if (c0 >= C) return;
  float* o = out + ((int64_t)k * C + c0) * 49;
  const int n = nch_wave * 49;
  for (int i = lane; i < n; i += 64) o[i] = (float)i;
}
extern "C" int probe_store(void* out, int K, int C, int nch_wave, int contig, void* stream) {
  dim3 g(K, (C + 4 * nch_wave - 1) / (4 * nch_wave));
  if (contig)
    hipLaunchKernelGGL(store_contig, g, dim3(256), 0, (hipStream_t)stream, (float*)out, C, nch_wave);
  else
    hipLaunchKernelGGL(store_pattern, g, dim3(256), 0, (hipStream_t)stream, (float*)out, C, nch_wave);
  return (int)hipGetLastError();
}
