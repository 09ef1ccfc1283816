// Small bandwidth kernels: global average pool fwd/bwd (torchvision avgpool+flatten),
// column sums (Linear bias gradients) and dtype casts.
#include "common.h"
#include "kernels.h"

namespace {

// x [Nb][HW][C] -> y [Nb][C]; one thread per (n, 8-channel chunk)
__global__ void k_avgpool_fwd(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int Nb,
                              int HW, int C) {
  const int CH = C / 8;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= Nb * CH) return;
  const int n = idx / CH, cc = idx % CH;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint16_t* src = x + (size_t)n * HW * C + cc * 8;
  for (int p = 0; p < HW; ++p) {
    const u32x4 v = *(const u32x4*)(src + (size_t)p * C);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[2 * e] += lo_bf(v[e]);
      acc[2 * e + 1] += hi_bf(v[e]);
    }
  }
  const float inv = 1.f / HW;
  u32x4 w;
#pragma unroll
  for (int e = 0; e < 4; ++e) w[e] = pack2bf(acc[2 * e] * inv, acc[2 * e + 1] * inv);
  *(u32x4*)(y + (size_t)n * C + cc * 8) = w;
}

__global__ void k_avgpool_bwd(const uint16_t* __restrict__ dy, uint16_t* __restrict__ dx, int Nb,
                              int HW, int C) {
  const int CH = C / 8;
  const size_t total = (size_t)Nb * HW * CH;
  const float inv = 1.f / HW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CH);
    const size_t n = i / ((size_t)HW * CH);
    const u32x4 v = *(const u32x4*)(dy + n * C + cc * 8);
    u32x4 w;
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = pack2bf(lo_bf(v[e]) * inv, hi_bf(v[e]) * inv);
    *(u32x4*)(dx + i * 8) = w;
  }
}

// Column sums in two deterministic levels: grid (C/64 strips, G row groups) writes partials
// ws[G][C]; k_colsum_final adds the G partials in order.  (One 64-column strip per block over
// all rows left a 2048-column, 1024-row head-bias gradient latency-bound at ~75 µs.)
__global__ void k_colsum(const uint16_t* __restrict__ x, int R, int C, float* __restrict__ ws) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int G = gridDim.y, g = blockIdx.y;
  const int per = (R + G - 1) / G;
  const int r0 = g * per, r1 = min(R, r0 + per);
  float a = 0.f;
  if (c < C)
#pragma unroll 4
    for (int r = r0 + rl; r < r1; r += 4) a += bf2f(x[(size_t)r * C + c]);
  red[rl][threadIdx.x & 63] = a;
  __syncthreads();
  if (rl == 0 && c < C)
    ws[(size_t)g * C + c] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                            red[3][threadIdx.x];
}

__global__ void k_colsum_final(const float* __restrict__ ws, int G, int C, float* __restrict__ out,
                               float beta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int g = 0; g < G; ++g) s += ws[(size_t)g * C + c];
  out[c] = beta != 0.f ? beta * out[c] + s : s;
}

__global__ void k_cast_f32_bf16(const float* __restrict__ x, uint16_t* __restrict__ y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

__global__ void k_cast_bf16_f32(const uint16_t* __restrict__ x, float* __restrict__ y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    y[i] = bf2f(x[i]);
}

int grid_for(size_t n, int cap = 8192) {
  size_t b = (n + 255) / 256;
  if (b > (size_t)cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

void avgpool_fwd(const uint16_t* x, uint16_t* y, int Nb, int HW, int C, hipStream_t s) {
  const int n = Nb * (C / 8);
  hipLaunchKernelGGL(k_avgpool_fwd, dim3((n + 255) / 256), dim3(256), 0, s, x, y, Nb, HW, C);
  HIP_CHECK_LAUNCH();
}

void avgpool_bwd(const uint16_t* dy, uint16_t* dx, int Nb, int HW, int C, hipStream_t s) {
  hipLaunchKernelGGL(k_avgpool_bwd, dim3(grid_for((size_t)Nb * HW * (C / 8))), dim3(256), 0, s, dy,
                     dx, Nb, HW, C);
  HIP_CHECK_LAUNCH();
}

int colsum_groups(int R) {
  int g = R / 64;
  return g < 1 ? 1 : (g > 32 ? 32 : g);
}

void colsum_bf16(const uint16_t* x, int R, int C, float* out, float beta, float* ws,
                 hipStream_t s) {
  const int G = colsum_groups(R);
  hipLaunchKernelGGL(k_colsum, dim3((C + 63) / 64, G), dim3(256), 0, s, x, R, C, ws);
  hipLaunchKernelGGL(k_colsum_final, dim3((C + 255) / 256), dim3(256), 0, s, ws, G, C, out, beta);
  HIP_CHECK_LAUNCH();
}

void cast_f32_bf16(const float* x, uint16_t* y, size_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_cast_f32_bf16, dim3(grid_for(n)), dim3(256), 0, s, x, y, n);
  HIP_CHECK_LAUNCH();
}

void cast_bf16_f32(const uint16_t* x, float* y, size_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_cast_bf16_f32, dim3(grid_for(n)), dim3(256), 0, s, x, y, n);
  HIP_CHECK_LAUNCH();
}
