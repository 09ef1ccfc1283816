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


// ---------------------------------------------------------------- split-K GEMM (small M)
// C[M][N] = f(A)[M][K] · B[N][K]ᵀ (+ bias) for the projection head's GEMM 2 (M 1,024 rows,
// N 128, K 2,048): the implicit-GEMM tiles give it 32 blocks whose 2,048-deep K loop is
// latency-bound (40 us, ~13 TF/s).  Here the K range is split: grid (M/64, N/64, KS) blocks
// each stage a 64-row slice of A and of B over K/KS columns in LDS (f = BatchNorm + ReLU of
// the A operand, per row segment and column, rounded to bf16 as the GEMM prologue does) and
// write a 64x64 fp32 partial; a second kernel sums the KS partials in a fixed order (same bits
// every run) and adds the bias.  4 waves, 32x32 per wave on v_mfma_f32_16x16x32_bf16; LDS rows
// padded by 16 bytes so the 16 rows of one b128 fragment read fall on distinct banks.
constexpr int SK_T = 64;
template <bool PRO>
__global__ __launch_bounds__(256) void k_gemm_sk(const uint16_t* __restrict__ A,
                                                 const uint16_t* __restrict__ B,
                                                 const float* __restrict__ sc,
                                                 const float* __restrict__ sh, int seg, int M,
                                                 int N, int K, int kslice,
                                                 float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) uint16_t sk_lds[];
  const int KP = kslice + 8;
  uint16_t* As = sk_lds;
  uint16_t* Bs = sk_lds + SK_T * KP;
  const int m0 = blockIdx.x * SK_T, n0 = blockIdx.y * SK_T, k0 = blockIdx.z * kslice;
  const int tid = threadIdx.x;
  const int CPR = kslice / 8;
  for (int c = tid; c < SK_T * CPR; c += 256) {
    const int r = c / CPR, ch = c - r * CPR;
    const int k = k0 + ch * 8;
    u32x4 v = *(const u32x4*)(A + (size_t)(m0 + r) * K + k);
    if (PRO) {
      const int sg = (m0 + r) / seg;
      const float* scs = sc + (size_t)sg * K + k;
      const float* shs = sh + (size_t)sg * K + k;
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = (e & 1) ? hi_bf(v[e >> 1]) : lo_bf(v[e >> 1]);
        const float y = fmaf(x, scs[e], shs[e]);
        f[e] = y > 0.f ? y : (y != y ? y : 0.f);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = pack2bf(f[2 * e], f[2 * e + 1]);
    }
    *(u32x4*)(As + r * KP + ch * 8) = v;
    *(u32x4*)(Bs + r * KP + ch * 8) = *(const u32x4*)(B + (size_t)(n0 + r) * K + k);
  }
  __syncthreads();
  const int lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int wm = (wid >> 1) * 32, wn = (wid & 1) * 32;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int kk = 0; kk < kslice; kk += 32) {
    bf16x8 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      a[i] = *(const bf16x8*)(As + (wm + i * 16 + li) * KP + kk + g * 8);
      b[i] = *(const bf16x8*)(Bs + (wn + i * 16 + li) * KP + kk + g * 8);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  // acc[i][j][r]: row 4 g + r of A-fragment i, row li of B-fragment j
  float* out = part + (size_t)blockIdx.z * M * N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(size_t)(m0 + wm + i * 16 + 4 * g + r) * N + n0 + wn + j * 16 + li] = acc[i][j][r];
}

// out[m][n] = bf16(Σ_ks part[ks][m][n] + bias[n]), ks in order; four columns per thread
__global__ void k_gemm_sk_reduce(const float* __restrict__ part, int KS, int M, int N,
                                 const float* __restrict__ bias, uint16_t* __restrict__ out) {
  const size_t i4 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n4 = (size_t)M * N / 4;
  if (i4 >= n4) return;
  const float4* p = (const float4*)part;
  float4 a = p[i4];
  for (int ks = 1; ks < KS; ++ks) {
    const float4 v = p[(size_t)ks * n4 + i4];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  if (bias != nullptr) {
    const int n = (int)((i4 * 4) % N);
    a.x += bias[n]; a.y += bias[n + 1]; a.z += bias[n + 2]; a.w += bias[n + 3];
  }
  *(u32x2*)(out + i4 * 4) = (u32x2){pack2bf(a.x, a.y), pack2bf(a.z, a.w)};
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

void gemm_sk(const uint16_t* A, const uint16_t* B, const float* sc, const float* sh, int seg,
             int M, int N, int K, int KS, float* part, const float* bias, uint16_t* out,
             hipStream_t s) {
  const int kslice = K / KS;
  const size_t lds = (size_t)2 * SK_T * (kslice + 8) * 2;
  const dim3 grid(M / SK_T, N / SK_T, KS);
  if (sc != nullptr)
    hipLaunchKernelGGL(k_gemm_sk<true>, grid, dim3(256), lds, s, A, B, sc, sh, seg, M, N, K,
                       kslice, part);
  else
    hipLaunchKernelGGL(k_gemm_sk<false>, grid, dim3(256), lds, s, A, B, sc, sh, seg, M, N, K,
                       kslice, part);
  HIP_CHECK_LAUNCH();
  const size_t n4 = (size_t)M * N / 4;
  hipLaunchKernelGGL(k_gemm_sk_reduce, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, part,
                     KS, M, N, bias, out);
  HIP_CHECK_LAUNCH();
}
