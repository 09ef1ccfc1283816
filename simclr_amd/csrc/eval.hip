// Remaining implicit kernels of the reference:
//   K2  MaxPool2d(3, 2, 1) of the ImageNet stem (torchvision ResNet, reference model.py:90-92
//       keeps it for resnet50 on 32x32 inputs) — NHWC bf16, forward records the window argmax
//       (one byte per output element) so the backward is a deterministic gather, no atomics;
//   K10 cross-entropy + top-k accuracy of the probes (reference eval.py:78,125-128) — one wave
//       per row: online logsumexp, loss, optional dlogits = (softmax - onehot)·scale, and the
//       target's rank (# classes scoring above it: top-k correct ⇔ rank < k, no sort);
//   K11 centroid weights (reference model.py:44-52): per-class feature sums in one pass over
//       the features, deterministic (each block owns a 64-column strip and walks every row).
#include "common.h"
#include "kernels.h"

namespace {

// ---------------------------------------------------------------------------- maxpool
// x [Nb][H][W][C] -> y [Nb][OH][OW][C], arg [Nb][OH][OW][C] (window tap 0..K*K-1); one thread
// per (output pixel, 8-channel chunk), 16-byte loads
__global__ void k_maxpool_fwd(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                              uint8_t* __restrict__ arg, int Nb, int H, int W, int C, int OH,
                              int OW, int K, int S, int P) {
  const int CH = C / 8;
  const size_t total = (size_t)Nb * OH * OW * CH;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CH);
    const size_t pix = i / CH;
    const int ow = (int)(pix % OW);
    const int oh = (int)((pix / OW) % OH);
    const int n = (int)(pix / ((size_t)OW * OH));
    float best[8];
    int bt[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bt[e] = 0; }
    for (int kh = 0; kh < K; ++kh) {
      const int ih = oh * S - P + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int iw = ow * S - P + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const u32x4 v = *(const u32x4*)(x + (((size_t)n * H + ih) * W + iw) * C + cc * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = (e & 1) ? hi_bf(v[e >> 1]) : lo_bf(v[e >> 1]);
          // strict > keeps the first maximum in window order, like PyTorch's kernel; NaN wins
          if (f > best[e] || f != f) { best[e] = f; bt[e] = kh * K + kw; }
        }
      }
    }
    u32x4 w;
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = pack2bf(best[2 * e], best[2 * e + 1]);
    *(u32x4*)(y + pix * C + cc * 8) = w;
    uint32_t a0 = 0, a1 = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a0 |= (uint32_t)bt[e] << (8 * e);
      a1 |= (uint32_t)bt[e + 4] << (8 * e);
    }
    *(u32x2*)(arg + pix * C + cc * 8) = (u32x2){a0, a1};
  }
}

// dx[n][ih][iw][c] = Σ over the output windows containing (ih, iw) whose argmax is this tap
__global__ void k_maxpool_bwd(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                              uint16_t* __restrict__ dx, int Nb, int H, int W, int C, int OH,
                              int OW, int K, int S, int P) {
  const int CH = C / 8;
  const size_t total = (size_t)Nb * H * W * CH;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CH);
    const size_t pix = i / CH;
    const int iw = (int)(pix % W);
    const int ih = (int)((pix / W) % H);
    const int n = (int)(pix / ((size_t)W * H));
    float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // oh such that oh*S - P <= ih <= oh*S - P + K - 1
    const int oh0 = max(0, (ih + P - K + S) / S), oh1 = min(OH - 1, (ih + P) / S);
    const int ow0 = max(0, (iw + P - K + S) / S), ow1 = min(OW - 1, (iw + P) / S);
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int kh = ih - (oh * S - P);
      if (kh < 0 || kh >= K) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int kw = iw - (ow * S - P);
        if (kw < 0 || kw >= K) continue;
        const size_t o = (((size_t)n * OH + oh) * OW + ow) * C + cc * 8;
        const u32x2 a = *(const u32x2*)(arg + o);
        const u32x4 v = *(const u32x4*)(dy + o);
        const int tap = kh * K + kw;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int t = (int)(((e < 4 ? a[0] : a[1]) >> (8 * (e & 3))) & 0xffu);
          if (t == tap) g[e] += (e & 1) ? hi_bf(v[e >> 1]) : lo_bf(v[e >> 1]);
        }
      }
    }
    u32x4 w;
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = pack2bf(g[2 * e], g[2 * e + 1]);
    *(u32x4*)(dx + pix * C + cc * 8) = w;
  }
}

// 2x2 space-to-depth of the zero-padded image for the ImageNet stem: a 7x7 / stride-2 / pad-P
// convolution over C <= 4 channels equals a 4x4 / stride-1 / unpadded one over
// xs[n][i][j][(dy * 2 + dx) * 4 + c] = img[n][2i + dy - P][2j + dx - P][c] (zero outside the
// image and for c >= creal) with the kernel folded the same way (models/fused.py _s2d_weight).
// K = 256 instead of 49 taps x 8 gathered channels = 392, every gather 32 contiguous bytes instead
// of 16 (tools/stem_s2d_probe.py: forward 1310 -> 889 us, weight gradient 1621 -> 858 us at
// 224x224, batch 1024).  One thread per (n, i, j, dy): two input pixels in, 16 bytes out.
__global__ void k_stem_s2d(const uint16_t* __restrict__ img, uint16_t* __restrict__ xs, int Nb,
                           int H, int W, int Cin, int creal, int HS, int WS, int P) {
  const size_t total = (size_t)Nb * HS * WS * 2;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const int dy = (int)(t & 1);
    const size_t pix = t >> 1;
    const int j = (int)(pix % WS);
    const size_t r = pix / WS;
    const int i = (int)(r % HS);
    const int n = (int)(r / HS);
    const int ih = 2 * i + dy - P;
    uint16_t v[8];
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int iw = 2 * j + dx - P;
      uint2 q = make_uint2(0u, 0u);
      if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
        q = *reinterpret_cast<const uint2*>(img + (((size_t)n * H + ih) * W + iw) * Cin);
      v[dx * 4 + 0] = (uint16_t)(q.x & 0xffffu);
      v[dx * 4 + 1] = creal > 1 ? (uint16_t)(q.x >> 16) : 0;
      v[dx * 4 + 2] = creal > 2 ? (uint16_t)(q.y & 0xffffu) : 0;
      v[dx * 4 + 3] = creal > 3 ? (uint16_t)(q.y >> 16) : 0;
    }
    uint4 o;
    o.x = v[0] | ((uint32_t)v[1] << 16);
    o.y = v[2] | ((uint32_t)v[3] << 16);
    o.z = v[4] | ((uint32_t)v[5] << 16);
    o.w = v[6] | ((uint32_t)v[7] << 16);
    *reinterpret_cast<uint4*>(xs + pix * 16 + dy * 8) = o;
  }
}


// ---------------------------------------------------------------------------- pooled stem
// The ImageNet-shape stem (reference model.py:90-92 keeps torchvision's 7x7/s2 conv -> BN ->
// ReLU -> MaxPool2d(3, 2, 1) for resnet50), fused around the max-pool:
//   forward   out = maxpool(relu(ss0[view]·a + ss1[view])) straight from the pre-BN conv output
//             a: the full-resolution BN + ReLU output is never written (the unfused path writes
//             it and reads it back).  Besides the window tap (one byte, for the backward) the
//             kernel keeps the pre-BN value at the argmax (asel), so the BatchNorm backward
//             partials Σg, Σg·x̂ come from pooled-size tensors (k_bn_bwd_reduce over out / asel:
//             g is zero off the argmax positions, and relu'(y[argmax]) = [out > 0]);
//   backward  da = A·g + B·a + D at full resolution, g gathered from the windows whose argmax
//             is this position (ReLU mask [out > 0]): max-pool backward, ReLU mask and the
//             BatchNorm input gradient in one pass (the unfused path scatters g, reduces over g
//             and a, and applies: three full-resolution passes).
// Values are compared after bf16 rounding, as the unfused BN-apply pass stores them; the first
// maximum in window order wins (strict >), NaN wins, as in k_maxpool_fwd.
__global__ void k_bn_relu_maxpool(const uint16_t* __restrict__ a, const float* __restrict__ ss,
                                  int S, uint16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                  uint16_t* __restrict__ asel, int Nb, int H, int W, int C,
                                  int OH, int OW, int K, int Sd, int P) {
  const int CH = C / 8;
  const int per_seg = Nb / S;
  const size_t total = (size_t)Nb * OH * OW * CH;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CH);
    const size_t pix = i / CH;
    const int ow = (int)(pix % OW);
    const int oh = (int)((pix / OW) % OH);
    const int n = (int)(pix / ((size_t)OW * OH));
    const int seg = n / per_seg;
    float sc[8], sh[8], best[8];
    int bt[8];
    uint32_t ba[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = ss[seg * C + cc * 8 + e];
      sh[e] = ss[S * C + seg * C + cc * 8 + e];
      best[e] = -INFINITY;
      bt[e] = 0;
      ba[e] = 0;
    }
    for (int kh = 0; kh < K; ++kh) {
      const int ih = oh * Sd - P + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int iw = ow * Sd - P + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const u32x4 v = *(const u32x4*)(a + (((size_t)n * H + ih) * W + iw) * C + cc * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t w = v[e >> 1];
          const float av = (e & 1) ? hi_bf(w) : lo_bf(w);
          float f = fmaf(av, sc[e], sh[e]);
          f = f > 0.f ? f : (f != f ? f : 0.f);
          f = bf2f(f2bf(f));
          if (f > best[e] || f != f) {
            best[e] = f;
            bt[e] = kh * K + kw;
            ba[e] = (e & 1) ? (w >> 16) : (w & 0xffffu);
          }
        }
      }
    }
    u32x4 wy, wa;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      wy[e] = pack2bf(best[2 * e], best[2 * e + 1]);
      wa[e] = ba[2 * e] | (ba[2 * e + 1] << 16);
    }
    *(u32x4*)(y + pix * C + cc * 8) = wy;
    *(u32x4*)(asel + pix * C + cc * 8) = wa;
    uint32_t a0 = 0, a1 = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a0 |= (uint32_t)bt[e] << (8 * e);
      a1 |= (uint32_t)bt[e + 4] << (8 * e);
    }
    *(u32x2*)(arg + pix * C + cc * 8) = (u32x2){a0, a1};
  }
}

// da[n][ih][iw][c] = A·g + B·a + D, g = Σ over the windows containing (ih, iw) whose argmax is
// this tap and whose pooled output is positive (the ReLU mask) of the pooled gradient
__global__ void k_maxpool_bwd_bn(const uint16_t* __restrict__ gy, const uint8_t* __restrict__ arg,
                                 const uint16_t* __restrict__ y, const uint16_t* __restrict__ a,
                                 const float* __restrict__ coef, int S, uint16_t* __restrict__ da,
                                 int Nb, int H, int W, int C, int OH, int OW, int K, int Sd,
                                 int P) {
  const int CH = C / 8;
  const int per_seg = Nb / S;
  const size_t total = (size_t)Nb * H * W * CH;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CH);
    const size_t pix = i / CH;
    const int iw = (int)(pix % W);
    const int ih = (int)((pix / W) % H);
    const int n = (int)(pix / ((size_t)W * H));
    const int seg = n / per_seg;
    float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int oh0 = max(0, (ih + P - K + Sd) / Sd), oh1 = min(OH - 1, (ih + P) / Sd);
    const int ow0 = max(0, (iw + P - K + Sd) / Sd), ow1 = min(OW - 1, (iw + P) / Sd);
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int kh = ih - (oh * Sd - P);
      if (kh < 0 || kh >= K) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int kw = iw - (ow * Sd - P);
        if (kw < 0 || kw >= K) continue;
        const size_t o = (((size_t)n * OH + oh) * OW + ow) * C + cc * 8;
        const u32x2 t8 = *(const u32x2*)(arg + o);
        const u32x4 v = *(const u32x4*)(gy + o);
        const u32x4 yv = *(const u32x4*)(y + o);
        const int tap = kh * K + kw;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int t = (int)(((e < 4 ? t8[0] : t8[1]) >> (8 * (e & 3))) & 0xffu);
          const float yy = (e & 1) ? hi_bf(yv[e >> 1]) : lo_bf(yv[e >> 1]);
          if (t == tap && yy > 0.f) g[e] += (e & 1) ? hi_bf(v[e >> 1]) : lo_bf(v[e >> 1]);
        }
      }
    }
    const u32x4 av = *(const u32x4*)(a + pix * C + cc * 8);
    u32x4 w;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float r[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = 2 * e + h;
        const int c = seg * C + cc * 8 + k;
        const float x = h ? hi_bf(av[e]) : lo_bf(av[e]);
        r[h] = coef[c] * g[k] + coef[S * C + c] * x + coef[2 * S * C + c];
      }
      w[e] = pack2bf(r[0], r[1]);
    }
    *(u32x4*)(da + pix * C + cc * 8) = w;
  }
}

// ---------------------------------------------------------------------------- CE + top-k
// logits [B][C] fp32, y [B] int64.  Per row: loss = lse - logit[y]; rank = #{j: logit[j] >
// logit[y]} + #{j < y: logit[j] == logit[y]} + #{j != y: logit[j] is NaN} (torch.topk orders NaN
// above every number); a NaN target logit or an out-of-range label gives rank C (never correct);
// dlogits (optional) = (softmax - onehot)·gscale.
// One 64-lane wave per row, 4 rows per block.
__global__ __launch_bounds__(256) void k_ce_topk(const float* __restrict__ logits,
                                                 const int64_t* __restrict__ y, int B, int C,
                                                 float gscale, float* __restrict__ loss,
                                                 int* __restrict__ rank,
                                                 float* __restrict__ dlogits) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float* z = logits + (size_t)row * C;
  const int t = (int)y[row];
  const float zt = (t >= 0 && t < C) ? z[t] : NAN;
  float m = -INFINITY, s = 0.f;
  int above = 0;
  for (int j = lane; j < C; j += 64) {
    const float v = z[j];
    above += (v > zt || (v == zt && j < t) || (v != v && j != t)) ? 1 : 0;
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; } else { s += __expf(v - m); }
  }
  // wave reduction of (m, s) and the count
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float m2 = __shfl_xor(m, off, 64), s2 = __shfl_xor(s, off, 64);
    const float mm = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mm)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
    m = mm;
    above += __shfl_xor(above, off, 64);
  }
  const float lse = m + __logf(s);
  if (lane == 0) {
    const bool valid = t >= 0 && t < C && zt == zt;
    loss[row] = lse - zt;             // NaN for an out-of-range label (as F.cross_entropy errors)
    rank[row] = valid ? above : C;    // never counted as correct
  }
  if (dlogits != nullptr) {
    float* d = dlogits + (size_t)row * C;
    for (int j = lane; j < C; j += 64) d[j] = (__expf(z[j] - lse) - (j == t ? 1.f : 0.f)) * gscale;
  }
}

// ---------------------------------------------------------------------------- centroid sums
// X [N][D] fp32, y [N] int64 -> part [G][NC][D], pcnt [G][NC]: block (strip, g) owns a 64-column
// strip and the rows r ≡ g (mod G), accumulating per-class sums in LDS in row order; then
// k_class_sums_final adds the G partials in order (deterministic, no atomics).
__global__ __launch_bounds__(64) void k_class_sums(const float* __restrict__ X,
                                                   const int64_t* __restrict__ y, int N, int D,
                                                   int NC, float* __restrict__ part,
                                                   float* __restrict__ pcnt) {
  extern __shared__ float acc[];  // [NC][64] + [NC]
  const int cl = threadIdx.x, d = blockIdx.x * 64 + cl;
  const int g = blockIdx.y, G = gridDim.y;
  float* cnt = acc + (size_t)NC * 64;
  for (int i = cl; i < NC * 64; i += 64) acc[i] = 0.f;
  for (int i = cl; i < NC; i += 64) cnt[i] = 0.f;
  __syncthreads();
  for (int r = g; r < N; r += G) {
    const int c = (int)y[r];
    if (c < 0 || c >= NC) continue;
    if (d < D) acc[c * 64 + cl] += X[(size_t)r * D + d];
    if (cl == 0) cnt[c] += 1.f;
  }
  __syncthreads();
  for (int c = 0; c < NC; ++c) {
    if (d < D) part[((size_t)g * NC + c) * D + d] = acc[c * 64 + cl];
  }
  if (blockIdx.x == 0)
    for (int c = cl; c < NC; c += 64) pcnt[(size_t)g * NC + c] = cnt[c];
}

__global__ void k_class_sums_final(const float* __restrict__ part, const float* __restrict__ pcnt,
                                   int G, int NC, int D, float* __restrict__ sums,
                                   float* __restrict__ counts) {
  const size_t n = (size_t)NC * D;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n + NC;
       i += (size_t)gridDim.x * blockDim.x) {
    float a = 0.f;
    if (i < n) {
      for (int g = 0; g < G; ++g) a += part[(size_t)g * n + i];
      sums[i] = a;
    } else {
      const size_t c = i - n;
      for (int g = 0; g < G; ++g) a += pcnt[(size_t)g * NC + c];
      counts[c] = a;
    }
  }
}

int grid_cap(size_t n) {
  size_t b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}

}  // namespace

void maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* arg, int Nb, int H, int W, int C,
                 int OH, int OW, int K, int S, int P, hipStream_t s) {
  hipLaunchKernelGGL(k_maxpool_fwd, dim3(grid_cap((size_t)Nb * OH * OW * (C / 8))), dim3(256), 0,
                     s, x, y, arg, Nb, H, W, C, OH, OW, K, S, P);
  HIP_CHECK_LAUNCH();
}

void maxpool_bwd(const uint16_t* dy, const uint8_t* arg, uint16_t* dx, int Nb, int H, int W,
                 int C, int OH, int OW, int K, int S, int P, hipStream_t s) {
  hipLaunchKernelGGL(k_maxpool_bwd, dim3(grid_cap((size_t)Nb * H * W * (C / 8))), dim3(256), 0, s,
                     dy, arg, dx, Nb, H, W, C, OH, OW, K, S, P);
  HIP_CHECK_LAUNCH();
}

void bn_relu_maxpool(const uint16_t* a, const float* ss, int S, uint16_t* y, uint8_t* arg,
                     uint16_t* asel, int Nb, int H, int W, int C, int OH, int OW, int K, int Sd,
                     int P, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_relu_maxpool, dim3(grid_cap((size_t)Nb * OH * OW * (C / 8))), dim3(256),
                     0, s, a, ss, S, y, arg, asel, Nb, H, W, C, OH, OW, K, Sd, P);
  HIP_CHECK_LAUNCH();
}

void stem_s2d(const uint16_t* img, uint16_t* xs, int Nb, int H, int W, int Cin, int creal,
              int HS, int WS, int P, hipStream_t s) {
  hipLaunchKernelGGL(k_stem_s2d, dim3(grid_cap((size_t)Nb * HS * WS * 2)), dim3(256), 0, s, img,
                     xs, Nb, H, W, Cin, creal, HS, WS, P);
  HIP_CHECK_LAUNCH();
}

void maxpool_bwd_bn(const uint16_t* gy, const uint8_t* arg, const uint16_t* y, const uint16_t* a,
                    const float* coef, int S, uint16_t* da, int Nb, int H, int W, int C, int OH,
                    int OW, int K, int Sd, int P, hipStream_t s) {
  hipLaunchKernelGGL(k_maxpool_bwd_bn, dim3(grid_cap((size_t)Nb * H * W * (C / 8))), dim3(256), 0,
                     s, gy, arg, y, a, coef, S, da, Nb, H, W, C, OH, OW, K, Sd, P);
  HIP_CHECK_LAUNCH();
}

void ce_topk(const float* logits, const int64_t* y, int B, int C, float gscale, float* loss,
             int* rank, float* dlogits, hipStream_t s) {
  hipLaunchKernelGGL(k_ce_topk, dim3((B + 3) / 4), dim3(256), 0, s, logits, y, B, C, gscale, loss,
                     rank, dlogits);
  HIP_CHECK_LAUNCH();
}

size_t class_sums_lds(int NC) { return ((size_t)NC * 64 + NC) * sizeof(float); }
int class_sums_groups(int N) { return N >= 4096 ? 32 : 1; }

void class_sums(const float* X, const int64_t* y, int N, int D, int NC, float* part, float* pcnt,
                float* sums, float* counts, hipStream_t s) {
  const int G = class_sums_groups(N);
  hipLaunchKernelGGL(k_class_sums, dim3((D + 63) / 64, G), dim3(64), class_sums_lds(NC), s, X, y,
                     N, D, NC, part, pcnt);
  HIP_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_class_sums_final, dim3(grid_cap((size_t)NC * D + NC)), dim3(256), 0, s, part,
                     pcnt, G, NC, D, sums, counts);
  HIP_CHECK_LAUNCH();
}
