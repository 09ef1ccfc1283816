// Fused LARS (Apex LARC, clip=False) + SGD momentum over the flat parameter store, gfx950.
//
// Reference: SGD(momentum=0.9, nesterov=False, weight_decay=0, two param groups from
// exclude_from_wt_decay) wrapped in apex.parallel.LARC(trust_coefficient=0.001, clip=False)
// (/root/reference/main.py:18-36, 85-94).  Apex runs a Python loop over all
// 65/164 parameters with two host-synchronising norm comparisons each, then SGD.step.
//
// Here: (1) lars_norms — one block per ≤16K-element chunk computes Σp² and Σg² (grad scaled by
// 1/world for the DDP average) into a per-chunk slot; (2) lars_update — one block per chunk sums
// its segment's chunk slots (deterministic), forms the trust ratio with Apex's "both norms
// non-zero" guard predicated in-kernel, folds weight decay, updates momentum and the fp32 master
// weight and rewrites the bf16 shadow weight the convolutions consume.  The learning rate is read
// from device memory (written by lr_schedule_step), so the whole step is host-sync free and
// hipGraph-capturable.
#include <math.h>
#include "common.h"
#include "kernels.h"

namespace {

constexpr int LARS_THREADS = 256;

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0) {
    for (int i = 0; i < LARS_THREADS / 64; ++i) t += red[i];
    red[LARS_THREADS / 64] = t;
  }
  __syncthreads();
  t = red[LARS_THREADS / 64];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(LARS_THREADS) void k_lars_norms(const float* __restrict__ p,
                                                             const float* __restrict__ g,
                                                             const int* __restrict__ chunk_beg,
                                                             const int* __restrict__ chunk_end,
                                                             float grad_scale,
                                                             float* __restrict__ norms) {
  __shared__ float red[LARS_THREADS / 64 + 1];
  const int c = blockIdx.x;
  const int beg = chunk_beg[c], end = chunk_end[c];
  float sp = 0.f, sg = 0.f;
  // beg/end are multiples of 4 except possibly the segment's end; four 16-byte loads of each
  // operand in flight per thread (one pair at a time ran at ~4 TB/s)
  int i = beg + threadIdx.x * 4;
  constexpr int ST = LARS_THREADS * 4;
  for (; i + 3 * ST + 3 < end; i += 4 * ST) {
    float4 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = *(const float4*)(p + i + u * ST);
      b[u] = *(const float4*)(g + i + u * ST);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sp += a[u].x * a[u].x + a[u].y * a[u].y + a[u].z * a[u].z + a[u].w * a[u].w;
      sg += b[u].x * b[u].x + b[u].y * b[u].y + b[u].z * b[u].z + b[u].w * b[u].w;
    }
  }
  for (; i + 3 < end; i += ST) {
    const float4 a = *(const float4*)(p + i);
    const float4 b = *(const float4*)(g + i);
    sp += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
    sg += b.x * b.x + b.y * b.y + b.z * b.z + b.w * b.w;
  }
  for (; i < end; ++i) {  // tail (< 4 elements), only reached by one thread
    sp += p[i] * p[i];
    sg += g[i] * g[i];
  }
  sp = block_sum(sp, red);
  sg = block_sum(sg, red);
  if (threadIdx.x == 0) {
    norms[2 * c] = sp;
    norms[2 * c + 1] = sg * grad_scale * grad_scale;
  }
}

// seg_flags bit0: apply LARS trust ratio; bit1: write bf16 shadow
__global__ __launch_bounds__(LARS_THREADS) void k_lars_update(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ mom,
    uint16_t* __restrict__ shadow, const int* __restrict__ chunk_seg,
    const int* __restrict__ chunk_beg, const int* __restrict__ chunk_end,
    const int* __restrict__ seg_chunk_beg, const int* __restrict__ seg_chunk_end,
    const float* __restrict__ seg_wd, const int* __restrict__ seg_flags,
    const float* __restrict__ norms, const float* __restrict__ lr_ptr, float momentum, float trust,
    float eps, float grad_scale, int nesterov) {
  __shared__ float red[LARS_THREADS / 64 + 1];
  const int c = blockIdx.x;
  const int seg = chunk_seg[c];
  const float wd = seg_wd[seg];
  const int flags = seg_flags[seg];
  // the segment's chunk slots summed by the whole block (fixed slot -> thread assignment and
  // reduction tree: deterministic); one thread walking them serially cost up to ~250 dependent
  // loads per block on the big 3x3 / head tensors
  float sp = 0.f, sg = 0.f;
  for (int k = seg_chunk_beg[seg] + threadIdx.x; k < seg_chunk_end[seg]; k += LARS_THREADS) {
    sp += norms[2 * k];
    sg += norms[2 * k + 1];
  }
  sp = block_sum(sp, red);
  sg = block_sum(sg, red);
  const float pn = sqrtf(sp), gn = sqrtf(sg);
  // Apex LARC: only when both norms are non-zero is wd folded and the grad rescaled
  float scale = grad_scale, wdf = 0.f;
  if (flags & 1) {
    if (pn != 0.f && gn != 0.f) {
      const float local = trust * pn / (gn + pn * wd + eps);
      scale = grad_scale * local;
      wdf = wd * local;
    }
  } else {
    wdf = wd;  // plain SGD weight decay
  }
  const float lr = lr_ptr[0];
  const int beg = chunk_beg[c], end = chunk_end[c];
  const bool write_shadow = (flags & 2) && shadow != nullptr;
  auto step1 = [&](float pv, float gv, float mv, float& bo) {
    const float d = gv * scale + wdf * pv;
    const float b = momentum * mv + d;  // mom starts at 0 == torch's buf=clone(d)
    bo = b;
    const float upd = nesterov ? d + momentum * b : b;
    return pv - lr * upd;
  };
  // 16-byte accesses (chunk starts are 64-element aligned; only a segment's end may not be a
  // multiple of 4: that tail of < 4 elements is reached by one thread)
  int i = beg + threadIdx.x * 4;
  for (; i + 3 < end; i += LARS_THREADS * 4) {
    const float4 pv = *(const float4*)(p + i);
    const float4 gv = *(const float4*)(g + i);
    const float4 mv = *(const float4*)(mom + i);
    float4 b, np;
    np.x = step1(pv.x, gv.x, mv.x, b.x);
    np.y = step1(pv.y, gv.y, mv.y, b.y);
    np.z = step1(pv.z, gv.z, mv.z, b.z);
    np.w = step1(pv.w, gv.w, mv.w, b.w);
    *(float4*)(mom + i) = b;
    *(float4*)(p + i) = np;
    if (write_shadow) *(u32x2*)(shadow + i) = (u32x2){pack2bf(np.x, np.y), pack2bf(np.z, np.w)};
  }
  for (; i < end; ++i) {
    float b;
    const float np = step1(p[i], g[i], mom[i], b);
    mom[i] = b;
    p[i] = np;
    if (write_shadow) shadow[i] = f2bf(np);
  }
}

// Reference LR closed form (lr_utils.py + CosineAnnealingLR stepped after the
// optimizer for step > warmup).  mode 0: warmup + cosine; mode 1: cosine from step 0 (probe);
// mode 2: constant.
__global__ void k_lr_step(int64_t* step, float* lr_out, double lr0, int64_t warmup, int64_t total,
                          int mode) {
  const int64_t s = step[0];
  double lr;
  if (mode == 2) {
    lr = lr0;
  } else if (mode == 1) {
    lr = total > 0 ? lr0 * 0.5 * (1.0 + cos(M_PI * (double)s / (double)total)) : lr0;
  } else if (s <= warmup) {
    lr = warmup > 0 ? (double)s / (double)warmup * lr0 : lr0;
  } else {
    const double T = (double)(total - warmup);
    lr = T > 0 ? lr0 * 0.5 * (1.0 + cos(M_PI * (double)(s - warmup - 1) / T)) : lr0;
  }
  lr_out[0] = (float)lr;
  step[0] = s + 1;
}

}  // namespace

void lars_norms(const float* p, const float* g, const int* chunk_beg, const int* chunk_end,
                int nchunks, float grad_scale, float* norms, hipStream_t s) {
  hipLaunchKernelGGL(k_lars_norms, dim3(nchunks), dim3(LARS_THREADS), 0, s, p, g, chunk_beg,
                     chunk_end, grad_scale, norms);
  HIP_CHECK_LAUNCH();
}

void lars_update(float* p, const float* g, float* mom, uint16_t* shadow, const int* chunk_seg,
                 const int* chunk_beg, const int* chunk_end, int nchunks, const int* seg_chunk_beg,
                 const int* seg_chunk_end, const float* seg_wd, const int* seg_flags,
                 const float* norms, const float* lr_ptr, float momentum, float trust, float eps,
                 float grad_scale, int nesterov, hipStream_t s) {
  hipLaunchKernelGGL(k_lars_update, dim3(nchunks), dim3(LARS_THREADS), 0, s, p, g, mom, shadow,
                     chunk_seg, chunk_beg, chunk_end, seg_chunk_beg, seg_chunk_end, seg_wd,
                     seg_flags, norms, lr_ptr, momentum, trust, eps, grad_scale, nesterov);
  HIP_CHECK_LAUNCH();
}

void lr_schedule_step(int64_t* step, float* lr_out, double lr0, int64_t warmup, int64_t total,
                      int mode, hipStream_t s) {
  hipLaunchKernelGGL(k_lr_step, dim3(1), dim3(1), 0, s, step, lr_out, lr0, warmup, total, mode);
  HIP_CHECK_LAUNCH();
}
