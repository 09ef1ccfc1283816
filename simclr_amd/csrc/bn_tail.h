// BatchNorm finalize fused into the tail of the producing conv kernel (conv.hip igemm_bn_tail).
//
// The conv epilogue already writes per-block Σ / Σ² (forward) or Σg / Σg·x̂ (dgrad modes 3/4)
// partial rows; the separate k_bn_reduce_fused launch that reduced and finalized them sat on the
// critical path ~100 times per ResNet-50 step (10 µs each plus its dispatch: removing them
// entirely measured 23.43 → 22.45 ms/step).  Here the conv's own blocks do it: a two-level
// last-arriver over the row-blocks of each channel tile (level-1 groups of `gr` row-blocks, then
// one level-2 pass over the groups' sums), summing in a fixed order (deterministic), followed
// by the finalize of that tile's channels — forward: mean / invstd, the scale-shift table of the
// consumer, running statistics, num_batches_tracked; backward: the input-gradient coefficients
// and dγ, dβ — and, at world > 1, the IPC statistics exchange (comm/ipc.py) in between.
// Publication across XCDs follows k_bn_reduce_fused: partial rows are written with agent-scope
// relaxed (write-through) stores, the writer drains them (vmcnt(0)) before its ticket
// increment, and the last arriver performs one agent-scope acquire before reading.
#pragma once
#include "common.h"
#include "kernels.h"  // IpcX, BnFin, BnTailArgs

constexpr int kTailMaxS = 2;
constexpr int kTailMaxCols = 256;
constexpr int kTailMaxWorld = 16;

// Cross-rank sum of the tile's [S][2][ncol] sums held in LDS `v` (index (sg*2+k)*ncol + j for
// column c0 + j; c0, ncol multiples of 64): the LL-word protocol of bn.hip bn_ipc_exchange —
// push this rank's slot to every arena, then spin on the W slots of the own arena (wall-clock
// bounded) and sum them in rank order.  `sh_ep` is LDS scratch of ncol/64 words.
__device__ inline void tail_ipc_exchange(const IpcX& x, int S, int C, int c0, int ncol, float* v,
                                         unsigned* sh_ep) {
  const int W = x.world;
  const int ngr = ncol / 64;
  if ((int)threadIdx.x < ngr) {
    const int g = c0 / 64 + threadIdx.x;
    const unsigned e = x.epoch[g] + 1u;
    x.epoch[g] = e;
    sh_ep[threadIdx.x] = e;
  }
  __syncthreads();
  const long long slot = 2LL * S * C;
  const int nval = S * 2 * ncol;
  for (int i = threadIdx.x; i < W * nval; i += blockDim.x) {
    const int r = i / nval, q = i - r * nval;
    const int sk = q / ncol, j = q - sk * ncol;
    const int sg = sk >> 1, k = sk & 1;
    const unsigned e = sh_ep[j >> 6];
    const long long base = x.site + (long long)(e & 1u) * W * slot;
    const uint64_t w = ((uint64_t)e << 32) | (uint64_t)__float_as_uint(v[q]);
    __hip_atomic_store(x.peers[r] + base + (long long)x.rank * slot + (long long)k * S * C +
                           (long long)sg * C + c0 + j,
                       w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  constexpr int MAXV = (kTailMaxS * 2 * kTailMaxCols + 255) / 256;
  float res[MAXV];
  const long long t0 = (long long)wall_clock64();
  bool dead = __hip_atomic_load(x.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
#pragma unroll
  for (int u = 0; u < MAXV; ++u) {
    res[u] = 0.f;
    const int q = threadIdx.x + u * (int)blockDim.x;
    if (q >= nval) continue;
    const int sk = q / ncol, j = q - sk * ncol;
    const int sg = sk >> 1, k = sk & 1;
    const unsigned e = sh_ep[j >> 6];
    const long long base = x.site + (long long)(e & 1u) * W * slot;
    const uint64_t* src = x.own + base + (long long)k * S * C + (long long)sg * C + c0 + j;
    uint64_t w[kTailMaxWorld];
#pragma unroll
    for (int r = 0; r < kTailMaxWorld; ++r)
      if (r < W) w[r] = __hip_atomic_load(src + r * slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // poll every pending slot per round (the rank loop is unrolled: w stays in registers with
    // static indices — no M0-relative gpr_idx addressing, see tools/isa_check.py)
    while (true) {
      bool pending = false;
#pragma unroll
      for (int r = 0; r < kTailMaxWorld; ++r)
        if (r < W && (unsigned)(w[r] >> 32) != e) {
          pending = true;
          w[r] = __hip_atomic_load(src + r * slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      if (!pending) break;
      if (dead || (long long)wall_clock64() - t0 > 200000000LL) {
        __hip_atomic_store(x.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dead = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < kTailMaxWorld; ++r)
      if (r < W) a += __uint_as_float((uint32_t)w[r]);
    res[u] = a;
  }
  __syncthreads();  // every thread done reading its local values before v is overwritten
#pragma unroll
  for (int u = 0; u < MAXV; ++u) {
    const int q = threadIdx.x + u * (int)blockDim.x;
    if (q < nval) v[q] = res[u];
  }
  __syncthreads();
}

// Finalize one channel c from the global per-segment sums g1/g2 (and, for dγ / dβ in mode 2,
// the rank-local sums l1/l2).  Same math as bn.hip k_bn_reduce_fused modes 1 / 2 (SyncBN's
// batch_norm_gather_stats_with_counts / batch_norm_backward_reduce, reference main.py:176).
__device__ inline void bn_fin_col(const BnFin& f, int c, const float* g1, const float* g2,
                                  const float* l1, const float* l2) {
  const int S = f.S, C = f.C;
  if (f.mode == 1) {
    float rm = f.rm ? f.rm[c] : 0.f, rv = f.rv ? f.rv[c] : 0.f;
    const float unbias = f.count > 1.f ? f.count / (f.count - 1.f) : 1.f;
    // compile-time trip count: a runtime-indexed register array would need M0-relative
    // (gpr_idx) addressing, which the opaque-DMA kernels must not use (tools/isa_check.py)
#pragma unroll
    for (int sg = 0; sg < kTailMaxS; ++sg) {
      if (sg >= S) break;
      const float mean = g1[sg] / f.count;
      float var = g2[sg] / f.count - mean * mean;
      var = var > 0.f ? var : 0.f;
      const float inv = rsqrtf(var + f.eps);
      f.mi[sg * C + c] = mean;
      f.mi[S * C + sg * C + c] = inv;
      if (f.ss != nullptr) {
        const float sc = (f.gamma ? f.gamma[c] : 1.f) * inv;
        f.ss[sg * C + c] = sc;
        f.ss[S * C + sg * C + c] = (f.beta ? f.beta[c] : 0.f) - mean * sc;
      }
      rm = (1.f - f.momentum) * rm + f.momentum * mean;
      rv = (1.f - f.momentum) * rv + f.momentum * var * unbias;
    }
    if (f.rm) f.rm[c] = rm;
    if (f.rv) f.rv[c] = rv;
  } else {
    const float gm = f.gamma ? f.gamma[c] : 1.f;
    float dg = 0.f, db = 0.f;
#pragma unroll
    for (int sg = 0; sg < kTailMaxS; ++sg) {
      if (sg >= S) break;
      db += l1[sg];
      dg += l2[sg];
      const float mean = f.mi[sg * C + c], inv = f.mi[S * C + sg * C + c];
      const float A = gm * inv;
      const float bb = g1[sg] / f.count, c2 = g2[sg] / f.count;
      f.coef[sg * C + c] = A;
      f.coef[S * C + sg * C + c] = -A * c2 * inv;
      f.coef[2 * S * C + sg * C + c] = -A * bb + A * c2 * inv * mean;
    }
    if (f.dgamma) f.dgamma[c] = dg;
    if (f.dbeta) f.dbeta[c] = db;
  }
}
