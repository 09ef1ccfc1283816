// Segmented (per-view) cross-replica BatchNorm for bf16 NHWC activations on gfx950.
//
// Replaces SyncBatchNorm's batch_norm_stats / gather_stats_with_counts / batch_norm_elemt and
// the backward_reduce / backward_elemt pair (torch/nn/modules/_functions.py:39-170) that the
// reference runs once per view per layer (/root/reference/main.py:112-113,176).
// Layout: x is [R, C] (R = S segments x Rs rows, C % 8 == 0), 16-byte vector accesses,
// per-thread fixed channel chunk so scale/shift live in registers, fp32 math, deterministic
// two-level reductions (block partials, then one reduce pass) — no float atomics.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

// partial layout: [S][nblk][2][C]
__global__ __launch_bounds__(256) void k_bn_stats(const uint16_t* __restrict__ x, int Rs, int C,
                                                  int nblk, float* __restrict__ partial) {
  const int TPR = C / 8 < 256 ? C / 8 : 256;
  const int RPB = 256 / TPR;
  const int seg = blockIdx.y;
  const int blk = blockIdx.x;
  const int tid = threadIdx.x;
  const int cchunk0 = tid % TPR;
  const int rlane = tid / TPR;
  __shared__ float red[256 * 2 * 8 / 8 * 8];  // [RPB][C chunk of this pass][2]
  const int rows_per_blk = (Rs + nblk - 1) / nblk;
  const int rbeg = blk * rows_per_blk;
  const int rend = min(Rs, rbeg + rows_per_blk);
  const uint16_t* xs = x + (size_t)seg * Rs * C;
  for (int cc = cchunk0; cc < C / 8; cc += TPR) {
    float s1[8], s2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
    if (rlane < RPB) {
      // rows >= rend read as zero through the buffer descriptor: they add nothing
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          (void*)xs, (short)0, (int)(uint32_t)((size_t)rend * C * 2), 0x00020000);
      for (int r0 = rbeg + rlane; r0 < rend; r0 += RPB * 4) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          v[u] = __builtin_amdgcn_raw_buffer_load_b128(
              rx, (uint32_t)(((size_t)(r0 + u * RPB) * C + cc * 8) * 2), 0, 0);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float a = lo_bf(v[u][e]), b = hi_bf(v[u][e]);
            s1[2 * e] += a; s2[2 * e] += a * a;
            s1[2 * e + 1] += b; s2[2 * e + 1] += b * b;
          }
      }
    }
    // reduce over RPB row lanes through LDS: red[rlane][cchunk][e][2]
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[((rlane * TPR + cchunk0) * 8 + e) * 2 + 0] = s1[e];
      red[((rlane * TPR + cchunk0) * 8 + e) * 2 + 1] = s2[e];
    }
    __syncthreads();
    // TPR*8 channels handled in this pass; threads cover them
    for (int t = tid; t < TPR * 8; t += 256) {
      float a = 0.f, b = 0.f;
      for (int r = 0; r < RPB; ++r) {
        a += red[(r * TPR * 8 + t) * 2 + 0];
        b += red[(r * TPR * 8 + t) * 2 + 1];
      }
      const int c = (cc - cchunk0) * 8 + t;  // channel base of this pass + t
      float* dst = partial + (((size_t)seg * nblk + blk) * 2) * C;
      dst[c] = a;
      dst[C + c] = b;
    }
  }
}

// Level-1 slice of a [S][nblk][2][C] partial array: one block = 64 channels x both halves
// (Σ, Σ²) = 32 float4 columns x 8 row lanes, summing rows [beg, end) of segment s.  16-byte loads
// and several rows in flight per thread: a 4 MB partial is read by a few hundred blocks in ~1 µs
// of DRAM time, so the pass is latency-bound and wants bytes-in-flight (guide §3, R3).
// Returns (in threads 0..31) the float4 sum of column j = tid: half = j >> 4, c = cg*64 + (j&15)*4.
__device__ __forceinline__ float4 l1_slice(const float* __restrict__ partial, int nblk, int C,
                                           int s, int cg, int beg, int end, float4 (*red)[32]) {
  const int j = threadIdx.x & 31;
  const int rl = threadIdx.x >> 5;
  const int c4 = cg * 64 + (j & 15) * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c4 < C) {
    const float* src = partial + (size_t)s * nblk * 2 * C + (j >> 4) * C + c4;
    // batches of U rows per thread, every load of a batch issued before the first is summed
    // (rows ascending per thread, as before: the same sums bit for bit).  The plain loop was
    // compiled as 4-deep load groups: one dependent ~µs trip per 4 rows of a cold slice
    constexpr int U = 8;
    for (int i0 = beg + rl; i0 < end; i0 += 8 * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = i0 + 8 * u < end ? *(const float4*)(src + (size_t)(i0 + 8 * u) * 2 * C)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
      }
    }
  }
  red[rl][j] = acc;
  __syncthreads();
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (threadIdx.x < 32) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {  // fixed order: deterministic
      const float4 v = red[q][j];
      r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    }
  }
  return r;
}

// Level 1: grid (ceil(C/64), S, G); each block sums a G-th of one segment's partial rows for 64
// channels -> level-2 partials [S][G][2][C].  Order of summation fixed => deterministic.
__global__ __launch_bounds__(256) void k_reduce_partials_l1(const float* __restrict__ partial,
                                                            int nblk, int S, int C, int G,
                                                            float* __restrict__ l2) {
  __shared__ float4 red[8][32];
  const int s = blockIdx.y, gz = blockIdx.z, cg = blockIdx.x;
  const int per = (nblk + G - 1) / G;
  const int beg = gz * per;
  const int end = min(nblk, beg + per);
  const float4 r = l1_slice(partial, nblk, C, s, cg, beg, end, red);
  const int j = threadIdx.x;
  const int c4 = cg * 64 + (j & 15) * 4;
  if (j < 32 && c4 < C)
    *(float4*)(l2 + (((size_t)s * G + gz) * 2) * C + (j >> 4) * C + c4) = r;
}

// Level 2: stats[2][S][C] = Σ_g l2[s][g][*][c]
__global__ void k_reduce_partials(const float* __restrict__ partial, int nblk, int S, int C,
                                  float* __restrict__ stats) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // over S*C
  if (idx >= S * C) return;
  const int s = idx / C, c = idx % C;
  float a = 0.f, b = 0.f;
  const float* src = partial + (size_t)s * nblk * 2 * C;
#pragma unroll 8
  for (int i = 0; i < nblk; ++i) {
    a += src[(size_t)i * 2 * C + c];
    b += src[(size_t)i * 2 * C + C + c];
  }
  stats[(size_t)s * C + c] = a;           // [2][S][C]
  stats[(size_t)S * C + s * C + c] = b;
}

// ---------------------------------------------------------------------------------------------
// One-launch BatchNorm reduction: partial [S][nblk][2][C] -> (per mode)
//   mode 0: stats [2][S][C]                    (the cross-rank all-reduce input)
//   mode 1: forward finalize (mean/invstd, scale/shift, running stats, num_batches_tracked)
//   mode 2: backward finalize (dγ, dβ, coef [3][S][C])
// Grid (ceil(C/64), S, G): every block sums a G-th of one segment's partial rows for 64
// channels into ws [S][G][2][C]; the last of the S·G blocks of a channel group to arrive (agent-
// scope release/acquire around a per-group ticket, cdna_hip_programming.md §5 item 2) sums the
// G slices in fixed order and finalizes: deterministic, and three launches become one.
// Tickets live in a persistent zeroed array; the last arriver resets its own ticket, so the op
// must stay on one stream (it does: the compute stream).
struct BnReduceArgs {
  const float* partial;
  int nblk, S, C, G, mode, direct;
  float* ws;
  unsigned* tickets;
  float* stats;  // mode 0 out
  // mode 1
  float count, eps, momentum;
  float* running_mean;
  float* running_var;
  float* mi;  // mode 1 out / mode 2 in
  int64_t* nbt;
  const float* gamma;
  const float* beta;
  float* ss;
  // mode 2
  float* dgamma;
  float* dbeta;
  float* coef;
  // IPC exchange (world > 1): see bn_ipc_exchange
  uint64_t* const* peers;
  uint64_t* own;
  long long site;
  unsigned* epoch;
  int* err;
  int world, rank;
};

constexpr int kMaxSeg = 4;  // BatchNorm segments (views) per launch handled by the reducer
constexpr int kMaxWorld = 16;

// Cross-rank sum of one channel group's [S][2][64] BatchNorm sums, replacing SyncBatchNorm's
// all_gather / all_reduce (reference main.py:176 → torch/nn/modules/_functions.py:74,159) for
// the latency-bound statistics exchange: no RCCL launch, no separate reduce / finalize kernels.
// Every rank's arena (fine-grained, uncached device memory, mapped into every peer with
// hipIpcOpenMemHandle) holds, per BatchNorm site, [parity][rank][2][S][C] 8-byte LL words:
// the float's bits in the low half and the exchange epoch in the high half, so one 64-bit
// store publishes value and flag together — no fence, no release/acquire, no L2 write-back
// (the reader spins on each word until its epoch matches).  The last-arriving block of the
// channel group pushes its slot to all ranks (system-scope relaxed stores through the peer
// mappings), then waits for the W slots in its own arena and sums them in rank order, so every
// rank finalizes from bitwise-identical statistics.  The epoch is a per-(site, group) counter
// that advances once per call on every rank (SPMD order); parity double-buffers the region so
// a rank running one call ahead never overwrites a slot a slower rank is still reading.  A
// bounded spin sets *err and continues rather than hang the GPU if a peer never arrives.
__device__ void bn_ipc_exchange(const BnReduceArgs& p, int cg, float (*fin)[2][64],
                                unsigned* sh_epoch) {
  const int S = p.S, C = p.C, W = p.world;
  if (threadIdx.x == 0) {
    const unsigned e = p.epoch[cg] + 1u;
    p.epoch[cg] = e;
    *sh_epoch = e;
  }
  __syncthreads();
  const unsigned e = *sh_epoch;
  const long long slot = 2LL * S * C;                 // words per rank slot
  const long long base = p.site + (long long)(e & 1u) * W * slot;
  const int nval = S * 2 * 64;                        // this group's values
  // push: value v = (sg, k, cl) to word [k][sg][c] of slot `rank` in every arena
  for (int i = threadIdx.x; i < W * nval; i += blockDim.x) {
    const int r = i / nval, v = i - r * nval;
    const int sg = v / 128, k = (v >> 6) & 1, cl = v & 63;
    const int c = cg * 64 + cl;
    if (c >= C) continue;
    const uint64_t w = ((uint64_t)e << 32) | (uint64_t)__float_as_uint(fin[sg][k][cl]);
    uint64_t* dst = p.peers[r] + base + (long long)p.rank * slot + (long long)k * S * C +
                    (long long)sg * C + c;
    __hip_atomic_store(dst, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // gather: every rank's word for this group, summed in rank order (identical on all ranks);
  // all W loads of a value are in flight before the first is checked
  static_assert(2 * kMaxSeg * 64 <= 2 * 256, "two values per thread at most");
  float res[2] = {0.f, 0.f};
  // wall-clock bound (100 MHz constant counter): 2 s per exchange, and none at all once an
  // earlier exchange timed out — a lost peer costs seconds, never a hung GPU
  const long long t0 = (long long)wall_clock64();
  bool dead = __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int v = threadIdx.x + j * 256;
    const int sg = v / 128, k = (v >> 6) & 1, cl = v & 63;
    const int c = cg * 64 + cl;
    if (v >= nval || c >= C) continue;
    const uint64_t* src = p.own + base + (long long)k * S * C + (long long)sg * C + c;
    uint64_t w[kMaxWorld];
#pragma unroll
    for (int r = 0; r < kMaxWorld; ++r)
      if (r < W) w[r] = __hip_atomic_load(src + r * slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // poll every pending slot per round (unrolled rank loop: w stays in registers)
    while (true) {
      bool pending = false;
#pragma unroll
      for (int r = 0; r < kMaxWorld; ++r)
        if (r < W && (unsigned)(w[r] >> 32) != e) {
          pending = true;
          w[r] = __hip_atomic_load(src + r * slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      if (!pending) break;
      if (dead || (long long)wall_clock64() - t0 > 200000000LL) {
        __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dead = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < kMaxWorld; ++r)
      if (r < W) a += __uint_as_float((uint32_t)w[r]);
    res[j] = a;
  }
  __syncthreads();  // every thread done reading its local sums before fin is overwritten
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int v = threadIdx.x + j * 256;
    const int sg = v / 128, k = (v >> 6) & 1, cl = v & 63;
    if (v < nval && cg * 64 + cl < C) fin[sg][k][cl] = res[j];
  }
  __syncthreads();
}

// IPC: the cross-rank exchange is compiled only into the world > 1 instantiation, so the
// single-GPU kernel keeps its small register / argument footprint
template <bool IPC>
__global__ __launch_bounds__(256) void k_bn_reduce_fused(BnReduceArgs p) {
  __shared__ float4 red4[kMaxSeg * 8][32];
  __shared__ float fin[kMaxSeg][2][64];
  __shared__ int last;
  const int cl = threadIdx.x & 63;
  const int lane = threadIdx.x >> 6;
  const int cg = blockIdx.x;
  const int c = cg * 64 + cl;
  const int C = p.C, S = p.S;
  int G = p.G;
  const float* src2 = p.ws;  // level-2 rows [S][G][2][C]
  if (p.direct) {
    // few partial rows: one block per channel group reads them all, no slices / ticket
    src2 = p.partial;
    G = p.nblk;
  } else {
  const int s = blockIdx.y, gz = blockIdx.z;
  const int per = (p.nblk + G - 1) / G;
  const int beg = gz * per;
  const int end = min(p.nblk, beg + per);
  const float4 r = l1_slice(p.partial, p.nblk, C, s, cg, beg, end, red4);
  // ---- publish this slice write-through (sc1: agent-scope relaxed atomic stores), so no
  // release fence is needed — an agent release would write back this XCD's whole dirty L2,
  // which right after a conv epilogue is megabytes (guide §6 Guideline 16, R1)
  {
    const int j = threadIdx.x;
    const int c4 = cg * 64 + (j & 15) * 4;
    if (j < 32 && c4 < C) {
      float* dst = p.ws + (((size_t)s * G + gz) * 2) * C + (j >> 4) * C + c4;
      __hip_atomic_store(dst + 0, r.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dst + 1, r.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dst + 2, r.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dst + 3, r.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old =
        __hip_atomic_fetch_add(&p.tickets[cg], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == (unsigned)(S * G - 1);
    if (last)  // reset for the next launch (stream-ordered)
      __hip_atomic_store(&p.tickets[cg], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  // consumer: no agent acquire — every slice was stored sc1 and drained before its block's
  // ticket add, and the last arriver reads every one of them with sc1 loads (L1 bypass;
  // guide §6 Guideline 16 Rule, MI355X_MICROARCH.md visibility table row 1: ticket form, the
  // other waves behind the barrier above), which saves the acquire's ~1.7 µs.  Every (segment,
  // slice) row of the 64-channel group is loaded at once by all 256 threads and combined
  // through LDS in a fixed order
  }  // !direct
  {
    const int j = threadIdx.x & 31, rl = threadIdx.x >> 5;
    const int c4 = cg * 64 + (j & 15) * 4;
    float4 acc[kMaxSeg];
#pragma unroll
    for (int sg = 0; sg < kMaxSeg; ++sg) acc[sg] = make_float4(0.f, 0.f, 0.f, 0.f);
    // one code path per load form (the cache-policy operand is an immediate): a per-load
    // select between them was compiled load -> wait -> load, serialising the batch
    const bool handoff = !p.direct;
    const float* rb = handoff ? p.ws : p.partial;
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)rb, (short)0, (int)((size_t)S * G * 2 * C * 4), 0x00020000);
    auto sum_rows = [&](auto aux) {
      constexpr int AUX = decltype(aux)::value;
      if (c4 >= C) return;
      const int base = (j >> 4) * C + c4;  // float offset of this thread's row-0 element
      constexpr int U = 4;
      for (int g0 = rl; g0 < G; g0 += 8 * U) {
        u32x4 v[kMaxSeg][U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int g = g0 + 8 * u;
#pragma unroll
          for (int sg = 0; sg < kMaxSeg; ++sg) {
            const bool ok = sg < S && g < G;
            // out-of-range rows read an offset past the resource: the buffer load returns 0
            const int off = ok ? (int)(((size_t)(sg * G + g) * 2 * C + base) * 4) : 0x7fffffff;
            v[sg][u] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, AUX);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int sg = 0; sg < kMaxSeg; ++sg) {
            acc[sg].x += __uint_as_float(v[sg][u][0]); acc[sg].y += __uint_as_float(v[sg][u][1]);
            acc[sg].z += __uint_as_float(v[sg][u][2]); acc[sg].w += __uint_as_float(v[sg][u][3]);
          }
        }
      }
    };
    if (handoff)
      sum_rows(std::integral_constant<int, 16>{});  // sc1
    else
      sum_rows(std::integral_constant<int, 0>{});
#pragma unroll
    for (int sg = 0; sg < kMaxSeg; ++sg) red4[sg * 8 + rl][j] = acc[sg];  // red4: [kMaxSeg*8][32]
  }
  __syncthreads();
  if (threadIdx.x < 32 * S) {
    const int j = threadIdx.x & 31, sg = threadIdx.x >> 5;
    float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 v = red4[sg * 8 + q][j];
      r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    }
    float* f = &fin[sg][j >> 4][(j & 15) * 4];
    f[0] = r.x; f[1] = r.y; f[2] = r.z; f[3] = r.w;
  }
  __syncthreads();
  float dg = 0.f, db = 0.f;
  if (IPC && p.world > 1 && p.mode != 0) {
    // SyncBN semantics: dγ, dβ are per-rank (summed later by the gradient all-reduce), the
    // normalisation statistics / input-gradient coefficients use the global sums
    if (p.mode == 2 && lane == 0 && c < C)
      for (int sg = 0; sg < S; ++sg) { db += fin[sg][0][cl]; dg += fin[sg][1][cl]; }
    __shared__ unsigned sh_epoch;
    bn_ipc_exchange(p, cg, fin, &sh_epoch);
  }
  if (p.mode == 1 && c == 0 && lane == 0 && p.nbt != nullptr) p.nbt[0] += S;  // one per view
  if (lane != 0 || c >= C) return;
  float rm = 0.f, rv = 0.f, gm = 1.f;
  const bool local_dgb = !(IPC && p.world > 1);
  if (p.mode == 1) {
    rm = p.running_mean ? p.running_mean[c] : 0.f;
    rv = p.running_var ? p.running_var[c] : 0.f;
  }
  if (p.mode == 2) gm = p.gamma ? p.gamma[c] : 1.f;
  const float unbias = p.count > 1.f ? p.count / (p.count - 1.f) : 1.f;
  for (int sg = 0; sg < S; ++sg) {
    const float s1 = fin[sg][0][cl], s2 = fin[sg][1][cl];
    if (p.mode == 0) {
      p.stats[sg * C + c] = s1;
      p.stats[S * C + sg * C + c] = s2;
      db += s1;  // written only when dβ / dγ outputs are given (BN-backward partials)
      dg += s2;
    } else if (p.mode == 1) {
      const float mean = s1 / p.count;
      float var = s2 / p.count - mean * mean;
      var = var > 0.f ? var : 0.f;
      const float inv = rsqrtf(var + p.eps);
      p.mi[sg * C + c] = mean;
      p.mi[S * C + sg * C + c] = inv;
      if (p.ss != nullptr) {
        const float sc = (p.gamma ? p.gamma[c] : 1.f) * inv;
        p.ss[sg * C + c] = sc;
        p.ss[S * C + sg * C + c] = (p.beta ? p.beta[c] : 0.f) - mean * sc;
      }
      rm = (1.f - p.momentum) * rm + p.momentum * mean;
      rv = (1.f - p.momentum) * rv + p.momentum * var * unbias;
    } else {
      if (local_dgb) {
        db += s1;
        dg += s2;
      }
      const float mean = p.mi[sg * C + c], inv = p.mi[S * C + sg * C + c];
      const float A = gm * inv;
      const float bb = s1 / p.count, c2 = s2 / p.count;
      p.coef[sg * C + c] = A;
      p.coef[S * C + sg * C + c] = -A * c2 * inv;
      p.coef[2 * S * C + sg * C + c] = -A * bb + A * c2 * inv * mean;
    }
  }
  if (lane != 0 || c >= C) return;
  if (p.mode == 1) {
    if (p.running_mean) p.running_mean[c] = rm;
    if (p.running_var) p.running_var[c] = rv;
  } else {
    if (p.dgamma) p.dgamma[c] = dg;
    if (p.dbeta) p.dbeta[c] = db;
  }
}

// stats [2][S][C] -> mean_invstd [2][S][C]; sequential running-stat updates per segment
// Optionally also the fused-apply table ss [2][S][C]: scale = γ·invstd, shift = β − mean·scale.
__global__ void k_bn_finalize(const float* __restrict__ stats, int S, int C, float count, float eps,
                              float momentum, float* running_mean, float* running_var,
                              float* __restrict__ mi, int64_t* nbt, const float* __restrict__ gamma,
                              const float* __restrict__ beta, float* __restrict__ ss) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt != nullptr) nbt[0] += S;  // num_batches_tracked: one per view
  if (c >= C) return;
  float rm = running_mean ? running_mean[c] : 0.f;
  float rv = running_var ? running_var[c] : 0.f;
  const float unbias = count > 1.f ? count / (count - 1.f) : 1.f;
  for (int s = 0; s < S; ++s) {
    const float mean = stats[s * C + c] / count;
    float var = stats[S * C + s * C + c] / count - mean * mean;
    var = var > 0.f ? var : 0.f;
    const float inv = rsqrtf(var + eps);
    mi[s * C + c] = mean;
    mi[S * C + s * C + c] = inv;
    if (ss != nullptr) {
      const float sc = (gamma ? gamma[c] : 1.f) * inv;
      ss[s * C + c] = sc;
      ss[S * C + s * C + c] = (beta ? beta[c] : 0.f) - mean * sc;
    }
    rm = (1.f - momentum) * rm + momentum * mean;
    rv = (1.f - momentum) * rv + momentum * var * unbias;
  }
  if (running_mean) running_mean[c] = rm;
  if (running_var) running_var[c] = rv;
}

// grid (nbx, S): segment-uniform scale/shift in registers, U rows in flight per thread through
// raw buffer loads (out-of-range rows read as zero, so the loads need no branches).
constexpr int UNR = 4;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(uint32_t)bytes, 0x00020000);
}

__global__ __launch_bounds__(256) void k_bn_apply(const uint16_t* __restrict__ x,
                                                  const uint16_t* __restrict__ res,
                                                  uint16_t* __restrict__ y,
                                                  const float* __restrict__ mi,
                                                  const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, int R, int C,
                                                  int S, int relu) {
  const int CH = C / 8;
  const int TPR = CH < 256 ? CH : 256;
  const int RPB = 256 / TPR;
  const int Rs = R / S;
  const int seg = blockIdx.y;
  const int cc0 = threadIdx.x % TPR;
  const int rl = threadIdx.x / TPR;
  if (rl >= RPB) return;
  const size_t sbase = (size_t)seg * Rs * C;
  const size_t sbytes = (size_t)Rs * C * 2;
  const __amdgpu_buffer_rsrc_t rx = rsrc(x + sbase, sbytes);
  const __amdgpu_buffer_rsrc_t rr = rsrc(res ? res + sbase : x + sbase, sbytes);
  for (int cc = cc0; cc < CH; cc += TPR) {
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = cc * 8 + e;
      const float mean = mi[seg * C + c], inv = mi[S * C + seg * C + c];
      const float g = gamma ? gamma[c] : 1.f;
      const float b = beta ? beta[c] : 0.f;
      sc[e] = g * inv;
      sh[e] = b - mean * g * inv;
    }
    for (int r0 = blockIdx.x * RPB * UNR + rl; r0 < Rs; r0 += gridDim.x * RPB * UNR) {
      u32x4 v[UNR], rv[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const uint32_t off = (uint32_t)(((size_t)(r0 + u * RPB) * C + cc * 8) * 2);
        v[u] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
        if (res) rv[u] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = r0 + u * RPB;
        if (r >= Rs) break;
        float o[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[2 * e] = lo_bf(v[u][e]) * sc[2 * e] + sh[2 * e];
          o[2 * e + 1] = hi_bf(v[u][e]) * sc[2 * e + 1] + sh[2 * e + 1];
        }
        if (res) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[2 * e] += lo_bf(rv[u][e]);
            o[2 * e + 1] += hi_bf(rv[u][e]);
          }
        }
        if (relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = fmaxf(o[e], 0.f);
        }
        u32x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = pack2bf(o[2 * e], o[2 * e + 1]);
        *(u32x4*)(y + sbase + (size_t)r * C + cc * 8) = w;
      }
    }
  }
}

// y = relu?(x·sc + sh [+ res | + res·rsc + rsh]) with precomputed [2][S][C] tables: the
// block-output apply of the fused ResNet executor (BN3 + downsample-BN + residual + ReLU in one
// pass; neither BN output is materialised separately).
template <int RES>  // 0 none, 1 plain residual, 2 affine residual
__global__ __launch_bounds__(256) void k_bn_apply_ss(const uint16_t* __restrict__ x,
                                                     const float* __restrict__ ss,
                                                     const uint16_t* __restrict__ res,
                                                     const float* __restrict__ rss,
                                                     uint16_t* __restrict__ y,
                                                     uint8_t* __restrict__ mask, int R, int C,
                                                     int S, int relu) {
  const int CH = C / 8;
  const int TPR = CH < 256 ? CH : 256;
  const int RPB = 256 / TPR;
  const int Rs = R / S;
  const int seg = blockIdx.y;
  const int cc0 = threadIdx.x % TPR;
  const int rl = threadIdx.x / TPR;
  if (rl >= RPB) return;
  const size_t sbase = (size_t)seg * Rs * C;
  const size_t sbytes = (size_t)Rs * C * 2;
  const __amdgpu_buffer_rsrc_t rx = rsrc(x + sbase, sbytes);
  const __amdgpu_buffer_rsrc_t rr = rsrc(RES ? res + sbase : x + sbase, sbytes);
  for (int cc = cc0; cc < CH; cc += TPR) {
    float sc[8], sh[8], rsc[8], rsh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = cc * 8 + e;
      sc[e] = ss[seg * C + c];
      sh[e] = ss[(S + seg) * C + c];
      if (RES == 2) {
        rsc[e] = rss[seg * C + c];
        rsh[e] = rss[(S + seg) * C + c];
      }
    }
    for (int r0 = blockIdx.x * RPB * UNR + rl; r0 < Rs; r0 += gridDim.x * RPB * UNR) {
      u32x4 v[UNR], rv[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const uint32_t off = (uint32_t)(((size_t)(r0 + u * RPB) * C + cc * 8) * 2);
        v[u] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
        if (RES) rv[u] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = r0 + u * RPB;
        if (r >= Rs) break;
        float o[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[2 * e] = lo_bf(v[u][e]) * sc[2 * e] + sh[2 * e];
          o[2 * e + 1] = hi_bf(v[u][e]) * sc[2 * e + 1] + sh[2 * e + 1];
          if (RES == 1) {
            o[2 * e] += lo_bf(rv[u][e]);
            o[2 * e + 1] += hi_bf(rv[u][e]);
          } else if (RES == 2) {
            o[2 * e] += lo_bf(rv[u][e]) * rsc[2 * e] + rsh[2 * e];
            o[2 * e + 1] += hi_bf(rv[u][e]) * rsc[2 * e + 1] + rsh[2 * e + 1];
          }
        }
        if (relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = fmaxf(o[e], 0.f);
        }
        u32x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = pack2bf(o[2 * e], o[2 * e + 1]);
        *(u32x4*)(y + sbase + (size_t)r * C + cc * 8) = w;
        if (mask != nullptr) {  // bit e = (y[c0 + e] > 0): the ReLU mask at 1/16 of y's bytes
          unsigned bits = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) bits |= (o[e] > 0.f ? 1u : 0u) << e;
          mask[(sbase + (size_t)r * C) / 8 + cc] = (uint8_t)bits;
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_bn_apply_eval(const uint16_t* __restrict__ x,
                                                       const uint16_t* __restrict__ res,
                                                       uint16_t* __restrict__ y,
                                                       const float* __restrict__ rmean,
                                                       const float* __restrict__ rvar,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps,
                                                       int R, int C, int relu) {
  const int CH = C / 8;
  const size_t total = (size_t)R * CH;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CH);
    const u32x4 v = *(const u32x4*)(x + i * 8);
    u32x4 rv = {0, 0, 0, 0};
    if (res) rv = *(const u32x4*)(res + i * 8);
    u32x4 w;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float o2[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = cc * 8 + 2 * e + h;
        const float inv = rsqrtf(rvar[c] + eps);
        const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
        float xv = h ? hi_bf(v[e]) : lo_bf(v[e]);
        float o = (xv - rmean[c]) * inv * g + b;
        if (res) o += h ? hi_bf(rv[e]) : lo_bf(rv[e]);
        if (relu) o = fmaxf(o, 0.f);
        o2[h] = o;
      }
      w[e] = pack2bf(o2[0], o2[1]);
    }
    *(u32x4*)(y + i * 8) = w;
  }
}

// Σg and Σg·x̂ partials, g = dy * (y > 0 if relu). partial layout [S][nblk][2][C]
__global__ __launch_bounds__(256) void k_bn_bwd_reduce(const uint16_t* __restrict__ dy,
                                                       const uint16_t* __restrict__ y,
                                                       const uint16_t* __restrict__ x,
                                                       const float* __restrict__ mi, int Rs,
                                                       int C, int S, int relu, int nblk,
                                                       float* __restrict__ partial) {
  const int TPR = C / 8 < 256 ? C / 8 : 256;
  const int RPB = 256 / TPR;
  const int seg = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x;
  const int cchunk0 = tid % TPR, rlane = tid / TPR;
  __shared__ float red[256 * 2 * 8];
  const int rows_per_blk = (Rs + nblk - 1) / nblk;
  const int rbeg = blk * rows_per_blk;
  const int rend = min(Rs, rbeg + rows_per_blk);
  const size_t base = (size_t)seg * Rs * C;
  for (int cc = cchunk0; cc < C / 8; cc += TPR) {
    float s1[8], s2[8], mean[8], inv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] = 0.f; s2[e] = 0.f;
      mean[e] = mi[seg * C + cc * 8 + e];
      inv[e] = mi[S * C + seg * C + cc * 8 + e];
    }
    if (rlane < RPB) {
      // rows >= rend read as zero (dy = 0 contributes nothing)
      const uint32_t nb = (uint32_t)((size_t)rend * C * 2);
      const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(dy + base),
                                                                          (short)0, (int)nb, 0x00020000);
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)(x + base),
                                                                          (short)0, (int)nb, 0x00020000);
      const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((relu ? y : x) + base), (short)0, (int)nb, 0x00020000);
      for (int r0 = rbeg + rlane; r0 < rend; r0 += RPB * 4) {
        u32x4 vd[4], vx[4], vy[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t off = (uint32_t)(((size_t)(r0 + u * RPB) * C + cc * 8) * 2);
          vd[u] = __builtin_amdgcn_raw_buffer_load_b128(rd, off, 0, 0);
          vx[u] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
          if (relu) vy[u] = __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int k = 2 * e + h;
              float g = h ? hi_bf(vd[u][e]) : lo_bf(vd[u][e]);
              if (relu) {
                const float yy = h ? hi_bf(vy[u][e]) : lo_bf(vy[u][e]);
                g = yy > 0.f ? g : 0.f;
              }
              const float xh = ((h ? hi_bf(vx[u][e]) : lo_bf(vx[u][e])) - mean[k]) * inv[k];
              s1[k] += g;
              s2[k] += g * xh;
            }
          }
      }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[((rlane * TPR + cchunk0) * 8 + e) * 2 + 0] = s1[e];
      red[((rlane * TPR + cchunk0) * 8 + e) * 2 + 1] = s2[e];
    }
    __syncthreads();
    for (int t = tid; t < TPR * 8; t += 256) {
      float a = 0.f, b = 0.f;
      for (int r = 0; r < RPB; ++r) {
        a += red[(r * TPR * 8 + t) * 2 + 0];
        b += red[(r * TPR * 8 + t) * 2 + 1];
      }
      const int c = (cc - cchunk0) * 8 + t;
      float* dst = partial + (((size_t)seg * nblk + blk) * 2) * C;
      dst[c] = a;
      dst[C + c] = b;
    }
  }
}

// sums [2][S][C] (Σg, Σg·x̂, already all-reduced) -> dγ, dβ (summed over segments) and
// coef [3][S][C] with dx = A·g + B·x + D
__global__ void k_bn_bwd_finalize(const float* __restrict__ sums, const float* __restrict__ mi,
                                  const float* __restrict__ gamma, int S, int C, float count,
                                  float* dgamma, float* dbeta, float* __restrict__ coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float dg = 0.f, db = 0.f;
  const float gm = gamma ? gamma[c] : 1.f;
  for (int s = 0; s < S; ++s) {
    const float sg = sums[s * C + c], sgx = sums[S * C + s * C + c];
    db += sg;
    dg += sgx;
    const float mean = mi[s * C + c], inv = mi[S * C + s * C + c];
    const float A = gm * inv;
    const float b = sg / count, c2 = sgx / count;
    coef[s * C + c] = A;
    coef[S * C + s * C + c] = -A * c2 * inv;
    coef[2 * S * C + s * C + c] = -A * b + A * c2 * inv * mean;
  }
  if (dgamma) dgamma[c] = dg;
  if (dbeta) dbeta[c] = db;
}

__global__ __launch_bounds__(256) void k_bn_bwd_apply(const uint16_t* __restrict__ dy,
                                                      const uint16_t* __restrict__ y,
                                                      const uint16_t* __restrict__ x,
                                                      const float* __restrict__ coef, int R,
                                                      int C, int S, int relu,
                                                      uint16_t* __restrict__ dx,
                                                      uint16_t* __restrict__ dres) {
  const int CH = C / 8;
  const int TPR = CH < 256 ? CH : 256;
  const int RPB = 256 / TPR;
  const int Rs = R / S;
  const int seg = blockIdx.y;
  const int cc0 = threadIdx.x % TPR;
  const int rl = threadIdx.x / TPR;
  if (rl >= RPB) return;
  const size_t sbase = (size_t)seg * Rs * C;
  const size_t sbytes = (size_t)Rs * C * 2;
  const __amdgpu_buffer_rsrc_t rd = rsrc(dy + sbase, sbytes);
  const __amdgpu_buffer_rsrc_t rx = rsrc(x + sbase, sbytes);
  const __amdgpu_buffer_rsrc_t ry = rsrc(relu ? y + sbase : x + sbase, sbytes);
  for (int cc = cc0; cc < CH; cc += TPR) {
    float A[8], B[8], D[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = cc * 8 + e;
      A[e] = coef[seg * C + c];
      B[e] = coef[S * C + seg * C + c];
      D[e] = coef[2 * S * C + seg * C + c];
    }
    for (int r0 = blockIdx.x * RPB * UNR + rl; r0 < Rs; r0 += gridDim.x * RPB * UNR) {
      u32x4 vd[UNR], vx[UNR], vy[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const uint32_t off = (uint32_t)(((size_t)(r0 + u * RPB) * C + cc * 8) * 2);
        vd[u] = __builtin_amdgcn_raw_buffer_load_b128(rd, off, 0, 0);
        vx[u] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
        if (relu) vy[u] = __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = r0 + u * RPB;
        if (r >= Rs) break;
        u32x4 wdx, wg;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float o[2], gg[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int k = 2 * e + h;
            float g = h ? hi_bf(vd[u][e]) : lo_bf(vd[u][e]);
            if (relu) {
              const float yy = h ? hi_bf(vy[u][e]) : lo_bf(vy[u][e]);
              g = yy > 0.f ? g : 0.f;
            }
            const float xv = h ? hi_bf(vx[u][e]) : lo_bf(vx[u][e]);
            o[h] = A[k] * g + B[k] * xv + D[k];
            gg[h] = g;
          }
          wdx[e] = pack2bf(o[0], o[1]);
          wg[e] = pack2bf(gg[0], gg[1]);
        }
        const size_t off = sbase + (size_t)r * C + cc * 8;
        *(u32x4*)(dx + off) = wdx;
        if (dres) *(u32x4*)(dres + off) = wg;
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_bn_bwd_apply2(const uint16_t* __restrict__ g,
                                                       const uint16_t* __restrict__ x1,
                                                       const float* __restrict__ coef1,
                                                       uint16_t* __restrict__ dx1,
                                                       const uint16_t* __restrict__ x2,
                                                       const float* __restrict__ coef2,
                                                       uint16_t* __restrict__ dx2, int R, int C,
                                                       int S) {
  const int CH = C / 8;
  const int TPR = CH < 256 ? CH : 256;
  const int RPB = 256 / TPR;
  const int Rs = R / S;
  const int seg = blockIdx.y;
  const int cc0 = threadIdx.x % TPR;
  const int rl = threadIdx.x / TPR;
  if (rl >= RPB) return;
  const size_t sbase = (size_t)seg * Rs * C;
  const size_t sbytes = (size_t)Rs * C * 2;
  const __amdgpu_buffer_rsrc_t rg = rsrc(g + sbase, sbytes);
  const __amdgpu_buffer_rsrc_t r1 = rsrc(x1 + sbase, sbytes);
  const __amdgpu_buffer_rsrc_t r2 = rsrc(x2 + sbase, sbytes);
  for (int cc = cc0; cc < CH; cc += TPR) {
    float A1[8], B1[8], D1[8], A2[8], B2[8], D2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = cc * 8 + e;
      A1[e] = coef1[seg * C + c]; B1[e] = coef1[(S + seg) * C + c]; D1[e] = coef1[(2 * S + seg) * C + c];
      A2[e] = coef2[seg * C + c]; B2[e] = coef2[(S + seg) * C + c]; D2[e] = coef2[(2 * S + seg) * C + c];
    }
    for (int r0 = blockIdx.x * RPB * UNR + rl; r0 < Rs; r0 += gridDim.x * RPB * UNR) {
      u32x4 vg[UNR], v1[UNR], v2[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const uint32_t off = (uint32_t)(((size_t)(r0 + u * RPB) * C + cc * 8) * 2);
        vg[u] = __builtin_amdgcn_raw_buffer_load_b128(rg, off, 0, 0);
        v1[u] = __builtin_amdgcn_raw_buffer_load_b128(r1, off, 0, 0);
        v2[u] = __builtin_amdgcn_raw_buffer_load_b128(r2, off, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = r0 + u * RPB;
        if (r >= Rs) break;
        u32x4 w1, w2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float g0 = lo_bf(vg[u][e]), g1 = hi_bf(vg[u][e]);
          w1[e] = pack2bf(A1[2 * e] * g0 + B1[2 * e] * lo_bf(v1[u][e]) + D1[2 * e],
                          A1[2 * e + 1] * g1 + B1[2 * e + 1] * hi_bf(v1[u][e]) + D1[2 * e + 1]);
          w2[e] = pack2bf(A2[2 * e] * g0 + B2[2 * e] * lo_bf(v2[u][e]) + D2[2 * e],
                          A2[2 * e + 1] * g1 + B2[2 * e + 1] * hi_bf(v2[u][e]) + D2[2 * e + 1]);
        }
        const size_t off = sbase + (size_t)r * C + cc * 8;
        *(u32x4*)(dx1 + off) = w1;
        *(u32x4*)(dx2 + off) = w2;
      }
    }
  }
}

int apply_grid(int R, int C, int S) {
  const int CH = C / 8;
  const int TPR = CH < 256 ? CH : 256;
  const int RPB = 256 / TPR;
  const int Rs = R / S;
  int blocks = (Rs + RPB * UNR - 1) / (RPB * UNR);
  // ~2 iterations of UNR rows per thread; cap the grid at ~8 blocks per CU per segment
  blocks = (blocks + 1) / 2;
  const int cap = 2048 / S;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  return blocks;
}

}  // namespace

int bn_stats_blocks_per_seg(int R, int C, int S) {
  const int Rs = R / S;
  const int CH = C / 8;
  const int TPR = CH < 256 ? CH : 256;
  const int RPB = 256 / TPR;
  // aim for ~1024 blocks total with >= 8 row-iterations per thread
  int nblk = 1024 / S;
  const int max_blk = Rs / (RPB * 8);
  if (nblk > max_blk) nblk = max_blk;
  if (nblk < 1) nblk = 1;
  return nblk;
}

void bn_stats_partial(const uint16_t* x, int R, int C, int S, float* partial, int* nblk_out,
                      hipStream_t s) {
  const int nblk = bn_stats_blocks_per_seg(R, C, S);
  if (nblk_out) *nblk_out = nblk;
  hipLaunchKernelGGL(k_bn_stats, dim3(nblk, S), dim3(256), 0, s, x, R / S, C, nblk, partial);
  HIP_CHECK_LAUNCH();
}

// measured: the one-pass (direct) reduce wins only for the smallest partials
int bn_reduce_direct_rows() { return 64; }

int bn_reduce_groups(int nblk) {
  // measured (tools/bench_reduce.py, r2): few slices beat many — the per-group ticket
  // atomics serialise and the consumer reads all
  constexpr int rows = 128, cap = 16;
  if (nblk <= rows) return 1;
  int g = (nblk + rows - 1) / rows;  // ~rows partial rows per level-1 block
  return g > cap ? cap : g;
}

void bn_reduce_partials(const float* partial, int nblk, int S, int C, float* stats, float* ws,
                        hipStream_t s) {
  const int n = S * C;
  const int G = bn_reduce_groups(nblk);
  if (G > 1) {
    hipLaunchKernelGGL(k_reduce_partials_l1, dim3((C + 63) / 64, S, G), dim3(256), 0, s, partial,
                       nblk, S, C, G, ws);
    HIP_CHECK_LAUNCH();
    partial = ws;
    nblk = G;
  }
  hipLaunchKernelGGL(k_reduce_partials, dim3((n + 255) / 256), dim3(256), 0, s, partial, nblk, S, C,
                     stats);
  HIP_CHECK_LAUNCH();
}

void bn_finalize(const float* stats, int S, int C, float count, float eps, float momentum,
                 float* running_mean, float* running_var, float* mean_invstd, int64_t* nbt,
                 const float* gamma, const float* beta, float* scale_shift, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_finalize, dim3((C + 255) / 256), dim3(256), 0, s, stats, S, C, count, eps,
                     momentum, running_mean, running_var, mean_invstd, nbt, gamma, beta,
                     scale_shift);
  HIP_CHECK_LAUNCH();
}

void bn_reduce_fused(const BnReduceFusedParams& q, hipStream_t s) {
  BnReduceArgs a{};
  a.partial = q.partial; a.nblk = q.nblk; a.S = q.S; a.C = q.C; a.mode = q.mode;
  a.G = bn_reduce_groups(q.nblk);
  a.direct = q.nblk <= bn_reduce_direct_rows();
  a.ws = q.ws; a.tickets = q.tickets; a.stats = q.stats;
  a.count = q.count; a.eps = q.eps; a.momentum = q.momentum;
  a.running_mean = q.running_mean; a.running_var = q.running_var; a.mi = q.mi; a.nbt = q.nbt;
  a.gamma = q.gamma; a.beta = q.beta; a.ss = q.ss;
  a.dgamma = q.dgamma; a.dbeta = q.dbeta; a.coef = q.coef;
  a.peers = q.ipc_peers; a.own = q.ipc_own; a.site = q.ipc_site; a.epoch = q.ipc_epoch;
  a.err = q.ipc_err; a.world = q.world; a.rank = q.rank;
  const dim3 grid = a.direct ? dim3((q.C + 63) / 64) : dim3((q.C + 63) / 64, q.S, a.G);
  if (a.world > 1 && a.peers != nullptr)
    hipLaunchKernelGGL(k_bn_reduce_fused<true>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_bn_reduce_fused<false>, grid, dim3(256), 0, s, a);
  HIP_CHECK_LAUNCH();
}

void bn_apply_ss(const uint16_t* x, const float* ss, const uint16_t* res, const float* rss,
                 uint16_t* y, uint8_t* mask, int R, int C, int S, int relu, hipStream_t s) {
  const dim3 grid(apply_grid(R, C, S), S);
  if (res == nullptr)
    hipLaunchKernelGGL(k_bn_apply_ss<0>, grid, dim3(256), 0, s, x, ss, res, rss, y, mask, R, C, S,
                       relu);
  else if (rss == nullptr)
    hipLaunchKernelGGL(k_bn_apply_ss<1>, grid, dim3(256), 0, s, x, ss, res, rss, y, mask, R, C, S,
                       relu);
  else
    hipLaunchKernelGGL(k_bn_apply_ss<2>, grid, dim3(256), 0, s, x, ss, res, rss, y, mask, R, C, S,
                       relu);
  HIP_CHECK_LAUNCH();
}

void bn_apply(const uint16_t* x, const uint16_t* res, uint16_t* y, const float* mi,
              const float* gamma, const float* beta, int R, int C, int S, int relu,
              hipStream_t s) {
  hipLaunchKernelGGL(k_bn_apply, dim3(apply_grid(R, C, S), S), dim3(256), 0, s, x, res, y, mi, gamma,
                     beta, R, C, S, relu);
  HIP_CHECK_LAUNCH();
}

void bn_apply_eval(const uint16_t* x, const uint16_t* res, uint16_t* y, const float* rmean,
                   const float* rvar, const float* gamma, const float* beta, float eps, int R,
                   int C, int relu, hipStream_t s) {
  const size_t total = (size_t)R * (C / 8);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_bn_apply_eval, dim3(blocks), dim3(256), 0, s, x, res, y, rmean, rvar, gamma,
                     beta, eps, R, C, relu);
  HIP_CHECK_LAUNCH();
}

void bn_bwd_reduce(const uint16_t* dy, const uint16_t* y, const uint16_t* x, const float* mi, int R,
                   int C, int S, int relu, float* partial, hipStream_t s) {
  const int nblk = bn_stats_blocks_per_seg(R, C, S);
  hipLaunchKernelGGL(k_bn_bwd_reduce, dim3(nblk, S), dim3(256), 0, s, dy, y, x, mi, R / S, C, S,
                     relu, nblk, partial);
  HIP_CHECK_LAUNCH();
}

void bn_bwd_finalize(const float* sums, const float* mi, const float* gamma, int S, int C,
                     float count, float* dgamma, float* dbeta, float* coef, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_bwd_finalize, dim3((C + 255) / 256), dim3(256), 0, s, sums, mi, gamma, S,
                     C, count, dgamma, dbeta, coef);
  HIP_CHECK_LAUNCH();
}

void bn_bwd_apply(const uint16_t* dy, const uint16_t* y, const uint16_t* x, const float* coef,
                  int R, int C, int S, int relu, uint16_t* dx, uint16_t* dres, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_bwd_apply, dim3(apply_grid(R, C, S), S), dim3(256), 0, s, dy, y, x, coef, R, C,
                     S, relu, dx, dres);
  HIP_CHECK_LAUNCH();
}

void bn_bwd_apply2(const uint16_t* g, const uint16_t* x1, const float* coef1, uint16_t* dx1,
                   const uint16_t* x2, const float* coef2, uint16_t* dx2, int R, int C, int S,
                   hipStream_t s) {
  hipLaunchKernelGGL(k_bn_bwd_apply2, dim3(apply_grid(R, C, S), S), dim3(256), 0, s, g, x1, coef1,
                     dx1, x2, coef2, dx2, R, C, S);
  HIP_CHECK_LAUNCH();
}
