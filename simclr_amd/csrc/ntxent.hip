// Fused NT-Xent (normalised temperature-scaled cross entropy) on gfx950, exact fp32 via the
// f32-input MFMA v_mfma_f32_16x16x4_f32 (cdna_hip_programming.md §3 'FP32-input MFMA').
//
// Reference: /root/reference/loss.py:33-65 — L2-normalise both views, three N×N GEMMs, two
// boolean-mask copies, two concats and two cross-entropies.  Mathematically
// (verified in SURVEY) that is the textbook NT-Xent over 2N anchors: for anchor i the logits are
// s_ij = ẑ_i·ẑ_j / τ over all j ≠ i, the target is the other view of the same image.
//
// Here the similarity matrix is never materialised:
//   fwd   : per 16-anchor tile × column split, S tiles on MFMA, online log-sum-exp, the positive
//           logit picked in-register; a finish kernel merges the splits -> per-row LSE, loss.
//   bwd   : dS = g·(softmax − onehot(pos)) recomputed tile by tile and immediately contracted with
//           the other side's ẑ on MFMA ("owned"/"partner" formulation: the row pass gives
//           Σ_j dS_ij ẑ_j, the column pass Σ_i dS_ij ẑ_i), splits summed by a reduce kernel,
//           then the normalisation backward.
// Columns may be the local rows (reference semantics) or an all-gather of every rank's ẑ
// (``loss.gather``): rows are then columns [col_offset, col_offset+R) of the gathered set.
//
// Data: zn [Ccols][D] fp32 row-major and znT [D][Ccols] fp32 (both produced by the normalise /
// transpose kernels), D % 4 == 0, D <= 256; R % 16 == 0, Ccols % 16 == 0.
#include "common.h"
#include "kernels.h"

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int pos_col(int r_local, int n_local, int col_offset) {
  return col_offset + (r_local < n_local ? r_local + n_local : r_local - n_local);
}

// z [R][D] bf16 -> zn [R][D] fp32 normalised, inv_norm [R]; one wave per row
__global__ void k_normalize(const uint16_t* __restrict__ z, int R, int D, float* __restrict__ zn,
                            float* __restrict__ inv_norm) {
  const int row = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (row >= R) return;
  float ss = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float v = bf2f(z[(size_t)row * D + d]);
    ss += v * v;
  }
  ss = wave_sum(ss);
  const float nrm = sqrtf(ss);
  const float inv = 1.f / fmaxf(nrm, 1e-12f);  // F.normalize eps
  for (int d = lane; d < D; d += 64) zn[(size_t)row * D + d] = bf2f(z[(size_t)row * D + d]) * inv;
  if (lane == 0) inv_norm[row] = inv;
}

// in [R][D] -> out [D][ldo] at columns [c0, c0 + R)
__global__ void k_transpose(const float* __restrict__ in, float* __restrict__ out, int R, int D,
                            int ldo, int c0) {
  __shared__ float t[32][33];
  const int r0 = blockIdx.x * 32, d0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: ty 0..7
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, d = d0 + tx;
    t[k][tx] = (r < R && d < D) ? in[(size_t)r * D + d] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int d = d0 + k, r = r0 + tx;
    if (d < D && r < R) out[(size_t)d * ldo + c0 + r] = t[tx][k];
  }
}

// S^T tile [partner q (16)][owned o (16)] = Σ_k Z[q][k] Z[o][k]; lane gets (q = 4g+i, o = li)
template <int D>
__device__ __forceinline__ f32x4_t sim_tile(const float* __restrict__ znT, int Ccols, int q0,
                                            const float* breg) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, li = lane & 15;
  f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
  constexpr int ksteps = D / 4;
#pragma unroll
  for (int ks = 0; ks < ksteps; ks += 2) {
    const float aq0 = znT[(size_t)(4 * ks + g) * Ccols + q0 + li];
    const float aq1 = znT[(size_t)(4 * (ks + 1) + g) * Ccols + q0 + li];
    a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(aq0, breg[ks], a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(aq1, breg[ks + 1], a1, 0, 0, 0);
  }
  return a0 + a1;
}

// Forward: grid (R/16, splits), one wave per block. Owned = anchor rows [r0, r0+16) (local),
// partners = columns [c_beg, c_end). Writes part[split][r][3] = (max, sumexp, pos logit or -inf)
template <int D>
__global__ __launch_bounds__(64) void k_ntxent_fwd(const float* __restrict__ znT, int R, int Ccols,
                                                   int col_offset, int n_local,
                                                   float inv_temp, int cols_per_split,
                                                   float* __restrict__ part, int c_lo, int c_hi,
                                                   int split_base) {
  const int lane = threadIdx.x;
  const int g = lane >> 4, li = lane & 15;
  const int r0 = blockIdx.x * 16;
  const int split = split_base + blockIdx.y;
  const int c_beg = c_lo + blockIdx.y * cols_per_split;
  int c_end = c_beg + cols_per_split;
  if (c_end > c_hi) c_end = c_hi;
  float breg[D / 4];
#pragma unroll
  for (int ks = 0; ks < D / 4; ++ks)
    breg[ks] = znT[(size_t)(4 * ks + g) * Ccols + col_offset + r0 + li];
  const int my_r = r0 + li;  // owned row of this lane (o = li)
  const int self_c = col_offset + my_r;
  const int pos_c = pos_col(my_r, n_local, col_offset);
  float m = -INFINITY, l = 0.f, spos = -INFINITY;
  for (int q0 = c_beg; q0 < c_end; q0 += 16) {
    const f32x4_t s = sim_tile<D>(znT, Ccols, q0, breg);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = q0 + 4 * g + i;
      const float v = s[i] * inv_temp;
      if (c == pos_c) spos = v;
      if (c != self_c) {
        if (v > m) {
          l = l * __expf(m - v) + 1.f;
          m = v;
        } else {
          l += __expf(v - m);
        }
      }
    }
  }
  // merge across the 4 lane groups (g) holding the same row
#pragma unroll
  for (int off = 16; off < 64; off <<= 1) {
    const float m2 = __shfl_xor(m, off, 64);
    const float l2 = __shfl_xor(l, off, 64);
    const float p2 = __shfl_xor(spos, off, 64);
    const float mn = fmaxf(m, m2);
    l = (mn == -INFINITY) ? 0.f : l * __expf(m - mn) + l2 * __expf(m2 - mn);
    m = mn;
    spos = fmaxf(spos, p2);
  }
  if (g == 0) {
    float* dst = part + ((size_t)split * R + my_r) * 3;
    dst[0] = m;
    dst[1] = l;
    dst[2] = spos;
  }
}

// merge splits -> lse[r], loss[r]
__global__ void k_ntxent_finish(const float* __restrict__ part, int R, int splits,
                                float* __restrict__ lse, float* __restrict__ loss) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  float m = -INFINITY, l = 0.f, sp = -INFINITY;
  for (int s = 0; s < splits; ++s) {
    const float* p = part + ((size_t)s * R + r) * 3;
    const float mn = fmaxf(m, p[0]);
    if (mn != -INFINITY) l = l * __expf(m - mn) + p[1] * __expf(p[0] - mn);
    m = mn;
    sp = fmaxf(sp, p[2]);
  }
  const float ls = m + logf(l);
  lse[r] = ls;
  loss[r] = ls - sp;
}

// Backward (owned/partner). ROW mode: owned = local anchor rows (lse by owned), partners =
// columns. COL mode: owned = columns [o0..), partners = local anchor rows (lse by partner).
// out[split][owned][D] += Σ_q w(q,o) ẑ_q ; w = gscale·(exp(s−lse_anchor) − [col==pos(anchor)])
template <bool ROW, int D>
__global__ __launch_bounds__(64) void k_ntxent_bwd(const float* __restrict__ zn,
                                                   const float* __restrict__ znT,
                                                   const float* __restrict__ lse, int R,
                                                   int Ccols, int col_offset, int n_local,
                                                   float inv_temp, float gscale,
                                                   const float* __restrict__ gout,
                                                   int partners_per_split,
                                                   float* __restrict__ out) {
  const int lane = threadIdx.x;
  const int g = lane >> 4, li = lane & 15;
  const int o0 = blockIdx.x * 16;  // ROW: local row index; COL: column index
  const int split = blockIdx.y;
  const int nown = ROW ? R : Ccols;
  const int npart = ROW ? Ccols : R;
  const int q_beg = split * partners_per_split;
  int q_end = q_beg + partners_per_split;
  if (q_end > npart) q_end = npart;
  const float gs = gscale * (gout ? gout[0] : 1.f);
  // owned operand (B of the similarity MFMA): column index in znT of owned item li
  const int own_col = ROW ? (col_offset + o0 + li) : (o0 + li);
  float breg[D / 4];
#pragma unroll
  for (int ks = 0; ks < D / 4; ++ks) breg[ks] = znT[(size_t)(4 * ks + g) * Ccols + own_col];
  float lse_own = 0.f;
  int self_c = -1, pos_c = -1;
  if (ROW) {
    const int r = o0 + li;
    lse_own = lse[r];
    self_c = col_offset + r;
    pos_c = pos_col(r, n_local, col_offset);
  }
  constexpr int nd = D / 16;
  f32x4_t acc[nd];
#pragma unroll
  for (int t = 0; t < nd; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  for (int q0 = q_beg; q0 < q_end; q0 += 16) {
    const int qcol0 = ROW ? q0 : (col_offset + q0);  // partner column index in znT / zn
    const f32x4_t s = sim_tile<D>(znT, Ccols, qcol0, breg);
    float w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = s[i] * inv_temp;
      if (ROW) {
        const int c = q0 + 4 * g + i;
        const float p = (c == self_c) ? 0.f : __expf(v - lse_own);
        w[i] = gs * (p - (c == pos_c ? 1.f : 0.f));
      } else {
        const int r = q0 + 4 * g + i;        // anchor (local row)
        const int c = o0 + li;               // owned column
        const float la = lse[r];
        const int sc = col_offset + r;
        const int pc = pos_col(r, n_local, col_offset);
        const float p = (c == sc) ? 0.f : __expf(v - la);
        w[i] = gs * (p - (c == pc ? 1.f : 0.f));
      }
    }
    // acc[o][d] += Σ_q w(q,o) Z[q][d]: A[o=li][k=g] = w[t] (q = 4g+t), B[k=g][d=li] = Z[q][d]
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float* zrow = zn + (size_t)(qcol0 + 4 * g + t) * D + li;
#pragma unroll
      for (int dt = 0; dt < nd; ++dt)
        acc[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[t], zrow[dt * 16], acc[dt], 0, 0, 0);
    }
  }
  // lane holds out[o = 4g+i][d = dt*16 + li]
  float* dst = out + (size_t)split * nown * D;
#pragma unroll
  for (int dt = 0; dt < nd; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dst[(size_t)(o0 + 4 * g + i) * D + dt * 16 + li] = acc[dt][i] * inv_temp;
}

// out[r][d] = Σ_s part[s][r][d]   (n elems per split)
__global__ void k_sum_splits(const float* __restrict__ part, int splits, size_t n,
                             float* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += part[(size_t)k * n + i];
    out[i] = s;
  }
}

// dz = (dẑ − ẑ (ẑ·dẑ)) · inv_norm ; one wave per row
__global__ void k_normalize_bwd(const float* __restrict__ zn, const float* __restrict__ inv_norm,
                                const float* __restrict__ dzn, int R, int D,
                                uint16_t* __restrict__ dz_bf16, float* __restrict__ dz_f32) {
  const int row = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (row >= R) return;
  float dot = 0.f;
  for (int d = lane; d < D; d += 64) dot += zn[(size_t)row * D + d] * dzn[(size_t)row * D + d];
  dot = wave_sum(dot);
  const float inv = inv_norm[row];
  for (int d = lane; d < D; d += 64) {
    const size_t i = (size_t)row * D + d;
    const float v = (dzn[i] - zn[i] * dot) * inv;
    if (dz_bf16) dz_bf16[i] = f2bf(v);
    if (dz_f32) dz_f32[i] = v;
  }
}

__global__ void k_reduce_loss(const float* __restrict__ loss, int R, float scale,
                              float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < R; i += blockDim.x) s += loss[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    out[0] = t * scale;
  }
}

// One-wave blocks, latency-bound on their L2 operand loads: each block should walk about 8
// partner tiles (128 columns), with at least 512 blocks (so the SIMDs have waves to switch
// between) and at most 4096 (the split partials grow with the count).  tools/ntxent_bench.py,
// R = 1024: at 8192 global negatives (8 ranks) the fixed 512-block rule took 85 + 107 + 327 µs
// (forward, column and row gradient passes), this one ~57 + 78 + 94; at 1024 columns it keeps
// 512.
int splits_for(int tiles, int ptiles, int tiles_per_block = 8) {
  long target = (long)tiles * ptiles / tiles_per_block;
  target = target < 512 ? 512 : (target > 4096 ? 4096 : target);
  int s = (int)((target + tiles - 1) / tiles);
  if (s > ptiles) s = ptiles;
  if (s < 1) s = 1;
  return s;
}

}  // namespace

// ------------------------------------------------------------------- host API (raw pointers)
void ntxent_normalize_f32(const uint16_t* z, int R, int D, float* zn, float* inv_norm,
                          hipStream_t s) {
  hipLaunchKernelGGL(k_normalize, dim3((R + 3) / 4), dim3(256), 0, s, z, R, D, zn, inv_norm);
  HIP_CHECK_LAUNCH();
}

void ntxent_transpose_cols(const float* in, float* out, int R, int D, int ldo, int c0,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_transpose, dim3((R + 31) / 32, (D + 31) / 32), dim3(256), 0, s, in, out, R,
                     D, ldo, c0);
  HIP_CHECK_LAUNCH();
}

void ntxent_transpose(const float* in, float* out, int R, int D, hipStream_t s) {
  ntxent_transpose_cols(in, out, R, D, R, 0, s);
}

// measured optimum (tools/ntxent_bench.py, 8192 columns): ~16 partner tiles per block for the
// forward (57 µs vs 74 at 8) and the column pass (73 vs 78), ~8 for the row pass (93 vs 110)
int ntxent_fwd_splits(int R, int Ccols) { return splits_for(R / 16, Ccols / 16, 16); }
int ntxent_bwd_splits(int nown, int npart) {
  return splits_for(nown / 16, npart / 16, nown <= npart ? 8 : 16);
}

// columns [c_lo, c_hi) of znT into splits [split_base, split_base + splits) of part
void ntxent_forward_range(const float* znT, int R, int Ccols, int D, int col_offset, int n_local,
                          float inv_temp, float* part, int c_lo, int c_hi, int splits,
                          int split_base, hipStream_t s) {
  const int ptiles = (c_hi - c_lo) / 16;
  const int per = ((ptiles + splits - 1) / splits) * 16;
#define FWD_CASE(DD)                                                                        \
  case DD:                                                                                  \
    hipLaunchKernelGGL(k_ntxent_fwd<DD>, dim3(R / 16, splits), dim3(64), 0, s, znT, R, Ccols, \
                       col_offset, n_local, inv_temp, per, part, c_lo, c_hi, split_base);   \
    break;
  switch (D) {
    FWD_CASE(32) FWD_CASE(64) FWD_CASE(128) FWD_CASE(256)
    default: fprintf(stderr, "ntxent: unsupported D=%d\n", D); abort();
  }
#undef FWD_CASE
  HIP_CHECK_LAUNCH();
}

void ntxent_finish(const float* part, int R, int splits, float* lse, float* loss, hipStream_t s) {
  hipLaunchKernelGGL(k_ntxent_finish, dim3((R + 255) / 256), dim3(256), 0, s, part, R, splits, lse,
                     loss);
  HIP_CHECK_LAUNCH();
}

void ntxent_forward(const float* znT, int R, int Ccols, int D, int col_offset, int n_local,
                    float inv_temp, float* part, int splits, float* lse, float* loss,
                    hipStream_t s) {
  ntxent_forward_range(znT, R, Ccols, D, col_offset, n_local, inv_temp, part, 0, Ccols, splits, 0,
                       s);
  ntxent_finish(part, R, splits, lse, loss, s);
}

void ntxent_backward_part(int row_mode, const float* zn, const float* znT, const float* lse, int R,
                          int Ccols, int D, int col_offset, int n_local, float inv_temp,
                          float gscale, const float* gout, float* part, int splits, float* out,
                          hipStream_t s) {
  const int nown = row_mode ? R : Ccols;
  const int npart = row_mode ? Ccols : R;
  const int ptiles = npart / 16;
  const int per = ((ptiles + splits - 1) / splits) * 16;
#define BWD_CASE(DD)                                                                          \
  case DD:                                                                                    \
    if (row_mode)                                                                             \
      hipLaunchKernelGGL((k_ntxent_bwd<true, DD>), dim3(nown / 16, splits), dim3(64), 0, s, zn, \
                         znT, lse, R, Ccols, col_offset, n_local, inv_temp, gscale, gout, per,  \
                         part);                                                               \
    else                                                                                      \
      hipLaunchKernelGGL((k_ntxent_bwd<false, DD>), dim3(nown / 16, splits), dim3(64), 0, s,    \
                         zn, znT, lse, R, Ccols, col_offset, n_local, inv_temp, gscale, gout,   \
                         per, part);                                                          \
    break;
  switch (D) {
    BWD_CASE(32) BWD_CASE(64) BWD_CASE(128) BWD_CASE(256)
    default: fprintf(stderr, "ntxent: unsupported D=%d\n", D); abort();
  }
#undef BWD_CASE
  HIP_CHECK_LAUNCH();
  const size_t n = (size_t)nown * D;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_sum_splits, dim3(blocks), dim3(256), 0, s, part, splits, n, out);
  HIP_CHECK_LAUNCH();
}

void ntxent_normalize_backward(const float* zn, const float* inv_norm, const float* dzn, int R,
                               int D, uint16_t* dz_bf16, float* dz_f32, hipStream_t s) {
  hipLaunchKernelGGL(k_normalize_bwd, dim3((R + 3) / 4), dim3(256), 0, s, zn, inv_norm, dzn, R, D,
                     dz_bf16, dz_f32);
  HIP_CHECK_LAUNCH();
}

void ntxent_reduce_loss(const float* loss_rows, int R, float scale, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce_loss, dim3(1), dim3(1024), 0, s, loss_rows, R, scale, out);
  HIP_CHECK_LAUNCH();
}
