// Host-side launchers of the simclr_amd gfx950 kernels (raw pointers + stream; no torch types,
// so the .hip translation units compile without the ATen headers).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

// Conv geometry for the implicit GEMM (see conv.hip / conv_hip.py for the derivations).
struct ConvGeom {
  int Nb, IH, IW, C;        // gathered input tensor NHWC (C % 8 == 0)
  int OH, OW;               // logical output grid (rows M = Nb*OH*OW)
  int KH, KW;               // taps
  int ish, isw, dh, dw;     // input = (oh*ish + kh*dh + ih0, ow*isw + kw*dw + iw0)
  int ih0, iw0;
  int N;                    // output channels (GEMM N)
  int OHp, OWp, osh, osw, ooh, oow, ldo;  // physical output mapping
};

// ---- conv.hip
// Optional fusions around the implicit GEMM (all pointers nullable / mode 0 = off).
struct ConvFusion {
  const float* pro_sc = nullptr;  // A/X-operand prologue: a = relu?(x*sc[seg][c] + sh[seg][c])
  const float* pro_sh = nullptr;
  int pro_seg_rows = 0;           // rows per segment (BM must divide it for igemm)
  int pro_relu = 0;
  int pro_S = 1;
  const float* pro_d = nullptr;   // igemm BN-backward prologue: a = sc·A + sh·A2 + d
  const uint16_t* A2 = nullptr;   //   second A-operand tensor (same geometry as A)
  const float* pro_rsc = nullptr; // igemm block-output prologue (pro_out != nullptr): a =
  const float* pro_rsh = nullptr; //   relu(A·sc + sh + A2·rsc + rsh), A2 = residual (rsc null:
  uint16_t* pro_out = nullptr;    //   identity), a and its ReLU bitmask stored to pro_out /
  uint8_t* pro_mask = nullptr;    //   pro_mask
  const uint16_t* dY2 = nullptr;  // wgrad dY-operand BN-backward prologue (coef [3][S][N])
  const float* dp_coef = nullptr;
  int dp_seg_rows = 0, dp_S = 1;
  int epi_mode = 0;               // igemm: 1 out = acc + a; 2 out = acc + (b > 0 ? a : 0);
  int epi_a_sub = 0;              // epi_a is the stride-2 subsampled [Nb][ceil(OH/2)][ceil(OW/2)][ldo]
                                  // tensor (a stride-2 1x1 downsample's compact dgrad): 0 at odd (oh, ow)
                                  // 3 out = (b*sc+sh > 0 ? acc : 0) + BN-bwd partials
                                  // 4 out = (b > 0 ? acc + a : 0) + BN-bwd partials vs c
  const uint16_t* epi_a = nullptr;
  const uint16_t* epi_b = nullptr;
  const uint16_t* epi_c = nullptr;  // mode 4: pre-BN activation for x̂
  const uint8_t* epi_mask = nullptr;  // mode 4: ReLU bitmask of the block input (see bn_apply_ss)
  const uint16_t* epi_c2 = nullptr;   // mode 4: second x̂ source (producer's downsample BN input)
  const float* epi_mi2 = nullptr;     //   and its mean/invstd [2][S][N]
  float* stats2 = nullptr;            //   partials Σg, Σg·x̂2 (layout of stats)
  const float* epi_ss = nullptr;  // mode 3: [2][S][N] scale/shift
  const float* epi_mi = nullptr;  // mode 3/4: [2][S][N] mean/invstd
  int epi_S = 1;
  int seg_rows = 0;               // rows per segment of the output (stats remap, mode 3)
  int stats_seg_blocks = 0;       // >0: segment-major stats rows (see conv.hip)
  int stats_base = 0;
};

int igemm_num_variants();
int igemm_variant_bm(int v);
int igemm_variant_bn(int v);
int igemm_default_variant(int N);
bool igemm_variant_glds(int v);  // LDS-DMA variant (see igemm_glds_ok)
bool igemm_glds_ok(const ConvGeom& g, bool pro, bool bn_bwd_pro);
// can tile variant v run this geometry with these operand prologues (single source of truth for
// the bindings' checks and the Python autotuner's candidate lists)
bool igemm_variant_is_patch(int v);
bool igemm_variant_ok(int v, const ConvGeom& g, bool pro, bool bn_bwd_pro);
bool igemm_dual_ok(int v, const ConvGeom& g);
bool igemm_variant_patch(int v);  // the LDS-resident-patch 3x3 kernel
bool igemm_patch_ok(const ConvGeom& g);  // block-output prologue (see igemm_glds)
int igemm_block_m(int N);
void conv_igemm_nt(const ConvGeom& g, const uint16_t* A, size_t a_elems, const uint16_t* B,
                   uint16_t* out, const float* bias, float* stats, const ConvFusion& f,
                   int variant, hipStream_t s);
int wgrad_num_variants();
// wgrad_xp's step-affine X addressing: set the mode (>= 0) and/or return it (SIMCLR_WGRAD_XLIN)
int wgrad_xlin(int mode);
int wgrad_default_variant(int N);
bool wgrad_variant_glds(int v);  // LDS-DMA variant (see wgrad_variant_ok)
int wgrad_variant_area(int v);   // output tile elements (BCO x BKK)
bool wgrad_variant_ok(int v, const ConvGeom& g, bool pro, bool dy_pro);
int wgrad_splits(const ConvGeom& g, int variant);
void conv_wgrad(const ConvGeom& g, const uint16_t* dY, const uint16_t* X, size_t x_elems,
                float* partial, int splits, float* out, int Creal, float beta,
                const ConvFusion& f, int variant, hipStream_t s);
// fused 1x1 backward (dgrad + wgrad + BN2-backward partials in one pass, Co = 256, Ci = 64)
size_t conv1x1_bwd_dual_lds();
void conv1x1_bwd_dual(const uint16_t* G, const uint16_t* A3, const float* coef, const uint16_t* X,
                      const float* xss, const float* xmi, const uint16_t* Wt, uint16_t* gm,
                      float* stats, float* wpart, int M, int CO, int CI, int S, int bps,
                      hipStream_t s, const uint16_t* Xraw = nullptr, bool dual8 = false);
void conv1x1_bwd_dual_s2(const uint16_t* G, const uint16_t* A3, const float* coef,
                         const uint16_t* X, const uint16_t* Wt, uint16_t* gm, float* wpart,
                         int Mo, int CO, int CI, int S, int bps, int H, int W, int OH, int OW,
                         hipStream_t s);
void wgrad_reduce_slabs(float* partial, int splits, float* out, size_t n, float beta,
                        hipStream_t s);
// output tiles of a weight-gradient launch (ticket words of the in-kernel split reduction)
int wgrad_tiles(const ConvGeom& g, int variant);
// one dgrad weight transform (see weight_transform_batch): Wt[ci][khs][kws][co] =
// W[co][kh0 + khs*sh][kw0 + kws*sw][ci]; blocks [blk0, blk0 + nblk) of the batch launch
struct WtDesc {
  const uint16_t* W;
  uint16_t* Wt;
  int Co, KH, KW, Ci, KHs, KWs, kh0, sh, kw0, sw, blk0, nblk;
};
static_assert(sizeof(WtDesc) == 64, "WtDesc layout");
void conv_weight_transform_batch(const WtDesc* d, int n, int total_blocks, hipStream_t s);
void conv_weight_transform(const uint16_t* W, uint16_t* Wt, int Co, int KH, int KW, int Ci,
                           int KHs, int KWs, int kh0, int sh, int kw0, int sw, hipStream_t s);

// ---- bn.hip  (x: [R, C] bf16 rows, S segments of R/S rows each)
void bn_stats_partial(const uint16_t* x, int R, int C, int S, float* partial, int* nblk_per_seg,
                      hipStream_t s);
int bn_stats_blocks_per_seg(int R, int C, int S);
int bn_reduce_groups(int nblk);  // level-1 groups; workspace = S*groups*2*C floats
int bn_reduce_direct_rows();      // bn_reduce_fused: partials with <= this many rows per segment are
                                  // reduced by one block per channel group (no slices / ticket)
void bn_reduce_partials(const float* partial, int nblk_per_seg, int S, int C, float* stats,
                        float* ws, hipStream_t s);
void bn_finalize(const float* stats, int S, int C, float count, float eps, float momentum,
                 float* running_mean, float* running_var, float* mean_invstd, int64_t* nbt,
                 const float* gamma, const float* beta, float* scale_shift, hipStream_t s);
// One-launch reduce of [S][nblk][2][C] partials + (mode 0) stats out, (1) forward finalize,
// (2) backward finalize.  ws = S*groups*2*C floats; tickets = >= ceil(C/64) zeroed uints.
struct BnReduceFusedParams {
  const float* partial = nullptr;
  int nblk = 0, S = 1, C = 0, mode = 0;
  float* ws = nullptr;
  unsigned* tickets = nullptr;
  float* stats = nullptr;
  float count = 1.f, eps = 1e-5f, momentum = 0.1f;
  float* running_mean = nullptr;
  float* running_var = nullptr;
  float* mi = nullptr;
  int64_t* nbt = nullptr;
  const float* gamma = nullptr;
  const float* beta = nullptr;
  float* ss = nullptr;
  float* dgamma = nullptr;
  float* dbeta = nullptr;
  float* coef = nullptr;
  // cross-rank exchange over IPC-mapped peer arenas (modes 1 / 2 at world > 1, see bn.hip)
  uint64_t* const* ipc_peers = nullptr;  // device array [world] of arena bases (own included)
  uint64_t* ipc_own = nullptr;           // this rank's arena base
  long long ipc_site = 0;                // word offset of this BatchNorm's region
  unsigned* ipc_epoch = nullptr;         // [ceil(C/64)] per-site exchange counters
  int* ipc_err = nullptr;                // set on a spin timeout
  int world = 1, rank = 0;
};
void bn_reduce_fused(const BnReduceFusedParams& q, hipStream_t s);
// words of one exchange region: 2 parities x world x [2][S][C] (LL words: value | epoch << 32)
inline long long bn_ipc_region_words(int world, int S, int C) {
  return 2LL * world * 2 * S * C;
}

// ---- comm.hip: one-shot IPC all-gather (op 0) / reduce-scatter (op 1) of 32-bit words over the
// peer-mapped arenas (LL words; site = 2 parities x world x n words, IPC_COLL_BLOCKS epoch
// counters)
constexpr int IPC_COLL_BLOCKS = 64;
long long ipc_coll_region_words(int world, int n);
void ipc_collective(int op, const uint32_t* src, uint32_t* dst, int n, uint64_t* const* peers,
                    uint64_t* own, long long site, unsigned* epoch, int* err, int world,
                    int rank, hipStream_t s);
// y = relu?(x*sc + sh + [res | res*rsc + rsh]); ss / rss are [2][S][C] scale/shift tables
// optional mask: uint8 [R][C/8], bit e of byte (r, c/8) = (y[r][c] > 0)
void bn_apply_ss(const uint16_t* x, const float* ss, const uint16_t* res, const float* rss,
                 uint16_t* y, uint8_t* mask, int R, int C, int S, int relu, hipStream_t s);
void bn_apply(const uint16_t* x, const uint16_t* res, uint16_t* y, const float* mean_invstd,
              const float* gamma, const float* beta, int R, int C, int S, int relu,
              hipStream_t s);
void bn_apply_eval(const uint16_t* x, const uint16_t* res, uint16_t* y, const float* rmean,
                   const float* rvar, const float* gamma, const float* beta, float eps, int R,
                   int C, int relu, hipStream_t s);
void bn_bwd_reduce(const uint16_t* dy, const uint16_t* y, const uint16_t* x,
                   const float* mean_invstd, int R, int C, int S, int relu, float* partial,
                   hipStream_t s);
void bn_bwd_finalize(const float* sums, const float* mean_invstd, const float* gamma, int S, int C,
                     float count, float* dgamma, float* dbeta, float* coef, hipStream_t s);
void bn_bwd_apply(const uint16_t* dy, const uint16_t* y, const uint16_t* x, const float* coef,
                  int R, int C, int S, int relu, uint16_t* dx, uint16_t* dres, hipStream_t s);
// two BatchNorms fed by the same gradient (residual block: last BN + downsample BN):
// dx1 = A1·g + B1·x1 + D1, dx2 = A2·g + B2·x2 + D2 in one pass over g
void bn_bwd_apply2(const uint16_t* g, const uint16_t* x1, const float* coef1, uint16_t* dx1,
                   const uint16_t* x2, const float* coef2, uint16_t* dx2, int R, int C, int S,
                   hipStream_t s);

// ---- misc.hip
void avgpool_fwd(const uint16_t* x, uint16_t* y, int Nb, int HW, int C, hipStream_t s);
void avgpool_bwd(const uint16_t* dy, uint16_t* dx, int Nb, int HW, int C, hipStream_t s);
int colsum_groups(int R);  // workspace = colsum_groups(R) * C floats
// split-K GEMM for small M: out = f(A)·Bᵀ (+ bias), f = BN + ReLU per (row segment, column)
// when sc != nullptr; part = [KS][M][N] fp32 scratch (misc.hip)
void gemm_sk(const uint16_t* A, const uint16_t* B, const float* sc, const float* sh, int seg,
             int M, int N, int K, int KS, float* part, const float* bias, uint16_t* out,
             hipStream_t s);
void colsum_bf16(const uint16_t* x, int R, int C, float* out, float beta, float* ws,
                 hipStream_t s);
void cast_f32_bf16(const float* x, uint16_t* y, size_t n, hipStream_t s);
void cast_bf16_f32(const uint16_t* x, float* y, size_t n, hipStream_t s);

// ---- ntxent.hip  (exact fp32 on v_mfma_f32_16x16x4_f32)
void ntxent_normalize_f32(const uint16_t* z, int R, int D, float* zn, float* inv_norm,
                          hipStream_t s);
void ntxent_transpose(const float* in, float* out, int R, int D, hipStream_t s);
// in [R][D] -> columns [c0, c0 + R) of out [D][ldo]
void ntxent_transpose_cols(const float* in, float* out, int R, int D, int ldo, int c0,
                           hipStream_t s);
// forward partials of the columns [c_lo, c_hi) into splits [split_base, +splits), and the merge
void ntxent_forward_range(const float* znT, int R, int Ccols, int D, int col_offset, int n_local,
                          float inv_temp, float* part, int c_lo, int c_hi, int splits,
                          int split_base, hipStream_t s);
void ntxent_finish(const float* part, int R, int splits, float* lse, float* loss, hipStream_t s);
int ntxent_fwd_splits(int R, int Ccols);
int ntxent_bwd_splits(int nown, int npart);
void ntxent_forward(const float* znT, int R, int Ccols, int D, int col_offset, int n_local,
                    float inv_temp, float* part, int splits, float* lse, float* loss,
                    hipStream_t s);
void ntxent_backward_part(int row_mode, const float* zn, const float* znT, const float* lse, int R,
                          int Ccols, int D, int col_offset, int n_local, float inv_temp,
                          float gscale, const float* gout, float* part, int splits, float* out,
                          hipStream_t s);
void ntxent_normalize_backward(const float* zn, const float* inv_norm, const float* dzn, int R,
                               int D, uint16_t* dz_bf16, float* dz_f32, hipStream_t s);
void ntxent_reduce_loss(const float* loss_rows, int R, float scale, float* out, hipStream_t s);

// ---- lars.hip (flat fp32 master / grad / momentum, bf16 shadow; per-segment table)
void lars_norms(const float* p, const float* g, const int* chunk_beg, const int* chunk_end,
                int nchunks, float grad_scale, float* norms, hipStream_t s);
void lars_update(float* p, const float* g, float* mom, uint16_t* shadow, const int* chunk_seg,
                 const int* chunk_beg, const int* chunk_end, int nchunks, const int* seg_chunk_beg,
                 const int* seg_chunk_end, const float* seg_wd, const int* seg_flags,
                 const float* norms, const float* lr_ptr, float momentum, float trust, float eps,
                 float grad_scale, int nesterov, hipStream_t s);
void lr_schedule_step(int64_t* step, float* lr_out, double lr0, int64_t warmup, int64_t total,
                      int mode, hipStream_t s);

// ---- augment.hip
void simclr_augment(const uint8_t* images, const int64_t* indices, int n, int views, int H, int W,
                    int OH, int OW, int Cpad, float strength, uint64_t seed, uint64_t counter,
                    int view_offset, int flags, uint16_t* out, float* params_out, hipStream_t s);

// ---- eval.hip: maxpool (K2), cross-entropy + top-k (K10), centroid class sums (K11)
void maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* arg, int Nb, int H, int W, int C,
                 int OH, int OW, int K, int S, int P, hipStream_t s);
void maxpool_bwd(const uint16_t* dy, const uint8_t* arg, uint16_t* dx, int Nb, int H, int W,
                 int C, int OH, int OW, int K, int S, int P, hipStream_t s);
// ImageNet stem as a 4x4 stride-1 conv: 2x2 space-to-depth of the P-padded image (C <= 4 real)
void stem_s2d(const uint16_t* img, uint16_t* xs, int Nb, int H, int W, int Cin, int creal,
              int HS, int WS, int P, hipStream_t s);
void bn_relu_maxpool(const uint16_t* a, const float* ss, int S, uint16_t* y, uint8_t* arg,
                     uint16_t* asel, int Nb, int H, int W, int C, int OH, int OW, int K, int Sd,
                     int P, hipStream_t s);
void maxpool_bwd_bn(const uint16_t* gy, const uint8_t* arg, const uint16_t* y, const uint16_t* a,
                    const float* coef, int S, uint16_t* da, int Nb, int H, int W, int C, int OH,
                    int OW, int K, int Sd, int P, hipStream_t s);
void ce_topk(const float* logits, const int64_t* y, int B, int C, float gscale, float* loss,
             int* rank, float* dlogits, hipStream_t s);
size_t class_sums_lds(int NC);
int class_sums_groups(int N);
void class_sums(const float* X, const int64_t* y, int N, int D, int NC, float* part, float* pcnt,
                float* sums, float* counts, hipStream_t s);

