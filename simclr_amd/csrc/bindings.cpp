// torch.ops.simclr_amd.* registrations for the gfx950 kernels.  Every op launches on the current
// HIP stream (so they compose with hipGraph capture and side-stream overlap) and validates the
// shapes / dtypes / devices the kernels assume before any launch (a bad shape must never reach a
// hand-written kernel: an out-of-bounds access can take the whole node down).
#include <ATen/core/Tensor.h>
#include <ATen/ops/empty.h>
#include <ATen/ops/zeros.h>
#include <ATen/hip/HIPContext.h>
#include <c10/util/Exception.h>
#include <torch/library.h>

#include <vector>

#include "kernels.h"

using at::Tensor;

namespace {

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

void check_dev(const Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, ": expected a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, ": expected dtype ", dt, " got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, ": expected a contiguous tensor");
}

const uint16_t* bf(const Tensor& t, const char* n) {
  check_dev(t, at::kBFloat16, n);
  return reinterpret_cast<const uint16_t*>(t.data_ptr());
}
uint16_t* bfw(const Tensor& t, const char* n) {
  check_dev(t, at::kBFloat16, n);
  return reinterpret_cast<uint16_t*>(t.data_ptr());
}
const float* f32(const Tensor& t, const char* n) {
  check_dev(t, at::kFloat, n);
  return t.data_ptr<float>();
}
float* f32w(const Tensor& t, const char* n) {
  check_dev(t, at::kFloat, n);
  return t.data_ptr<float>();
}
const float* optf32(const c10::optional<Tensor>& t, const char* n) {
  return (t.has_value() && t->defined()) ? f32(*t, n) : nullptr;
}
float* optf32w(const c10::optional<Tensor>& t, const char* n) {
  return (t.has_value() && t->defined()) ? f32w(*t, n) : nullptr;
}
const uint16_t* optbf(const c10::optional<Tensor>& t, const char* n) {
  return (t.has_value() && t->defined()) ? bf(*t, n) : nullptr;
}
uint16_t* optbfw(const c10::optional<Tensor>& t, const char* n) {
  return (t.has_value() && t->defined()) ? bfw(*t, n) : nullptr;
}
const int* i32(const Tensor& t, const char* n) {
  check_dev(t, at::kInt, n);
  return t.data_ptr<int>();
}

ConvGeom geom_from(const std::vector<int64_t>& v) {
  TORCH_CHECK(v.size() == 22, "conv geometry must have 22 entries");
  ConvGeom g;
  int* p = &g.Nb;
  for (int i = 0; i < 22; ++i) p[i] = (int)v[i];
  TORCH_CHECK(g.C % 8 == 0, "conv: gathered channels must be a multiple of 8, got ", g.C);
  TORCH_CHECK(g.N > 0 && g.Nb > 0 && g.OH > 0 && g.OW > 0, "conv: empty problem");
  return g;
}

// ------------------------------------------------------------------------------- conv
ConvFusion fusion_from(const c10::optional<Tensor>& pro_sc, const c10::optional<Tensor>& pro_sh,
                       int64_t pro_seg_rows, bool pro_relu, int64_t pro_S, int64_t epi_mode,
                       const c10::optional<Tensor>& epi_a, const c10::optional<Tensor>& epi_b,
                       int64_t C, int64_t out_numel) {
  ConvFusion f;
  f.pro_sc = optf32(pro_sc, "pro_sc");
  f.pro_sh = optf32(pro_sh, "pro_sh");
  TORCH_CHECK((f.pro_sc == nullptr) == (f.pro_sh == nullptr), "prologue needs scale and shift");
  if (f.pro_sc) {
    TORCH_CHECK(pro_sc->numel() >= pro_S * C && pro_sh->numel() >= pro_S * C,
                "prologue scale/shift must be [S][C]");
  }
  f.pro_seg_rows = (int)pro_seg_rows;
  f.pro_relu = pro_relu ? 1 : 0;
  f.pro_S = (int)pro_S;
  f.epi_mode = (int)epi_mode;
  f.epi_a = optbf(epi_a, "epi_a");
  f.epi_b = optbf(epi_b, "epi_b");
  TORCH_CHECK(epi_mode >= 0 && epi_mode <= 4, "epi_mode");
  if (epi_mode == 1 || epi_mode == 2 || epi_mode == 4)
    TORCH_CHECK(f.epi_a && epi_a->numel() >= out_numel, "epilogue operand a");
  if (epi_mode == 2 || epi_mode == 3)
    TORCH_CHECK(f.epi_b && epi_b->numel() >= out_numel, "epilogue operand b");
  return f;
}

unsigned* tickets_for(const Tensor& like, int64_t n, int64_t slot);


void igemm(const Tensor& A, const Tensor& B, const Tensor& out, const c10::optional<Tensor>& bias,
           const c10::optional<Tensor>& stats, std::vector<int64_t> gv,
           const c10::optional<Tensor>& pro_sc, const c10::optional<Tensor>& pro_sh,
           int64_t pro_seg_rows, bool pro_relu, int64_t epi_mode,
           const c10::optional<Tensor>& epi_a, const c10::optional<Tensor>& epi_b,
           int64_t variant, const c10::optional<Tensor>& epi_ss,
           const c10::optional<Tensor>& epi_mi, int64_t seg_rows, int64_t stats_seg_blocks,
           int64_t stats_base, const c10::optional<Tensor>& epi_c,
           const c10::optional<Tensor>& epi_mask, const c10::optional<Tensor>& epi_c2,
           const c10::optional<Tensor>& epi_mi2, const c10::optional<Tensor>& stats2,
           const c10::optional<Tensor>& pro_d, const c10::optional<Tensor>& A2,
           const c10::optional<Tensor>& pro_rss, const c10::optional<Tensor>& pro_out,
           const c10::optional<Tensor>& pro_mask) {
  const ConvGeom g = geom_from(gv);
  // bit 8 of epi_mode: epi_a is the stride-2 subsampled residual (conv.hip epi_load_batch)
  const bool epi_sub = (epi_mode & 256) != 0;
  epi_mode &= 255;
  TORCH_CHECK(A.numel() == (int64_t)g.Nb * g.IH * g.IW * g.C, "igemm: A numel mismatch");
  TORCH_CHECK(A.numel() * 2 < (int64_t)1 << 31, "igemm: A larger than 2 GiB");
  const int64_t K = (int64_t)g.KH * g.KW * g.C;
  TORCH_CHECK(B.numel() == (int64_t)g.N * K, "igemm: B numel mismatch");
  TORCH_CHECK(g.ldo % 8 == 0 && g.N % 8 == 0, "igemm: N/ldo must be multiples of 8");
  TORCH_CHECK(out.numel() >= (int64_t)g.Nb * g.OHp * g.OWp * g.ldo, "igemm: out too small");
  TORCH_CHECK(out.numel() * 2 < ((int64_t)1 << 31) * 2, "igemm: out too large");
  if (variant < 0 || variant >= igemm_num_variants()) variant = igemm_default_variant(g.N);
  const int64_t M = (int64_t)g.Nb * g.OH * g.OW;
  const int bm = igemm_variant_bm((int)variant);
  const bool has_pd = pro_d.has_value() && pro_d->defined();
  // pro_out: the block-output prologue's output (dual) — or, with the BN-backward prologue on a
  // patch variant, the materialised prologue result (the weight gradient's dY)
  const bool dual = pro_out.has_value() && pro_out->defined() && !has_pd;
  if (dual) {
    TORCH_CHECK(igemm_dual_ok((int)variant, g),
                "igemm: block-output prologue needs a 2-stage LDS-DMA variant (igemm_dual_ok) on "
                "a 1x1 / stride-1 / unpadded convolution");
  } else if (igemm_variant_glds((int)variant)) {
    TORCH_CHECK(igemm_variant_ok((int)variant, g, pro_sc.has_value() && pro_sc->defined(),
                                 pro_d.has_value() && pro_d->defined()),
                "igemm: LDS-DMA variant needs C % 64 == 0 and its prologues (BN-apply, "
                "BN-backward) only on unpadded 1x1 convolutions (2-stage tiles whose staging fits)");
  }
  if (bias.has_value() && bias->defined()) TORCH_CHECK(bias->numel() == g.N, "igemm: bias size");
  const bool has_stats = stats.has_value() && stats->defined();
  if (has_stats && stats_seg_blocks == 0)
    TORCH_CHECK(stats->numel() >= ((M + bm - 1) / bm) * 2 * g.N, "igemm: stats buffer too small");
  const bool direct = g.osh == 1 && g.osw == 1 && g.ooh == 0 && g.oow == 0 && g.OHp == g.OH &&
                      g.OWp == g.OW;
  const int64_t sub_numel = (int64_t)g.Nb * ((g.OH + 1) / 2) * ((g.OW + 1) / 2) * g.ldo;
  if (epi_sub) {
    TORCH_CHECK(epi_mode == 1 || epi_mode == 2 || epi_mode == 4,
                "igemm: a subsampled residual needs epilogue mode 1, 2 or 4");
    TORCH_CHECK(direct, "igemm: a subsampled residual needs a direct (stride-1) output");
    TORCH_CHECK(epi_a.has_value() && epi_a->defined() && epi_a->numel() == sub_numel,
                "igemm: subsampled residual must be [Nb][ceil(OH/2)][ceil(OW/2)][ldo]");
  }
  ConvFusion f = fusion_from(pro_sc, pro_sh, pro_seg_rows, pro_relu, 1, epi_mode, epi_a, epi_b,
                             g.C, epi_sub ? sub_numel : out.numel());
  f.epi_a_sub = epi_sub ? 1 : 0;
  if (epi_sub && epi_mode == 2)
    TORCH_CHECK(epi_b->numel() >= out.numel(), "epilogue operand b");
  f.seg_rows = (int)seg_rows;
  f.stats_seg_blocks = (int)stats_seg_blocks;
  f.stats_base = (int)stats_base;
  if (seg_rows > 0)
    TORCH_CHECK(seg_rows % bm == 0 && M % seg_rows == 0,
                "igemm: segment rows must be a multiple of the tile rows and divide M");
  if (stats_seg_blocks > 0) {
    TORCH_CHECK(has_stats && seg_rows > 0, "igemm: stats remap needs stats and seg_rows");
    const int64_t nseg = M / seg_rows;
    TORCH_CHECK(stats_base >= 0 && stats_base + seg_rows / bm <= stats_seg_blocks,
                "igemm: stats remap window out of range");
    TORCH_CHECK(stats->numel() >= nseg * stats_seg_blocks * 2 * g.N,
                "igemm: remapped stats buffer too small");
  }
  if (epi_mode == 3 || epi_mode == 4) {
    TORCH_CHECK(seg_rows > 0, "igemm mode 3/4 needs seg_rows");
    TORCH_CHECK(!f.pro_sc || epi_mode == 3 || (pro_d.has_value() && pro_d->defined()),
                "igemm: the BN-apply prologue takes epilogue mode 3 only (mode 4: BN-backward)");
    const int64_t nseg = M / seg_rows;
    f.epi_mi = optf32(epi_mi, "epi_mi");
    f.epi_S = (int)nseg;
    TORCH_CHECK(f.epi_mi && epi_mi->numel() >= 2 * nseg * g.N,
                "igemm mode 3/4: mean/invstd table must be [2][S][N]");
    if (epi_mode == 3) {
      f.epi_ss = optf32(epi_ss, "epi_ss");
      TORCH_CHECK(f.epi_ss && epi_ss->numel() >= 2 * nseg * g.N,
                  "igemm mode 3: scale/shift table must be [2][S][N]");
    } else {
      f.epi_c = optbf(epi_c, "epi_c");
      TORCH_CHECK(f.epi_c && epi_c->numel() >= out.numel(), "igemm mode 4: epilogue operand c");
      if (epi_mask.has_value() && epi_mask->defined()) {
        check_dev(*epi_mask, at::kByte, "epi_mask");
        TORCH_CHECK(epi_mask->numel() * 8 >= out.numel(), "igemm mode 4: mask size");
        f.epi_mask = epi_mask->data_ptr<uint8_t>();
      }
      if (stats2.has_value() && stats2->defined()) {
        f.stats2 = f32w(*stats2, "stats2");
        f.epi_c2 = optbf(epi_c2, "epi_c2");
        f.epi_mi2 = optf32(epi_mi2, "epi_mi2");
        TORCH_CHECK(has_stats && f.epi_c2 && f.epi_mi2 && epi_c2->numel() >= out.numel() &&
                        epi_mi2->numel() >= 2 * nseg * g.N && stats2->numel() >= stats->numel(),
                    "igemm mode 4: second BN stream needs c2, mi2 [2][S][N] and stats2");
      }
    }
  }
  if (f.pro_sc) {
    TORCH_CHECK(pro_seg_rows > 0 && pro_seg_rows % bm == 0 && M % pro_seg_rows == 0,
                "igemm prologue: segment rows must be a multiple of the tile rows");
    TORCH_CHECK(pro_sc->numel() >= (M / pro_seg_rows) * g.C, "igemm prologue: [S][C] size");
  }
  if (pro_d.has_value() && pro_d->defined()) {
    TORCH_CHECK(f.pro_sc, "igemm BN-backward prologue needs pro_sc (A) and pro_sh (B)");
    // the BN-backward prologue + mode-4 epilogue is not instantiated for tiles above 256 x 128
    // (the 256 x 256 tile with both fusions drains its DMA pipeline): conv.hip launch_glds
    TORCH_CHECK(!(igemm_variant_glds((int)variant) && epi_mode == 4 &&
                  igemm_variant_bm((int)variant) * igemm_variant_bn((int)variant) > 256 * 128),
                "igemm: BN-backward prologue + mode-4 epilogue needs an LDS-DMA tile of at most "
                "256 x 128 (variant ", variant, ")");
    TORCH_CHECK(pro_d->numel() >= (M / pro_seg_rows) * g.C, "igemm prologue: d [S][C] size");
    TORCH_CHECK(A2.has_value() && A2->numel() == A.numel(), "igemm prologue: A2 must match A");
    TORCH_CHECK(epi_mode == 0 || epi_mode == 3 || epi_mode == 4,
                "igemm BN-backward prologue: epilogue 0, 3 or 4");
    f.pro_d = f32(*pro_d, "pro_d");
    f.A2 = bf(*A2, "A2");
    if (pro_out.has_value() && pro_out->defined()) {
      TORCH_CHECK(igemm_variant_patch((int)variant) && (epi_mode == 0 || epi_mode == 3),
                  "igemm: the materialised BN-backward operand (pro_out) needs a patch variant "
                  "and epilogue 0 or 3");
      TORCH_CHECK(pro_out->numel() == A.numel(), "igemm: pro_out must match A");
      const char* o0 = static_cast<const char*>(pro_out->data_ptr());
      const char* o1 = o0 + pro_out->numel() * 2;
      for (const Tensor* t : {&A, &*A2, &out}) {
        const char* t0 = static_cast<const char*>(t->data_ptr());
        const char* t1 = t0 + t->numel() * t->element_size();
        TORCH_CHECK(!(o0 < t1 && t0 < o1), "igemm: pro_out must not alias A, A2 or out");
      }
      f.pro_out = bfw(*pro_out, "pro_out");
    }
  }
  if (dual) {
    TORCH_CHECK(f.pro_sc && f.pro_sh && !f.pro_d && epi_mode == 0 && !(bias.has_value() && bias->defined()),
                "igemm block-output prologue: scale/shift tables, no other fusion");
    TORCH_CHECK(A2.has_value() && A2->numel() == A.numel(), "igemm block-output prologue: residual");
    TORCH_CHECK(pro_out->numel() == A.numel(), "igemm block-output prologue: out size");
    TORCH_CHECK(pro_mask.has_value() && pro_mask->defined() && pro_mask->numel() * 8 >= A.numel(),
                "igemm block-output prologue: mask size");
    check_dev(*pro_mask, at::kByte, "pro_mask");
    // the nb == 0 column of blocks writes relu(bn(A) + res) while the other column blocks
    // still read A / A2: the kernel applies ReLU unconditionally and the output must not alias
    TORCH_CHECK(pro_relu, "igemm block-output prologue: always applies ReLU (pro_relu required)");
    auto overlaps = [](const Tensor& a, const Tensor& b) {
      const char* a0 = static_cast<const char*>(a.data_ptr());
      const char* b0 = static_cast<const char*>(b.data_ptr());
      const char* a1 = a0 + a.numel() * a.element_size();
      const char* b1 = b0 + b.numel() * b.element_size();
      return a0 < b1 && b0 < a1;
    };
    TORCH_CHECK(!overlaps(*pro_out, A) && !overlaps(*pro_out, *A2) && !overlaps(*pro_out, out) &&
                    !overlaps(*pro_mask, A) && !overlaps(*pro_mask, *A2) && !overlaps(*pro_mask, out),
                "igemm block-output prologue: out / mask must not alias A, the residual or the "
                "conv output");
    f.A2 = bf(*A2, "A2");
    f.pro_out = bfw(*pro_out, "pro_out");
    f.pro_mask = pro_mask->data_ptr<uint8_t>();
    if (pro_rss.has_value() && pro_rss->defined()) {
      const int64_t nseg = M / pro_seg_rows;
      TORCH_CHECK(pro_rss->numel() >= 2 * nseg * g.C, "igemm block-output prologue: rss [2][S][C]");
      f.pro_rsc = f32(*pro_rss, "pro_rss");
      f.pro_rsh = f.pro_rsc + nseg * g.C;
    }
  }
  conv_igemm_nt(g, bf(A, "A"), (size_t)A.numel(), bf(B, "B"), bfw(out, "out"), optf32(bias, "bias"),
                optf32w(stats, "stats"), f, (int)variant, cur_stream());
}

int64_t igemm_bm(int64_t N) { return igemm_block_m((int)N); }
int64_t igemm_nvariants() { return igemm_num_variants(); }
int64_t igemm_vbm(int64_t v) { return igemm_variant_bm((int)v); }
int64_t igemm_vbn(int64_t v) { return igemm_variant_bn((int)v); }
bool igemm_vglds(int64_t v) { return igemm_variant_glds((int)v); }
bool igemm_gldsok(std::vector<int64_t> gv, bool pro, bool bn_bwd_pro) {
  return igemm_glds_ok(geom_from(gv), pro, bn_bwd_pro);
}
int64_t wgrad_nvariants() { return wgrad_num_variants(); }
int64_t wgrad_xlin_op(int64_t mode) { return wgrad_xlin((int)mode); }
bool wgrad_vglds(int64_t v) { return wgrad_variant_glds((int)v); }
bool igemm_vok(int64_t v, std::vector<int64_t> gv, bool pro, bool bnb) {
  return igemm_variant_ok((int)v, geom_from(gv), pro, bnb);
}
bool igemm_dok(int64_t v, std::vector<int64_t> gv) { return igemm_dual_ok((int)v, geom_from(gv)); }
bool wgrad_vok(int64_t v, std::vector<int64_t> gv, bool pro, bool dpro) {
  return wgrad_variant_ok((int)v, geom_from(gv), pro, dpro);
}

int64_t wgrad_nsplit(std::vector<int64_t> gv, int64_t variant) {
  return wgrad_splits(geom_from(gv), (int)variant);
}

int64_t wgrad_ntiles(std::vector<int64_t> gv, int64_t variant) {
  return wgrad_tiles(geom_from(gv), (int)variant);
}

void wgrad(const Tensor& dY, const Tensor& X, const Tensor& partial, const Tensor& out,
           std::vector<int64_t> gv, int64_t splits, int64_t creal, double beta,
           const c10::optional<Tensor>& pro_sc, const c10::optional<Tensor>& pro_sh,
           int64_t pro_seg_rows, bool pro_relu, int64_t pro_S, int64_t variant,
           const c10::optional<Tensor>& dY2, const c10::optional<Tensor>& dp_coef,
           int64_t dp_seg_rows, int64_t dp_S) {
  const ConvGeom g = geom_from(gv);
  const int64_t M = (int64_t)g.Nb * g.OH * g.OW;
  const int64_t K = (int64_t)g.KH * g.KW * g.C;
  TORCH_CHECK(dY.numel() == M * g.N, "wgrad: dY numel mismatch");
  TORCH_CHECK(X.numel() == (int64_t)g.Nb * g.IH * g.IW * g.C, "wgrad: X numel mismatch");
  TORCH_CHECK(partial.numel() >= splits * g.N * K, "wgrad: partial too small");
  TORCH_CHECK(out.numel() == (int64_t)g.N * g.KH * g.KW * creal, "wgrad: out numel mismatch");
  TORCH_CHECK(creal <= g.C && creal > 0, "wgrad: bad creal");
  TORCH_CHECK(pro_S >= 1 && pro_S <= 2, "wgrad prologue supports at most 2 segments");
  if (wgrad_variant_glds((int)variant))
    TORCH_CHECK(wgrad_variant_ok((int)variant, g, pro_sc.has_value() && pro_sc->defined(),
                                 dY2.has_value() && dY2->defined()),
                "wgrad: LDS-DMA variant needs C % 64 == 0, no dY prologue, and an X prologue only "
                "on unpadded 1x1 convolutions");
  ConvFusion f = fusion_from(pro_sc, pro_sh, pro_seg_rows, pro_relu, pro_S, 0, c10::nullopt,
                             c10::nullopt, g.C, 0);
  if (f.pro_sc) {
    // the prologue is indexed by *input* rows, which equal output rows only for 1x1/stride-1
    TORCH_CHECK(pro_seg_rows > 0 && (int64_t)g.Nb % pro_S == 0, "wgrad prologue geometry");
  }
  if (dY2.has_value() && dY2->defined()) {
    TORCH_CHECK(dY2->numel() == dY.numel(), "wgrad: dY2 must match dY");
    TORCH_CHECK(dp_coef.has_value() && dp_coef->numel() >= 3 * dp_S * g.N, "wgrad: dp_coef [3][S][N]");
    const int64_t iters = (M + 63) / 64;
    const int64_t ips = (iters + splits - 1) / splits;
    // a split may straddle at most one segment boundary (the kernel holds two coefficient sets)
    TORCH_CHECK(dp_seg_rows > 0 && M % dp_seg_rows == 0 && M / dp_seg_rows == dp_S &&
                    (dp_S <= 2 || dp_seg_rows % (ips * 64) == 0) && dp_seg_rows % 64 == 0,
                "wgrad dY prologue: 64-row segments, and every split inside one segment when "
                "there are more than two");
    TORCH_CHECK(!wgrad_variant_glds((int)variant),
                "wgrad dY prologue: register-staged variants only");
    f.dY2 = bf(*dY2, "dY2");
    f.dp_coef = f32(*dp_coef, "dp_coef");
    f.dp_seg_rows = (int)dp_seg_rows;
    f.dp_S = (int)dp_S;
  }
  conv_wgrad(g, bf(dY, "dY"), bf(X, "X"), (size_t)X.numel(), f32w(partial, "partial"), (int)splits,
             f32w(out, "out"), (int)creal, (float)beta, f, (int)variant, cur_stream());
}


// fused 1x1 backward of a bottleneck conv3 (conv.hip conv1x1_bwd_dual): returns nothing; writes
// gm [M][Ci], stats [S*bps][2][Ci] (BN2-backward partials), wpart [S*bps][Co][Ci] (dW slabs)
void conv1x1_bwd_dual_op(const Tensor& G, const c10::optional<Tensor>& A3,
                         const c10::optional<Tensor>& coef, const Tensor& X,
                         const c10::optional<Tensor>& xss, const c10::optional<Tensor>& xmi,
                         const Tensor& Wt, const Tensor& gm,
                         const Tensor& stats, const Tensor& wpart, int64_t S, int64_t bps,
                         const c10::optional<Tensor>& Xraw, bool dual8) {
  const int64_t CI = gm.size(-1);
  const int64_t M = gm.numel() / CI;
  const int64_t CO = G.numel() / M;
  const uint16_t* xr = optbf(Xraw, "Xraw");
  TORCH_CHECK((CO == 256 && CI == 64 && xr == nullptr) || (CO == 512 && CI == 128),
              "conv1x1_bwd_dual: (Co, Ci) = (256, 64) or (512, 128); a pre-applied X (Xraw "
              "given) only with (512, 128)");
  if (xr != nullptr) TORCH_CHECK(Xraw->numel() == M * CI, "conv1x1_bwd_dual: Xraw size");
  TORCH_CHECK(G.numel() == M * CO && X.numel() == M * CI && Wt.numel() == CI * CO,
              "conv1x1_bwd_dual: operand sizes");
  TORCH_CHECK(S >= 1 && S <= 2 && bps >= 1 && M % S == 0 && (M / S) % (64 * bps) == 0,
              "conv1x1_bwd_dual: every block's rows must lie in one segment (64-row tiles)");
  const float* xs = optf32(xss, "xss");
  const float* xm = optf32(xmi, "xmi");
  // no BN2 tables: the plain form (a downsample conv; no mask, no partials) — (256, 64) only
  TORCH_CHECK((xs == nullptr) == (xm == nullptr), "conv1x1_bwd_dual: xss and xmi together");
  TORCH_CHECK(xs != nullptr || (CO == 256 && CI == 64 && xr == nullptr),
              "conv1x1_bwd_dual: the plain form is (Co, Ci) = (256, 64) only");
  if (xs != nullptr) {
    TORCH_CHECK(xss->numel() >= 2 * S * CI && xmi->numel() >= 2 * S * CI,
                "conv1x1_bwd_dual: BN2 tables");
    TORCH_CHECK(stats.numel() >= S * bps * 2 * CI, "conv1x1_bwd_dual: stats size");
  }
  TORCH_CHECK(wpart.numel() >= S * bps * CO * CI, "conv1x1_bwd_dual: wpart size");
  TORCH_CHECK(M * CO * 2 < (int64_t(1) << 31), "conv1x1_bwd_dual: 32-bit buffer offsets");
  const uint16_t* a3 = optbf(A3, "A3");
  const float* cf = optf32(coef, "coef");
  if (a3 != nullptr) {
    TORCH_CHECK(A3->numel() == G.numel() && cf != nullptr && coef->numel() >= 3 * S * CO,
                "conv1x1_bwd_dual: lazy BN-backward needs A3 [M][Co] and coef [3][S][Co]");
  }
  conv1x1_bwd_dual(bf(G, "G"), a3, cf, bf(X, "X"), xs, xm,
                   bf(Wt, "Wt"), bfw(gm, "gm"), f32w(stats, "stats"), f32w(wpart, "wpart"),
                   (int)M, (int)CO, (int)CI, (int)S, (int)bps, cur_stream(), xr, dual8);
}

// 1x1 stride-2 downsample backward (layer2.0): X [N][H][W][Ci] block input, gm [N][OH][OW][Ci]
void conv1x1_bwd_dual_s2_op(const Tensor& G, const c10::optional<Tensor>& A3,
                            const c10::optional<Tensor>& coef, const Tensor& X, const Tensor& Wt,
                            const Tensor& gm, const Tensor& wpart, int64_t S, int64_t bps) {
  TORCH_CHECK(X.dim() == 4 && gm.dim() == 4, "conv1x1_bwd_dual_s2: NHWC 4-D X and gm");
  const int64_t N = X.size(0), H = X.size(1), W = X.size(2), CI = X.size(3);
  const int64_t OH = gm.size(1), OW = gm.size(2);
  TORCH_CHECK(gm.size(0) == N && gm.size(3) == CI && OH == (H + 1) / 2 && OW == (W + 1) / 2,
              "conv1x1_bwd_dual_s2: gm is the stride-2 output map");
  const int64_t Mo = N * OH * OW;
  const int64_t CO = G.numel() / Mo;
  TORCH_CHECK(CO == 512 && CI == 256 && G.numel() == Mo * CO && Wt.numel() == CI * CO,
              "conv1x1_bwd_dual_s2: (Co, Ci) = (512, 256) only");
  TORCH_CHECK(S >= 1 && S <= 2 && N % S == 0 && bps >= 1 && (Mo / S) % (64 * bps) == 0,
              "conv1x1_bwd_dual_s2: every block's rows must lie in one segment");
  TORCH_CHECK(wpart.numel() >= S * bps * CO * CI, "conv1x1_bwd_dual_s2: wpart size");
  TORCH_CHECK(Mo * CO * 2 < (int64_t(1) << 31) && X.numel() * 2 < (int64_t(1) << 31),
              "conv1x1_bwd_dual_s2: 32-bit buffer offsets");
  const uint16_t* a3 = optbf(A3, "A3");
  const float* cf = optf32(coef, "coef");
  TORCH_CHECK(a3 == nullptr && cf == nullptr,
              "conv1x1_bwd_dual_s2: dY must be materialised (no lazy BN-backward form)");
  conv1x1_bwd_dual_s2(bf(G, "G"), a3, cf, bf(X, "X"), bf(Wt, "Wt"), bfw(gm, "gm"),
                      f32w(wpart, "wpart"), (int)Mo, (int)CO, (int)CI, (int)S, (int)bps, (int)H,
                      (int)W, (int)OH, (int)OW, cur_stream());
}

void wgrad_reduce_slabs_op(const Tensor& partial, int64_t splits, const Tensor& out, double beta) {
  const int64_t n = out.numel();
  TORCH_CHECK(n % 4 == 0 && partial.numel() >= splits * n && splits >= 1,
              "wgrad_reduce_slabs: sizes");
  wgrad_reduce_slabs(f32w(partial, "partial"), (int)splits, f32w(out, "out"), (size_t)n,
                     (float)beta, cur_stream());
}

void weight_transform(const Tensor& W, const Tensor& Wt, std::vector<int64_t> p) {
  TORCH_CHECK(p.size() == 10, "weight_transform params");
  const int Co = p[0], KH = p[1], KW = p[2], Ci = p[3], KHs = p[4], KWs = p[5];
  TORCH_CHECK(W.numel() == (int64_t)Co * KH * KW * Ci, "weight_transform: W numel");
  TORCH_CHECK(Wt.numel() == (int64_t)Ci * KHs * KWs * Co, "weight_transform: Wt numel");
  for (int a = 0; a < KHs; ++a) {
    const int kh = (int)p[6] + a * (int)p[7];
    TORCH_CHECK(kh >= 0 && kh < KH, "weight_transform: kh out of range");
  }
  for (int a = 0; a < KWs; ++a) {
    const int kw = (int)p[8] + a * (int)p[9];
    TORCH_CHECK(kw >= 0 && kw < KW, "weight_transform: kw out of range");
  }
  conv_weight_transform(bf(W, "W"), bfw(Wt, "Wt"), Co, KH, KW, Ci, KHs, KWs, p[6], p[7], p[8], p[9],
                        cur_stream());
}

// Batched dgrad weight transforms: plan (validate + device descriptor table, eager) and launch.
// The plan holds raw pointers: the caller keeps every W / Wt tensor alive and unmoved while
// it is used (FusedStages caches it next to the tensors and rebuilds it when they change).
Tensor weight_transform_plan(const std::vector<Tensor>& Ws, const std::vector<Tensor>& Wts,
                             std::vector<int64_t> p) {
  const size_t n = Ws.size();
  TORCH_CHECK(n > 0 && Wts.size() == n && p.size() == 10 * n, "weight_transform_plan sizes");
  Tensor host = at::empty({(int64_t)(n * sizeof(WtDesc) / 8) + 1},
                          at::TensorOptions().dtype(at::kLong));
  WtDesc* d = reinterpret_cast<WtDesc*>(host.data_ptr<int64_t>());
  int blk = 0;
  for (size_t i = 0; i < n; ++i) {
    const int64_t* q = p.data() + 10 * i;
    const int Co = q[0], KH = q[1], KW = q[2], Ci = q[3], KHs = q[4], KWs = q[5];
    TORCH_CHECK(Ws[i].numel() == (int64_t)Co * KH * KW * Ci, "weight_transform_plan: W numel");
    TORCH_CHECK(Wts[i].numel() == (int64_t)Ci * KHs * KWs * Co, "weight_transform_plan: Wt numel");
    TORCH_CHECK(Ws[i].device() == Wts[0].device() && Wts[i].device() == Wts[0].device(),
                "weight_transform_plan: one device");
    for (int a = 0; a < KHs; ++a)
      TORCH_CHECK(q[6] + a * q[7] >= 0 && q[6] + a * q[7] < KH, "weight_transform_plan: kh");
    for (int a = 0; a < KWs; ++a)
      TORCH_CHECK(q[8] + a * q[9] >= 0 && q[8] + a * q[9] < KW, "weight_transform_plan: kw");
    const int nb = ((Co + 63) / 64) * ((Ci + 63) / 64) * KHs * KWs;  // 64x64 tiles per tap
    d[i] = WtDesc{bf(Ws[i], "W"), bfw(Wts[i], "Wt"), Co, KH, KW, Ci, KHs, KWs, (int)q[6],
                  (int)q[7], (int)q[8], (int)q[9], blk, nb};
    blk += nb;
  }
  // host table [n descriptors | total block count]; the caller moves the descriptors to the
  // device once and keeps the count on the host (no sync per launch, graph-capturable)
  host.data_ptr<int64_t>()[n * sizeof(WtDesc) / 8] = blk;
  return host;
}

void weight_transform_batch(const Tensor& table, int64_t total_blocks) {
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kLong && table.numel() % 8 == 0 &&
                  table.numel() > 0 && total_blocks > 0,
              "weight_transform_batch: device descriptors from weight_transform_plan");
  conv_weight_transform_batch(reinterpret_cast<const WtDesc*>(table.data_ptr<int64_t>()),
                              (int)(table.numel() / 8), (int)total_blocks, cur_stream());
}

// ------------------------------------------------------------------------------- batch norm
void check_rc(const Tensor& x, int64_t S, const char* n) {
  TORCH_CHECK(x.dim() >= 2, n, ": rank");
  const int64_t C = x.size(-1);
  TORCH_CHECK(C % 8 == 0, n, ": channels must be a multiple of 8");
  const int64_t CH = C / 8;
  TORCH_CHECK(CH <= 256 || CH % 256 == 0, n, ": unsupported channel count");
  TORCH_CHECK((x.numel() / C) % S == 0, n, ": rows not divisible by segments");
}

int64_t bn_blocks(int64_t R, int64_t C, int64_t S) {
  return bn_stats_blocks_per_seg((int)R, (int)C, (int)S);
}

void bn_stats(const Tensor& x, int64_t S, const Tensor& partial) {
  check_rc(x, S, "bn_stats");
  const int C = x.size(-1), R = x.numel() / C;
  const int nblk = bn_stats_blocks_per_seg(R, C, S);
  TORCH_CHECK(partial.numel() >= (int64_t)S * nblk * 2 * C, "bn_stats: partial too small");
  bn_stats_partial(bf(x, "x"), R, C, S, f32w(partial, "partial"), nullptr, cur_stream());
}

void bn_reduce(const Tensor& partial, int64_t nblk, int64_t S, int64_t C, const Tensor& stats) {
  TORCH_CHECK(partial.numel() >= S * nblk * 2 * C && stats.numel() >= 2 * S * C, "bn_reduce sizes");
  const int G = bn_reduce_groups((int)nblk);
  TORCH_CHECK(G == 1 || C % 4 == 0, "bn_reduce: C must be a multiple of 4 (float4 partial rows)");
  at::Tensor ws;
  float* wsp = nullptr;
  if (G > 1) {
    ws = at::empty({S * G * 2 * C}, stats.options());
    wsp = ws.data_ptr<float>();
  }
  bn_reduce_partials(f32(partial, "partial"), nblk, S, C, f32w(stats, "stats"), wsp, cur_stream());
}

void bn_final(const Tensor& stats, int64_t S, int64_t C, double count, double eps, double momentum,
              const c10::optional<Tensor>& rm, const c10::optional<Tensor>& rv, const Tensor& mi,
              const c10::optional<Tensor>& nbt, const c10::optional<Tensor>& gamma,
              const c10::optional<Tensor>& beta, const c10::optional<Tensor>& ss) {
  if (ss.has_value() && ss->defined()) TORCH_CHECK(ss->numel() >= 2 * S * C, "bn_finalize: ss size");
  if (gamma.has_value() && gamma->defined()) TORCH_CHECK(gamma->numel() == C, "bn_finalize: gamma");
  if (beta.has_value() && beta->defined()) TORCH_CHECK(beta->numel() == C, "bn_finalize: beta");
  TORCH_CHECK(stats.numel() >= 2 * S * C && mi.numel() >= 2 * S * C, "bn_finalize sizes");
  int64_t* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    check_dev(*nbt, at::kLong, "num_batches_tracked");
    nb = nbt->data_ptr<int64_t>();
  }
  bn_finalize(f32(stats, "stats"), S, C, (float)count, (float)eps, (float)momentum,
              optf32w(rm, "running_mean"), optf32w(rv, "running_var"), f32w(mi, "mean_invstd"), nb,
              optf32(gamma, "gamma"), optf32(beta, "beta"), optf32w(ss, "ss"), cur_stream());
}

// persistent zeroed ticket arrays for the last-arriver reductions, per device and per slot:
// reductions that may run concurrently (different streams) must use different slots
constexpr int kTicketSlots = 4;  // 0/1 BN reduce per stream, 2/3 conv tails per stream
constexpr int64_t kTicketStride = 4096;
unsigned* tickets_for(const Tensor& like, int64_t n, int64_t slot) {
  static std::vector<Tensor> per_dev;
  TORCH_CHECK(slot >= 0 && slot < kTicketSlots, "ticket slot out of range");
  TORCH_CHECK(n <= kTicketStride, "too many channel groups for the ticket array");
  const int d = like.get_device();
  if ((int)per_dev.size() <= d) per_dev.resize(d + 1);
  if (!per_dev[d].defined()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(cur_stream(), &cs);
    TORCH_CHECK(cs == hipStreamCaptureStatusNone,
                "bn ticket array must be allocated before graph capture");
    per_dev[d] = at::zeros({kTicketSlots * kTicketStride}, like.options().dtype(at::kInt));
  }
  return reinterpret_cast<unsigned*>(per_dev[d].data_ptr<int>()) + slot * kTicketStride;
}

void bn_reduce_fused_op(const Tensor& partial, int64_t nblk, int64_t S, int64_t C, int64_t mode,
                        const c10::optional<Tensor>& stats, double count, double eps,
                        double momentum, const c10::optional<Tensor>& rm,
                        const c10::optional<Tensor>& rv, const c10::optional<Tensor>& mi,
                        const c10::optional<Tensor>& nbt, const c10::optional<Tensor>& gamma,
                        const c10::optional<Tensor>& beta, const c10::optional<Tensor>& ss,
                        const c10::optional<Tensor>& dgamma, const c10::optional<Tensor>& dbeta,
                        const c10::optional<Tensor>& coef, int64_t ticket_slot,
                        const c10::optional<Tensor>& ipc_peers,
                        const c10::optional<Tensor>& ipc_arena, int64_t ipc_site,
                        const c10::optional<Tensor>& ipc_epoch,
                        const c10::optional<Tensor>& ipc_err, int64_t world, int64_t rank) {
  TORCH_CHECK(mode >= 0 && mode <= 2, "bn_reduce_fused: mode");
  TORCH_CHECK(nblk > 0 && partial.numel() >= S * nblk * 2 * C, "bn_reduce_fused: partial size");
  TORCH_CHECK(C % 4 == 0, "bn_reduce_fused: C must be a multiple of 4 (float4 partial rows)");
  TORCH_CHECK(S >= 1 && S <= 4, "bn_reduce_fused: at most 4 segments");
  BnReduceFusedParams q;
  q.partial = f32(partial, "partial");
  q.nblk = (int)nblk; q.S = (int)S; q.C = (int)C; q.mode = (int)mode;
  const int G = bn_reduce_groups((int)nblk);
  at::Tensor ws = at::empty({S * G * 2 * C}, partial.options());
  q.ws = ws.data_ptr<float>();
  q.tickets = tickets_for(partial, (C + 63) / 64, ticket_slot);
  q.count = (float)count; q.eps = (float)eps; q.momentum = (float)momentum;
  if (mode == 0) {
    TORCH_CHECK(stats.has_value() && stats->numel() >= 2 * S * C, "bn_reduce_fused: stats");
    q.stats = f32w(*stats, "stats");
    // optional: the local dβ = Σ_s Σg, dγ = Σ_s Σg·x̂ of a BatchNorm backward's partials (the
    // distributed path all-reduces `stats` for the input-gradient coefficients afterwards)
    q.dgamma = optf32w(dgamma, "dgamma");
    q.dbeta = optf32w(dbeta, "dbeta");
  } else if (mode == 1) {
    TORCH_CHECK(mi.has_value() && mi->numel() >= 2 * S * C, "bn_reduce_fused: mi");
    q.mi = f32w(*mi, "mi");
    q.running_mean = optf32w(rm, "running_mean");
    q.running_var = optf32w(rv, "running_var");
    if (nbt.has_value() && nbt->defined()) {
      check_dev(*nbt, at::kLong, "num_batches_tracked");
      q.nbt = nbt->data_ptr<int64_t>();
    }
    q.gamma = optf32(gamma, "gamma");
    q.beta = optf32(beta, "beta");
    if (ss.has_value() && ss->defined()) TORCH_CHECK(ss->numel() >= 2 * S * C, "bn_reduce_fused: ss");
    q.ss = optf32w(ss, "ss");
  } else {
    TORCH_CHECK(mi.has_value() && mi->numel() >= 2 * S * C, "bn_reduce_fused: mi");
    TORCH_CHECK(coef.has_value() && coef->numel() >= 3 * S * C, "bn_reduce_fused: coef");
    q.mi = const_cast<float*>(f32(*mi, "mi"));
    q.gamma = optf32(gamma, "gamma");
    q.dgamma = optf32w(dgamma, "dgamma");
    q.dbeta = optf32w(dbeta, "dbeta");
    q.coef = f32w(*coef, "coef");
  }
  if (q.gamma) TORCH_CHECK(gamma->numel() == C, "bn_reduce_fused: gamma size");
  if (q.beta) TORCH_CHECK(beta->numel() == C, "bn_reduce_fused: beta size");
  if (q.dgamma) TORCH_CHECK(dgamma->numel() == C, "bn_reduce_fused: dgamma size");
  if (q.dbeta) TORCH_CHECK(dbeta->numel() == C, "bn_reduce_fused: dbeta size");
  if (world > 1) {
    // IPC statistics exchange (bn.hip bn_ipc_exchange): every rank's arena must hold this
    // site's region, the peer table one base per rank, the epochs one counter per channel group
    TORCH_CHECK(mode == 1 || mode == 2, "bn_reduce_fused: the IPC exchange finalizes (mode 1/2)");
    TORCH_CHECK(world <= 16 && rank >= 0 && rank < world, "bn_reduce_fused: world / rank");
    TORCH_CHECK(ipc_peers.has_value() && ipc_arena.has_value() && ipc_epoch.has_value() &&
                    ipc_err.has_value(), "bn_reduce_fused: IPC exchange needs peers, arena, epoch, err");
    check_dev(*ipc_peers, at::kLong, "ipc_peers");
    check_dev(*ipc_arena, at::kLong, "ipc_arena");
    check_dev(*ipc_epoch, at::kInt, "ipc_epoch");
    check_dev(*ipc_err, at::kInt, "ipc_err");
    TORCH_CHECK(ipc_peers->numel() == world, "bn_reduce_fused: peer table size");
    TORCH_CHECK(ipc_epoch->numel() >= (C + 63) / 64, "bn_reduce_fused: epoch counters");
    TORCH_CHECK(ipc_site >= 0 && ipc_site + bn_ipc_region_words((int)world, (int)S, (int)C) <=
                                    ipc_arena->numel(),
                "bn_reduce_fused: IPC site region outside the arena");
    q.ipc_peers = reinterpret_cast<uint64_t* const*>(ipc_peers->data_ptr<int64_t>());
    q.ipc_own = reinterpret_cast<uint64_t*>(ipc_arena->data_ptr<int64_t>());
    q.ipc_site = ipc_site;
    q.ipc_epoch = reinterpret_cast<unsigned*>(ipc_epoch->data_ptr<int>());
    q.ipc_err = ipc_err->data_ptr<int>();
    q.world = (int)world;
    q.rank = (int)rank;
  }
  bn_reduce_fused(q, cur_stream());
}

// one-shot IPC all-gather (op 0: dst [W][n] <- every rank's src [n]) or reduce-scatter (op 1:
// dst [n] <- sum over ranks of src [W][n] row `rank`) of 32-bit words (comm.hip)
void ipc_collective_op(int64_t op, const Tensor& src, const Tensor& dst, const Tensor& peers,
                       const Tensor& arena, int64_t site, const Tensor& epoch, const Tensor& err,
                       int64_t world, int64_t rank) {
  TORCH_CHECK(op == 0 || op == 1, "ipc_collective: op 0 (all-gather) or 1 (reduce-scatter)");
  const bool words = src.element_size() == 4 && dst.element_size() == 4;
  const bool pairs = op == 0 && src.element_size() == 2 && dst.element_size() == 2;
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.is_contiguous() && dst.is_contiguous() &&
                  (words || pairs),
              "ipc_collective: contiguous 32-bit (or bf16 pairs for the all-gather) GPU tensors");
  const int64_t nbytes = src.numel() * src.element_size();
  TORCH_CHECK(nbytes % 4 == 0, "ipc_collective: payload must be whole 32-bit words");
  const int64_t n = op == 0 ? nbytes / 4 : nbytes / 4 / world;
  TORCH_CHECK(world >= 1 && world <= 16 && rank >= 0 && rank < world, "ipc_collective: world");
  TORCH_CHECK(dst.numel() * dst.element_size() == (op == 0 ? world * n * 4 : n * 4),
              "ipc_collective: dst size");
  TORCH_CHECK(op == 0 || src.numel() * src.element_size() == world * n * 4,
              "ipc_collective: reduce-scatter src must be [world][n] words");
  check_dev(peers, at::kLong, "ipc_peers");
  check_dev(arena, at::kLong, "ipc_arena");
  check_dev(epoch, at::kInt, "ipc_epoch");
  check_dev(err, at::kInt, "ipc_err");
  TORCH_CHECK(peers.numel() == world, "ipc_collective: peer table size");
  TORCH_CHECK(epoch.numel() >= IPC_COLL_BLOCKS, "ipc_collective: epoch counters");
  TORCH_CHECK(site >= 0 && site + ipc_coll_region_words((int)world, (int)n) <= arena.numel(),
              "ipc_collective: site outside the arena");
  ipc_collective((int)op, static_cast<const uint32_t*>(src.data_ptr()),
                 static_cast<uint32_t*>(dst.data_ptr()), (int)n,
                 reinterpret_cast<uint64_t* const*>(peers.data_ptr<int64_t>()),
                 reinterpret_cast<uint64_t*>(arena.data_ptr<int64_t>()), site,
                 reinterpret_cast<unsigned*>(epoch.data_ptr<int>()), err.data_ptr<int>(),
                 (int)world, (int)rank, cur_stream());
}

void bn_apply_ss_op(const Tensor& x, const Tensor& ss, const c10::optional<Tensor>& res,
                    const c10::optional<Tensor>& rss, const Tensor& y, int64_t S, bool relu,
                    const c10::optional<Tensor>& mask) {
  check_rc(x, S, "bn_apply_ss");
  const int C = x.size(-1), R = x.numel() / C;
  TORCH_CHECK(y.numel() == x.numel(), "bn_apply_ss: y size");
  TORCH_CHECK(ss.numel() >= 2 * S * C, "bn_apply_ss: ss size");
  const bool has_res = res.has_value() && res->defined();
  if (has_res) TORCH_CHECK(res->numel() == x.numel(), "bn_apply_ss: res size");
  if (rss.has_value() && rss->defined())
    TORCH_CHECK(has_res && rss->numel() >= 2 * S * C, "bn_apply_ss: rss needs res, [2][S][C]");
  uint8_t* mk = nullptr;
  if (mask.has_value() && mask->defined()) {
    check_dev(*mask, at::kByte, "mask");
    TORCH_CHECK(mask->numel() * 8 == x.numel(), "bn_apply_ss: mask must be [R][C/8] uint8");
    mk = mask->data_ptr<uint8_t>();
  }
  bn_apply_ss(bf(x, "x"), f32(ss, "ss"), optbf(res, "res"), optf32(rss, "rss"), bfw(y, "y"), mk, R,
              C, S, relu ? 1 : 0, cur_stream());
}

void bn_apply_op(const Tensor& x, const c10::optional<Tensor>& res, const Tensor& y,
                 const Tensor& mi, const c10::optional<Tensor>& gamma,
                 const c10::optional<Tensor>& beta, int64_t S, bool relu) {
  check_rc(x, S, "bn_apply");
  const int C = x.size(-1), R = x.numel() / C;
  TORCH_CHECK(y.numel() == x.numel(), "bn_apply: y size");
  if (res.has_value() && res->defined()) TORCH_CHECK(res->numel() == x.numel(), "bn_apply: res size");
  TORCH_CHECK(mi.numel() >= 2 * S * C, "bn_apply: mean_invstd size");
  bn_apply(bf(x, "x"), optbf(res, "res"), bfw(y, "y"), f32(mi, "mi"), optf32(gamma, "gamma"),
           optf32(beta, "beta"), R, C, S, relu ? 1 : 0, cur_stream());
}

void bn_apply_eval_op(const Tensor& x, const c10::optional<Tensor>& res, const Tensor& y,
                      const Tensor& rm, const Tensor& rv, const c10::optional<Tensor>& gamma,
                      const c10::optional<Tensor>& beta, double eps, bool relu) {
  check_rc(x, 1, "bn_apply_eval");
  const int C = x.size(-1), R = x.numel() / C;
  TORCH_CHECK(y.numel() == x.numel(), "bn_apply_eval: y size");
  bn_apply_eval(bf(x, "x"), optbf(res, "res"), bfw(y, "y"), f32(rm, "rm"), f32(rv, "rv"),
                optf32(gamma, "gamma"), optf32(beta, "beta"), (float)eps, R, C, relu ? 1 : 0,
                cur_stream());
}

void bn_bwd_reduce_op(const Tensor& dy, const c10::optional<Tensor>& y, const Tensor& x,
                      const Tensor& mi, int64_t S, bool relu, const Tensor& partial) {
  check_rc(x, S, "bn_bwd_reduce");
  const int C = x.size(-1), R = x.numel() / C;
  TORCH_CHECK(dy.numel() == x.numel(), "bn_bwd_reduce: dy size");
  TORCH_CHECK(!relu || (y.has_value() && y->numel() == x.numel()), "bn_bwd_reduce: y needed");
  const int nblk = bn_stats_blocks_per_seg(R, C, S);
  TORCH_CHECK(partial.numel() >= (int64_t)S * nblk * 2 * C, "bn_bwd_reduce: partial too small");
  bn_bwd_reduce(bf(dy, "dy"), optbf(y, "y"), bf(x, "x"), f32(mi, "mi"), R, C, S, relu ? 1 : 0,
                f32w(partial, "partial"), cur_stream());
}

void bn_bwd_final(const Tensor& sums, const Tensor& mi, const c10::optional<Tensor>& gamma,
                  int64_t S, int64_t C, double count, const c10::optional<Tensor>& dgamma,
                  const c10::optional<Tensor>& dbeta, const Tensor& coef) {
  TORCH_CHECK(sums.numel() >= 2 * S * C && coef.numel() >= 3 * S * C, "bn_bwd_finalize sizes");
  bn_bwd_finalize(f32(sums, "sums"), f32(mi, "mi"), optf32(gamma, "gamma"), S, C, (float)count,
                  optf32w(dgamma, "dgamma"), optf32w(dbeta, "dbeta"), f32w(coef, "coef"),
                  cur_stream());
}

void bn_bwd_apply_op(const Tensor& dy, const c10::optional<Tensor>& y, const Tensor& x,
                     const Tensor& coef, int64_t S, bool relu, const Tensor& dx,
                     const c10::optional<Tensor>& dres) {
  check_rc(x, S, "bn_bwd_apply");
  const int C = x.size(-1), R = x.numel() / C;
  TORCH_CHECK(dy.numel() == x.numel() && dx.numel() == x.numel(), "bn_bwd_apply sizes");
  TORCH_CHECK(!relu || (y.has_value() && y->numel() == x.numel()), "bn_bwd_apply: y needed");
  bn_bwd_apply(bf(dy, "dy"), optbf(y, "y"), bf(x, "x"), f32(coef, "coef"), R, C, S, relu ? 1 : 0,
               bfw(dx, "dx"), optbfw(dres, "dres"), cur_stream());
}

void bn_bwd_apply2_op(const Tensor& g, const Tensor& x1, const Tensor& coef1, const Tensor& dx1,
                      const Tensor& x2, const Tensor& coef2, const Tensor& dx2, int64_t S) {
  check_rc(x1, S, "bn_bwd_apply2");
  const int C = x1.size(-1), R = x1.numel() / C;
  TORCH_CHECK(g.numel() == x1.numel() && x2.numel() == x1.numel() && dx1.numel() == x1.numel() &&
                  dx2.numel() == x1.numel(), "bn_bwd_apply2 sizes");
  TORCH_CHECK(coef1.numel() >= 3 * S * C && coef2.numel() >= 3 * S * C, "bn_bwd_apply2 coef");
  bn_bwd_apply2(bf(g, "g"), bf(x1, "x1"), f32(coef1, "coef1"), bfw(dx1, "dx1"), bf(x2, "x2"),
                f32(coef2, "coef2"), bfw(dx2, "dx2"), R, C, S, cur_stream());
}

// ------------------------------------------------------------------------------- misc
void avgpool_fwd_op(const Tensor& x, const Tensor& y, int64_t Nb, int64_t HW, int64_t C) {
  TORCH_CHECK(C % 8 == 0 && x.numel() == Nb * HW * C && y.numel() == Nb * C, "avgpool_fwd sizes");
  avgpool_fwd(bf(x, "x"), bfw(y, "y"), Nb, HW, C, cur_stream());
}
void avgpool_bwd_op(const Tensor& dy, const Tensor& dx, int64_t Nb, int64_t HW, int64_t C) {
  TORCH_CHECK(C % 8 == 0 && dx.numel() == Nb * HW * C && dy.numel() == Nb * C, "avgpool_bwd sizes");
  avgpool_bwd(bf(dy, "dy"), bfw(dx, "dx"), Nb, HW, C, cur_stream());
}
void colsum_op(const Tensor& x, const Tensor& out, double beta) {
  const int C = x.size(-1), R = x.numel() / C;
  TORCH_CHECK(out.numel() == C, "colsum sizes");
  at::Tensor ws = at::empty({(int64_t)colsum_groups(R) * C}, out.options());
  colsum_bf16(bf(x, "x"), R, C, f32w(out, "out"), (float)beta, ws.data_ptr<float>(), cur_stream());
}
void cast_to_bf16(const Tensor& x, const Tensor& y) {
  TORCH_CHECK(x.numel() == y.numel(), "cast sizes");
  cast_f32_bf16(f32(x, "x"), bfw(y, "y"), x.numel(), cur_stream());
}
void cast_to_f32(const Tensor& x, const Tensor& y) {
  TORCH_CHECK(x.numel() == y.numel(), "cast sizes");
  cast_bf16_f32(bf(x, "x"), f32w(y, "y"), x.numel(), cur_stream());
}

// ------------------------------------------------------------------------------- nt-xent
void nt_normalize(const Tensor& z, const Tensor& zn, const Tensor& inv_norm) {
  TORCH_CHECK(z.dim() == 2, "nt_normalize: z must be 2-D");
  const int R = z.size(0), D = z.size(1);
  TORCH_CHECK(zn.numel() == (int64_t)R * D && inv_norm.numel() == R, "nt_normalize sizes");
  ntxent_normalize_f32(bf(z, "z"), R, D, f32w(zn, "zn"), f32w(inv_norm, "inv_norm"), cur_stream());
}
void nt_transpose(const Tensor& in, const Tensor& out) {
  const int R = in.size(0), D = in.size(1);
  TORCH_CHECK(out.numel() == (int64_t)R * D, "nt_transpose sizes");
  ntxent_transpose(f32(in, "in"), f32w(out, "out"), R, D, cur_stream());
}
void check_nt(int R, int Ccols, int D, int col_offset, int n_local) {
  TORCH_CHECK(R % 16 == 0 && Ccols % 16 == 0, "ntxent: rows/cols must be multiples of 16");
  TORCH_CHECK(D == 32 || D == 64 || D == 128 || D == 256, "ntxent: D must be 32/64/128/256");
  TORCH_CHECK(2 * n_local == R, "ntxent: R must be 2*n_local");
  TORCH_CHECK(col_offset >= 0 && col_offset + R <= Ccols, "ntxent: bad col_offset");
}
int64_t nt_fwd_splits(int64_t R, int64_t C) { return ntxent_fwd_splits(R, C); }
// rows [R][D] -> columns [c0, c0 + R) of out [D][Ccols]
void nt_transpose_cols(const Tensor& in, const Tensor& out, int64_t c0) {
  const int R = in.size(0), D = in.size(1);
  TORCH_CHECK(out.dim() == 2 && out.size(0) == D && c0 >= 0 && c0 + R <= out.size(1),
              "nt_transpose_cols: out must be [D][Ccols] with room for columns [c0, c0 + R)");
  ntxent_transpose_cols(f32(in, "in"), f32w(out, "out"), R, D, (int)out.size(1), (int)c0,
                        cur_stream());
}
// forward partials of columns [c_lo, c_hi) into splits [split_base, split_base + splits)
void nt_forward_range(const Tensor& znT, int64_t R, int64_t col_offset, int64_t n_local,
                      double inv_temp, const Tensor& part, int64_t c_lo, int64_t c_hi,
                      int64_t splits, int64_t split_base) {
  const int D = znT.size(0), Ccols = znT.size(1);
  check_nt(R, Ccols, D, col_offset, n_local);
  TORCH_CHECK(c_lo >= 0 && c_lo < c_hi && c_hi <= Ccols && c_lo % 16 == 0 && c_hi % 16 == 0 &&
                  splits >= 1 && split_base >= 0 && part.numel() >= (split_base + splits) * R * 3,
              "nt_forward_range: column window / splits");
  ntxent_forward_range(f32(znT, "znT"), R, Ccols, D, col_offset, n_local, (float)inv_temp,
                       f32w(part, "part"), c_lo, c_hi, splits, split_base, cur_stream());
}
void nt_finish(const Tensor& part, int64_t R, int64_t splits, const Tensor& lse,
               const Tensor& loss) {
  TORCH_CHECK(part.numel() >= splits * R * 3 && lse.numel() == R && loss.numel() == R,
              "nt_finish sizes");
  ntxent_finish(f32(part, "part"), R, splits, f32w(lse, "lse"), f32w(loss, "loss"), cur_stream());
}
int64_t nt_bwd_splits(int64_t nown, int64_t npart) { return ntxent_bwd_splits(nown, npart); }
void nt_forward(const Tensor& znT, int64_t R, int64_t col_offset, int64_t n_local, double inv_temp,
                const Tensor& part, int64_t splits, const Tensor& lse, const Tensor& loss) {
  const int D = znT.size(0), Ccols = znT.size(1);
  check_nt(R, Ccols, D, col_offset, n_local);
  TORCH_CHECK(part.numel() >= splits * R * 3 && lse.numel() == R && loss.numel() == R,
              "nt_forward sizes");
  ntxent_forward(f32(znT, "znT"), R, Ccols, D, col_offset, n_local, (float)inv_temp,
                 f32w(part, "part"), splits, f32w(lse, "lse"), f32w(loss, "loss"), cur_stream());
}
void nt_backward_part(bool row_mode, const Tensor& zn, const Tensor& znT, const Tensor& lse,
                      int64_t R, int64_t col_offset, int64_t n_local, double inv_temp,
                      double gscale, const c10::optional<Tensor>& gout, const Tensor& part,
                      int64_t splits, const Tensor& out) {
  const int D = znT.size(0), Ccols = znT.size(1);
  check_nt(R, Ccols, D, col_offset, n_local);
  TORCH_CHECK(zn.numel() == (int64_t)Ccols * D, "nt_backward: zn size");
  const int64_t nown = row_mode ? R : Ccols;
  TORCH_CHECK(part.numel() >= splits * nown * D && out.numel() == nown * D, "nt_backward sizes");
  ntxent_backward_part(row_mode ? 1 : 0, f32(zn, "zn"), f32(znT, "znT"), f32(lse, "lse"), R, Ccols,
                       D, col_offset, n_local, (float)inv_temp, (float)gscale, optf32(gout, "gout"),
                       f32w(part, "part"), splits, f32w(out, "out"), cur_stream());
}
void nt_normalize_backward(const Tensor& zn, const Tensor& inv_norm, const Tensor& dzn,
                           const c10::optional<Tensor>& dz_bf16, const c10::optional<Tensor>& dz_f32) {
  const int R = zn.size(0), D = zn.size(1);
  TORCH_CHECK(dzn.numel() == (int64_t)R * D, "nt_normalize_backward sizes");
  ntxent_normalize_backward(f32(zn, "zn"), f32(inv_norm, "inv_norm"), f32(dzn, "dzn"), R, D,
                            optbfw(dz_bf16, "dz_bf16"), optf32w(dz_f32, "dz_f32"), cur_stream());
}
void nt_reduce_loss(const Tensor& loss_rows, double scale, const Tensor& out) {
  ntxent_reduce_loss(f32(loss_rows, "loss_rows"), loss_rows.numel(), (float)scale, f32w(out, "out"),
                     cur_stream());
}

// ------------------------------------------------------------------------------- lars
void lars_norms_op(const Tensor& p, const Tensor& g, const Tensor& chunk_beg,
                   const Tensor& chunk_end, double grad_scale, const Tensor& norms) {
  const int nchunks = chunk_beg.numel();
  TORCH_CHECK(norms.numel() >= 2 * nchunks && p.numel() == g.numel(), "lars_norms sizes");
  lars_norms(f32(p, "p"), f32(g, "g"), i32(chunk_beg, "chunk_beg"), i32(chunk_end, "chunk_end"),
             nchunks, (float)grad_scale, f32w(norms, "norms"), cur_stream());
}
void lars_update_op(const Tensor& p, const Tensor& g, const Tensor& mom,
                    const c10::optional<Tensor>& shadow, const Tensor& chunk_seg,
                    const Tensor& chunk_beg, const Tensor& chunk_end, const Tensor& seg_chunk_beg,
                    const Tensor& seg_chunk_end, const Tensor& seg_wd, const Tensor& seg_flags,
                    const Tensor& norms, const Tensor& lr, double momentum, double trust, double eps,
                    double grad_scale, bool nesterov) {
  const int nchunks = chunk_beg.numel();
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == mom.numel(), "lars_update sizes");
  if (shadow.has_value() && shadow->defined())
    TORCH_CHECK(shadow->numel() == p.numel(), "lars_update: shadow size");
  lars_update(f32w(p, "p"), f32(g, "g"), f32w(mom, "mom"), optbfw(shadow, "shadow"),
              i32(chunk_seg, "chunk_seg"), i32(chunk_beg, "chunk_beg"), i32(chunk_end, "chunk_end"),
              nchunks, i32(seg_chunk_beg, "seg_chunk_beg"), i32(seg_chunk_end, "seg_chunk_end"),
              f32(seg_wd, "seg_wd"), i32(seg_flags, "seg_flags"), f32(norms, "norms"),
              f32(lr, "lr"), (float)momentum, (float)trust, (float)eps, (float)grad_scale,
              nesterov ? 1 : 0, cur_stream());
}
void lr_step_op(const Tensor& step, const Tensor& lr, double lr0, int64_t warmup, int64_t total,
                int64_t mode) {
  check_dev(step, at::kLong, "step");
  lr_schedule_step(step.data_ptr<int64_t>(), f32w(lr, "lr"), lr0, warmup, total, (int)mode,
                   cur_stream());
}

// ------------------------------------------------------------------------------- augment
void augment_op(const Tensor& images, const c10::optional<Tensor>& indices, int64_t n,
                int64_t views, int64_t OH, int64_t OW, int64_t Cpad, double strength, int64_t seed,
                int64_t counter, int64_t view_offset, int64_t flags, const Tensor& out,
                const c10::optional<Tensor>& params) {
  check_dev(images, at::kByte, "images");
  TORCH_CHECK(images.dim() == 4 && images.size(3) == 3, "augment: images must be [N,H,W,3] uint8");
  const int H = images.size(1), W = images.size(2);
  TORCH_CHECK(Cpad >= 3, "augment: Cpad >= 3");
  TORCH_CHECK(out.numel() == views * n * OH * OW * Cpad, "augment: out size");
  const int64_t* idx = nullptr;
  if (indices.has_value() && indices->defined()) {
    check_dev(*indices, at::kLong, "indices");
    TORCH_CHECK(indices->numel() >= n, "augment: indices size");
    idx = indices->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(n <= images.size(0), "augment: n > dataset");
  }
  if (!(flags & 1)) TORCH_CHECK(OH == H && OW == W, "augment: plain mode needs OH==H, OW==W");
  float* po = nullptr;
  if (params.has_value() && params->defined()) {
    TORCH_CHECK(params->numel() >= views * n * 16, "augment: params size");
    po = f32w(*params, "params");
  }
  simclr_augment(images.data_ptr<uint8_t>(), idx, n, views, H, W, OH, OW, Cpad, (float)strength,
                 (uint64_t)seed, (uint64_t)counter, view_offset, flags, bfw(out, "out"), po,
                 cur_stream());
}

// ---- eval.hip: maxpool (K2), cross-entropy + top-k (K10), centroid class sums (K11)
void maxpool_fwd_op(const Tensor& x, const Tensor& y, const Tensor& arg, int64_t K, int64_t S,
                    int64_t P) {
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4, "maxpool: NHWC 4-D tensors expected");
  const int Nb = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int OH = (H + 2 * P - K) / S + 1, OW = (W + 2 * P - K) / S + 1;
  TORCH_CHECK(C % 8 == 0 && K >= 1 && K * K <= 255 && S >= 1 && P >= 0 && P < K,
              "maxpool: C % 8 == 0, K*K <= 255, 0 <= P < K");
  TORCH_CHECK(y.size(0) == Nb && y.size(1) == OH && y.size(2) == OW && y.size(3) == C,
              "maxpool: output shape");
  check_dev(arg, at::kByte, "arg");
  TORCH_CHECK(arg.numel() == y.numel(), "maxpool: argmax size");
  maxpool_fwd(bf(x, "x"), bfw(y, "y"), arg.data_ptr<uint8_t>(), Nb, H, W, C, OH, OW, (int)K,
              (int)S, (int)P, cur_stream());
}

void maxpool_bwd_op(const Tensor& dy, const Tensor& arg, const Tensor& dx, int64_t K, int64_t S,
                    int64_t P) {
  TORCH_CHECK(dy.dim() == 4 && dx.dim() == 4, "maxpool_bwd: NHWC 4-D tensors expected");
  const int Nb = dx.size(0), H = dx.size(1), W = dx.size(2), C = dx.size(3);
  const int OH = (H + 2 * P - K) / S + 1, OW = (W + 2 * P - K) / S + 1;
  TORCH_CHECK(C % 8 == 0 && K * K <= 255 && P < K, "maxpool_bwd: geometry");
  TORCH_CHECK(dy.size(0) == Nb && dy.size(1) == OH && dy.size(2) == OW && dy.size(3) == C,
              "maxpool_bwd: dy shape");
  check_dev(arg, at::kByte, "arg");
  TORCH_CHECK(arg.numel() == dy.numel(), "maxpool_bwd: argmax size");
  maxpool_bwd(bf(dy, "dy"), arg.data_ptr<uint8_t>(), bfw(dx, "dx"), Nb, H, W, C, OH, OW, (int)K,
              (int)S, (int)P, cur_stream());
}

// split-K small-M GEMM (projection head GEMM 2): out = relu(bn(A))·Bᵀ + bias
void gemm_sk_op(const Tensor& A, const Tensor& B, const c10::optional<Tensor>& sc,
                const c10::optional<Tensor>& sh, int64_t seg, int64_t KS, const Tensor& part,
                const c10::optional<Tensor>& bias, const Tensor& out) {
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && out.dim() == 2, "gemm_sk: 2-D operands");
  const int64_t M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K && out.size(0) == M && out.size(1) == N, "gemm_sk: shapes");
  TORCH_CHECK(M % 64 == 0 && N % 64 == 0 && KS >= 1 && K % (KS * 32) == 0 && K / KS <= 512,
              "gemm_sk: M, N multiples of 64; K / KS a multiple of 32, at most 512");
  TORCH_CHECK(part.numel() >= KS * M * N, "gemm_sk: partial scratch size");
  TORCH_CHECK(sc.has_value() == sh.has_value(), "gemm_sk: sc and sh together");
  if (sc.has_value()) {
    TORCH_CHECK(seg >= 1 && M % seg == 0, "gemm_sk: row segments");
    TORCH_CHECK(sc->numel() >= (M / seg) * K && sh->numel() >= (M / seg) * K,
                "gemm_sk: per-segment scale / shift tables");
  }
  if (bias.has_value()) TORCH_CHECK(bias->numel() == N, "gemm_sk: bias size");
  gemm_sk(bf(A, "A"), bf(B, "B"), sc.has_value() ? f32(*sc, "sc") : nullptr,
          sh.has_value() ? f32(*sh, "sh") : nullptr, (int)seg, (int)M, (int)N, (int)K, (int)KS,
          f32w(part, "part"), bias.has_value() ? f32(*bias, "bias") : nullptr, bfw(out, "out"),
          cur_stream());
}

// ImageNet stem: 2x2 space-to-depth of the zero-padded image (7x7/s2 -> 4x4/s1 conv)
void stem_s2d_op(const Tensor& img, int64_t creal, int64_t P, const Tensor& xs) {
  TORCH_CHECK(img.dim() == 4 && xs.dim() == 4, "stem_s2d: NHWC 4-D");
  const int Nb = img.size(0), H = img.size(1), W = img.size(2), Cin = img.size(3);
  TORCH_CHECK(Cin % 4 == 0 && creal >= 1 && creal <= 4 && P >= 0, "stem_s2d: channels / pad");
  TORCH_CHECK((H + 2 * P) % 2 == 0 && (W + 2 * P) % 2 == 0, "stem_s2d: padded size must be even");
  TORCH_CHECK(xs.size(0) == Nb && xs.size(1) == (H + 2 * P) / 2 && xs.size(2) == (W + 2 * P) / 2 &&
                  xs.size(3) == 16, "stem_s2d: output shape");
  stem_s2d(bf(img, "img"), bfw(xs, "xs"), Nb, H, W, Cin, (int)creal, (int)xs.size(1),
           (int)xs.size(2), (int)P, cur_stream());
}

// pooled ImageNet stem: BN + ReLU + max-pool forward, max-pool + ReLU-mask + BN backward
void bn_relu_maxpool_op(const Tensor& a, const Tensor& ss, int64_t S, const Tensor& y,
                        const Tensor& arg, const Tensor& asel, int64_t K, int64_t Sd, int64_t P) {
  TORCH_CHECK(a.dim() == 4 && y.dim() == 4 && asel.dim() == 4, "bn_relu_maxpool: NHWC 4-D");
  const int Nb = a.size(0), H = a.size(1), W = a.size(2), C = a.size(3);
  const int OH = (H + 2 * P - K) / Sd + 1, OW = (W + 2 * P - K) / Sd + 1;
  TORCH_CHECK(C % 8 == 0 && K >= 1 && K * K <= 255 && Sd >= 1 && P >= 0 && P < K,
              "bn_relu_maxpool: geometry");
  TORCH_CHECK(S >= 1 && Nb % S == 0, "bn_relu_maxpool: images must split evenly into views");
  TORCH_CHECK(y.size(0) == Nb && y.size(1) == OH && y.size(2) == OW && y.size(3) == C &&
                  asel.sizes() == y.sizes(), "bn_relu_maxpool: output shapes");
  TORCH_CHECK(ss.numel() == 2 * S * C, "bn_relu_maxpool: scale/shift table [2][S][C]");
  check_dev(arg, at::kByte, "arg");
  TORCH_CHECK(arg.numel() == y.numel(), "bn_relu_maxpool: argmax size");
  bn_relu_maxpool(bf(a, "a"), f32(ss, "ss"), (int)S, bfw(y, "y"), arg.data_ptr<uint8_t>(),
                  bfw(asel, "asel"), Nb, H, W, C, OH, OW, (int)K, (int)Sd, (int)P, cur_stream());
}

void maxpool_bwd_bn_op(const Tensor& gy, const Tensor& arg, const Tensor& y, const Tensor& a,
                       const Tensor& coef, int64_t S, const Tensor& da, int64_t K, int64_t Sd,
                       int64_t P) {
  TORCH_CHECK(a.dim() == 4 && da.dim() == 4 && gy.dim() == 4 && y.dim() == 4,
              "maxpool_bwd_bn: NHWC 4-D");
  const int Nb = a.size(0), H = a.size(1), W = a.size(2), C = a.size(3);
  const int OH = (H + 2 * P - K) / Sd + 1, OW = (W + 2 * P - K) / Sd + 1;
  TORCH_CHECK(C % 8 == 0 && K * K <= 255 && Sd >= 1 && P >= 0 && P < K, "maxpool_bwd_bn: geometry");
  TORCH_CHECK(S >= 1 && Nb % S == 0, "maxpool_bwd_bn: images must split evenly into views");
  TORCH_CHECK(gy.size(0) == Nb && gy.size(1) == OH && gy.size(2) == OW && gy.size(3) == C &&
                  y.sizes() == gy.sizes() && da.sizes() == a.sizes(),
              "maxpool_bwd_bn: shapes");
  TORCH_CHECK(coef.numel() == 3 * S * C, "maxpool_bwd_bn: coef [3][S][C]");
  check_dev(arg, at::kByte, "arg");
  TORCH_CHECK(arg.numel() == gy.numel(), "maxpool_bwd_bn: argmax size");
  maxpool_bwd_bn(bf(gy, "gy"), arg.data_ptr<uint8_t>(), bf(y, "y"), bf(a, "a"), f32(coef, "coef"),
                 (int)S, bfw(da, "da"), Nb, H, W, C, OH, OW, (int)K, (int)Sd, (int)P, cur_stream());
}

void ce_topk_op(const Tensor& logits, const Tensor& y, double gscale, const Tensor& loss,
                const Tensor& rank, const c10::optional<Tensor>& dlogits) {
  TORCH_CHECK(logits.dim() == 2, "ce_topk: logits [B][C]");
  const int B = logits.size(0), C = logits.size(1);
  check_dev(y, at::kLong, "y");
  check_dev(rank, at::kInt, "rank");
  TORCH_CHECK(y.numel() == B && loss.numel() == B && rank.numel() == B, "ce_topk: row counts");
  float* dl = optf32w(dlogits, "dlogits");
  if (dl) TORCH_CHECK(dlogits->numel() == (int64_t)B * C, "ce_topk: dlogits size");
  ce_topk(f32(logits, "logits"), y.data_ptr<int64_t>(), B, C, (float)gscale, f32w(loss, "loss"),
          rank.data_ptr<int>(), dl, cur_stream());
}

void class_sums_op(const Tensor& X, const Tensor& y, int64_t NC, const Tensor& sums,
                   const Tensor& counts) {
  TORCH_CHECK(X.dim() == 2, "class_sums: X [N][D]");
  const int N = X.size(0), D = X.size(1);
  check_dev(y, at::kLong, "y");
  TORCH_CHECK(y.numel() == N, "class_sums: labels");
  TORCH_CHECK(NC >= 1 && class_sums_lds((int)NC) <= 64 * 1024, "class_sums: at most ~250 classes");
  TORCH_CHECK(sums.numel() == NC * D && counts.numel() == NC, "class_sums: output sizes");
  const int G = class_sums_groups(N);
  at::Tensor part = at::empty({(int64_t)G * NC * D}, X.options());
  at::Tensor pcnt = at::empty({(int64_t)G * NC}, X.options());
  class_sums(f32(X, "X"), y.data_ptr<int64_t>(), N, D, (int)NC, part.data_ptr<float>(),
             pcnt.data_ptr<float>(), f32w(sums, "sums"), f32w(counts, "counts"), cur_stream());
}

}  // namespace


TORCH_LIBRARY(simclr_amd, m) {
  m.def("maxpool_fwd(Tensor x, Tensor(a!) y, Tensor(b!) arg, int K, int S, int P) -> ()", &maxpool_fwd_op);
  m.def("maxpool_bwd(Tensor dy, Tensor arg, Tensor(a!) dx, int K, int S, int P) -> ()", &maxpool_bwd_op);
  m.def("stem_s2d(Tensor img, int creal, int P, Tensor(a!) xs) -> ()", &stem_s2d_op);
  m.def("gemm_sk(Tensor A, Tensor B, Tensor? sc, Tensor? sh, int seg, int KS, Tensor(a!) part, "
        "Tensor? bias, Tensor(b!) out) -> ()", &gemm_sk_op);
  m.def("bn_relu_maxpool(Tensor a, Tensor ss, int S, Tensor(a!) y, Tensor(b!) arg, Tensor(c!) asel, "
        "int K, int Sd, int P) -> ()", &bn_relu_maxpool_op);
  m.def("maxpool_bwd_bn(Tensor gy, Tensor arg, Tensor y, Tensor a, Tensor coef, int S, Tensor(a!) da, "
        "int K, int Sd, int P) -> ()", &maxpool_bwd_bn_op);
  m.def("ce_topk(Tensor logits, Tensor y, float gscale, Tensor(a!) loss, Tensor(b!) rank, Tensor(c!)? dlogits=None) -> ()", &ce_topk_op);
  m.def("class_sums(Tensor X, Tensor y, int NC, Tensor(a!) sums, Tensor(b!) counts) -> ()", &class_sums_op);
  m.def("igemm(Tensor A, Tensor B, Tensor(a!) out, Tensor? bias, Tensor(b!)? stats, int[] geom, Tensor? pro_sc=None, Tensor? pro_sh=None, int pro_seg_rows=0, bool pro_relu=False, int epi_mode=0, Tensor? epi_a=None, Tensor? epi_b=None, int variant=-1, Tensor? epi_ss=None, Tensor? epi_mi=None, int seg_rows=0, int stats_seg_blocks=0, int stats_base=0, Tensor? epi_c=None, Tensor? epi_mask=None, Tensor? epi_c2=None, Tensor? epi_mi2=None, Tensor(c!)? stats2=None, Tensor? pro_d=None, Tensor? A2=None, Tensor? pro_rss=None, Tensor(d!)? pro_out=None, Tensor(e!)? pro_mask=None) -> ()", &igemm);
  m.def("igemm_dual_ok(int v, int[] geom) -> bool", &igemm_dok);
  m.def("igemm_bm(int N) -> int", &igemm_bm);
  m.def("igemm_nvariants() -> int", &igemm_nvariants);
  m.def("igemm_variant_bm(int v) -> int", &igemm_vbm);
  m.def("igemm_variant_bn(int v) -> int", &igemm_vbn);
  m.def("igemm_variant_glds(int v) -> bool", &igemm_vglds);
  m.def("igemm_glds_ok(int[] geom, bool pro, bool bn_bwd_pro) -> bool", &igemm_gldsok);
  m.def("wgrad_nvariants() -> int", &wgrad_nvariants);
  m.def("wgrad_xlin(int mode=-1) -> int", &wgrad_xlin_op);
  m.def("wgrad_variant_glds(int v) -> bool", &wgrad_vglds);
  m.def("igemm_variant_patch(int v) -> bool", [](int64_t v) {
    return v >= 0 && v < igemm_num_variants() && igemm_variant_patch((int)v);
  });
  m.def("wgrad_variant_area(int v) -> int", [](int64_t v) -> int64_t {
    TORCH_CHECK(v >= 0 && v < wgrad_num_variants(), "wgrad variant out of range");
    return wgrad_variant_area((int)v);
  });
  m.def("igemm_variant_ok(int v, int[] geom, bool pro, bool bn_bwd_pro) -> bool", &igemm_vok);
  m.def("wgrad_variant_ok(int v, int[] geom, bool pro, bool dy_pro) -> bool", &wgrad_vok);
  m.def("wgrad_splits(int[] geom, int variant=-1) -> int", &wgrad_nsplit);
  m.def("wgrad_tiles(int[] geom, int variant=-1) -> int", &wgrad_ntiles);
  m.def("conv1x1_bwd_dual_s2(Tensor G, Tensor? A3, Tensor? coef, Tensor X, Tensor Wt, "
        "Tensor(a!) gm, Tensor(b!) wpart, int S, int bps) -> ()", &conv1x1_bwd_dual_s2_op);
  m.def("conv1x1_bwd_dual(Tensor G, Tensor? A3, Tensor? coef, Tensor X, Tensor? xss, Tensor? xmi, Tensor Wt, Tensor(a!) gm, Tensor(b!) stats, Tensor(c!) wpart, int S, int bps, Tensor? Xraw=None, bool dual8=False) -> ()", &conv1x1_bwd_dual_op);
  m.def("wgrad_reduce_slabs(Tensor(a!) partial, int splits, Tensor(b!) out, float beta=0.0) -> ()", &wgrad_reduce_slabs_op);
  m.def("wgrad(Tensor dY, Tensor X, Tensor(a!) partial, Tensor(b!) out, int[] geom, int splits, int creal, float beta, Tensor? pro_sc=None, Tensor? pro_sh=None, int pro_seg_rows=0, bool pro_relu=False, int pro_S=1, int variant=-1, Tensor? dY2=None, Tensor? dp_coef=None, int dp_seg_rows=0, int dp_S=1) -> ()", &wgrad);
  m.def("weight_transform(Tensor W, Tensor(a!) Wt, int[] p) -> ()", &weight_transform);
  m.def("weight_transform_plan(Tensor[] Ws, Tensor[] Wts, int[] p) -> Tensor", &weight_transform_plan);
  m.def("weight_transform_batch(Tensor table, int total_blocks) -> ()", &weight_transform_batch);
  m.def("bn_blocks(int R, int C, int S) -> int", &bn_blocks);
  m.def("bn_stats(Tensor x, int S, Tensor(a!) partial) -> ()", &bn_stats);
  m.def("bn_reduce(Tensor partial, int nblk, int S, int C, Tensor(a!) stats) -> ()", &bn_reduce);
  m.def("bn_finalize(Tensor stats, int S, int C, float count, float eps, float momentum, Tensor(a!)? rm, Tensor(b!)? rv, Tensor(c!) mi, Tensor(d!)? nbt, Tensor? gamma=None, Tensor? beta=None, Tensor(e!)? ss=None) -> ()", &bn_final);
  m.def("ipc_collective(int op, Tensor src, Tensor(a!) dst, Tensor peers, Tensor(b!) arena, int site, Tensor(c!) epoch, Tensor(d!) err, int world, int rank) -> ()", &ipc_collective_op);
  m.def("ipc_coll_blocks() -> int", []() -> int64_t { return IPC_COLL_BLOCKS; });
  m.def("bn_reduce_fused(Tensor partial, int nblk, int S, int C, int mode, Tensor(a!)? stats=None, float count=1.0, float eps=1e-5, float momentum=0.1, Tensor(b!)? rm=None, Tensor(c!)? rv=None, Tensor(d!)? mi=None, Tensor(e!)? nbt=None, Tensor? gamma=None, Tensor? beta=None, Tensor(f!)? ss=None, Tensor(g!)? dgamma=None, Tensor(h!)? dbeta=None, Tensor(i!)? coef=None, int ticket_slot=0, Tensor? ipc_peers=None, Tensor(j!)? ipc_arena=None, int ipc_site=0, Tensor(k!)? ipc_epoch=None, Tensor(l!)? ipc_err=None, int world=1, int rank=0) -> ()", &bn_reduce_fused_op);
  // the ticket arrays are allocated outside any capture: Trainer.capture() calls this first
  m.def("bn_tickets_init(Tensor like) -> ()", [](const Tensor& like) { (void)tickets_for(like, 0, 0); });
  m.def("bn_apply_ss(Tensor x, Tensor ss, Tensor? res, Tensor? rss, Tensor(a!) y, int S, bool relu, Tensor(b!)? mask=None) -> ()", &bn_apply_ss_op);
  m.def("bn_apply(Tensor x, Tensor? res, Tensor(a!) y, Tensor mi, Tensor? gamma, Tensor? beta, int S, bool relu) -> ()", &bn_apply_op);
  m.def("bn_apply_eval(Tensor x, Tensor? res, Tensor(a!) y, Tensor rm, Tensor rv, Tensor? gamma, Tensor? beta, float eps, bool relu) -> ()", &bn_apply_eval_op);
  m.def("bn_bwd_reduce(Tensor dy, Tensor? y, Tensor x, Tensor mi, int S, bool relu, Tensor(a!) partial) -> ()", &bn_bwd_reduce_op);
  m.def("bn_bwd_finalize(Tensor sums, Tensor mi, Tensor? gamma, int S, int C, float count, Tensor(a!)? dgamma, Tensor(b!)? dbeta, Tensor(c!) coef) -> ()", &bn_bwd_final);
  m.def("bn_bwd_apply(Tensor dy, Tensor? y, Tensor x, Tensor coef, int S, bool relu, Tensor(a!) dx, Tensor(b!)? dres) -> ()", &bn_bwd_apply_op);
  m.def("bn_bwd_apply2(Tensor g, Tensor x1, Tensor coef1, Tensor(a!) dx1, Tensor x2, Tensor coef2, Tensor(b!) dx2, int S) -> ()", &bn_bwd_apply2_op);
  m.def("avgpool_fwd(Tensor x, Tensor(a!) y, int Nb, int HW, int C) -> ()", &avgpool_fwd_op);
  m.def("avgpool_bwd(Tensor dy, Tensor(a!) dx, int Nb, int HW, int C) -> ()", &avgpool_bwd_op);
  m.def("colsum(Tensor x, Tensor(a!) out, float beta) -> ()", &colsum_op);
  m.def("cast_to_bf16(Tensor x, Tensor(a!) y) -> ()", &cast_to_bf16);
  m.def("cast_to_f32(Tensor x, Tensor(a!) y) -> ()", &cast_to_f32);
  m.def("nt_normalize(Tensor z, Tensor(a!) zn, Tensor(b!) inv_norm) -> ()", &nt_normalize);
  m.def("nt_transpose(Tensor x, Tensor(a!) out) -> ()", &nt_transpose);
  m.def("nt_transpose_cols(Tensor x, Tensor(a!) out, int c0) -> ()", &nt_transpose_cols);
  m.def("nt_forward_range(Tensor znT, int R, int col_offset, int n_local, float inv_temp, Tensor(a!) part, int c_lo, int c_hi, int splits, int split_base) -> ()", &nt_forward_range);
  m.def("nt_finish(Tensor part, int R, int splits, Tensor(a!) lse, Tensor(b!) loss) -> ()", &nt_finish);
  m.def("nt_fwd_splits(int R, int C) -> int", &nt_fwd_splits);
  m.def("nt_bwd_splits(int nown, int npart) -> int", &nt_bwd_splits);
  m.def("nt_forward(Tensor znT, int R, int col_offset, int n_local, float inv_temp, Tensor(a!) part, int splits, Tensor(b!) lse, Tensor(c!) loss) -> ()", &nt_forward);
  m.def("nt_backward_part(bool row_mode, Tensor zn, Tensor znT, Tensor lse, int R, int col_offset, int n_local, float inv_temp, float gscale, Tensor? gout, Tensor(a!) part, int splits, Tensor(b!) out) -> ()", &nt_backward_part);
  m.def("nt_normalize_backward(Tensor zn, Tensor inv_norm, Tensor dzn, Tensor(a!)? dz_bf16, Tensor(b!)? dz_f32) -> ()", &nt_normalize_backward);
  m.def("nt_reduce_loss(Tensor loss_rows, float scale, Tensor(a!) out) -> ()", &nt_reduce_loss);
  m.def("lars_norms(Tensor p, Tensor g, Tensor chunk_beg, Tensor chunk_end, float grad_scale, Tensor(a!) norms) -> ()", &lars_norms_op);
  m.def("lars_update(Tensor(a!) p, Tensor g, Tensor(b!) mom, Tensor(c!)? shadow, Tensor chunk_seg, Tensor chunk_beg, Tensor chunk_end, Tensor seg_chunk_beg, Tensor seg_chunk_end, Tensor seg_wd, Tensor seg_flags, Tensor norms, Tensor lr, float momentum, float trust, float eps, float grad_scale, bool nesterov) -> ()", &lars_update_op);
  m.def("lr_step(Tensor(a!) step, Tensor(b!) lr, float lr0, int warmup, int total, int mode) -> ()", &lr_step_op);
  m.def("augment(Tensor images, Tensor? indices, int n, int views, int OH, int OW, int Cpad, float strength, int seed, int counter, int view_offset, int flags, Tensor(a!) out, Tensor(b!)? params) -> ()", &augment_op);
}
