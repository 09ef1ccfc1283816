// Host-side invariants of the kernel launchers, built with AddressSanitizer + UBSan by
// tests/test_host_sanitizers.py (sanitizer builds of the C++ host code; GPU-side
// sanitizers are unavailable on this pool).  Only host logic runs here — the tile-variant
// admissibility / split planning of conv.hip, the BatchNorm reduction planning of bn.hip and
// the split / workspace arithmetic of ntxent.hip and eval.hip — over every convolution of
// ResNet-18/50 at the CIFAR (32x32) and ImageNet (224x224) shapes, in all three passes.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../simclr_amd/csrc/kernels.h"

namespace {

int failures = 0;
#define EXPECT(cond, ...)                                  \
  do {                                                     \
    if (!(cond)) {                                         \
      std::fprintf(stderr, "FAIL %s: ", #cond);            \
      std::fprintf(stderr, __VA_ARGS__);                   \
      std::fprintf(stderr, "\n");                          \
      ++failures;                                          \
    }                                                      \
  } while (0)

ConvGeom fwd_geom(int N, int H, int W, int C, int k, int s, int p, int Co) {
  const int OH = (H + 2 * p - k) / s + 1, OW = (W + 2 * p - k) / s + 1;
  return ConvGeom{N, H, W, C, OH, OW, k, k, s, s, 1, 1, -p, -p, Co, OH, OW, 1, 1, 0, 0, Co};
}

struct Conv { int C, Co, k, s, H; };

std::vector<Conv> resnet_convs(bool bottleneck, int H0, bool imagenet_stem) {
  std::vector<Conv> v;
  int H = H0;
  if (imagenet_stem) { v.push_back({8, 64, 7, 2, H}); H = (H + 6 - 7) / 2 + 1; H = (H + 2 - 3) / 2 + 1; }
  else v.push_back({8, 64, 3, 1, H});
  int inpl = 64;
  const int planes[4] = {64, 128, 256, 512}, blocks[4] = {bottleneck ? 3 : 2, bottleneck ? 4 : 2,
                                                          bottleneck ? 6 : 2, bottleneck ? 3 : 2};
  for (int l = 0; l < 4; ++l) {
    for (int b = 0; b < blocks[l]; ++b) {
      const int s = (b == 0 && l > 0) ? 2 : 1;
      const int out = bottleneck ? planes[l] * 4 : planes[l];
      if (bottleneck) {
        v.push_back({inpl, planes[l], 1, 1, H});
        v.push_back({planes[l], planes[l], 3, s, H});
        const int Ho = (H + 2 - 3) / s + 1;
        v.push_back({planes[l], out, 1, 1, Ho});
      } else {
        v.push_back({inpl, planes[l], 3, s, H});
        const int Ho = (H + 2 - 3) / s + 1;
        v.push_back({planes[l], planes[l], 3, 1, Ho});
      }
      if (b == 0 && (s != 1 || inpl != out)) v.push_back({inpl, out, 1, s, H});
      H = (H + 2 - 3) / s + 1;
      inpl = out;
    }
  }
  return v;
}

void check_net(const char* name, bool bottleneck, int H0, bool imagenet, int batch) {
  for (const Conv& c : resnet_convs(bottleneck, H0, imagenet)) {
    const int p = c.k / 2;
    const ConvGeom g = fwd_geom(batch, c.H, c.H, c.C, c.k, c.s, p, c.Co);
    const long long M = (long long)g.Nb * g.OH * g.OW;
    int ok = 0;
    for (int v = 0; v < igemm_num_variants(); ++v) {
      const int bm = igemm_variant_bm(v), bn = igemm_variant_bn(v);
      EXPECT(bm > 0 && bn > 0 && bm % 16 == 0 && bn % 16 == 0, "%s variant %d tile %dx%d", name, v,
             bm, bn);
      ok += igemm_variant_ok(v, g, false, false) ? 1 : 0;
      (void)igemm_dual_ok(v, g);
    }
    EXPECT(ok > 0, "%s: no igemm variant for C=%d Co=%d k=%d s=%d H=%d", name, c.C, c.Co, c.k, c.s, c.H);
    int wok = 0;
    for (int v = 0; v < wgrad_num_variants(); ++v) {
      if (!wgrad_variant_ok(v, g, false, false)) continue;
      ++wok;
      const int sp = wgrad_splits(g, v);
      EXPECT(sp >= 1 && (long long)sp <= (M + 63) / 64, "%s wgrad splits %d for M=%lld", name, sp, M);
    }
    EXPECT(wok > 0 || c.C % 8 != 0, "%s: no wgrad variant for C=%d Co=%d k=%d", name, c.C, c.Co, c.k);
    const int nb = bn_stats_blocks_per_seg((int)(M / 2), c.Co, 2);
    EXPECT(nb >= 1, "%s bn blocks", name);
    const int G = bn_reduce_groups(nb);
    EXPECT(G >= 1 && G <= nb, "%s bn groups %d of %d rows", name, G, nb);
    EXPECT(bn_ipc_region_words(8, 2, c.Co) == 2LL * 8 * 2 * 2 * c.Co, "%s ipc region", name);
  }
}

}  // namespace

int main() {
  for (int batch : {64, 1024}) {
    check_net("resnet50-cifar", true, 32, false, batch);
    check_net("resnet18-cifar", false, 36, false, batch);
    check_net("resnet50-imagenet@32", true, 32, true, batch);
  }
  check_net("resnet50-imagenet@224", true, 224, true, 256);
  for (int R : {128, 1024, 8192})
    for (int Cc : {R, 8 * R}) {
      EXPECT(ntxent_fwd_splits(R, Cc) >= 1, "nt fwd splits");
      EXPECT(ntxent_bwd_splits(R, Cc) >= 1, "nt bwd splits");
    }
  for (int N : {10, 5000, 50000}) EXPECT(class_sums_groups(N) >= 1, "class sums groups");
  EXPECT(class_sums_lds(100) <= 64 * 1024, "class sums lds");
  EXPECT(colsum_groups(1024) >= 1 && colsum_groups(1) >= 1, "colsum groups");
  std::printf("host_check: %d failure(s)\n", failures);
  return failures ? 1 : 0;
}
