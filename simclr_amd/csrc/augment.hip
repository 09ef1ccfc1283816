// On-device SimCLR augmentation (gfx950): one workgroup per (image, view).
//
// Reference: create_simclr_data_augmentation (/root/reference/dataset.py:19-38) run by 8 CPU
// DataLoader workers per GPU through PIL:
//   RandomResizedCrop(32, scale=(0.08,1), ratio=(3/4,4/3), bilinear) → RandomHorizontalFlip(0.5)
//   → RandomApply([ColorJitter(0.8s,0.8s,0.8s,0.2s)], p=0.8) → RandomGrayscale(0.2) → ToTensor.
// The uint8 dataset lives in HBM once (CIFAR-10 = 150 MB); per step only an index vector moves.
// Parameters follow torchvision's samplers (10-attempt rejection sampling with the central-crop
// fallback, jitter factors U[max(0,1-x), 1+x], random op order per image); pixel math follows
// PIL (half-pixel-centre bilinear with edge clamp, uint8 rounding between ops, blend truncation,
// ITU-R 601-2 luma with PIL's fixed-point rounding, contrast against the rounded mean luma).
// Hue uses a float HSV round trip (PIL's uint8 HSV differs by quantisation only).
// Output: bf16 NHWC with the channel dim zero-padded to Cpad (8) for 16-byte conv gathers.
// RNG: counter-based splitmix64 keyed by (seed, step counter, view, dataset index) — independent
// of rank count and launch order.
#include <math.h>
#include "common.h"
#include "kernels.h"

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct Rng {
  uint64_t key;
  uint64_t ctr;
  __device__ float uniform() {  // [0, 1)
    const uint64_t r = splitmix64(key ^ (0xD1B54A32D192ED03ull * (++ctr)));
    return (float)(r >> 40) * (1.0f / 16777216.0f);
  }
  __device__ float uniform(float a, float b) { return a + (b - a) * uniform(); }
  __device__ int randint(int lo, int hi_excl) {  // [lo, hi)
    const uint64_t r = splitmix64(key ^ (0xD1B54A32D192ED03ull * (++ctr)));
    return lo + (int)(r % (uint64_t)(hi_excl - lo));
  }
};

struct AugParams {
  int ci, cj, ch, cw;   // crop
  int flip;
  int jitter;           // jitter applied
  int order[4];         // 0 brightness 1 contrast 2 saturation 3 hue
  float fb, fc, fs, fh;
  int gray;
};

__device__ void sample_params(Rng& rng, int H, int W, float strength, AugParams& P) {
  // RandomResizedCrop.get_params
  const float area = (float)(H * W);
  const float lr0 = logf(3.f / 4.f), lr1 = logf(4.f / 3.f);
  bool found = false;
  for (int t = 0; t < 10 && !found; ++t) {
    const float target = area * rng.uniform(0.08f, 1.0f);
    const float ar = expf(rng.uniform(lr0, lr1));
    const int w = (int)rintf(sqrtf(target * ar));
    const int h = (int)rintf(sqrtf(target / ar));
    if (w > 0 && w <= W && h > 0 && h <= H) {
      P.ci = rng.randint(0, H - h + 1);
      P.cj = rng.randint(0, W - w + 1);
      P.ch = h;
      P.cw = w;
      found = true;
    }
  }
  if (!found) {
    const float in_ratio = (float)W / (float)H;
    int w, h;
    if (in_ratio < 3.f / 4.f) {
      w = W; h = (int)rintf(w / (3.f / 4.f));
    } else if (in_ratio > 4.f / 3.f) {
      h = H; w = (int)rintf(h * (4.f / 3.f));
    } else {
      w = W; h = H;
    }
    P.ci = (H - h) / 2; P.cj = (W - w) / 2; P.ch = h; P.cw = w;
  }
  P.flip = rng.uniform() < 0.5f;
  // RandomApply(p=0.8): applied unless p < rand
  P.jitter = !(0.8f < rng.uniform());
  // ColorJitter.get_params: randperm(4) then factors
  int ord[4] = {0, 1, 2, 3};
  for (int i = 3; i > 0; --i) {
    const int j = rng.randint(0, i + 1);
    const int t = ord[i]; ord[i] = ord[j]; ord[j] = t;
  }
  for (int i = 0; i < 4; ++i) P.order[i] = ord[i];
  const float b = 0.8f * strength, c = 0.8f * strength, s = 0.8f * strength, h = 0.2f * strength;
  P.fb = rng.uniform(fmaxf(0.f, 1.f - b), 1.f + b);
  P.fc = rng.uniform(fmaxf(0.f, 1.f - c), 1.f + c);
  P.fs = rng.uniform(fmaxf(0.f, 1.f - s), 1.f + s);
  P.fh = rng.uniform(-h, h);
  P.gray = rng.uniform() < 0.2f;
}

__device__ __forceinline__ float clip_trunc(float v) {  // PIL blend: clip then truncate to uint8
  return v <= 0.f ? 0.f : (v >= 255.f ? 255.f : floorf(v));
}

__device__ __forceinline__ int luma(float r, float g, float b) {  // PIL L24 fixed point
  return ((int)r * 19595 + (int)g * 38470 + (int)b * 7471 + 0x8000) >> 16;
}

__device__ void rgb2hsv(float r, float g, float b, float& h, float& s, float& v) {
  const float mx = fmaxf(r, fmaxf(g, b)), mn = fminf(r, fminf(g, b));
  v = mx;
  const float d = mx - mn;
  s = mx > 0.f ? d / mx : 0.f;
  if (d <= 0.f) { h = 0.f; return; }
  float hh;
  if (mx == r) hh = (g - b) / d;
  else if (mx == g) hh = 2.f + (b - r) / d;
  else hh = 4.f + (r - g) / d;
  hh /= 6.f;
  h = hh - floorf(hh);
}

__device__ void hsv2rgb(float h, float s, float v, float& r, float& g, float& b) {
  const float h6 = h * 6.f;
  const int i = ((int)floorf(h6)) % 6;
  const float f = h6 - floorf(h6);
  const float p = v * (1.f - s), q = v * (1.f - s * f), t = v * (1.f - s * (1.f - f));
  switch (i) {
    case 0: r = v; g = t; b = p; break;
    case 1: r = q; g = v; b = p; break;
    case 2: r = p; g = v; b = t; break;
    case 3: r = p; g = q; b = v; break;
    case 4: r = t; g = p; b = v; break;
    default: r = v; g = p; b = q; break;
  }
}

constexpr int AUG_THREADS = 256;
constexpr int MAX_PIX_PER_THREAD = 16;  // up to 64x64 outputs

__global__ __launch_bounds__(AUG_THREADS) void k_augment(const uint8_t* __restrict__ images,
                                                         const int64_t* __restrict__ indices,
                                                         int n, int H, int W, int OH, int OW,
                                                         int Cpad, float strength, uint64_t seed,
                                                         uint64_t counter, int view_offset,
                                                         int flags, uint16_t* __restrict__ out,
                                                         float* __restrict__ params_out) {
  __shared__ AugParams P;
  __shared__ int red[AUG_THREADS / 64];
  const int b = blockIdx.x, view = blockIdx.y + view_offset;
  const int64_t idx = indices ? indices[b] : (int64_t)b;
  const uint8_t* img = images + (size_t)idx * H * W * 3;
  const bool augment = flags & 1;
  if (threadIdx.x == 0) {
    if (augment) {
      Rng rng{splitmix64(seed ^ splitmix64(counter * 0x9E3779B97F4A7C15ull + (uint64_t)view) ^
                         splitmix64((uint64_t)idx + 0x632BE59BD9B4E019ull)), 0};
      sample_params(rng, H, W, strength, P);
    } else {
      P.ci = 0; P.cj = 0; P.ch = H; P.cw = W; P.flip = 0; P.jitter = 0; P.gray = 0;
      P.fb = P.fc = P.fs = 1.f; P.fh = 0.f;
      for (int i = 0; i < 4; ++i) P.order[i] = i;
    }
    if (params_out) {
      float* po = params_out + ((size_t)blockIdx.y * n + b) * 16;
      po[0] = P.ci; po[1] = P.cj; po[2] = P.ch; po[3] = P.cw; po[4] = P.flip; po[5] = P.jitter;
      for (int i = 0; i < 4; ++i) po[6 + i] = P.order[i];
      po[10] = P.fb; po[11] = P.fc; po[12] = P.fs; po[13] = P.fh; po[14] = P.gray; po[15] = 0.f;
    }
  }
  __syncthreads();
  const int npix = OH * OW;
  float R[MAX_PIX_PER_THREAD], G[MAX_PIX_PER_THREAD], B[MAX_PIX_PER_THREAD];
  const int myn = (npix - (int)threadIdx.x + AUG_THREADS - 1) / AUG_THREADS;
  // resized crop (+ flip), rounded to uint8 like PIL
  const float sy = (float)P.ch / OH, sx = (float)P.cw / OW;
#pragma unroll
  for (int k = 0; k < MAX_PIX_PER_THREAD; ++k) {
    if (k >= myn) break;
    const int p = threadIdx.x + k * AUG_THREADS;
    const int oy = p / OW;
    int ox = p - oy * OW;
    if (P.flip) ox = OW - 1 - ox;
    float fy = (oy + 0.5f) * sy - 0.5f;
    float fx = (ox + 0.5f) * sx - 0.5f;
    fy = fminf(fmaxf(fy, 0.f), (float)(P.ch - 1));
    fx = fminf(fmaxf(fx, 0.f), (float)(P.cw - 1));
    const int y0 = (int)floorf(fy), x0 = (int)floorf(fx);
    const int y1 = min(y0 + 1, P.ch - 1), x1 = min(x0 + 1, P.cw - 1);
    const float wy = fy - y0, wx = fx - x0;
    const uint8_t* p00 = img + ((size_t)(P.ci + y0) * W + (P.cj + x0)) * 3;
    const uint8_t* p01 = img + ((size_t)(P.ci + y0) * W + (P.cj + x1)) * 3;
    const uint8_t* p10 = img + ((size_t)(P.ci + y1) * W + (P.cj + x0)) * 3;
    const uint8_t* p11 = img + ((size_t)(P.ci + y1) * W + (P.cj + x1)) * 3;
    float c3[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float top = p00[c] + wx * (p01[c] - p00[c]);
      const float bot = p10[c] + wx * (p11[c] - p10[c]);
      const float v = top + wy * (bot - top);
      c3[c] = fminf(fmaxf(floorf(v + 0.5f), 0.f), 255.f);
    }
    R[k] = c3[0]; G[k] = c3[1]; B[k] = c3[2];
  }
  if (P.jitter) {
    for (int oi = 0; oi < 4; ++oi) {
      const int op = P.order[oi];
      if (op == 0) {  // brightness: blend(black, img, f)
#pragma unroll
        for (int k = 0; k < MAX_PIX_PER_THREAD; ++k) {
          if (k >= myn) break;
          R[k] = clip_trunc(R[k] * P.fb); G[k] = clip_trunc(G[k] * P.fb); B[k] = clip_trunc(B[k] * P.fb);
        }
      } else if (op == 1) {  // contrast: blend(mean luma, img, f)
        int s = 0;
#pragma unroll
        for (int k = 0; k < MAX_PIX_PER_THREAD; ++k) {
          if (k >= myn) break;
          s += luma(R[k], G[k], B[k]);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        __syncthreads();
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        int tot = 0;
        for (int w = 0; w < AUG_THREADS / 64; ++w) tot += red[w];
        const float mean = floorf((float)tot / npix + 0.5f);
#pragma unroll
        for (int k = 0; k < MAX_PIX_PER_THREAD; ++k) {
          if (k >= myn) break;
          R[k] = clip_trunc(mean + P.fc * (R[k] - mean));
          G[k] = clip_trunc(mean + P.fc * (G[k] - mean));
          B[k] = clip_trunc(mean + P.fc * (B[k] - mean));
        }
      } else if (op == 2) {  // saturation: blend(gray, img, f)
#pragma unroll
        for (int k = 0; k < MAX_PIX_PER_THREAD; ++k) {
          if (k >= myn) break;
          const float l = (float)luma(R[k], G[k], B[k]);
          R[k] = clip_trunc(l + P.fs * (R[k] - l));
          G[k] = clip_trunc(l + P.fs * (G[k] - l));
          B[k] = clip_trunc(l + P.fs * (B[k] - l));
        }
      } else {  // hue
#pragma unroll
        for (int k = 0; k < MAX_PIX_PER_THREAD; ++k) {
          if (k >= myn) break;
          float h, s, v, r, g, bb;
          rgb2hsv(R[k] / 255.f, G[k] / 255.f, B[k] / 255.f, h, s, v);
          h += P.fh;
          h -= floorf(h);
          hsv2rgb(h, s, v, r, g, bb);
          R[k] = fminf(fmaxf(floorf(r * 255.f + 0.5f), 0.f), 255.f);
          G[k] = fminf(fmaxf(floorf(g * 255.f + 0.5f), 0.f), 255.f);
          B[k] = fminf(fmaxf(floorf(bb * 255.f + 0.5f), 0.f), 255.f);
        }
      }
    }
  }
  const size_t obase = ((size_t)blockIdx.y * n + b) * npix;
  const float inv255 = 1.f / 255.f;
#pragma unroll
  for (int k = 0; k < MAX_PIX_PER_THREAD; ++k) {
    if (k >= myn) break;
    const int p = threadIdx.x + k * AUG_THREADS;
    float r = R[k], g = G[k], bb = B[k];
    if (P.gray) {
      const float l = (float)luma(r, g, bb);
      r = g = bb = l;
    }
    uint16_t* o = out + (obase + p) * Cpad;
    if (Cpad == 8) {
      u32x4 w;
      w[0] = pack2bf(r * inv255, g * inv255);
      w[1] = pack2bf(bb * inv255, 0.f);
      w[2] = 0; w[3] = 0;
      *(u32x4*)o = w;
    } else {
      o[0] = f2bf(r * inv255); o[1] = f2bf(g * inv255); o[2] = f2bf(bb * inv255);
      for (int c = 3; c < Cpad; ++c) o[c] = 0;
    }
  }
}

// ---- ImageNet-shape outputs (BASELINE config 5: 224x224) --------------------------------
// The register-resident kernel above holds every output pixel of an image (<= 64x64) across
// the colour ops, because contrast blends against the mean luma of the image as it is at that
// point of the random op order.  For large outputs the block instead walks the pixels twice:
// pass 1 recomputes crop + the ops before contrast and reduces the luma sum; pass 2 recomputes
// them, applies contrast with the mean and the remaining ops and writes.  Every per-pixel op is
// deterministic, so both passes see identical values (recompute instead of a scratch image).
__device__ __forceinline__ void crop_pixel(const AugParams& P, const uint8_t* img, int W, int OH,
                                           int OW, int p, float& r, float& g, float& b) {
  const float sy = (float)P.ch / OH, sx = (float)P.cw / OW;
  const int oy = p / OW;
  int ox = p - oy * OW;
  if (P.flip) ox = OW - 1 - ox;
  float fy = (oy + 0.5f) * sy - 0.5f;
  float fx = (ox + 0.5f) * sx - 0.5f;
  fy = fminf(fmaxf(fy, 0.f), (float)(P.ch - 1));
  fx = fminf(fmaxf(fx, 0.f), (float)(P.cw - 1));
  const int y0 = (int)floorf(fy), x0 = (int)floorf(fx);
  const int y1 = min(y0 + 1, P.ch - 1), x1 = min(x0 + 1, P.cw - 1);
  const float wy = fy - y0, wx = fx - x0;
  const uint8_t* p00 = img + ((size_t)(P.ci + y0) * W + (P.cj + x0)) * 3;
  const uint8_t* p01 = img + ((size_t)(P.ci + y0) * W + (P.cj + x1)) * 3;
  const uint8_t* p10 = img + ((size_t)(P.ci + y1) * W + (P.cj + x0)) * 3;
  const uint8_t* p11 = img + ((size_t)(P.ci + y1) * W + (P.cj + x1)) * 3;
  float c3[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float top = p00[c] + wx * (p01[c] - p00[c]);
    const float bot = p10[c] + wx * (p11[c] - p10[c]);
    const float v = top + wy * (bot - top);
    c3[c] = fminf(fmaxf(floorf(v + 0.5f), 0.f), 255.f);
  }
  r = c3[0]; g = c3[1]; b = c3[2];
}

// one colour op (brightness / saturation / hue) on one pixel; contrast is handled by the caller
__device__ __forceinline__ void pixel_op(const AugParams& P, int op, float& R, float& G,
                                         float& B) {
  if (op == 0) {
    R = clip_trunc(R * P.fb); G = clip_trunc(G * P.fb); B = clip_trunc(B * P.fb);
  } else if (op == 2) {
    const float l = (float)luma(R, G, B);
    R = clip_trunc(l + P.fs * (R - l));
    G = clip_trunc(l + P.fs * (G - l));
    B = clip_trunc(l + P.fs * (B - l));
  } else if (op == 3) {
    float h, s, v, r, g, bb;
    rgb2hsv(R / 255.f, G / 255.f, B / 255.f, h, s, v);
    h += P.fh;
    h -= floorf(h);
    hsv2rgb(h, s, v, r, g, bb);
    R = fminf(fmaxf(floorf(r * 255.f + 0.5f), 0.f), 255.f);
    G = fminf(fmaxf(floorf(g * 255.f + 0.5f), 0.f), 255.f);
    B = fminf(fmaxf(floorf(bb * 255.f + 0.5f), 0.f), 255.f);
  }
}

__global__ __launch_bounds__(AUG_THREADS) void k_augment_large(
    const uint8_t* __restrict__ images, const int64_t* __restrict__ indices, int n, int H, int W,
    int OH, int OW, int Cpad, float strength, uint64_t seed, uint64_t counter, int view_offset,
    int flags, uint16_t* __restrict__ out, float* __restrict__ params_out) {
  __shared__ AugParams P;
  __shared__ long long red[AUG_THREADS / 64];
  const int b = blockIdx.x, view = blockIdx.y + view_offset;
  const int64_t idx = indices ? indices[b] : (int64_t)b;
  const uint8_t* img = images + (size_t)idx * H * W * 3;
  if (threadIdx.x == 0) {
    if (flags & 1) {
      Rng rng{splitmix64(seed ^ splitmix64(counter * 0x9E3779B97F4A7C15ull + (uint64_t)view) ^
                         splitmix64((uint64_t)idx + 0x632BE59BD9B4E019ull)), 0};
      sample_params(rng, H, W, strength, P);
    } else {
      P.ci = 0; P.cj = 0; P.ch = H; P.cw = W; P.flip = 0; P.jitter = 0; P.gray = 0;
      P.fb = P.fc = P.fs = 1.f; P.fh = 0.f;
      for (int i = 0; i < 4; ++i) P.order[i] = i;
    }
    if (params_out) {
      float* po = params_out + ((size_t)blockIdx.y * n + b) * 16;
      po[0] = P.ci; po[1] = P.cj; po[2] = P.ch; po[3] = P.cw; po[4] = P.flip; po[5] = P.jitter;
      for (int i = 0; i < 4; ++i) po[6 + i] = P.order[i];
      po[10] = P.fb; po[11] = P.fc; po[12] = P.fs; po[13] = P.fh; po[14] = P.gray; po[15] = 0.f;
    }
  }
  __syncthreads();
  const int npix = OH * OW;
  int kc = 4;  // position of contrast in the op order (4: none / jitter off)
  if (P.jitter)
    for (int i = 0; i < 4; ++i)
      if (P.order[i] == 1) kc = i;
  float mean = 0.f;
  if (kc < 4) {  // pass 1: mean luma of the image as contrast sees it
    long long s = 0;
    for (int p = threadIdx.x; p < npix; p += AUG_THREADS) {
      float r, g, bb;
      crop_pixel(P, img, W, OH, OW, p, r, g, bb);
      for (int i = 0; i < kc; ++i) pixel_op(P, P.order[i], r, g, bb);
      s += luma(r, g, bb);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    long long tot = 0;
    for (int w = 0; w < AUG_THREADS / 64; ++w) tot += red[w];
    mean = floorf((float)((double)tot / npix) + 0.5f);
  }
  const size_t obase = ((size_t)blockIdx.y * n + b) * npix;
  const float inv255 = 1.f / 255.f;
  for (int p = threadIdx.x; p < npix; p += AUG_THREADS) {  // pass 2
    float r, g, bb;
    crop_pixel(P, img, W, OH, OW, p, r, g, bb);
    if (P.jitter)
      for (int i = 0; i < 4; ++i) {
        if (i == kc) {
          r = clip_trunc(mean + P.fc * (r - mean));
          g = clip_trunc(mean + P.fc * (g - mean));
          bb = clip_trunc(mean + P.fc * (bb - mean));
        } else {
          pixel_op(P, P.order[i], r, g, bb);
        }
      }
    if (P.gray) {
      const float l = (float)luma(r, g, bb);
      r = g = bb = l;
    }
    uint16_t* o = out + (obase + p) * Cpad;
    if (Cpad == 8) {
      u32x4 w;
      w[0] = pack2bf(r * inv255, g * inv255);
      w[1] = pack2bf(bb * inv255, 0.f);
      w[2] = 0; w[3] = 0;
      *(u32x4*)o = w;
    } else {
      o[0] = f2bf(r * inv255); o[1] = f2bf(g * inv255); o[2] = f2bf(bb * inv255);
      for (int c = 3; c < Cpad; ++c) o[c] = 0;
    }
  }
}

}  // namespace

void simclr_augment(const uint8_t* images, const int64_t* indices, int n, int views, int H, int W,
                    int OH, int OW, int Cpad, float strength, uint64_t seed, uint64_t counter,
                    int view_offset, int flags, uint16_t* out, float* params_out, hipStream_t s) {
  if (OH * OW > AUG_THREADS * MAX_PIX_PER_THREAD) {  // two-pass kernel, any size
    hipLaunchKernelGGL(k_augment_large, dim3(n, views), dim3(AUG_THREADS), 0, s, images, indices,
                       n, H, W, OH, OW, Cpad, strength, seed, counter, view_offset, flags, out,
                       params_out);
    HIP_CHECK_LAUNCH();
    return;
  }
  hipLaunchKernelGGL(k_augment, dim3(n, views), dim3(AUG_THREADS), 0, s, images, indices, n, H, W,
                     OH, OW, Cpad, strength, seed, counter, view_offset, flags, out, params_out);
  HIP_CHECK_LAUNCH();
}
