// Memory-bound helpers of the encoder / fusion hot path (NHWC):
//  - input staging: NCHW fp32 volume stack -> gated NHWC (SEBlock modality
//    attention, model_module.py:25-43 used at :649-650) + per-pixel channel
//    mean for the reconstruction target (train_fusion.py:735-737)
//  - per-(n,c) spatial reductions (SE squeeze, GroupNorm(C,C) statistics,
//    AdaptiveAvgPool2d(1), SE/gate gradients)
//  - channel scaling (SE excite), GroupNorm(C,C) apply of the gated mix
//    alpha*f_b + (1-alpha)*f (model_module.py:673-675, :688-690)
//  - maxpool 3x3/s2/p1 (timm stem), nearest 2x upsample (AdaptiveAvgPool2d
//    (64,64) of a 32x32 map, model_module.py:531-534, :707-710), bilinear
//    resize (align_corners=False), column statistics for BN on non-conv inputs
//  - MaskGuidedSpatialAttention (model_module.py:49-97) forward/backward
#include <algorithm>

#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

static inline int gsz(long long n, int b = 256) {
  long long g = (n + b - 1) / b;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

// ---------------------------------------------------------- input staging
template <typename T>
__global__ void k_input_prep(const float* __restrict__ x, int N, int C, int H, int W, const float* __restrict__ gate,
                             T* __restrict__ y, int Cp, float* __restrict__ cmean) {
  const long long HW = (long long)H * W;
  const long long total = (long long)N * HW;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / HW, p = i - n * HW;
    const float* src = x + n * C * HW + p;
    float s = 0.f;
    if (y) {
      T* dst = y + i * Cp;
      for (int c = 0; c < Cp; ++c) {
        float v = 0.f;
        if (c < C) {
          v = src[c * HW];
          s += v;
          if (gate) v *= gate[n * C + c];
        }
        dst[c] = Cvt<T>::store(v);
      }
    } else {
      for (int c = 0; c < C; ++c) s += src[c * HW];
    }
    if (cmean) cmean[i] = s / (float)C;
  }
}

// per (n,c) mean of an NCHW fp32 tensor: block per (n,c)
__global__ void k_nchw_mean(const float* __restrict__ x, long long HW, float* __restrict__ out) {
  __shared__ float red[16];
  const float* p = x + (long long)blockIdx.x * HW;
  float s = 0.f;
  for (long long i = threadIdx.x; i < HW; i += blockDim.x) s += p[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[blockIdx.x] = s / (float)HW;
}

// out[n][c] = scale * sum_hw a[n,hw,c] * (b ? b[n,hw,c] : 1); block = (n, 64-channel group), 4 row lanes
template <typename T>
// block = CW channel lanes x R = 256 / CW pixel lanes (CW = C rounded up to a
// power of two, <= 64): a 1-channel map (the gating's mask-logit means) uses
// all 256 threads instead of 4; pixel lanes combined by a fixed-order tree
__global__ void k_nhwc_reduce(const T* __restrict__ a, int lda, const T* __restrict__ b, int ldb, int HW, int C,
                              float scale, float* __restrict__ out, int accumulate) {
  __shared__ float red[256];
  int CW = 1;
  while (CW < C && CW < 64) CW <<= 1;
  const int R = 256 / CW;
  const int cl = threadIdx.x % CW, rl = threadIdx.x / CW;
  const int n = blockIdx.x, c = blockIdx.y * 64 + cl;
  float s = 0.f;
  if (c < C && cl < 64) {
    const T* pa = a + (long long)n * HW * lda + c;
    const T* pb = b ? b + (long long)n * HW * ldb + c : nullptr;
#pragma unroll 4
    for (int p = rl; p < HW; p += R) {
      const float v = ld(pa + (long long)p * lda);
      s += pb ? v * ld(pb + (long long)p * ldb) : v;
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int st = R >> 1; st > 0; st >>= 1) {
    if (rl < st) red[threadIdx.x] += red[threadIdx.x + st * CW];
    __syncthreads();
  }
  if (rl == 0 && c < C) {
    const float r = red[cl] * scale;
    out[n * C + c] = accumulate ? out[n * C + c] + r : r;
  }
}

// y = x * gate[n][c]
template <typename T>
__global__ void k_channel_scale(const T* __restrict__ x, int ldx, const float* __restrict__ gate,
                                T* __restrict__ y, int ldy, long long N, int HW, int C) {
  const long long total = N * HW * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / C;
    const int c = (int)(i - row * C);
    const long long n = row / HW;
    st(y + row * ldy + c, ld(x + row * ldx + c) * gate[n * C + c]);
  }
}

// z = sig(w)*a + (1-sig(w))*b
template <typename T>
__global__ void k_mix(const T* __restrict__ a, int lda, const T* __restrict__ b, int ldb, const float* __restrict__ wlogit,
                      T* __restrict__ z, int ldz, long long M, int C) {
  const float al = 1.f / (1.f + __expf(-wlogit[0]));
  const long long total = M * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long m = i / C;
    const int c = (int)(i - m * C);
    st(z + m * ldz + c, al * ld(a + m * lda + c) + (1.f - al) * ld(b + m * ldb + c));
  }
}

// GroupNorm(C, C): y = (z - mean[n][c]) * rsqrt(var + eps) * g[c] + b[c]; var = m2 - mean^2
template <typename T>
__global__ void k_gn_apply(const T* __restrict__ z, int ldz, const float* __restrict__ mean,
                           const float* __restrict__ m2, const float* __restrict__ g, const float* __restrict__ b,
                           float eps, T* __restrict__ y, int ldy, long long N, int HW, int C) {
  const long long total = N * HW * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / C;
    const int c = (int)(i - row * C);
    const long long n = row / HW;
    const float mu = mean[n * C + c];
    const float var = fmaxf(m2[n * C + c] - mu * mu, 0.f);
    const float v = (ld(z + row * ldz + c) - mu) * rsqrtf(var + eps) * g[c] + b[c];
    st(y + row * ldy + c, v);
  }
}

__device__ __forceinline__ void ldf8(const float* p, float v[8]) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// k_gn_apply on 8-channel 16-B vectors with 32-bit index math (C % 8 == 0, rows * C < 2^31): the
// same per-element arithmetic, one 16-B load / store per thread instead of eight 2-B ones and two
// 64-bit divisions per element
template <typename T>
__global__ void __launch_bounds__(256) k_gn_apply8(const T* __restrict__ z, int ldz, const float* __restrict__ mean,
                                                   const float* __restrict__ m2, const float* __restrict__ g,
                                                   const float* __restrict__ b, float eps, T* __restrict__ y, int ldy,
                                                   int rows, int HW, int C) {
  const int cv = C >> 3, total = rows * cv;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int row = i / cv;
    const int c0 = (i - row * cv) * 8;
    const int nc = (row / HW) * C + c0;
    float v[8], mu[8], q[8], gg[8], bb[8];
    ld8(z + (size_t)row * ldz + c0, v);
    ldf8(mean + nc, mu);
    ldf8(m2 + nc, q);
    ldf8(g + c0, gg);
    ldf8(b + c0, bb);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float var = fmaxf(q[k] - mu[k] * mu[k], 0.f);
      v[k] = (v[k] - mu[k]) * rsqrtf(var + eps) * gg[k] + bb[k];
    }
    st8(y + (size_t)row * ldy + c0, v);
  }
}

// k_gn_bwd_apply on 8-channel vectors (same conditions and arithmetic as k_gn_apply8 / k_gn_bwd_apply)
template <typename T>
__global__ void __launch_bounds__(256) k_gn_bwd_apply8(const T* __restrict__ dy, int lddy, const T* __restrict__ z,
                                                       int ldz, const float* __restrict__ mean,
                                                       const float* __restrict__ m2, const float* __restrict__ s1,
                                                       const float* __restrict__ s2, const float* __restrict__ g,
                                                       float eps, T* __restrict__ dz, int lddz, int rows, int HW, int C) {
  const int cv = C >> 3, total = rows * cv;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int row = i / cv;
    const int c0 = (i - row * cv) * 8;
    const int nc = (row / HW) * C + c0;
    float d[8], zz[8], mu[8], q[8], a1[8], a2[8], gg[8];
    ld8(dy + (size_t)row * lddy + c0, d);
    ld8(z + (size_t)row * ldz + c0, zz);
    ldf8(mean + nc, mu);
    ldf8(m2 + nc, q);
    ldf8(s1 + nc, a1);
    ldf8(s2 + nc, a2);
    ldf8(g + c0, gg);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float rs = rsqrtf(fmaxf(q[k] - mu[k] * mu[k], 0.f) + eps);
      const float xh = (zz[k] - mu[k]) * rs;
      d[k] = gg[k] * rs / (float)HW * ((float)HW * d[k] - a1[k] - xh * a2[k]);
    }
    st8(dz + (size_t)row * lddz + c0, d);
  }
}

// GroupNorm(C,C) backward given per-(n,c) sums S1 = sum dy, S2 = sum dy*xhat:
// dz = g*rstd/HW * (HW*dy - S1 - xhat*S2)
template <typename T>
__global__ void k_gn_bwd_apply(const T* __restrict__ dy, int lddy, const T* __restrict__ z, int ldz,
                               const float* __restrict__ mean, const float* __restrict__ m2,
                               const float* __restrict__ s1, const float* __restrict__ s2,
                               const float* __restrict__ g, float eps, T* __restrict__ dz, int lddz, long long N,
                               int HW, int C) {
  const long long total = N * HW * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / C;
    const int c = (int)(i - row * C);
    const long long n = row / HW;
    const float mu = mean[n * C + c];
    const float rs = rsqrtf(fmaxf(m2[n * C + c] - mu * mu, 0.f) + eps);
    const float xh = (ld(z + row * ldz + c) - mu) * rs;
    const float v = g[c] * rs / (float)HW * ((float)HW * ld(dy + row * lddy + c) - s1[n * C + c] - xh * s2[n * C + c]);
    st(dz + row * lddz + c, v);
  }
}

// S2[n][c] = sum_hw dy * xhat  (xhat from z, mean, m2)
template <typename T>
__global__ void k_gn_bwd_reduce(const T* __restrict__ dy, int lddy, const T* __restrict__ z, int ldz,
                                const float* __restrict__ mean, const float* __restrict__ m2, float eps, int HW, int C,
                                float* __restrict__ s1, float* __restrict__ s2) {
  __shared__ float red[4][64][2];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int n = blockIdx.x, c = blockIdx.y * 64 + cl;
  float a = 0.f, q = 0.f;
  if (c < C) {
    const float mu = mean[n * C + c];
    const float rs = rsqrtf(fmaxf(m2[n * C + c] - mu * mu, 0.f) + eps);
    for (int p = rl; p < HW; p += 4) {
      const long long row = (long long)n * HW + p;
      const float g = ld(dy + row * lddy + c);
      a += g;
      q += g * (ld(z + row * ldz + c) - mu) * rs;
    }
  }
  red[rl][cl][0] = a;
  red[rl][cl][1] = q;
  __syncthreads();
  if (rl == 0 && c < C) {
    s1[n * C + c] = red[0][cl][0] + red[1][cl][0] + red[2][cl][0] + red[3][cl][0];
    s2[n * C + c] = red[0][cl][1] + red[1][cl][1] + red[2][cl][1] + red[3][cl][1];
  }
}

// k_gn_bwd_reduce on 8-channel vectors: block = 32 pixel lanes x 8 channel lanes
// of 8 channels (64 channels of one sample), 16-B loads -- the scalar form reads
// 2 B per lane over 4 pixel lanes (~0.3 TB/s at one block per 64 channels and sample)
template <typename T>
__global__ void __launch_bounds__(256) k_gn_bwd_reduce8(const T* __restrict__ dy, int lddy, const T* __restrict__ z,
                                                        int ldz, const float* __restrict__ mean,
                                                        const float* __restrict__ m2, float eps, int HW, int C,
                                                        float* __restrict__ s1, float* __restrict__ s2) {
  __shared__ float red[32][65 * 2];
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int n = blockIdx.x, c0 = blockIdx.y * 64 + cl * 8;
  float a[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { a[e] = 0.f; q[e] = 0.f; }
  if (c0 < C) {
    float mu[8], rs[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mu[e] = mean[n * C + c0 + e];
      rs[e] = rsqrtf(fmaxf(m2[n * C + c0 + e] - mu[e] * mu[e], 0.f) + eps);
    }
    for (int p = rl; p < HW; p += 32) {
      const long long row = (long long)n * HW + p;
      float g[8], zv[8];
      ld8(dy + row * lddy + c0, g);
      ld8(z + row * ldz + c0, zv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a[e] += g[e];
        q[e] += g[e] * (zv[e] - mu[e]) * rs[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[rl][(cl * 8 + e) * 2] = a[e];
    red[rl][(cl * 8 + e) * 2 + 1] = q[e];
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int c = threadIdx.x >> 1, w = threadIdx.x & 1;
    float t = 0.f;
#pragma unroll 8
    for (int r = 0; r < 32; ++r) t += red[r][c * 2 + w];
    const int cg = blockIdx.y * 64 + c;
    if (cg < C) (w ? s2 : s1)[n * C + cg] = t;
  }
}

// ------------------------------------------------------------- max pool
template <typename T>
__global__ void k_maxpool(const T* __restrict__ x, int N, int H, int W, int C, int ldx, T* __restrict__ y, int Ho,
                          int Wo, int ldy, int k, int s, int p) {
  const long long total = (long long)N * Ho * Wo * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long pix = i / C;
    const int n = (int)(pix / (Ho * Wo));
    const int rem = (int)(pix - (long long)n * Ho * Wo);
    const int ho = rem / Wo, wo = rem % Wo;
    float m = -INFINITY;
    for (int r = 0; r < k; ++r) {
      const int hi = ho * s - p + r;
      if (hi < 0 || hi >= H) continue;
      for (int q = 0; q < k; ++q) {
        const int wi = wo * s - p + q;
        if (wi < 0 || wi >= W) continue;
        const float v = ld(x + ((size_t)(n * H + hi) * W + wi) * ldx + c);
        if (v > m || isnan(v)) m = v;
      }
    }
    st(y + pix * ldy + c, m);
  }
}

// ------------------------------------------------------ 2x2 average pool (ResNet-D shortcut)
// timm resnet.py downsample_avg's pool in front of the 1x1 projection: same = 0 is
// AvgPool2d(2, s, ceil_mode=True, count_include_pad=False) -- windows clipped at the input edge and
// divided by their in-range count; same = 1 is AvgPool2dSame(2, 1) of a dilated stage -- pad_same adds
// one zero row / column at the bottom / right, which avg_pool2d then counts (divisor always 4).
// One thread per output element (NHWC, channel fastest: coalesced); fp32 sums.
template <typename T>
__global__ void k_avgpool2(const T* __restrict__ x, int N, int H, int W, int C, int ldx, T* __restrict__ y, int Ho,
                           int Wo, int ldy, int s, int same) {
  const long long total = (long long)N * Ho * Wo * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long pix = i / C;
    const int n = (int)(pix / ((long long)Ho * Wo));
    const int rem = (int)(pix - (long long)n * Ho * Wo);
    const int ho = rem / Wo, wo = rem - (rem / Wo) * Wo;
    float sum = 0.f;
    int cnt = 0;
    for (int r = 0; r < 2; ++r) {
      const int hi = ho * s + r;
      if (hi >= H) continue;
      for (int q = 0; q < 2; ++q) {
        const int wi = wo * s + q;
        if (wi >= W) continue;
        sum += ld(x + ((size_t)(n * H + hi) * W + wi) * ldx + c);
        ++cnt;
      }
    }
    st(y + pix * ldy + c, sum / (float)(same ? 4 : cnt));
  }
}

// backward: each input element sums dy / divisor over the (at most 2x2) windows that contain it
template <typename T>
__global__ void k_avgpool2_bwd(const T* __restrict__ dy, int N, int H, int W, int C, int Ho, int Wo, int lddy,
                               T* __restrict__ dx, int lddx, int s, int same) {
  const long long total = (long long)N * H * W * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long pix = i / C;
    const int n = (int)(pix / ((long long)H * W));
    const int rem = (int)(pix - (long long)n * H * W);
    const int hi = rem / W, wi = rem - (rem / W) * W;
    float acc = 0.f;
    for (int r = 0; r < 2; ++r) {
      const int th = hi - r;  // window row start ho * s
      if (th < 0 || th % s) continue;
      const int ho = th / s;
      if (ho >= Ho) continue;
      const int rows = min(th + 2, H) - th;
      for (int q = 0; q < 2; ++q) {
        const int tw = wi - q;
        if (tw < 0 || tw % s) continue;
        const int wo = tw / s;
        if (wo >= Wo) continue;
        const int cols = min(tw + 2, W) - tw;
        acc += ld(dy + ((size_t)(n * Ho + ho) * Wo + wo) * lddy + c) / (float)(same ? 4 : rows * cols);
      }
    }
    st(dx + pix * lddx + c, acc);
  }
}

// backward: each input element receives dy of every window whose (first) argmax it is
template <typename T>
__global__ void k_maxpool_bwd(const T* __restrict__ x, int N, int H, int W, int C, int ldx, const T* __restrict__ dy,
                              int Ho, int Wo, int lddy, T* __restrict__ dx, int lddx, int k, int s, int p) {
  const long long total = (long long)N * H * W * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long pix = i / C;
    const int n = (int)(pix / (H * W));
    const int rem = (int)(pix - (long long)n * H * W);
    const int h = rem / W, w = rem % W;
    float g = 0.f;
    const int ho_lo = max(0, (h + p - k + s) / s), ho_hi = min(Ho - 1, (h + p) / s);
    const int wo_lo = max(0, (w + p - k + s) / s), wo_hi = min(Wo - 1, (w + p) / s);
    for (int ho = ho_lo; ho <= ho_hi; ++ho)
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        // recompute the window argmax with torch's rule (max_pool2d_with_indices): the index
        // starts at the window's first valid element and moves on `v > max || isnan(v)`
        float m = -INFINITY;
        int am = -1;
        for (int r = 0; r < k; ++r) {
          const int hi = ho * s - p + r;
          if (hi < 0 || hi >= H) continue;
          for (int q = 0; q < k; ++q) {
            const int wi = wo * s - p + q;
            if (wi < 0 || wi >= W) continue;
            const float v = ld(x + ((size_t)(n * H + hi) * W + wi) * ldx + c);
            if (am < 0) am = hi * W + wi;
            if (v > m || isnan(v)) { m = v; am = hi * W + wi; }
          }
        }
        if (am == h * W + w) g += ld(dy + ((size_t)(n * Ho + ho) * Wo + wo) * lddy + c);
      }
    st(dx + pix * lddx + c, g);
  }
}

// 8 channels per thread (16-B loads): the window argmax recompute per candidate
// output reads 16-B vectors instead of scalars
template <typename T>
__global__ void k_maxpool_bwd8(const T* __restrict__ x, int N, int H, int W, int C, int ldx, const T* __restrict__ dy,
                               int Ho, int Wo, int lddy, T* __restrict__ dx, int lddx, int k, int s, int p) {
  const int C8 = C >> 3;
  const long long total = (long long)N * H * W * C8;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C8) * 8;
    const long long pix = i / C8;
    const int n = (int)(pix / (H * W));
    const int rem = (int)(pix - (long long)n * H * W);
    const int h = rem / W, w = rem % W;
    float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int ho_lo = max(0, (h + p - k + s) / s), ho_hi = min(Ho - 1, (h + p) / s);
    const int wo_lo = max(0, (w + p - k + s) / s), wo_hi = min(Wo - 1, (w + p) / s);
    for (int ho = ho_lo; ho <= ho_hi; ++ho)
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        float m[8];
        int am[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) { m[e] = -INFINITY; am[e] = -1; }
        for (int r = 0; r < k; ++r) {
          const int hi = ho * s - p + r;
          if (hi < 0 || hi >= H) continue;
          for (int q = 0; q < k; ++q) {
            const int wi = wo * s - p + q;
            if (wi < 0 || wi >= W) continue;
            float v[8];
            ld8(x + ((size_t)(n * H + hi) * W + wi) * ldx + c, v);
            const int pos = hi * W + wi;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              if (am[e] < 0) am[e] = pos;  // torch: the first valid element until a max / NaN replaces it
              if (v[e] > m[e] || isnan(v[e])) { m[e] = v[e]; am[e] = pos; }
            }
          }
        }
        float d[8];
        ld8(dy + ((size_t)(n * Ho + ho) * Wo + wo) * lddy + c, d);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (am[e] == rem) g[e] += d[e];
      }
    st8(dx + pix * lddx + c, g);
  }
}

// ----------------------------------------------------------- resampling
template <typename T>
__global__ void k_up_nearest(const T* __restrict__ x, int ldx, T* __restrict__ y, int N, int H, int W, int C, int r) {
  const long long total = (long long)N * r * H * r * W * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long long t = i / C;
    const int wo = (int)(t % (r * W)); t /= (r * W);
    const int ho = (int)(t % (r * H));
    const int n = (int)(t / (r * H));
    y[i] = x[((size_t)(n * H + ho / r) * W + wo / r) * ldx + c];
  }
}

// sum of the r x r replicas (backward of nearest r-x upsample)
template <typename T>
__global__ void k_up_nearest_bwd(const T* __restrict__ dy, T* __restrict__ dx, int N, int H, int W, int C, int r) {
  const long long total = (long long)N * H * W * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long long t = i / C;
    const int w = (int)(t % W); t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float s = 0.f;
    for (int a = 0; a < r; ++a)
      for (int b = 0; b < r; ++b) s += ld(dy + ((size_t)(n * r * H + r * h + a) * r * W + r * w + b) * C + c);
    st(dx + i, s);
  }
}

__device__ __forceinline__ void lin_idx(int o, int in, int out, int& i0, int& i1, float& l1) {
  const float scale = (float)in / (float)out;
  float src = (o + 0.5f) * scale - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
}

// bilinear resize, align_corners=False (torch upsample_bilinear2d semantics)
template <typename T>
__global__ void k_bilinear(const T* __restrict__ x, int N, int Hi, int Wi, int C, int ldx, T* __restrict__ y, int Ho,
                           int Wo, int ldy) {
  const long long total = (long long)N * Ho * Wo * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long pix = i / C;
    const int n = (int)(pix / (Ho * Wo));
    const int rem = (int)(pix - (long long)n * Ho * Wo);
    const int ho = rem / Wo, wo = rem % Wo;
    int h0, h1, w0, w1;
    float lh, lw;
    lin_idx(ho, Hi, Ho, h0, h1, lh);
    lin_idx(wo, Wi, Wo, w0, w1, lw);
    const T* b = x + (size_t)n * Hi * Wi * ldx + c;
    const float v = (1.f - lh) * ((1.f - lw) * ld(b + ((size_t)h0 * Wi + w0) * ldx) + lw * ld(b + ((size_t)h0 * Wi + w1) * ldx)) +
                    lh * ((1.f - lw) * ld(b + ((size_t)h1 * Wi + w0) * ldx) + lw * ld(b + ((size_t)h1 * Wi + w1) * ldx));
    st(y + pix * ldy + c, v);
  }
}

// transpose of k_bilinear: dx[n,hi,wi,c] = sum over outputs of weight * dy (gather form)
template <typename T>
__global__ void k_bilinear_bwd(const T* __restrict__ dy, int N, int Ho, int Wo, int C, int lddy, T* __restrict__ dx,
                               int Hi, int Wi, int lddx) {
  const long long total = (long long)N * Hi * Wi * C;
  const float sh = (float)Ho / (float)Hi, sw = (float)Wo / (float)Wi;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long pix = i / C;
    const int n = (int)(pix / (Hi * Wi));
    const int rem = (int)(pix - (long long)n * Hi * Wi);
    const int hi = rem / Wi, wi = rem % Wi;
    // outputs whose source index lies within (hi-1, hi+1)
    const int ho_lo = max(0, (int)floorf((hi - 1 + 0.5f) * sh - 0.5f) - 1);
    const int ho_hi = min(Ho - 1, (int)ceilf((hi + 1 + 0.5f) * sh - 0.5f) + 1);
    const int wo_lo = max(0, (int)floorf((wi - 1 + 0.5f) * sw - 0.5f) - 1);
    const int wo_hi = min(Wo - 1, (int)ceilf((wi + 1 + 0.5f) * sw - 0.5f) + 1);
    float acc = 0.f;
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      int h0, h1;
      float lh;
      lin_idx(ho, Hi, Ho, h0, h1, lh);
      float wh = 0.f;
      if (h0 == hi) wh += 1.f - lh;
      if (h1 == hi) wh += lh;
      if (wh == 0.f) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        int w0, w1;
        float lw;
        lin_idx(wo, Wi, Wo, w0, w1, lw);
        float ww = 0.f;
        if (w0 == wi) ww += 1.f - lw;
        if (w1 == wi) ww += lw;
        if (ww == 0.f) continue;
        acc += wh * ww * ld(dy + ((size_t)(n * Ho + ho) * Wo + wo) * lddy + c);
      }
    }
    st(dx + pix * lddx + c, acc);
  }
}

// column stats: partials[tile][c] = (sum, sum^2) over 256-row tiles
template <typename T>
__global__ void k_col_stats(const T* __restrict__ x, int ldx, long long M, int C, float* __restrict__ part) {
  __shared__ float red[4][64][2];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  const long long r0 = (long long)blockIdx.x * 256;
  float s = 0.f, q = 0.f;
  if (c < C)
    for (int r = rl; r < 256; r += 4) {
      const long long m = r0 + r;
      if (m >= M) break;
      const float v = ld(x + m * ldx + c);
      s += v;
      q += v * v;
    }
  red[rl][cl][0] = s;
  red[rl][cl][1] = q;
  __syncthreads();
  if (rl == 0 && c < C)
    *(float2*)(part + ((size_t)blockIdx.x * C + c) * 2) =
        make_float2(red[0][cl][0] + red[1][cl][0] + red[2][cl][0] + red[3][cl][0],
                    red[0][cl][1] + red[1][cl][1] + red[2][cl][1] + red[3][cl][1]);
}

// the same partials from 8-channel vectors (16-B bf16 loads): block = CVt
// channel vectors x R = 256 / CVt row lanes over one 256-row tile, every
// thread's rows in flight together (the scalar form issued one 2-B load per
// row and channel: ~20 us for a 32k x 64 map)
template <typename T>
__global__ void __launch_bounds__(256) k_col_stats8(const T* __restrict__ x, int ldx, long long M, int C, int CVt,
                                                    float* __restrict__ part) {
  __shared__ float red[256 * 16];
  const int R = 256 / CVt;
  const int cvl = threadIdx.x % CVt, rl = threadIdx.x / CVt;
  const int cv = blockIdx.y * CVt + cvl;
  const long long r0 = (long long)blockIdx.x * 256;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s[j] = 0.f; q[j] = 0.f; }
  if (cv * 8 < C) {
#pragma unroll 4
    for (int r = rl; r < 256; r += R) {
      const long long m = r0 + r;
      if (m < M) {
        float v[8];
        ld8(x + m * ldx + cv * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[j] += v[j]; q[j] = fmaf(v[j], v[j], q[j]); }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[threadIdx.x * 16 + j] = s[j]; red[threadIdx.x * 16 + 8 + j] = q[j]; }
  __syncthreads();
  for (int t = threadIdx.x; t < CVt * 8; t += 256) {
    const int v = t >> 3, j = t & 7;
    float ss = 0.f, qq = 0.f;
    for (int r = 0; r < R; ++r) {
      ss += red[(r * CVt + v) * 16 + j];
      qq += red[(r * CVt + v) * 16 + 8 + j];
    }
    const int c = (blockIdx.y * CVt + v) * 8 + j;
    if (c < C) *(float2*)(part + ((size_t)blockIdx.x * C + c) * 2) = make_float2(ss, qq);
  }
}

// ------------------------------------------ mask-guided spatial attention
// mask m[n][p] (single channel, already at the feature resolution)
// h[c] = w1[c]*m ; GroupNorm(1,16) over (c,p) per sample: mean = mean(w1)*mean(m),
// E[h^2] = mean(w1^2)*mean(m^2) ; u_c = gelu((h-mu)*rs*g[c]+b[c]) ;
// A = clamp(sig(sum_c w2[c] u_c + b2), 1e-4, 1-1e-4) ; out = f * (1 + gamma*A)
// stats[n] = (sum m, sum m^2) computed by k_mask_stats.
template <typename T>
__global__ void k_mask_stats(const T* __restrict__ m, int HW, float* __restrict__ stats) {
  __shared__ float red[16];
  const T* p = m + (long long)blockIdx.x * HW;
  float s = 0.f, q = 0.f;
  for (int i = threadIdx.x; i < HW; i += blockDim.x) {
    const float v = ld(p + i);
    s += v;
    q += v * v;
  }
  s = block_sum(s, red);
  q = block_sum(q, red);
  if (threadIdx.x == 0) {
    stats[blockIdx.x * 2] = s;
    stats[blockIdx.x * 2 + 1] = q;
  }
}

struct MaskAttnP {
  const float* w1;  // [16]
  const float* g;   // [16]
  const float* b;   // [16]
  const float* w2;  // [16]
  const float* b2;  // [1]
  const float* gamma;  // [1]
  float eps;
  int hid;
};

__device__ __forceinline__ void mask_attn_stats(const MaskAttnP& P, const float* stats, int n, int HW, float& mu,
                                                float& rs) {
  float mw = 0.f, mw2 = 0.f;
  for (int c = 0; c < P.hid; ++c) { mw += P.w1[c]; mw2 += P.w1[c] * P.w1[c]; }
  mw /= P.hid;
  mw2 /= P.hid;
  const float mm = stats[2 * n] / HW, mm2 = stats[2 * n + 1] / HW;
  mu = mw * mm;
  const float var = fmaxf(mw2 * mm2 - mu * mu, 0.f);
  rs = rsqrtf(var + P.eps);
}

template <typename T>
__global__ void k_mask_attn_fwd(const T* __restrict__ f, int ldf, const T* __restrict__ m, MaskAttnP P,
                                const float* __restrict__ stats, T* __restrict__ out, int ldo, T* __restrict__ A_out,
                                long long N, int HW, int C) {
  const long long total = N * HW;
  for (long long i = (long long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); i < total;
       i += (long long)gridDim.x * (blockDim.x / 64)) {
    const int lane = threadIdx.x & 63;
    const int n = (int)(i / HW);
    float mu, rs;
    mask_attn_stats(P, stats, n, HW, mu, rs);
    const float mv = ld(m + i);
    float z = P.b2[0];
    for (int c = 0; c < P.hid; ++c) z += P.w2[c] * gelu_f((P.w1[c] * mv - mu) * rs * P.g[c] + P.b[c]);
    float A = sigmoid_f(z);
    A = fminf(fmaxf(A, 1e-4f), 1.f - 1e-4f);
    const float sc = 1.f + P.gamma[0] * A;
    for (int c = lane; c < C; c += 64) st(out + i * ldo + c, ld(f + i * ldf + c) * sc);
    if (lane == 0 && A_out) st(A_out + i, A);
  }
}


// ===================================================== 8-channel vector forms
// One thread = 8 consecutive channels of one pixel (16-B bf16 / 32-B f32
// accesses). Used when C, the leading dimensions and the pointers allow it.

// Stage 1 of out[n][c] (+)= scale * sum_hw a (*b) [and out_sq += scale*sum a^2]:
// grid (N, channel groups, S row splits), block 256 = CVt channel vectors
// (8 channels each) x R = 256/CVt row lanes; each block writes its partial
// sums to ws[s][n][c] (and ws[S*N*C + ...] for squares). Stage 2 sums the S
// partials in a fixed order. Deterministic, no atomics, no memset.
template <typename T>
__global__ void __launch_bounds__(256) k_nhwc_reduce8(const T* __restrict__ a, int lda, const T* __restrict__ b,
                                                      int ldb, int HW, int C, int CVt, int rpb, int sq,
                                                      float* __restrict__ ws) {
  __shared__ float red[256 * 8];
  const int CV = C >> 3;
  const int R = 256 / CVt;
  const int cvl = threadIdx.x % CVt, rl = threadIdx.x / CVt;
  const int n = blockIdx.x, N = gridDim.x;
  const int cv = blockIdx.y * CVt + cvl;
  const int p0 = blockIdx.z * rpb, p1 = min(HW, p0 + rpb);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float acq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (rl < R && cv < CV) {
    const T* pa = a + ((long long)n * HW) * lda + cv * 8;
    const T* pb = b ? b + ((long long)n * HW) * ldb + cv * 8 : nullptr;
#pragma unroll 4
    for (int p = p0 + rl; p < p1; p += R) {
      float va[8];
      ld8(pa + (long long)p * lda, va);
      if (pb) {
        float vb[8];
        ld8(pb + (long long)p * ldb, vb);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(va[j], vb[j], acc[j]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          acc[j] += va[j];
          acq[j] = fmaf(va[j], va[j], acq[j]);
        }
      }
    }
  }
  const size_t plane = (size_t)N * C;
  for (int pass = 0; pass < (sq ? 2 : 1); ++pass) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = pass ? acq[j] : acc[j];
    __syncthreads();
    for (int t = threadIdx.x; t < CVt * 8; t += 256) {
      const int v = t >> 3, jj = t & 7;
      float sum = 0.f;
      for (int r = 0; r < R; ++r) sum += red[(r * CVt + v) * 8 + jj];
      const int c = (blockIdx.y * CVt + v) * 8 + jj;
      if (blockIdx.y * CVt + v < CV)
        ws[(size_t)pass * gridDim.z * plane + (size_t)blockIdx.z * plane + (size_t)n * C + c] = sum;
    }
  }
}

__global__ void k_nhwc_reduce_fin(const float* __restrict__ ws, int S, long long NC, float scale,
                                  float* __restrict__ out, float* __restrict__ out_sq, int accumulate) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < NC * (out_sq ? 2 : 1);
       i += (long long)gridDim.x * blockDim.x) {
    const int pass = i >= NC;
    const long long e = pass ? i - NC : i;
    const float* p = ws + (size_t)pass * S * NC + e;
    float v = 0.f;
    for (int z = 0; z < S; ++z) v += p[(size_t)z * NC];
    float* o = pass ? out_sq + e : out + e;
    *o = accumulate ? *o + v * scale : v * scale;
  }
}

// per-(n,c) mean of NCHW fp32: block per plane, float4 loads, 4 in flight
__global__ void __launch_bounds__(256) k_nchw_mean4(const float* __restrict__ x, long long HW, float inv,
                                                    float* __restrict__ out) {
  __shared__ float red[16];
  const float* p = x + (long long)blockIdx.x * HW;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  long long i = threadIdx.x * 4;
  for (; i + 3 * 1024 < HW; i += 4 * 1024) {
    const float4 a = *(const float4*)(p + i), b = *(const float4*)(p + i + 1024);
    const float4 c = *(const float4*)(p + i + 2048), d = *(const float4*)(p + i + 3072);
    s0 += (a.x + a.y) + (a.z + a.w);
    s1 += (b.x + b.y) + (b.z + b.w);
    s2 += (c.x + c.y) + (c.z + c.w);
    s3 += (d.x + d.y) + (d.z + d.w);
  }
  for (; i < HW; i += 1024) {
    const float4 a = *(const float4*)(p + i);
    s0 += (a.x + a.y) + (a.z + a.w);
  }
  float s = block_sum((s0 + s1) + (s2 + s3), red);
  if (threadIdx.x == 0) out[blockIdx.x] = s * inv;
}

// input staging with 16-B stores: one thread = one pixel, Cp % 8 == 0
template <typename T>
__global__ void k_input_prep8(const float* __restrict__ x, int N, int C, int H, int W, const float* __restrict__ gate,
                              T* __restrict__ y, int Cp, float* __restrict__ cmean) {
  const long long HW = (long long)H * W;
  const long long total = (long long)N * HW;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / HW, p = i - n * HW;
    const float* src = x + n * C * HW + p;
    float s = 0.f;
    for (int c0 = 0; c0 < Cp; c0 += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        float t = 0.f;
        if (c < C) {
          t = src[c * HW];
          s += t;
          if (gate) t *= gate[n * C + c];
        }
        v[j] = t;
      }
      st8(y + i * Cp + c0, v);
    }
    if (cmean) cmean[i] = s / (float)C;
  }
}

template <typename T, typename I = long long>
__global__ void k_up_nearest8(const T* __restrict__ x, int ldx, T* __restrict__ y, int N, int H, int W, int C, int r) {
  const int CV = C >> 3;
  const I total = (long long)N * r * H * r * W * CV;
  for (I i = (I)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (I)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    I t = i / CV;
    const int wo = (int)(t % (r * W)); t /= (r * W);
    const int ho = (int)(t % (r * H));
    const int n = (int)(t / (r * H));
    float v[8];
    ld8(x + ((size_t)(n * H + ho / r) * W + wo / r) * ldx + cv * 8, v);
    st8(y + i * 8, v);
  }
}

// Max pool forward that also records, per output element, the window
// position (r*k + q, one byte) of its maximum with torch's rule
// (max_pool2d_with_indices: start at the window's first valid element, move
// on `v > max || isnan(v)`, so an all -inf window routes its gradient to the
// first element and the last NaN wins), exactly the element k_maxpool_bwd8
// re-derives -- so the backward needs no window re-scan (k_maxpool_bwd_idx8).
template <typename T>
__global__ void k_maxpool_idx8(const T* __restrict__ x, int N, int H, int W, int C, int ldx, T* __restrict__ y,
                               int Ho, int Wo, int ldy, unsigned char* __restrict__ idx, int k, int s, int p) {
  const int CV = C >> 3;
  const int total = N * Ho * Wo * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV, pix = i / CV;
    const int n = pix / (Ho * Wo), rem = pix - n * Ho * Wo;
    const int ho = rem / Wo, wo = rem - ho * Wo;
    float m[8];
    unsigned am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { m[j] = -INFINITY; am[j] = 255u; }
    for (int r = 0; r < k; ++r) {
      const int hi = ho * s - p + r;
      if (hi < 0 || hi >= H) continue;
      for (int q = 0; q < k; ++q) {
        const int wi = wo * s - p + q;
        if (wi < 0 || wi >= W) continue;
        float v[8];
        ld8(x + ((size_t)(n * H + hi) * W + wi) * ldx + cv * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (am[j] == 255u) am[j] = (unsigned)(r * k + q);
          if (v[j] > m[j] || isnan(v[j])) { m[j] = v[j]; am[j] = (unsigned)(r * k + q); }
        }
      }
    }
    st8(y + (size_t)pix * ldy + cv * 8, m);
    uint2 packed;
    packed.x = am[0] | (am[1] << 8) | (am[2] << 16) | (am[3] << 24);
    packed.y = am[4] | (am[5] << 8) | (am[6] << 16) | (am[7] << 24);
    *(uint2*)(idx + (size_t)i * 8) = packed;
  }
}

// dx from the recorded window positions: each input element sums dy over the
// windows (ho outer, wo inner, as k_maxpool_bwd8) whose recorded maximum is it
template <typename T>
__global__ void k_maxpool_bwd_idx8(const T* __restrict__ dy, int N, int H, int W, int C, int Ho, int Wo, int lddy,
                                   const unsigned char* __restrict__ idx, T* __restrict__ dx, int lddx, int k, int s,
                                   int p) {
  const int CV = C >> 3;
  const int total = N * H * W * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV, pix = i / CV;
    const int n = pix / (H * W), rem = pix - n * H * W;
    const int h = rem / W, w = rem - h * W;
    float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int ho_lo = max(0, (h + p - k + s) / s), ho_hi = min(Ho - 1, (h + p) / s);
    const int wo_lo = max(0, (w + p - k + s) / s), wo_hi = min(Wo - 1, (w + p) / s);
    for (int ho = ho_lo; ho <= ho_hi; ++ho)
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const unsigned code = (unsigned)((h + p - ho * s) * k + (w + p - wo * s));
        const int op = (n * Ho + ho) * Wo + wo;
        const uint2 pk = *(const uint2*)(idx + ((size_t)op * CV + cv) * 8);
        unsigned hit = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const unsigned b = ((e < 4 ? pk.x : pk.y) >> (8 * (e & 3))) & 255u;
          hit |= (b == code ? 1u : 0u) << e;
        }
        if (hit) {
          float d[8];
          ld8(dy + (size_t)op * lddy + cv * 8, d);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (hit & (1u << e)) g[e] += d[e];
        }
      }
    st8(dx + (size_t)pix * lddx + cv * 8, g);
  }
}

template <typename T>
__global__ void k_maxpool8(const T* __restrict__ x, int N, int H, int W, int C, int ldx, T* __restrict__ y, int Ho,
                           int Wo, int ldy, int k, int s, int p) {
  const int CV = C >> 3;
  const long long total = (long long)N * Ho * Wo * CV;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    const long long pix = i / CV;
    const int n = (int)(pix / (Ho * Wo));
    const int rem = (int)(pix - (long long)n * Ho * Wo);
    const int ho = rem / Wo, wo = rem % Wo;
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
    if (k == 3) {
      // the stem's 3x3 window: all nine 16-B loads in flight before any compare (the runtime-k loop
      // below waits out one load latency per tap); out-of-range taps are skipped exactly as there
      Vec8<T> vv[9];
      bool ok[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int hi = ho * s - p + t / 3, wi = wo * s - p + t % 3;
        ok[t] = hi >= 0 && hi < H && wi >= 0 && wi < W;
        vv[t] = ok[t] ? ldv8(x + ((size_t)(n * H + hi) * W + wi) * ldx + cv * 8) : zero8<T>();
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (!ok[t]) continue;
        float v[8];
        unpack8(vv[t], v);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (v[j] > m[j] || isnan(v[j])) m[j] = v[j];
      }
    } else {
      for (int r = 0; r < k; ++r) {
        const int hi = ho * s - p + r;
        if (hi < 0 || hi >= H) continue;
        for (int q = 0; q < k; ++q) {
          const int wi = wo * s - p + q;
          if (wi < 0 || wi >= W) continue;
          float v[8];
          ld8(x + ((size_t)(n * H + hi) * W + wi) * ldx + cv * 8, v);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (v[j] > m[j] || isnan(v[j])) m[j] = v[j];
        }
      }
    }
    st8(y + pix * ldy + cv * 8, m);
  }
}

template <typename T, typename I = long long>
__global__ void k_channel_scale8(const T* __restrict__ x, int ldx, const float* __restrict__ gate,
                                 T* __restrict__ y, int ldy, long long N, int HW, int C) {
  const int CV = C >> 3;
  const I total = N * HW * CV;
  for (I i = (I)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (I)gridDim.x * blockDim.x) {
    const I row = i / CV;
    const int c = (int)(i - row * CV) * 8;
    const I n = row / HW;
    float v[8];
    ld8(x + row * ldx + c, v);
    const float4 g0 = *(const float4*)(gate + n * C + c), g1 = *(const float4*)(gate + n * C + c + 4);
    v[0] *= g0.x; v[1] *= g0.y; v[2] *= g0.z; v[3] *= g0.w;
    v[4] *= g1.x; v[5] *= g1.y; v[6] *= g1.z; v[7] *= g1.w;
    st8(y + row * ldy + c, v);
  }
}

template <typename T, typename I = long long>
__global__ void k_mix8(const T* __restrict__ a, int lda, const T* __restrict__ b, int ldb,
                       const float* __restrict__ wlogit, T* __restrict__ z, int ldz, long long M, int C) {
  const float al = 1.f / (1.f + __expf(-wlogit[0]));
  const int CV = C >> 3;
  const I total = M * CV;
  for (I i = (I)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (I)gridDim.x * blockDim.x) {
    const I m = i / CV;
    const int c = (int)(i - m * CV) * 8;
    float va[8], vb[8];
    ld8(a + m * lda + c, va);
    ld8(b + m * ldb + c, vb);
#pragma unroll
    for (int j = 0; j < 8; ++j) va[j] = al * va[j] + (1.f - al) * vb[j];
    st8(z + m * ldz + c, va);
  }
}

}  // namespace dmf

using namespace dmf;

static inline bool a16(const void* p) { return p == nullptr || (((uintptr_t)p) & 15) == 0; }
static inline bool v8ok(int C, int ld0, int ld1, const void* p0, const void* p1, const void* p2 = nullptr) {
  return C % 8 == 0 && ld0 % 8 == 0 && ld1 % 8 == 0 && a16(p0) && a16(p1) && a16(p2);
}

extern "C" int dmf_input_prep(int dtype, const float* x, int N, int C, int H, int W, const float* gate, void* y, int Cp,
                              float* chan_mean, void* stream) {
  DMF_CHECK_ARG(x && (y || chan_mean) && Cp >= C, "dmf_input_prep: bad args");
  const long long total = (long long)N * H * W;
  if (total == 0) return 0;
  if (y && Cp % 8 == 0 && a16(y)) {
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_input_prep8<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, x, N, C, H, W,
                         gate, (T*)y, Cp, chan_mean));
  } else DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_input_prep<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, x, N, C, H, W, gate,
                       (T*)y, Cp, chan_mean));
  DMF_LAUNCH_CHECK("dmf_input_prep");
  return 0;
}

extern "C" int dmf_nchw_mean(const float* x, int NC, long long HW, float* out, void* stream) {
  DMF_CHECK_ARG(x && out && NC > 0 && HW > 0, "dmf_nchw_mean: bad args");
  if (HW % 4 == 0 && a16(x)) {
    hipLaunchKernelGGL(k_nchw_mean4, dim3(NC), dim3(256), 0, (hipStream_t)stream, x, HW, 1.f / (float)HW, out);
  } else {
    hipLaunchKernelGGL(k_nchw_mean, dim3(NC), dim3(256), 0, (hipStream_t)stream, x, HW, out);
  }
  DMF_LAUNCH_CHECK("dmf_nchw_mean");
  return 0;
}

// split plan of the vector path: (CVt, groups, S, rows per split)
static void nhwc_reduce_plan(int N, int HW, int C, int& CVt, int& groups, int& S, int& rpb) {
  const int CV = C / 8;
  CVt = CV < 32 ? CV : 32;
  groups = cdiv(CV, CVt);
  const int R = 256 / CVt;
  // >= ~1024 blocks chip-wide, each split >= 8 passes of R rows
  S = std::max(1, std::min(cdiv(1024, N * groups), cdiv(HW, 8 * R)));
  rpb = cdiv(HW, S);
  rpb = cdiv(rpb, R) * R;
  S = cdiv(HW, rpb);
}

extern "C" int dmf_nhwc_reduce_splits(int N, int HW, int C) {
  if (C % 8 != 0) return 0;
  int CVt, groups, S, rpb;
  nhwc_reduce_plan(N, HW, C, CVt, groups, S, rpb);
  return S;
}

extern "C" int dmf_nhwc_reduce_ws_size(int N, int HW, int C) {
  if (C % 8 != 0) return 0;
  int CVt, groups, S, rpb;
  nhwc_reduce_plan(N, HW, C, CVt, groups, S, rpb);
  return 2 * S * N * C;
}

extern "C" int dmf_nhwc_reduce(int dtype, const void* a, int lda, const void* b, int ldb, int N, int HW, int C,
                               float scale, float* out, float* out_sq, int accumulate, float* workspace,
                               void* stream) {
  DMF_CHECK_ARG(a && (out || workspace) && N > 0 && HW > 0 && C > 0, "dmf_nhwc_reduce: bad args");
  DMF_CHECK_ARG(out || (v8ok(C, lda, b ? ldb : 8, a, b) && !out_sq),
                "dmf_nhwc_reduce: the stage-1-only form (out == NULL) needs the 8-channel vector layout");
  DMF_CHECK_ARG(!(b && out_sq), "dmf_nhwc_reduce: out_sq is for the plain (b == NULL) form");
  hipStream_t st = (hipStream_t)stream;
  if (workspace && v8ok(C, lda, b ? ldb : 8, a, b)) {
    int CVt, groups, S, rpb;
    nhwc_reduce_plan(N, HW, C, CVt, groups, S, rpb);
    const dim3 g8(N, groups, S);
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_nhwc_reduce8<T>, g8, dim3(256), 0, st, (const T*)a, lda, (const T*)b, ldb,
                         HW, C, CVt, rpb, out_sq ? 1 : 0, workspace));
    const long long nc = (long long)N * C;
    if (!out) {  // stage 1 only: the consumer (dmf_se_mlp) sums the S partial planes itself
      DMF_LAUNCH_CHECK("dmf_nhwc_reduce");
      return 0;
    }
    hipLaunchKernelGGL(k_nhwc_reduce_fin, dim3(gsz(nc * (out_sq ? 2 : 1))), dim3(256), 0, st, workspace, S, nc, scale,
                       out, out_sq, accumulate);
    DMF_LAUNCH_CHECK("dmf_nhwc_reduce");
    return 0;
  }
  dim3 grid(N, cdiv(C, 64));
  for (int pass = 0; pass < (out_sq ? 2 : 1); ++pass) {
    const void* bb = pass ? a : b;
    const int ldbb = pass ? lda : ldb;
    float* o = pass ? out_sq : out;
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_nhwc_reduce<T>, grid, dim3(256), 0, st, (const T*)a, lda, (const T*)bb,
                         ldbb, HW, C, scale, o, accumulate));
  }
  DMF_LAUNCH_CHECK("dmf_nhwc_reduce");
  return 0;
}

extern "C" int dmf_channel_scale(int dtype, const void* x, int ldx, const float* gate, void* y, int ldy, int N, int HW,
                                 int C, void* stream) {
  DMF_CHECK_ARG(x && gate && y, "dmf_channel_scale: bad args");
  const long long total = (long long)N * HW * C;
  if (total == 0) return 0;
  if (v8ok(C, ldx, ldy, x, y, gate)) {
    // 32-bit index math when every offset fits (a 64-bit div per chunk otherwise)
    if ((long long)N * HW * std::max(ldx, ldy) < (1LL << 30))
      DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((k_channel_scale8<T, int>), dim3(gsz(total / 8)), dim3(256), 0,
                                                      (hipStream_t)stream, (const T*)x, ldx, gate, (T*)y, ldy,
                                                      (long long)N, HW, C));
    else
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_channel_scale8<T>, dim3(gsz(total / 8)), dim3(256), 0, (hipStream_t)stream,
                         (const T*)x, ldx, gate, (T*)y, ldy, (long long)N, HW, C));
    DMF_LAUNCH_CHECK("dmf_channel_scale");
    return 0;
  }
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_channel_scale<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, (const T*)x,
                       ldx, gate, (T*)y, ldy, (long long)N, HW, C));
  DMF_LAUNCH_CHECK("dmf_channel_scale");
  return 0;
}

extern "C" int dmf_mix(int dtype, const void* a, int lda, const void* b, int ldb, const float* wlogit, void* z, int ldz,
                       long long M, int C, void* stream) {
  DMF_CHECK_ARG(a && b && wlogit && z, "dmf_mix: bad args");
  if (M * C == 0) return 0;
  if (v8ok(C, lda, ldb, a, b) && ldz % 8 == 0 && a16(z)) {
    if (M * std::max(std::max(lda, ldb), std::max(ldz, C)) < (1LL << 30))
      DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((k_mix8<T, int>), dim3(gsz(M * C / 8)), dim3(256), 0,
                                                      (hipStream_t)stream, (const T*)a, lda, (const T*)b, ldb, wlogit,
                                                      (T*)z, ldz, M, C));
    else
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_mix8<T>, dim3(gsz(M * C / 8)), dim3(256), 0, (hipStream_t)stream, (const T*)a,
                         lda, (const T*)b, ldb, wlogit, (T*)z, ldz, M, C));
    DMF_LAUNCH_CHECK("dmf_mix");
    return 0;
  }
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_mix<T>, dim3(gsz(M * C)), dim3(256), 0, (hipStream_t)stream, (const T*)a, lda,
                       (const T*)b, ldb, wlogit, (T*)z, ldz, M, C));
  DMF_LAUNCH_CHECK("dmf_mix");
  return 0;
}

extern "C" int dmf_gn_apply(int dtype, const void* z, int ldz, const float* mean, const float* m2, const float* gamma,
                            const float* beta, float eps, void* y, int ldy, int N, int HW, int C, void* stream) {
  DMF_CHECK_ARG(z && mean && m2 && gamma && beta && y, "dmf_gn_apply: bad args");
  const long long total = (long long)N * HW * C;
  if (total == 0) return 0;
  const long long rows = (long long)N * HW;
  if (v8ok(C, ldz, ldy, z, y) && a16(mean) && a16(m2) && a16(gamma) && a16(beta) && rows * C < (1LL << 31) &&
      rows * ldz < (1LL << 31) && rows * ldy < (1LL << 31)) {
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_gn_apply8<T>, dim3(gsz(total / 8)), dim3(256), 0,
                                                    (hipStream_t)stream, (const T*)z, ldz, mean, m2, gamma, beta, eps,
                                                    (T*)y, ldy, (int)rows, HW, C));
    DMF_LAUNCH_CHECK("dmf_gn_apply");
    return 0;
  }
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_gn_apply<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, (const T*)z, ldz,
                       mean, m2, gamma, beta, eps, (T*)y, ldy, (long long)N, HW, C));
  DMF_LAUNCH_CHECK("dmf_gn_apply");
  return 0;
}

extern "C" int dmf_gn_bwd(int dtype, const void* dy, int lddy, const void* z, int ldz, const float* mean,
                          const float* m2, const float* gamma, float eps, float* s1, float* s2, void* dz, int lddz,
                          int N, int HW, int C, void* stream) {
  DMF_CHECK_ARG(dy && z && mean && m2 && gamma && s1 && s2 && dz, "dmf_gn_bwd: bad args");
  dim3 grid(N, cdiv(C, 64));
  const long long total = (long long)N * HW * C;
  const long long rows = (long long)N * HW;
  const bool apply8 = v8ok(C, lddy, ldz, dy, z, dz) && lddz % 8 == 0 && a16(mean) && a16(m2) && a16(s1) &&
                      a16(s2) && a16(gamma) && rows * C < (1LL << 31) && rows * lddy < (1LL << 31) &&
                      rows * ldz < (1LL << 31) && rows * lddz < (1LL << 31);
  DMF_DISPATCH_DTYPE(dtype, T, if (v8ok(C, lddy, ldz, dy, z))
      hipLaunchKernelGGL(k_gn_bwd_reduce8<T>, grid, dim3(256), 0, (hipStream_t)stream, (const T*)dy, lddy,
                         (const T*)z, ldz, mean, m2, eps, HW, C, s1, s2);
    else
      hipLaunchKernelGGL(k_gn_bwd_reduce<T>, grid, dim3(256), 0, (hipStream_t)stream, (const T*)dy, lddy,
                         (const T*)z, ldz, mean, m2, eps, HW, C, s1, s2);
    if (apply8)
      hipLaunchKernelGGL(k_gn_bwd_apply8<T>, dim3(gsz(total / 8)), dim3(256), 0, (hipStream_t)stream, (const T*)dy,
                         lddy, (const T*)z, ldz, mean, m2, s1, s2, gamma, eps, (T*)dz, lddz, (int)rows, HW, C);
    else
      hipLaunchKernelGGL(k_gn_bwd_apply<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, (const T*)dy,
                         lddy, (const T*)z, ldz, mean, m2, s1, s2, gamma, eps, (T*)dz, lddz, (long long)N, HW,
                         C));
  DMF_LAUNCH_CHECK("dmf_gn_bwd");
  return 0;
}

extern "C" int dmf_maxpool2d(int dtype, const void* x, int N, int H, int W, int C, int ldx, void* y, int Ho, int Wo,
                             int ldy, int k, int s, int p, void* stream) {
  DMF_CHECK_ARG(x && y && k > 0 && s > 0, "dmf_maxpool2d: bad args");
  const long long total = (long long)N * Ho * Wo * C;
  if (total == 0) return 0;
  if (v8ok(C, ldx, ldy, x, y)) {
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_maxpool8<T>, dim3(gsz(total / 8)), dim3(256), 0, (hipStream_t)stream,
                         (const T*)x, N, H, W, C, ldx, (T*)y, Ho, Wo, ldy, k, s, p));
    DMF_LAUNCH_CHECK("dmf_maxpool2d");
    return 0;
  }
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_maxpool<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, (const T*)x, N, H,
                       W, C, ldx, (T*)y, Ho, Wo, ldy, k, s, p));
  DMF_LAUNCH_CHECK("dmf_maxpool2d");
  return 0;
}

// output size of the 2x2 average pool (see k_avgpool2): same -> H; else ceil((H - 2) / s) + 1, the last
// window dropped when it would start past the input (torch ceil_mode with no padding)
static inline int avgpool2_out(int H, int s, int same) {
  if (same) return H;
  int o = (H - 2 + s - 1) / s + 1;
  if ((o - 1) * s >= H) --o;
  return o;
}

extern "C" int dmf_avgpool2d(int dtype, const void* x, int N, int H, int W, int C, int ldx, void* y, int Ho, int Wo,
                             int ldy, int s, int same, void* stream) {
  DMF_CHECK_ARG(x && y && (s == 1 || s == 2) && (same == 0 || (same == 1 && s == 1)) && H >= 2 && W >= 2,
                "dmf_avgpool2d: bad args (s=%d same=%d H=%d W=%d)", s, same, H, W);
  DMF_CHECK_ARG(Ho == avgpool2_out(H, s, same) && Wo == avgpool2_out(W, s, same) && ldx >= C && ldy >= C,
                "dmf_avgpool2d: output %dx%d does not match the pool of %dx%d", Ho, Wo, H, W);
  const long long total = (long long)N * Ho * Wo * C;
  if (total == 0) return 0;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_avgpool2<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream,
                       (const T*)x, N, H, W, C, ldx, (T*)y, Ho, Wo, ldy, s, same));
  DMF_LAUNCH_CHECK("dmf_avgpool2d");
  return 0;
}

extern "C" int dmf_avgpool2d_bwd(int dtype, const void* dy, int N, int H, int W, int C, int Ho, int Wo, int lddy,
                                 void* dx, int lddx, int s, int same, void* stream) {
  DMF_CHECK_ARG(dy && dx && (s == 1 || s == 2) && (same == 0 || (same == 1 && s == 1)) && H >= 2 && W >= 2,
                "dmf_avgpool2d_bwd: bad args");
  DMF_CHECK_ARG(Ho == avgpool2_out(H, s, same) && Wo == avgpool2_out(W, s, same) && lddy >= C && lddx >= C,
                "dmf_avgpool2d_bwd: shapes");
  const long long total = (long long)N * H * W * C;
  if (total == 0) return 0;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_avgpool2_bwd<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream,
                       (const T*)dy, N, H, W, C, Ho, Wo, lddy, (T*)dx, lddx, s, same));
  DMF_LAUNCH_CHECK("dmf_avgpool2d_bwd");
  return 0;
}

extern "C" int dmf_maxpool2d_idx(int dtype, const void* x, int N, int H, int W, int C, int ldx, void* y, int Ho, int Wo,
                                 int ldy, void* idx, int k, int s, int p, void* stream) {
  DMF_CHECK_ARG(x && y && idx && k >= 1 && k * k <= 255, "dmf_maxpool2d_idx: bad args");
  DMF_CHECK_ARG(v8ok(C, ldx, ldy, x, y) && ((uintptr_t)idx % 8) == 0, "dmf_maxpool2d_idx: needs C, strides % 8 == 0");
  const long long total = (long long)N * Ho * Wo * C;
  DMF_CHECK_ARG(total < (1LL << 31) && (long long)N * H * W * C < (1LL << 31), "dmf_maxpool2d_idx: too large");
  if (total == 0) return 0;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_maxpool_idx8<T>, dim3(gsz(total / 8)), dim3(256), 0, (hipStream_t)stream,
                       (const T*)x, N, H, W, C, ldx, (T*)y, Ho, Wo, ldy, (unsigned char*)idx, k, s, p));
  DMF_LAUNCH_CHECK("dmf_maxpool2d_idx");
  return 0;
}

extern "C" int dmf_maxpool2d_bwd_idx(int dtype, const void* dy, int N, int H, int W, int C, int Ho, int Wo, int lddy,
                                     const void* idx, void* dx, int lddx, int k, int s, int p, void* stream) {
  DMF_CHECK_ARG(dy && idx && dx && k >= 1 && k * k <= 255, "dmf_maxpool2d_bwd_idx: bad args");
  DMF_CHECK_ARG(v8ok(C, lddy, lddx, dy, dx) && ((uintptr_t)idx % 8) == 0, "dmf_maxpool2d_bwd_idx: needs C, strides % 8 == 0");
  const long long total = (long long)N * H * W * C;
  DMF_CHECK_ARG(total < (1LL << 31), "dmf_maxpool2d_bwd_idx: too large");
  if (total == 0) return 0;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_maxpool_bwd_idx8<T>, dim3(gsz(total / 8)), dim3(256), 0, (hipStream_t)stream,
                       (const T*)dy, N, H, W, C, Ho, Wo, lddy, (const unsigned char*)idx, (T*)dx, lddx, k, s,
                       p));
  DMF_LAUNCH_CHECK("dmf_maxpool2d_bwd_idx");
  return 0;
}

extern "C" int dmf_maxpool2d_bwd(int dtype, const void* x, int N, int H, int W, int C, int ldx, const void* dy, int Ho,
                                 int Wo, int lddy, void* dx, int lddx, int k, int s, int p, void* stream) {
  DMF_CHECK_ARG(x && dy && dx, "dmf_maxpool2d_bwd: bad args");
  const long long total = (long long)N * H * W * C;
  if (total == 0) return 0;
  if (v8ok(C, ldx, lddy, x, dy, dx) && lddx % 8 == 0) {
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_maxpool_bwd8<T>, dim3(gsz(total / 8)), dim3(256), 0, (hipStream_t)stream,
                         (const T*)x, N, H, W, C, ldx, (const T*)dy, Ho, Wo, lddy, (T*)dx, lddx, k, s, p));
    DMF_LAUNCH_CHECK("dmf_maxpool2d_bwd");
    return 0;
  }
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_maxpool_bwd<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, (const T*)x,
                       N, H, W, C, ldx, (const T*)dy, Ho, Wo, lddy, (T*)dx, lddx, k, s, p));
  DMF_LAUNCH_CHECK("dmf_maxpool2d_bwd");
  return 0;
}

extern "C" int dmf_upsample_nearest(int dtype, const void* x, int ldx, void* y, int N, int H, int W, int C, int r,
                                    void* stream) {
  DMF_CHECK_ARG(x && y && r >= 1, "dmf_upsample_nearest: bad args");
  const long long total = (long long)N * r * r * H * W * C;
  if (total == 0) return 0;
  if (v8ok(C, ldx, 8, x, y)) {
    if (total < (1LL << 30) && (long long)N * H * W * ldx < (1LL << 30))
      DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((k_up_nearest8<T, int>), dim3(gsz(total / 8)), dim3(256), 0,
                                                      (hipStream_t)stream, (const T*)x, ldx, (T*)y, N, H, W, C, r));
    else
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_up_nearest8<T>, dim3(gsz(total / 8)), dim3(256), 0, (hipStream_t)stream,
                         (const T*)x, ldx, (T*)y, N, H, W, C, r));
    DMF_LAUNCH_CHECK("dmf_upsample_nearest");
    return 0;
  }
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_up_nearest<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, (const T*)x,
                       ldx, (T*)y, N, H, W, C, r));
  DMF_LAUNCH_CHECK("dmf_upsample_nearest");
  return 0;
}

extern "C" int dmf_upsample_nearest_bwd(int dtype, const void* dy, void* dx, int N, int H, int W, int C, int r,
                                        void* stream) {
  DMF_CHECK_ARG(dy && dx && r >= 1, "dmf_upsample_nearest_bwd: bad args");
  const long long total = (long long)N * H * W * C;
  if (total == 0) return 0;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_up_nearest_bwd<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream,
                       (const T*)dy, (T*)dx, N, H, W, C, r));
  DMF_LAUNCH_CHECK("dmf_upsample_nearest_bwd");
  return 0;
}

extern "C" int dmf_bilinear(int dtype, const void* x, int N, int Hi, int Wi, int C, int ldx, void* y, int Ho, int Wo,
                            int ldy, void* stream) {
  DMF_CHECK_ARG(x && y, "dmf_bilinear: bad args");
  const long long total = (long long)N * Ho * Wo * C;
  if (total == 0) return 0;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_bilinear<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, (const T*)x, N,
                       Hi, Wi, C, ldx, (T*)y, Ho, Wo, ldy));
  DMF_LAUNCH_CHECK("dmf_bilinear");
  return 0;
}

extern "C" int dmf_bilinear_bwd(int dtype, const void* dy, int N, int Ho, int Wo, int C, int lddy, void* dx, int Hi,
                                int Wi, int lddx, void* stream) {
  DMF_CHECK_ARG(dy && dx, "dmf_bilinear_bwd: bad args");
  const long long total = (long long)N * Hi * Wi * C;
  if (total == 0) return 0;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_bilinear_bwd<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, (const T*)dy,
                       N, Ho, Wo, C, lddy, (T*)dx, Hi, Wi, lddx));
  DMF_LAUNCH_CHECK("dmf_bilinear_bwd");
  return 0;
}

extern "C" int dmf_col_stats_tiles(long long M) { return (int)((M + 255) / 256); }

extern "C" int dmf_col_stats(int dtype, const void* x, int ldx, long long M, int C, float* partials, void* stream) {
  DMF_CHECK_ARG(x && partials && M > 0 && C > 0, "dmf_col_stats: bad args");
  const int es = is16(dtype) ? 2 : 4;
  if (C % 8 == 0 && ldx % 8 == 0 && ((uintptr_t)x % (8 * es)) == 0) {
    const int CVt = std::min(32, C / 8);
    dim3 g8((unsigned)((M + 255) / 256), (unsigned)cdiv(C / 8, CVt));
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_col_stats8<T>, g8, dim3(256), 0, (hipStream_t)stream, (const T*)x, ldx, M, C, CVt,
                         partials));
    DMF_LAUNCH_CHECK("dmf_col_stats");
    return 0;
  }
  dim3 grid((unsigned)((M + 255) / 256), (unsigned)cdiv(C, 64));
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_col_stats<T>, grid, dim3(256), 0, (hipStream_t)stream, (const T*)x, ldx, M, C,
                       partials));
  DMF_LAUNCH_CHECK("dmf_col_stats");
  return 0;
}

extern "C" int dmf_mask_attn_fwd(int dtype, const void* f, int ldf, const void* m, int N, int HW, int C,
                                 const float* w1, const float* gn_w, const float* gn_b, const float* w2,
                                 const float* b2, const float* gamma, int hidden, float eps, float* stats, void* out,
                                 int ldo, void* A_out, void* stream) {
  DMF_CHECK_ARG(f && m && w1 && gn_w && gn_b && w2 && b2 && gamma && stats && out && hidden > 0,
                "dmf_mask_attn_fwd: bad args");
  MaskAttnP P{w1, gn_w, gn_b, w2, b2, gamma, eps, hidden};
  const long long total = (long long)N * HW;
  const int grid = (int)((total + 3) / 4 > 16384 ? 16384 : (total + 3) / 4);
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_mask_stats<T>, dim3(N), dim3(256), 0, (hipStream_t)stream, (const T*)m, HW, stats);
    hipLaunchKernelGGL(k_mask_attn_fwd<T>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const T*)f, ldf,
                       (const T*)m, P, stats, (T*)out, ldo, (T*)A_out, (long long)N, HW, C));
  DMF_LAUNCH_CHECK("dmf_mask_attn_fwd");
  return 0;
}

// ------------------------------------------------ adaptive average pooling
// nn.AdaptiveAvgPool2d((Ho, Wo)) on NHWC (model_module.py:534 proj_pool when
// the map size does not divide proj_dim, e.g. 48 -> 64 at S=384): output bin
// i covers input rows [floor(i*H/Ho), ceil((i+1)*H/Ho)). One thread per
// (output pixel, channel); the backward gathers, per input pixel, the bins
// that contain it (no atomics).
namespace dmf {
__device__ __forceinline__ int ap_lo(int i, int in, int out) { return (int)(((long long)i * in) / out); }
__device__ __forceinline__ int ap_hi(int i, int in, int out) { return (int)(((long long)(i + 1) * in + out - 1) / out); }

template <typename T>
__global__ void k_adaptive_avgpool(const T* __restrict__ x, int ldx, T* __restrict__ y, int ldy, int N, int H, int W,
                                   int C, int Ho, int Wo) {
  const long long total = (long long)N * Ho * Wo * C;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    const long long p = e / C;
    const int j = (int)(p % Wo), i = (int)((p / Wo) % Ho), n = (int)(p / ((long long)Wo * Ho));
    const int h0 = ap_lo(i, H, Ho), h1 = ap_hi(i, H, Ho), w0 = ap_lo(j, W, Wo), w1 = ap_hi(j, W, Wo);
    float s = 0.f;
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) s += ld(x + ((size_t)(n * H + h) * W + w) * ldx + c);
    st(y + p * ldy + c, s / (float)((h1 - h0) * (w1 - w0)));
  }
}

template <typename T>
__global__ void k_adaptive_avgpool_bwd(const T* __restrict__ dy, int lddy, T* __restrict__ dx, int lddx, int N, int H,
                                       int W, int C, int Ho, int Wo) {
  const long long total = (long long)N * H * W * C;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    const long long p = e / C;
    const int w = (int)(p % W), h = (int)((p / W) % H), n = (int)(p / ((long long)W * H));
    // candidate output bins: floor(h*Ho/H) - 1 .. ceil((h+1)*Ho/H) (clamped)
    const int i0 = max(0, (int)(((long long)h * Ho) / H) - 1), i1 = min(Ho, (int)(((long long)(h + 1) * Ho + H - 1) / H) + 1);
    const int j0 = max(0, (int)(((long long)w * Wo) / W) - 1), j1 = min(Wo, (int)(((long long)(w + 1) * Wo + W - 1) / W) + 1);
    float s = 0.f;
    for (int i = i0; i < i1; ++i) {
      const int a0 = ap_lo(i, H, Ho), a1 = ap_hi(i, H, Ho);
      if (h < a0 || h >= a1) continue;
      for (int j = j0; j < j1; ++j) {
        const int b0 = ap_lo(j, W, Wo), b1 = ap_hi(j, W, Wo);
        if (w < b0 || w >= b1) continue;
        s += ld(dy + ((size_t)(n * Ho + i) * Wo + j) * lddy + c) / (float)((a1 - a0) * (b1 - b0));
      }
    }
    st(dx + p * lddx + c, s);
  }
}
// the same on 8-channel (16-B) vectors with 32-bit index math: one thread per (output pixel, 8 channels),
// the window summed in the same (h, w) order per channel (bit-identical to k_adaptive_avgpool); the
// scalar form's 64-bit div / mod per element made it ~3x a copy of its bytes
template <typename T>
__global__ void __launch_bounds__(256) k_adaptive_avgpool8(const T* __restrict__ x, int ldx, T* __restrict__ y, int ldy,
                                                           int N, int H, int W, int C, int Ho, int Wo, int total8) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= total8) return;
  const int C8 = C >> 3;
  const int c = (e % C8) * 8;
  const int p = e / C8;
  const int j = p % Wo, q = p / Wo, i = q % Ho, n = q / Ho;
  const int h0 = ap_lo(i, H, Ho), h1 = ap_hi(i, H, Ho), w0 = ap_lo(j, W, Wo), w1 = ap_hi(j, W, Wo);
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.f;
  for (int h = h0; h < h1; ++h)
    for (int w = w0; w < w1; ++w) {
      float v[8];
      ld8(x + ((size_t)(n * H + h) * W + w) * ldx + c, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += v[k];
    }
  const float d = (float)((h1 - h0) * (w1 - w0));
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = s[k] / d;
  st8(y + (size_t)p * ldy + c, s);
}
}  // namespace dmf

extern "C" int dmf_adaptive_avgpool2d(int dtype, const void* x, int N, int H, int W, int C, int ldx, void* y, int Ho,
                                      int Wo, int ldy, void* stream) {
  DMF_CHECK_ARG(x && y && N > 0 && H > 0 && W > 0 && C > 0 && Ho > 0 && Wo > 0, "dmf_adaptive_avgpool2d: bad args");
  const long long total = (long long)N * Ho * Wo * C;
  if (C % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0 &&
      total / 8 < (1LL << 31) && (long long)N * H * W * ldx < (1LL << 31)) {
    const int total8 = (int)(total / 8);
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_adaptive_avgpool8<T>, dim3((unsigned)cdiv(total8, 256)), dim3(256),
                                                    0, (hipStream_t)stream, (const T*)x, ldx, (T*)y, ldy, N, H, W, C,
                                                    Ho, Wo, total8));
    DMF_LAUNCH_CHECK("dmf_adaptive_avgpool2d");
    return 0;
  }
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_adaptive_avgpool<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream,
                       (const T*)x, ldx, (T*)y, ldy, N, H, W, C, Ho, Wo));
  DMF_LAUNCH_CHECK("dmf_adaptive_avgpool2d");
  return 0;
}

extern "C" int dmf_adaptive_avgpool2d_bwd(int dtype, const void* dy, int N, int Ho, int Wo, int C, int lddy, void* dx,
                                          int H, int W, int lddx, void* stream) {
  DMF_CHECK_ARG(dy && dx && N > 0 && H > 0 && W > 0 && C > 0 && Ho > 0 && Wo > 0,
                "dmf_adaptive_avgpool2d_bwd: bad args");
  const long long total = (long long)N * H * W * C;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_adaptive_avgpool_bwd<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream,
                       (const T*)dy, lddy, (T*)dx, lddx, N, H, W, C, Ho, Wo));
  DMF_LAUNCH_CHECK("dmf_adaptive_avgpool2d_bwd");
  return 0;
}
