// GPU data path: the reference's CPU preprocessing of
// the DWI / DCE stacks, batched over volumes on the device.
//   DWINormalize            dataset.py:9-41     per-(volume, channel) z-score (unbiased std,
//                                               clamp 1e-6), clip [-3, 3], map to [0, 1];
//                                               the ADC slot (last channel) stays 0 (quirk Q12)
//   compute_adc_map         preprocess_helpers.py:133-167  per-pixel least-squares slope of
//                                               log(max(S, eps)) on the b-values, ADC = -slope
//   preprocess_adc          preprocess_helpers.py:39-49    log1p(max(adc, 0)) -> clip [0, 3e-3] / 3e-3
//   NyulStandardizer        preprocess_helpers.py:52-120   per-image percentiles (numpy 'linear')
//                                               at the landmarks, then np.interp twice
//   train augmentation      prepare_single_model.py:107-113  torchvision RandomAffine(90, (0.1, 0.1),
//                                               (0.1, 0.1)) -> RandomHorizontalFlip -> RandomVerticalFlip
//                                               as ONE nearest-neighbour gather per output pixel (the
//                                               per-volume parameters drawn on the host in torchvision's
//                                               order), then Resize (bilinear, antialias) as two
//                                               separable passes (W then H, as aten's upsample_*_aa)
// Percentiles are exact order statistics: a multi-target radix select over
// the order-preserving uint32 image of the float keys (4 passes of 8-bit
// digits, one 256-bin LDS histogram per target rank), one block per
// (volume, channel) plane. np.percentile's arithmetic is restated exactly
// (virtual index (n-1)*q/100 in double, _lerp with the float32 difference).
#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

// ------------------------------------------------------------ block sums
__device__ __forceinline__ double dp_block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double r = 0.0;
  for (int i = 0; i < nw; ++i) r += red[i];
  return r;
}

// one block per (n, c) plane
__global__ void __launch_bounds__(1024) k_dwi_normalize(const float* __restrict__ x, int C, long long HW, int adc,
                                                        float zlo, float zhi, float* __restrict__ y) {
  __shared__ double red[16];
  const int plane = blockIdx.x, c = plane % C;
  const float* xp = x + (size_t)plane * HW;
  float* yp = y + (size_t)plane * HW;
  if (adc && c == C - 1) {  // the reference leaves the ADC slot zero (out = zeros_like)
    for (long long i = threadIdx.x; i < HW; i += blockDim.x) yp[i] = 0.f;
    return;
  }
  double s = 0.0;
  for (long long i = threadIdx.x; i < HW; i += blockDim.x) s += (double)xp[i];
  const double mean_d = dp_block_sum(s, red) / (double)HW;
  double q = 0.0;
  for (long long i = threadIdx.x; i < HW; i += blockDim.x) {
    const double d = (double)xp[i] - mean_d;
    q += d * d;
  }
  const double var = HW > 1 ? dp_block_sum(q, red) / (double)(HW - 1) : 0.0;
  // torch: float32 mean / std scalars, then float32 elementwise
  const float mean = (float)mean_d;
  const float sd = fmaxf((float)sqrt(var), 1e-6f);
  const float span = zhi - zlo;
  for (long long i = threadIdx.x; i < HW; i += blockDim.x) {
    float z = (xp[i] - mean) / sd;
    z = fminf(fmaxf(z, zlo), zhi);
    yp[i] = (z - zlo) / span;
  }
}

// one thread per pixel; mode bit 0: preprocess_adc on the result
__global__ void k_adc_map(const float* __restrict__ dwi, int C, long long HW, long long total,
                          const float* __restrict__ bvals, float eps, int pre, float* __restrict__ adc) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / HW, p = i - n * HW;
    const float* s = dwi + (size_t)n * C * HW + p;
    float mb = 0.f, ml = 0.f;
    for (int c = 0; c < C; ++c) {
      mb += bvals[c];
      ml += logf(fmaxf(s[(size_t)c * HW], eps));
    }
    mb /= (float)C;
    ml /= (float)C;
    float cov = 0.f, var = 0.f;
    for (int c = 0; c < C; ++c) {
      const float db = bvals[c] - mb;
      cov += db * (logf(fmaxf(s[(size_t)c * HW], eps)) - ml);
      var += db * db;
    }
    float a = -(cov / (var + eps));
    if (pre) a = fminf(fmaxf(log1pf(fmaxf(a, 0.f)), 0.f), 3e-3f) / 3e-3f;
    adc[i] = a;
  }
}

// ------------------------------------------------------------ percentiles
__device__ __forceinline__ unsigned f2key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

constexpr int DP_MAXT = 64;  // distinct order statistics per plane

// one block (1024 threads) per plane: ranks[T] (ascending) -> keys[T]
__global__ void __launch_bounds__(1024) k_plane_select(const float* __restrict__ x, long long HW,
                                                       const int* __restrict__ ranks, int T,
                                                       float* __restrict__ vals) {
  extern __shared__ unsigned hist[];  // [T][256]
  __shared__ unsigned prefix[DP_MAXT], remaining[DP_MAXT];
  const float* xp = x + (size_t)blockIdx.x * HW;
  if (threadIdx.x < T) {
    prefix[threadIdx.x] = 0u;
    remaining[threadIdx.x] = (unsigned)ranks[threadIdx.x];
  }
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < T * 256; i += blockDim.x) hist[i] = 0u;
    __syncthreads();
    for (long long i = threadIdx.x; i < HW; i += blockDim.x) {
      const unsigned k = f2key(xp[i]);
      const unsigned hi = shift == 24 ? 0u : (k >> (shift + 8));
      const unsigned d = (k >> shift) & 255u;
      unsigned last = 0xffffffffu;  // targets sharing a prefix share one bin: count once per prefix
      for (int t = 0; t < T; ++t) {
        if (prefix[t] == hi && prefix[t] != last) {
          // the first target with this prefix owns the histogram row
          atomicAdd(&hist[t * 256 + d], 1u);
          last = prefix[t];
        }
      }
    }
    __syncthreads();
    // one thread per target: owner row = first target with the same prefix;
    // every target reads the old prefixes before any is updated
    unsigned new_r = 0u, new_p = 0u;
    if (threadIdx.x < T) {
      const int t = threadIdx.x;
      int owner = t;
      while (owner > 0 && prefix[owner - 1] == prefix[t]) --owner;
      const unsigned* h = hist + owner * 256;
      unsigned r = remaining[t], acc = 0u;
      int d = 0;
      for (; d < 255; ++d) {
        if (acc + h[d] > r) break;
        acc += h[d];
      }
      new_r = r - acc;
      new_p = (prefix[t] << 8) | (unsigned)d;
    }
    __syncthreads();
    if (threadIdx.x < T) {
      remaining[threadIdx.x] = new_r;
      prefix[threadIdx.x] = new_p;
    }
    __syncthreads();
  }
  if (threadIdx.x < T) vals[(size_t)blockIdx.x * T + threadIdx.x] = key2f(prefix[threadIdx.x]);
}

// numpy 'linear' percentile from the order statistics: pos = (n-1)*q/100,
// lo = floor(pos), g = pos - lo; _lerp(v[lo], v[lo+1], g) with the float32
// difference (numpy subtracts in the input dtype) -> double
__global__ void k_plane_percentiles(const float* __restrict__ vals, int T, const int* __restrict__ lo_idx,
                                    const int* __restrict__ hi_idx, const double* __restrict__ gam, int L,
                                    int planes, double* __restrict__ perc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= planes * L) return;
  const int pl = i / L, l = i - pl * L;
  const float a = vals[(size_t)pl * T + lo_idx[l]], b = vals[(size_t)pl * T + hi_idx[l]];
  const double g = gam[l];
  const double diff = (double)(b - a);  // float32 subtraction, as numpy
  perc[i] = g >= 0.5 ? (double)b - diff * (1.0 - g) : (double)a + diff * g;
}

// np.interp (numpy/_core/src/multiarray/compiled_base.c arr_interp), double
__device__ __forceinline__ double np_interp(double x, const double* xp, const double* fp, int n) {
  if (x > xp[n - 1]) return fp[n - 1];
  if (x < xp[0]) return fp[0];
  int j = 0;  // largest j with xp[j] <= x
  while (j + 1 < n && xp[j + 1] <= x) ++j;
  if (j == n - 1) return fp[j];
  if (xp[j] == x) return fp[j];
  const double slope = (fp[j + 1] - fp[j]) / (xp[j + 1] - xp[j]);
  double r = slope * (x - xp[j]) + fp[j];
  if (isnan(r)) {
    r = slope * (x - xp[j + 1]) + fp[j + 1];
    if (isnan(r) && fp[j] == fp[j + 1]) r = fp[j];
  }
  return r;
}

// NyulStandardizer.transform: per element, orig percentiles -> average
// landmarks -> standard scale (two np.interp); block per (plane, slice)
__global__ void __launch_bounds__(256) k_nyul_apply(const float* __restrict__ x, long long HW, int C,
                                                    const double* __restrict__ perc, const double* __restrict__ avg,
                                                    const double* __restrict__ scale, int L,
                                                    float* __restrict__ y) {
  __shared__ double sp[32], sa[32], ss[32];
  const int plane = blockIdx.y, c = plane % C;
  if (threadIdx.x < L) {
    sp[threadIdx.x] = perc[(size_t)plane * L + threadIdx.x];
    sa[threadIdx.x] = avg[(size_t)c * L + threadIdx.x];
    ss[threadIdx.x] = scale[threadIdx.x];
  }
  __syncthreads();
  const float* xp = x + (size_t)plane * HW;
  float* yp = y + (size_t)plane * HW;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += (long long)gridDim.x * blockDim.x) {
    const double m = np_interp((double)xp[i], sp, sa, L);
    yp[i] = (float)np_interp(m, sa, ss, L);
  }
}

// ------------------------------------------------------------ augmentation
// torchvision F.affine on a tensor (inverse matrix m[6] in centred pixel
// coordinates, _get_inverse_affine_matrix) = grid_sample(nearest, zeros,
// align_corners=False) of the grid that _gen_affine_grid builds; then the
// flips (applied AFTER the affine: out(i, j) = affine(i', j') with i' / j'
// mirrored). The float32 operation order follows torch's: base grid
// (j - W/2 + 0.5, i - H/2 + 0.5, 1) times theta^T / (W/2, H/2) (bmm, k = 0..2),
// unnormalise ((g + 1) * W - 1) / 2, round half to even (nearbyint).
// params[n] = {m0..m5, hflip, vflip}. One thread per output pixel, all
// channels (NCHW planes).
__global__ void __launch_bounds__(256) k_affine_flip(const float* __restrict__ x, int C, int H, int W,
                                                     const float* __restrict__ params, float* __restrict__ y) {
  const int n = blockIdx.y;
  const long long HW = (long long)H * W;
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  if (pix >= HW) return;
  const float* pm = params + n * 8;
  int i = (int)(pix / W), j = (int)(pix - (long long)i * W);
  if (pm[7] != 0.f) i = H - 1 - i;
  if (pm[6] != 0.f) j = W - 1 - j;
  const float hw = __fmul_rn(0.5f, (float)W), hh = __fmul_rn(0.5f, (float)H);
  const float bx = __fadd_rn(__fadd_rn((float)j, -__fmul_rn((float)W, 0.5f)), 0.5f);
  const float by = __fadd_rn(__fadd_rn((float)i, -__fmul_rn((float)H, 0.5f)), 0.5f);
  const float t00 = __fdiv_rn(pm[0], hw), t10 = __fdiv_rn(pm[1], hw), t20 = __fdiv_rn(pm[2], hw);
  const float t01 = __fdiv_rn(pm[3], hh), t11 = __fdiv_rn(pm[4], hh), t21 = __fdiv_rn(pm[5], hh);
  const float gx = __fadd_rn(__fadd_rn(__fmul_rn(bx, t00), __fmul_rn(by, t10)), t20);
  const float gy = __fadd_rn(__fadd_rn(__fmul_rn(bx, t01), __fmul_rn(by, t11)), t21);
  const float ix = __fdiv_rn(__fadd_rn(__fmul_rn(__fadd_rn(gx, 1.f), (float)W), -1.f), 2.f);
  const float iy = __fdiv_rn(__fadd_rn(__fmul_rn(__fadd_rn(gy, 1.f), (float)H), -1.f), 2.f);
  const float rx = rintf(ix), ry = rintf(iy);
  const bool in = rx >= 0.f && rx < (float)W && ry >= 0.f && ry < (float)H;
  const long long src = in ? (long long)ry * W + (long long)rx : 0;
  const float* xp = x + (long long)n * C * HW;
  float* yp = y + (long long)n * C * HW + pix;
  for (int c = 0; c < C; ++c) yp[c * HW] = in ? xp[c * HW + src] : 0.f;
}

// Resize, bilinear with antialias (aten _upsample_bilinear2d_aa, the kernel
// torchvision's tensor Resize runs): per output index o along one axis,
// scale = in/out, support = scale >= 1 ? scale : 1, centre = scale * (o + 0.5),
// window [max(int(centre - support + 0.5), 0), min(int(centre + support + 0.5), in)),
// triangle weights on (k + xmin - centre + 0.5) / max(scale, 1), normalised.
// axis 0: along W (rows of length Win -> Wout), axis 1: along H.
__device__ __forceinline__ float aa_tri(float v) {
  v = fabsf(v);
  return v < 1.f ? 1.f - v : 0.f;
}

__global__ void __launch_bounds__(256) k_resize_aa(const float* __restrict__ x, long long planes, int Hin, int Win,
                                                   int Hout, int Wout, int axis, float* __restrict__ y) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long per = (long long)Hout * Wout;
  if (idx >= planes * per) return;
  const long long pl = idx / per;
  const int r = (int)(idx - pl * per);
  const int oi = r / Wout, oj = r - (r / Wout) * Wout;
  const int in_size = axis == 0 ? Win : Hin, out_size = axis == 0 ? Wout : Hout, o = axis == 0 ? oj : oi;
  const float scale = (float)in_size / (float)out_size;
  const float support = scale >= 1.f ? scale : 1.f;
  const float invscale = scale >= 1.f ? 1.f / scale : 1.f;
  const float centre = scale * ((float)o + 0.5f);
  int xmin = (int)(centre - support + 0.5f);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(centre + support + 0.5f);
  if (xmax > in_size) xmax = in_size;
  float tot = 0.f;
  for (int k = xmin; k < xmax; ++k) tot += aa_tri(((float)(k - xmin) + (float)xmin - centre + 0.5f) * invscale);
  const float* xp = x + pl * (long long)Hin * Win;
  float acc = 0.f;
  for (int k = xmin; k < xmax; ++k) {
    float w = aa_tri(((float)(k - xmin) + (float)xmin - centre + 0.5f) * invscale);
    if (tot != 0.f) w /= tot;
    acc += w * (axis == 0 ? xp[(long long)oi * Win + k] : xp[(long long)k * Win + oj]);
  }
  y[idx] = acc;
}

}  // namespace dmf

using namespace dmf;

extern "C" int dmf_dwi_normalize(const float* x, int N, int C, long long HW, int adc, float z_lo, float z_hi, float* y,
                                 void* stream) {
  DMF_CHECK_ARG(x && y && N > 0 && C > 0 && HW > 0 && z_hi > z_lo, "dmf_dwi_normalize: bad args");
  hipLaunchKernelGGL(k_dwi_normalize, dim3(N * C), dim3(1024), 0, (hipStream_t)stream, x, C, HW, adc, z_lo, z_hi, y);
  DMF_LAUNCH_CHECK("dmf_dwi_normalize");
  return 0;
}

extern "C" int dmf_adc_map(const float* dwi, int N, int C, long long HW, const float* bvals, float eps, int preprocess,
                           float* adc, void* stream) {
  DMF_CHECK_ARG(dwi && bvals && adc && N > 0 && C > 1 && HW > 0, "dmf_adc_map: bad args");
  const long long total = (long long)N * HW;
  long long g = (total + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(k_adc_map, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, dwi, C, HW, total, bvals, eps,
                     preprocess, adc);
  DMF_LAUNCH_CHECK("dmf_adc_map");
  return 0;
}

extern "C" int dmf_plane_select(const float* x, int planes, long long HW, const int* ranks, int T, float* vals,
                                void* stream) {
  DMF_CHECK_ARG(x && ranks && vals && planes > 0 && HW > 0 && T > 0 && T <= DP_MAXT, "dmf_plane_select: bad args");
  DMF_CHECK_ARG(HW < (1LL << 32), "dmf_plane_select: plane too large");
  hipLaunchKernelGGL(k_plane_select, dim3(planes), dim3(1024), (size_t)T * 256 * 4, (hipStream_t)stream, x, HW, ranks,
                     T, vals);
  DMF_LAUNCH_CHECK("dmf_plane_select");
  return 0;
}

extern "C" int dmf_plane_percentiles(const float* vals, int T, const int* lo_idx, const int* hi_idx,
                                     const double* gamma, int L, int planes, double* perc, void* stream) {
  DMF_CHECK_ARG(vals && lo_idx && hi_idx && gamma && perc && L > 0 && planes > 0, "dmf_plane_percentiles: bad args");
  const int n = planes * L;
  hipLaunchKernelGGL(k_plane_percentiles, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, vals, T, lo_idx,
                     hi_idx, gamma, L, planes, perc);
  DMF_LAUNCH_CHECK("dmf_plane_percentiles");
  return 0;
}

extern "C" int dmf_nyul_apply(const float* x, int planes, int C, long long HW, const double* perc, const double* avg,
                              const double* scale, int L, float* y, void* stream) {
  DMF_CHECK_ARG(x && perc && avg && scale && y && planes > 0 && C > 0 && L >= 2 && L <= 32, "dmf_nyul_apply: bad args");
  long long gx = (HW + 255) / 256;
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(k_nyul_apply, dim3((unsigned)gx, planes), dim3(256), 0, (hipStream_t)stream, x, HW, C, perc, avg,
                     scale, L, y);
  DMF_LAUNCH_CHECK("dmf_nyul_apply");
  return 0;
}

extern "C" int dmf_affine_flip(const float* x, int N, int C, int H, int W, const float* params, float* y,
                               void* stream) {
  DMF_CHECK_ARG(x && params && y && N > 0 && C > 0 && H > 0 && W > 0 && N < 65536, "dmf_affine_flip: bad args");
  DMF_CHECK_ARG(x != y, "dmf_affine_flip: in-place is not supported (the gather reads arbitrary source pixels)");
  const long long HW = (long long)H * W;
  hipLaunchKernelGGL(k_affine_flip, dim3((unsigned)((HW + 255) / 256), (unsigned)N), dim3(256), 0,
                     (hipStream_t)stream, x, C, H, W, params, y);
  DMF_LAUNCH_CHECK("dmf_affine_flip");
  return 0;
}

extern "C" int dmf_resize_aa(const float* x, long long planes, int Hin, int Win, int Hout, int Wout, float* tmp,
                             float* y, void* stream) {
  DMF_CHECK_ARG(x && y && planes > 0 && Hin > 0 && Win > 0 && Hout > 0 && Wout > 0, "dmf_resize_aa: bad args");
  hipStream_t st = (hipStream_t)stream;
  const float* cur = x;
  int h = Hin, w = Win;
  if (Wout != Win) {  // horizontal pass first (aten order), into tmp unless it is the only pass
    float* dst = Hout != Hin ? tmp : y;
    DMF_CHECK_ARG(dst, "dmf_resize_aa: a two-pass resize needs tmp [planes][Hin][Wout]");
    const long long tot = planes * (long long)Hin * Wout;
    hipLaunchKernelGGL(k_resize_aa, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, cur, planes, Hin, Win, Hin,
                       Wout, 0, dst);
    cur = dst;
    w = Wout;
  }
  if (Hout != Hin) {
    const long long tot = planes * (long long)Hout * w;
    hipLaunchKernelGGL(k_resize_aa, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, cur, planes, h, w, Hout,
                       w, 1, y);
  } else if (Wout == Win) {
    DMF_CHECK_ARG(hipMemcpyAsync(y, x, planes * (long long)Hin * Win * sizeof(float), hipMemcpyDeviceToDevice, st) ==
                      hipSuccess,
                  "dmf_resize_aa: copy failed");
  }
  DMF_LAUNCH_CHECK("dmf_resize_aa");
  return 0;
}
