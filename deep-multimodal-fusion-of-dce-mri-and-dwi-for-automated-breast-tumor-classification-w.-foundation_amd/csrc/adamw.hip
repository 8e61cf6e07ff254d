// Multi-tensor AdamW (torch.optim.AdamW, amsgrad=False, as built by
// LightningFusionOptimizerFactory._build_optimizer, selector_helpers.py:
// 632-685 / _get_base_optimizer :617-629) in ONE launch over a chunk table,
// plus a multi-tensor copy used to pack/unpack gradient buckets for the
// RCCL all-reduce. Step counts live on the device (graph-replay safe).
//   p <- p * (1 - lr*wd); m <- m + (1-b1)(g-m); v <- b2 v + (1-b2) g^2
//   p <- p - lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

// tensors: [T][6] int64 = p, g, m, v, group, numel ; chunks: [n][3] = tensor, begin, end
__global__ void k_adamw(const long long* __restrict__ chunks, const long long* __restrict__ tensors,
                        const float* __restrict__ hyper, const int* __restrict__ steps, float gscale) {
  const long long* ch = chunks + 3 * blockIdx.x;
  const int t = (int)ch[0];
  const long long b = ch[1], e = ch[2];
  const long long* td = tensors + 6 * t;
  float* p = (float*)td[0];
  const float* g = (const float*)td[1];
  float* m = (float*)td[2];
  float* v = (float*)td[3];
  const float* hp = hyper + 5 * td[4];
  const float lr = hp[0], wd = hp[1], b1 = hp[2], b2 = hp[3], eps = hp[4];
  const int step = steps[t];
  const double bc1 = 1.0 - pow((double)b1, (double)step);
  const double bc2 = 1.0 - pow((double)b2, (double)step);
  const float step_size = (float)(lr / bc1);
  const float bc2s = (float)sqrt(bc2);
  const float decay = 1.f - lr * wd;
  for (long long i = b + threadIdx.x; i < e; i += blockDim.x) {
    const float gi = g[i] * gscale;
    float pi = p[i] * decay;
    float mi = m[i];
    mi = mi + (1.f - b1) * (gi - mi);
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    const float denom = sqrtf(vi) / bc2s + eps;
    pi = pi - step_size * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

__global__ void k_steps_inc(int* steps, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) steps[i] += 1;
}

// pairs: [T][2] int64 = src, dst ; dst[i] = src[i] * scale
__global__ void k_multi_copy(const long long* __restrict__ chunks, const long long* __restrict__ pairs, float scale) {
  const long long* ch = chunks + 3 * blockIdx.x;
  const long long* pr = pairs + 2 * ch[0];
  const float* src = (const float*)pr[0];
  float* dst = (float*)pr[1];
  if (scale == 0.f) {  // zero fill (grad reset), NaN-safe
    for (long long i = ch[1] + threadIdx.x; i < ch[2]; i += blockDim.x) dst[i] = 0.f;
  } else {
    for (long long i = ch[1] + threadIdx.x; i < ch[2]; i += blockDim.x) dst[i] = src[i] * scale;
  }
}

}  // namespace dmf

using namespace dmf;

extern "C" int dmf_adamw_multi(int nchunks, const long long* chunks, const long long* tensors, const float* hyper,
                               const int* steps, float grad_scale, void* stream) {
  DMF_CHECK_ARG(nchunks >= 0 && chunks && tensors && hyper && steps, "dmf_adamw_multi: bad args");
  if (nchunks == 0) return 0;
  hipLaunchKernelGGL(k_adamw, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, chunks, tensors, hyper, steps,
                     grad_scale);
  DMF_LAUNCH_CHECK("dmf_adamw_multi");
  return 0;
}

extern "C" int dmf_steps_inc(int* steps, int n, void* stream) {
  DMF_CHECK_ARG(steps && n >= 0, "dmf_steps_inc: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_steps_inc, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, steps, n);
  DMF_LAUNCH_CHECK("dmf_steps_inc");
  return 0;
}

extern "C" int dmf_multi_copy(int nchunks, const long long* chunks, const long long* pairs, float scale,
                              void* stream) {
  DMF_CHECK_ARG(nchunks >= 0 && chunks && pairs, "dmf_multi_copy: bad args");
  if (nchunks == 0) return 0;
  hipLaunchKernelGGL(k_multi_copy, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, chunks, pairs, scale);
  DMF_LAUNCH_CHECK("dmf_multi_copy");
  return 0;
}
