// Multi-tensor AdamW (torch.optim.AdamW, amsgrad=False, as built by
// LightningFusionOptimizerFactory._build_optimizer, selector_helpers.py:
// 632-685 / _get_base_optimizer :617-629) in ONE launch over a chunk table,
// plus a multi-tensor copy used to pack/unpack gradient buckets for the
// RCCL all-reduce. Step counts live on the device (graph-replay safe).
// Dynamic loss scaling ("16-mixed": torch.amp.GradScaler, as Lightning runs
// it): amp = {scale, found_inf} on the device; a non-finite check over the
// gradients sets found_inf, the update then skips every tensor (and the
// step counters) and unscales by 1/scale inside the same pass, and
// k_amp_update applies _amp_update_scale_'s growth / backoff rule.
//   p <- p * (1 - lr*wd); m <- m + (1-b1)(g-m); v <- b2 v + (1-b2) g^2
//   p <- p - lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

// tensors: [T][6] int64 = p, g, m, v, group, numel ; chunks: [n][3] = tensor, begin, end
__global__ void k_adamw(const long long* __restrict__ chunks, const long long* __restrict__ tensors,
                        const float* __restrict__ hyper, const int* __restrict__ steps, float gscale,
                        const float* __restrict__ amp) {
  if (amp) {
    if (amp[1] != 0.f) return;  // found_inf: the whole step is skipped
    gscale = gscale / amp[0];
  }
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

__global__ void k_steps_inc(int* steps, int n, const float* __restrict__ amp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (amp && amp[1] != 0.f) return;
  if (i < n) steps[i] += 1;
}

// found_inf (amp[1]) <- 1 if any gradient element of the table is inf / nan
// (torch._amp_foreach_non_finite_check_and_unscale_'s test; the unscale
// itself is folded into k_adamw). Benign race: every writer stores 1.
__global__ void k_amp_nonfinite(const long long* __restrict__ chunks, const long long* __restrict__ tensors,
                                float* __restrict__ amp) {
  const long long* ch = chunks + 3 * blockIdx.x;
  const float* g = (const float*)tensors[6 * ch[0] + 1];
  bool bad = false;
  for (long long i = ch[1] + threadIdx.x; i < ch[2]; i += blockDim.x) bad |= !isfinite(g[i]);
  const bool wave_bad = __any(bad);
  if (wave_bad && (threadIdx.x & 63) == 0) amp[1] = 1.f;
}

// torch._amp_update_scale_: found_inf -> scale *= backoff, tracker = 0;
// else tracker += 1 and, at growth_interval, scale *= growth (if finite), tracker = 0.
__global__ void k_amp_update(float* amp, int* tracker, float growth, float backoff, int interval) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (amp[1] != 0.f) {
    amp[0] *= backoff;
    tracker[0] = 0;
  } else {
    const int t = tracker[0] + 1;
    if (t == interval) {
      const float ns = amp[0] * growth;
      if (isfinite(ns)) amp[0] = ns;
      tracker[0] = 0;
    } else {
      tracker[0] = t;
    }
  }
  amp[1] = 0.f;  // ready for the next step's check
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
                     grad_scale, (const float*)nullptr);
  DMF_LAUNCH_CHECK("dmf_adamw_multi");
  return 0;
}

extern "C" int dmf_adamw_multi_amp(int nchunks, const long long* chunks, const long long* tensors, const float* hyper,
                                   int* steps, int nsteps, float grad_scale, const float* amp, void* stream) {
  DMF_CHECK_ARG(nchunks >= 0 && chunks && tensors && hyper && steps && amp && nsteps >= 0,
                "dmf_adamw_multi_amp: bad args");
  hipStream_t st = (hipStream_t)stream;
  if (nsteps > 0) hipLaunchKernelGGL(k_steps_inc, dim3(cdiv(nsteps, 256)), dim3(256), 0, st, steps, nsteps, amp);
  if (nchunks > 0)
    hipLaunchKernelGGL(k_adamw, dim3(nchunks), dim3(256), 0, st, chunks, tensors, hyper, steps, grad_scale, amp);
  DMF_LAUNCH_CHECK("dmf_adamw_multi_amp");
  return 0;
}

extern "C" int dmf_amp_nonfinite(int nchunks, const long long* chunks, const long long* tensors, float* amp,
                                 void* stream) {
  DMF_CHECK_ARG(nchunks >= 0 && chunks && tensors && amp, "dmf_amp_nonfinite: bad args");
  if (nchunks == 0) return 0;
  hipLaunchKernelGGL(k_amp_nonfinite, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, chunks, tensors, amp);
  DMF_LAUNCH_CHECK("dmf_amp_nonfinite");
  return 0;
}

extern "C" int dmf_amp_update(float* amp, int* tracker, float growth, float backoff, int interval, void* stream) {
  DMF_CHECK_ARG(amp && tracker && interval > 0, "dmf_amp_update: bad args");
  hipLaunchKernelGGL(k_amp_update, dim3(1), dim3(64), 0, (hipStream_t)stream, amp, tracker, growth, backoff, interval);
  DMF_LAUNCH_CHECK("dmf_amp_update");
  return 0;
}

extern "C" int dmf_steps_inc(int* steps, int n, void* stream) {
  DMF_CHECK_ARG(steps && n >= 0, "dmf_steps_inc: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_steps_inc, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, steps, n,
                     (const float*)nullptr);
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
