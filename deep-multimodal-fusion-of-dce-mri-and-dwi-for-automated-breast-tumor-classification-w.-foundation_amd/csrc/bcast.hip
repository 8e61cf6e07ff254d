// Per-(n,c) broadcast helpers used by the backward of the squeeze/excite and
// global-average-pool paths (SEBlock model_module.py:41-43, ClassificationHead
// :364-369, FusionModel classifier/pvec :944-949, :986):
//   y = x * gate[n][c] + add[n][c] * add_scale          (dmf_channel_affine)
//   y (+)= vec[n][c] * scale   for every pixel          (dmf_broadcast_hw)
//   g[n][c] = sum_hw dy_nhwc[n,hw,c] * x_nchw[n,c,hw]  (dmf_gate_grad_nchw,
//            modality-attention gate gradient against the raw fp32 input)
#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

static inline int gsz(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

template <typename T>
__global__ void k_channel_affine(const T* __restrict__ x, int ldx, const float* __restrict__ gate,
                                 const float* __restrict__ add, float add_scale, T* __restrict__ y, int ldy,
                                 long long N, int HW, int C) {
  const long long total = N * HW * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / C;
    const int c = (int)(i - row * C);
    const long long n = row / HW;
    float v = x ? ld(x + row * ldx + c) * (gate ? gate[n * C + c] : 1.f) : 0.f;
    if (add) v += add[n * C + c] * add_scale;
    st(y + row * ldy + c, v);
  }
}

template <typename T>
__global__ void k_broadcast_hw(const float* __restrict__ vec, float scale, T* __restrict__ y, int ldy, long long N,
                               int HW, int C, int accumulate) {
  const long long total = N * HW * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / C;
    const int c = (int)(i - row * C);
    const long long n = row / HW;
    float v = vec[n * C + c] * scale;
    if (accumulate) v += ld(y + row * ldy + c);
    st(y + row * ldy + c, v);
  }
}

// 8-channel vector form, 32-bit index math (the scalar form's 64-bit divisions
// per element: ~12 us on a 32 x 32 x 32 x 128 map)
template <typename T>
__global__ void __launch_bounds__(256) k_broadcast_hw8(const float* __restrict__ vec, float scale, T* __restrict__ y,
                                                       int ldy, int N, int HW, int C, int accumulate) {
  const int CV = C >> 3;
  const int total = N * HW * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV, row = i / CV, n = row / HW;
    const float* src = vec + (size_t)n * C + cv * 8;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = src[k] * scale;
    T* p = y + (size_t)row * ldy + cv * 8;
    if (accumulate) {
      float o[8];
      ld8(p, o);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += o[k];
    }
    st8(p, v);
  }
}

// block per (n, c)
template <typename T>
__global__ void k_gate_grad_nchw(const T* __restrict__ dy, int lddy, const float* __restrict__ x, int C, int HW,
                                 float* __restrict__ out) {
  __shared__ float red[16];
  const int n = blockIdx.x / C, c = blockIdx.x % C;
  const float* px = x + ((size_t)n * C + c) * HW;
  const T* pd = dy + (size_t)n * HW * lddy + c;
  float s = 0.f;
  for (int p = threadIdx.x; p < HW; p += blockDim.x) s += px[p] * ld(pd + (size_t)p * lddy);
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[n * C + c] = s;
}

}  // namespace dmf

using namespace dmf;

extern "C" int dmf_channel_affine(int dtype, const void* x, int ldx, const float* gate, const float* add,
                                  float add_scale, void* y, int ldy, int N, int HW, int C, void* stream) {
  DMF_CHECK_ARG(y && (x || add), "dmf_channel_affine: bad args");
  const long long total = (long long)N * HW * C;
  if (total == 0) return 0;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_channel_affine<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream,
                       (const T*)x, ldx, gate, add, add_scale, (T*)y, ldy, (long long)N, HW, C));
  DMF_LAUNCH_CHECK("dmf_channel_affine");
  return 0;
}

extern "C" int dmf_broadcast_hw(int dtype, const float* vec, float scale, void* y, int ldy, int N, int HW, int C,
                                int accumulate, void* stream) {
  DMF_CHECK_ARG(vec && y, "dmf_broadcast_hw: bad args");
  const long long total = (long long)N * HW * C;
  if (total == 0) return 0;
  if (C % 8 == 0 && ldy % 8 == 0 && ((uintptr_t)y % 16) == 0 && (long long)N * HW * ldy < (1LL << 31)) {
    const long long t8 = total / 8;
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_broadcast_hw8<T>, dim3(gsz(t8)), dim3(256), 0, (hipStream_t)stream, vec, scale,
                         (T*)y, ldy, N, HW, C, accumulate));
    DMF_LAUNCH_CHECK("dmf_broadcast_hw");
    return 0;
  }
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_broadcast_hw<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, vec, scale,
                       (T*)y, ldy, (long long)N, HW, C, accumulate));
  DMF_LAUNCH_CHECK("dmf_broadcast_hw");
  return 0;
}

extern "C" int dmf_gate_grad_nchw(int dtype, const void* dy, int lddy, const float* x, int N, int C, int HW,
                                  float* out, void* stream) {
  DMF_CHECK_ARG(dy && x && out && N > 0 && C > 0, "dmf_gate_grad_nchw: bad args");
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_gate_grad_nchw<T>, dim3(N * C), dim3(256), 0, (hipStream_t)stream, (const T*)dy,
                       lddy, x, C, HW, out));
  DMF_LAUNCH_CHECK("dmf_gate_grad_nchw");
  return 0;
}
