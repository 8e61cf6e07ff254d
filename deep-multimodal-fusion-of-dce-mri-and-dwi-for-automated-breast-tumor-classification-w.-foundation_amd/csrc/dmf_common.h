// Shared device/host helpers for the gfx950 kernels behind include/dmf_hip.h.
// Error model: every C-ABI entry point returns 0 on success or a negative
// code; the message is kept in a thread-local buffer read by
// dmf_last_error() (the Python boundary turns it into RuntimeError, never an
// abort -- SURVEY.md 8(b) "Errors").
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include "../../include/dmf_hip.h"

namespace dmf {

// ---------------------------------------------------------------- errors
void set_error(const char* fmt, ...);

#define DMF_CHECK_ARG(cond, ...)                                   \
  do {                                                             \
    if (!(cond)) {                                                 \
      ::dmf::set_error(__VA_ARGS__);                               \
      return -1;                                                   \
    }                                                              \
  } while (0)

#define DMF_LAUNCH_CHECK(what)                                     \
  do {                                                             \
    hipError_t e_ = hipGetLastError();                             \
    if (e_ != hipSuccess) {                                        \
      ::dmf::set_error("%s: launch failed: %s", what,              \
                       hipGetErrorString(e_));                     \
      return -2;                                                   \
    }                                                              \
  } while (0)

// ------------------------------------------------------------ numerics
typedef uint16_t bf16_t;  // raw storage of a bfloat16

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even, NaN preserving (hipcc lowers to v_cvt_pk_bf16_f32)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&h);
}

typedef _Float16 f16_t;   // IEEE binary16 storage (the "16-mixed" compute dtype)

// 16-bit storage dtypes (8 elements per 16-B chunk, 16-bit MFMA operands)
__host__ __device__ inline bool is16(int dt) { return dt == DMF_BF16 || dt == DMF_F16; }
// run the statements with T bound to the storage type of dtype (bf16 / f16 / f32)
#define DMF_DISPATCH_DTYPE(dtype, T, ...)          \
  do {                                             \
    switch (dtype) {                               \
      case DMF_BF16: {                             \
        typedef ::dmf::bf16_t T;                   \
        __VA_ARGS__;                               \
      } break;                                     \
      case DMF_F16: {                              \
        typedef ::dmf::f16_t T;                    \
        __VA_ARGS__;                               \
      } break;                                     \
      default: {                                   \
        typedef float T;                           \
        __VA_ARGS__;                               \
      } break;                                     \
    }                                              \
  } while (0)

__device__ __forceinline__ float h2f(uint32_t bits16) { return (float)__builtin_bit_cast(_Float16, (uint16_t)bits16); }
// round-to-nearest-even (v_cvt_f16_f32); overflow to +-inf as torch's fp16 autocast
__device__ __forceinline__ uint32_t f2h(float f) { return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)f); }

template <typename T> struct Cvt;
template <> struct Cvt<float> {
  __device__ __forceinline__ static float load(float v) { return v; }
  __device__ __forceinline__ static float store(float v) { return v; }
};
template <> struct Cvt<bf16_t> {
  __device__ __forceinline__ static float load(bf16_t v) { return bf2f(v); }
  __device__ __forceinline__ static bf16_t store(float v) { return f2bf(v); }
};
template <> struct Cvt<f16_t> {
  __device__ __forceinline__ static float load(f16_t v) { return (float)v; }
  __device__ __forceinline__ static f16_t store(float v) { return (f16_t)v; }
};
template <typename T> __device__ __forceinline__ float ld(const T* p) { return Cvt<T>::load(*p); }
// is T a 16-bit storage type (bf16 / f16: 8 elements per 16-B chunk, 16-bit MFMA operands)
template <typename T> struct Is16 { static constexpr bool value = sizeof(T) == 2; };

// one 16x16x32 MFMA on 16-B fragments of 16-bit elements of storage type T (bf16 or f16: the two run
// at the same rate on gfx950), fp32 accumulation
typedef __attribute__((ext_vector_type(8))) short dmf_s16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 dmf_h16x8;
typedef __attribute__((ext_vector_type(4))) float dmf_f32x4;
template <typename T>
__device__ __forceinline__ dmf_f32x4 mfma16(const uint4& a, const uint4& b, dmf_f32x4 c) {
  if constexpr (__is_same(T, f16_t))
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(dmf_h16x8, a), __builtin_bit_cast(dmf_h16x8, b), c,
                                                  0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(dmf_s16x8, a), __builtin_bit_cast(dmf_s16x8, b),
                                                   c, 0, 0, 0);
}

// the two 16-bit elements of a 32-bit word (low element first) <-> floats, per storage type
template <typename T> struct B16;
template <> struct B16<bf16_t> {
  __device__ __forceinline__ static float lo(uint32_t w) { return __uint_as_float(w << 16); }
  __device__ __forceinline__ static float hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
  __device__ __forceinline__ static uint32_t pack(float l, float h) { return (uint32_t)f2bf(l) | ((uint32_t)f2bf(h) << 16); }
};
template <> struct B16<f16_t> {
  __device__ __forceinline__ static float lo(uint32_t w) { return h2f(w & 0xffffu); }
  __device__ __forceinline__ static float hi(uint32_t w) { return h2f(w >> 16); }
  __device__ __forceinline__ static uint32_t pack(float l, float h) { return f2h(l) | (f2h(h) << 16); }
};
template <typename T> __device__ __forceinline__ void st(T* p, float v) { *p = Cvt<T>::store(v); }

// 8-element vector access (16 B for bf16, 32 B for f32); p must be aligned
__device__ __forceinline__ void ld8(const bf16_t* p, float v[8]) {
  const uint4 u = *(const uint4*)p;
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void ld8(const f16_t* p, float v[8]) {
  const uint4 u = *(const uint4*)p;
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = h2f(w[i] & 0xffffu);
    v[2 * i + 1] = h2f(w[i] >> 16);
  }
}
__device__ __forceinline__ void ld8(const float* p, float v[8]) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8(bf16_t* p, const float v[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
  *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ void st8(f16_t* p, const float v[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = f2h(v[2 * i]) | (f2h(v[2 * i + 1]) << 16);
  *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ void st8(float* p, const float v[8]) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// raw 8-element vectors, so a kernel can put several rows' loads in flight before it converts any
template <typename T> struct Vec8 { uint4 u; };
template <> struct Vec8<float> { float4 a, b; };
template <typename T> __device__ __forceinline__ Vec8<T> ldv8(const T* p) { return Vec8<T>{*(const uint4*)p}; }
template <> __device__ __forceinline__ Vec8<float> ldv8(const float* p) {
  return Vec8<float>{*(const float4*)p, *(const float4*)(p + 4)};
}
template <typename T> __device__ __forceinline__ Vec8<T> zero8() { return Vec8<T>{make_uint4(0, 0, 0, 0)}; }
template <> __device__ __forceinline__ Vec8<float> zero8<float>() {
  return Vec8<float>{make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
}
template <typename T> __device__ __forceinline__ void unpack8(const Vec8<T>& r, float v[8]) {
  const uint32_t w[4] = {r.u.x, r.u.y, r.u.z, r.u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = B16<T>::lo(w[i]);
    v[2 * i + 1] = B16<T>::hi(w[i]);
  }
}
template <> __device__ __forceinline__ void unpack8(const Vec8<float>& r, float v[8]) {
  v[0] = r.a.x; v[1] = r.a.y; v[2] = r.a.z; v[3] = r.a.w;
  v[4] = r.b.x; v[5] = r.b.y; v[6] = r.b.z; v[7] = r.b.w;
}

// erf for the GELUs: Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7 absolute), odd extension -- one
// v_rcp_f32, one v_exp_f32 and five FMAs. ocml's erff made a GELU BN apply VALU-bound (tools/apply_bench.py,
// C = 256, M = 32768: 13.5 us against 7.7 for the ReLU apply and 4.7 for a copy of the same bytes).
// NaN propagates. (Round 4 reverted it while the training step was not bitwise reproducible and run-to-run
// noise was mistaken for its effect; with fixed-order reductions it changes results by the 1.5e-7 only.)
__device__ __forceinline__ float erf_gelu(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  const float p = fmaf(fmaf(fmaf(fmaf(1.061405429f, t, -1.453152027f), t, 1.421413741f), t, -0.284496736f), t,
                       0.254829592f) * t;
  return copysignf(1.0f - p * __expf(-ax * ax), x);
}
// exact (erf) GELU, as torch nn.GELU() default (erf to 1.5e-7)
__device__ __forceinline__ float gelu_f(float x) {
  return 0.5f * x * (1.0f + erf_gelu(x * 0.70710678118654752440f));
}
// the same on two values with the packed fp32 VALU (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth per
// instruction; the reciprocal and exponential stay scalar): ~12 instead of ~20 VALU instructions per value
typedef float dmf_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ dmf_f2 gelu_f2(dmf_f2 x) {
  const dmf_f2 z = x * 0.70710678118654752440f;
  const dmf_f2 az = __builtin_elementwise_abs(z);
  const dmf_f2 d = __builtin_elementwise_fma(az, (dmf_f2)0.3275911f, (dmf_f2)1.0f);
  const dmf_f2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  dmf_f2 p = __builtin_elementwise_fma((dmf_f2)1.061405429f, t, (dmf_f2)-1.453152027f);
  p = __builtin_elementwise_fma(p, t, (dmf_f2)1.421413741f);
  p = __builtin_elementwise_fma(p, t, (dmf_f2)-0.284496736f);
  p = __builtin_elementwise_fma(p, t, (dmf_f2)0.254829592f) * t;
  const dmf_f2 q = -az * az;
  const dmf_f2 e = {__expf(q.x), __expf(q.y)};
  const dmf_f2 r = (dmf_f2)1.0f - p * e;
  const dmf_f2 erf = {copysignf(r.x, z.x), copysignf(r.y, z.y)};
  return 0.5f * x * ((dmf_f2)1.0f + erf);
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float cdf = 0.5f * (1.0f + erf_gelu(x * 0.70710678118654752440f));
  const float pdf = 0.39894228040143267794f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + __expf(-x)); }

// --------------------------------------------------------- reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// block-wide sum for blockDim.x multiple of 64 (<=1024); red needs 16 floats
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += red[i];
  return r;
}


// ------------------------------------------------------ batch-norm finalize
// One channel: batch statistics (sum s, sum of squares q over `count` rows,
// double) -> (scale, shift) of y = x*scale + shift; running-stat update with
// momentum and the unbiased variance (n = unbias_count if > 0 else count);
// eval mode reads the running stats. Shared by dmf_bn_finalize and the conv
// epilogue's last-arriving-block finalizer.
struct BnFin {
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  long long* nbt;
  float momentum, eps;
  double count, unbias_count;
  int training;
  float* ss;    // [2][C]
  float* save;  // [2][C] mean, invstd (nullable)
};

__device__ __forceinline__ void bn_fin_channel(const BnFin& f, int c, int C, double s, double q) {
  float mean, var;
  if (f.training) {
    const double m = s / f.count;
    double v = q / f.count - m * m;
    if (v < 0.0) v = 0.0;
    mean = (float)m;
    var = (float)v;
    if (f.running_mean) {
      f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * mean;
      const double n_ = f.unbias_count > 0.0 ? f.unbias_count : f.count;
      const double unb = n_ > 1.0 ? v * n_ / (n_ - 1.0) : v;
      f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * (float)unb;
    }
  } else {
    mean = f.running_mean[c];
    var = f.running_var[c];
  }
  const float inv = rsqrtf(var + f.eps);
  const float g = f.gamma ? f.gamma[c] : 1.f, b = f.beta ? f.beta[c] : 0.f;
  f.ss[c] = g * inv;
  f.ss[C + c] = b - mean * g * inv;
  if (f.save) {
    f.save[c] = mean;
    f.save[C + c] = inv;
  }
}

// ----------------------------------------------------- counter-based RNG
// Philox-4x32-10; (seed, offset) live in device memory so captured graphs
// draw fresh dropout masks on every replay.
__device__ __forceinline__ void philox(uint32_t key0, uint32_t key1, uint32_t c0, uint32_t c1,
                                       uint32_t c2, uint32_t c3, uint32_t out[4]) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one v_mad_u64_u32 per product instead of v_mul_hi_u32 + v_mul_lo_u32 (both quarter rate)
    const uint64_t p0 = (uint64_t)M0 * c0, p1 = (uint64_t)M1 * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ key0, n2 = hi0 ^ c3 ^ key1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    key0 += W0; key1 += W1;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// Bernoulli(1-p) keep flags of elements e..e+3 (e % 4 == 0) of dropout site
// `site`: Philox on (seed, offset) read from device memory (graph replays
// draw fresh masks), counter = (e/4, site, offset).
// the same with (seed, offset) already in registers: a kernel whose loop holds inline-asm barriers with
// "memory" clobbers would otherwise reload rng[0], rng[1] (a scalar-load round trip) before every call
__device__ __forceinline__ void dropout_keep4v(unsigned long long seed, unsigned long long off, int site,
                                               unsigned long long e, float p, bool keep[4]) {
  uint32_t r[4];
  philox((uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)(e >> 2), (uint32_t)(e >> 34), (uint32_t)site,
         (uint32_t)off, r);
  const uint32_t thr = (uint32_t)fminf(p * 4294967296.0f, 4294967295.0f);
#pragma unroll
  for (int i = 0; i < 4; ++i) keep[i] = r[i] >= thr;
}
__device__ __forceinline__ void dropout_keep4(const unsigned long long* rng, int site, unsigned long long e,
                                              float p, bool keep[4]) {
  const unsigned long long seed = rng[0], off = rng[1];
  uint32_t r[4];
  philox((uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)(e >> 2), (uint32_t)(e >> 34), (uint32_t)site,
         (uint32_t)off, r);
  const uint32_t thr = (uint32_t)fminf(p * 4294967296.0f, 4294967295.0f);
#pragma unroll
  for (int i = 0; i < 4; ++i) keep[i] = r[i] >= thr;
}

__host__ __device__ inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// bijective XCD-aware remap of a linear block id (T1): blocks b and b+8 share
// an XCD; give each XCD a contiguous range of logical tiles.
__device__ __forceinline__ int xcd_remap(int b, int nblk) {
  const int q = nblk / 8, r = nblk % 8, xcd = b % 8, loc = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// ------------------------------------------------ raw buffer loads / LDS-DMA
// Out-of-range lanes (tile edges, zero padding) get an offset past the buffer
// and read zeros from the range check: no branches, no 64-bit address math.
constexpr unsigned BUF_OOB = 0x80000000u;
constexpr int BUF_FLAGS = 0x00020000;
typedef int v4i_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4i_t buf_rsrc(const void* p, long long bytes) {
  const unsigned long long u = (unsigned long long)p;
  return v4i_t{(int)(unsigned)u, (int)(unsigned)(u >> 32), (int)bytes, BUF_FLAGS};
}
// One LDS-DMA wave-instruction: 64 lanes x 16 B from rsrc+voff(+soff) to LDS
// [lds, lds + 1 KiB). Inline asm so the compiler neither tracks it (it would
// drain vmcnt(0) before every ds_read it cannot disambiguate) nor reorders it
// across LDS accesses; m0 is saved and restored. lds and soff are wave-uniform by contract; the
// readfirstlane keeps them in SGPRs where the compiler cannot prove it (a no-op on SGPR values).
__device__ __forceinline__ void dma16(v4i_t rsrc, unsigned voff, unsigned soff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds)),
                 "s"(__builtin_amdgcn_readfirstlane(soff))
               : "memory");
}


}  // namespace dmf
