// Token-stream kernels of the hybrid TransformerStage (configuration 5,
// transformer_model.py:7-175) around the bf16 GEMMs of gemm.hip:
//   * LayerNorm forward with a bf16 output (the next GEMM's A operand) and
//     the saved (mean, rstd) -- PatchEmbed.norm :29, TransformerBlock.norm1/2 :71-73;
//   * LayerNorm backward fused with the residual-stream gradient add and the
//     gamma/beta column reductions;
//   * the LayerScale/dropout branch backward of x + drop(y) * gamma (:79-80,
//     proj_drop :115, MLP drop :133): dy, dgamma and the linear's dbias in one pass;
//   * column sums (qkv bias grad) and the f32 -> bf16 weight cast.
// The branch backward also comes in f32 (the parity mode; the f32 column
// sums are dense.hip's dmf_colsum_f32).
// Token rows are R = B * N, channels E contiguous (E % 256 == 0, E <= 1024).
#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

constexpr int TK_JMAX = 4;        // float4 column groups per lane: E <= 64 * 4 * TK_JMAX
constexpr int TK_ROWS = 32;       // rows per block in the column-reducing kernels (8 per wave)

// LayerNorm forward: one wave per row, x [R][E] (f32 or bf16) -> y [R][ldy] (f32 or bf16)
__device__ __forceinline__ float4 tk_ld4(const float* p) { return *(const float4*)p; }
__device__ __forceinline__ float4 tk_ld4(const bf16_t* p) {
  const uint2 u = *(const uint2*)p;
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ void tk_st4(float* p, float4 v) { *(float4*)p = v; }
__device__ __forceinline__ void tk_st4(bf16_t* p, float4 v) {
  uint2 u;
  u.x = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
  u.y = (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16);
  *(uint2*)p = u;
}

template <typename TX, typename TY>
__global__ void __launch_bounds__(256) k_ln_fwd(const TX* __restrict__ x, int ldx, long long R, int E,
                                                const float* __restrict__ g, const float* __restrict__ b, float eps,
                                                TY* __restrict__ y, int ldy, float* __restrict__ save) {
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  const int nj = E >> 8;
  const TX* px = x + r * ldx;
  float4 v[TK_JMAX];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < TK_JMAX; ++j)
    if (j < nj) {
      v[j] = tk_ld4(px + j * 256 + lane * 4);
      s += v[j].x + v[j].y + v[j].z + v[j].w;
    }
  const float mean = wave_sum(s) / E;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < TK_JMAX; ++j)
    if (j < nj) {
      const float a = v[j].x - mean, bb = v[j].y - mean, c = v[j].z - mean, d = v[j].w - mean;
      q += a * a + bb * bb + c * c + d * d;
    }
  const float rs = rsqrtf(wave_sum(q) / E + eps);
#pragma unroll
  for (int j = 0; j < TK_JMAX; ++j)
    if (j < nj) {
      const int c = j * 256 + lane * 4;
      const float4 gg = *(const float4*)(g + c), bb = *(const float4*)(b + c);
      tk_st4(y + r * ldy + c, make_float4((v[j].x - mean) * rs * gg.x + bb.x, (v[j].y - mean) * rs * gg.y + bb.y,
                                          (v[j].z - mean) * rs * gg.z + bb.z, (v[j].w - mean) * rs * gg.w + bb.w));
    }
  if (lane == 0 && save) { save[2 * r] = mean; save[2 * r + 1] = rs; }
}

// block-reduce per-lane column partials acc[j] (4 waves) into this block's slab row (the
// launcher then sums the slab rows in block order: deterministic, no atomics)
__device__ __forceinline__ void tk_col_flush(float* red, const float4 (&acc)[TK_JMAX], int nj, float* out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int E = nj * 256;
#pragma unroll
  for (int j = 0; j < TK_JMAX; ++j)
    if (j < nj) *(float4*)(red + wid * E + j * 256 + lane * 4) = acc[j];
  __syncthreads();
  for (int c = threadIdx.x; c < E; c += 256) {
    out[c] = (red[c] + red[E + c]) + (red[2 * E + c] + red[3 * E + c]);
  }
  __syncthreads();
}

// dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat)) (+ dres);
// dgamma += sum dy*xhat, dbeta += sum dy (column reductions: one slab row per block, slab0 / slab1)
template <typename TX>
__global__ void __launch_bounds__(256) k_ln_bwd(const float* __restrict__ dy, const TX* __restrict__ x, int ldx,
                                                const float* __restrict__ save, long long R, int E,
                                                const float* __restrict__ g, const float* dres, float* dx,
                                                float* __restrict__ slab0, float* __restrict__ slab1) {
  extern __shared__ float red[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nj = E >> 8;
  float4 ag[TK_JMAX], ab[TK_JMAX];
#pragma unroll
  for (int j = 0; j < TK_JMAX; ++j) ag[j] = ab[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  const long long r0 = (long long)blockIdx.x * TK_ROWS;
  for (int i = wid; i < TK_ROWS; i += 4) {
    const long long r = r0 + i;
    if (r >= R) break;
    const float mean = save[2 * r], rs = save[2 * r + 1];
    float4 xh[TK_JMAX], gd[TK_JMAX];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < TK_JMAX; ++j)
      if (j < nj) {
        const int c = j * 256 + lane * 4;
        const float4 xv = tk_ld4(x + r * ldx + c), dv = *(const float4*)(dy + r * E + c);
        const float4 gg = *(const float4*)(g + c);
        xh[j] = make_float4((xv.x - mean) * rs, (xv.y - mean) * rs, (xv.z - mean) * rs, (xv.w - mean) * rs);
        gd[j] = make_float4(dv.x * gg.x, dv.y * gg.y, dv.z * gg.z, dv.w * gg.w);
        s1 += gd[j].x + gd[j].y + gd[j].z + gd[j].w;
        s2 += gd[j].x * xh[j].x + gd[j].y * xh[j].y + gd[j].z * xh[j].z + gd[j].w * xh[j].w;
        ag[j].x += dv.x * xh[j].x; ag[j].y += dv.y * xh[j].y; ag[j].z += dv.z * xh[j].z; ag[j].w += dv.w * xh[j].w;
        ab[j].x += dv.x; ab[j].y += dv.y; ab[j].z += dv.z; ab[j].w += dv.w;
      }
    s1 = wave_sum(s1) / E;
    s2 = wave_sum(s2) / E;
#pragma unroll
    for (int j = 0; j < TK_JMAX; ++j)
      if (j < nj) {
        const int c = j * 256 + lane * 4;
        float4 o = make_float4(rs * (gd[j].x - s1 - xh[j].x * s2), rs * (gd[j].y - s1 - xh[j].y * s2),
                               rs * (gd[j].z - s1 - xh[j].z * s2), rs * (gd[j].w - s1 - xh[j].w * s2));
        if (dres) {
          const float4 d0 = *(const float4*)(dres + r * E + c);
          o.x += d0.x; o.y += d0.y; o.z += d0.z; o.w += d0.w;
        }
        *(float4*)(dx + r * E + c) = o;
      }
  }
  if (slab0) tk_col_flush(red, ag, nj, slab0 + (size_t)blockIdx.x * E);
  if (slab1) tk_col_flush(red, ab, nj, slab1 + (size_t)blockIdx.x * E);
}

// Branch backward of out = res + drop(y) * gamma, given gout = d out (f32):
//   dy = keep/(1-p) * gamma * gout (bf16, the linear's output grad),
//   dgamma += sum gout * drop(y), dbias += sum dy. Dropout element index r*E + c at `site`.
template <typename T>
__global__ void __launch_bounds__(256) k_lsdrop_bwd(const float* __restrict__ gout, const T* __restrict__ yaux,
                                                    long long R, int E, const float* __restrict__ gamma, float p,
                                                    const unsigned long long* rng, int site,
                                                    T* __restrict__ dy, float* __restrict__ slab0,
                                                    float* __restrict__ slab1) {
  const unsigned long long rseed_ = rng ? rng[0] : 0ull, roff_ = rng ? rng[1] : 0ull;  // read once (see dropout_keep4v)
  extern __shared__ float red[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nj = E >> 8;
  const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
  float4 ag[TK_JMAX], ab[TK_JMAX];
#pragma unroll
  for (int j = 0; j < TK_JMAX; ++j) ag[j] = ab[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  const long long r0 = (long long)blockIdx.x * TK_ROWS;
  for (int i = wid; i < TK_ROWS; i += 4) {
    const long long r = r0 + i;
    if (r >= R) break;
#pragma unroll
    for (int j = 0; j < TK_JMAX; ++j)
      if (j < nj) {
        const int c = j * 256 + lane * 4;
        const float4 go = *(const float4*)(gout + r * E + c);
        const float4 gg = *(const float4*)(gamma + c);
        const float4 y4 = tk_ld4(yaux + r * E + c);
        const float yv[4] = {y4.x, y4.y, y4.z, y4.w};
        float m[4] = {ks, ks, ks, ks};
        if (p > 0.f) {
          bool keep[4];
          dropout_keep4v(rseed_, roff_, site, (unsigned long long)(r * E + c), p, keep);
#pragma unroll
          for (int q = 0; q < 4; ++q) m[q] = keep[q] ? ks : 0.f;
        }
        const float d0 = m[0] * gg.x * go.x, d1 = m[1] * gg.y * go.y, d2 = m[2] * gg.z * go.z,
                    d3 = m[3] * gg.w * go.w;
        ag[j].x += go.x * m[0] * yv[0]; ag[j].y += go.y * m[1] * yv[1];
        ag[j].z += go.z * m[2] * yv[2]; ag[j].w += go.w * m[3] * yv[3];
        ab[j].x += d0; ab[j].y += d1; ab[j].z += d2; ab[j].w += d3;
        tk_st4(dy + r * E + c, make_float4(d0, d1, d2, d3));
      }
  }
  if (slab0) tk_col_flush(red, ag, nj, slab0 + (size_t)blockIdx.x * E);
  if (slab1) tk_col_flush(red, ab, nj, slab1 + (size_t)blockIdx.x * E);
}

// slab[r / 64][c] = sum over the 64-row band of X[r][c] (bf16 X, C % 8 == 0); block = 256 column
// chunks of 8 x 64 rows; the launcher sums the bands in order
__device__ __forceinline__ void tk_ld8(const bf16_t* p, float* v) { ld8(p, v); }
__device__ __forceinline__ void tk_ld8(const float* p, float* v) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <typename T>
__global__ void __launch_bounds__(256) k_tok_colsum(const T* __restrict__ X, int ldx, long long R, int C,
                                                float* __restrict__ out) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= C) return;
  const long long r0 = (long long)blockIdx.y * 64;
  const long long r1 = r0 + 64 < R ? r0 + 64 : R;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (long long r = r0; r < r1; ++r) {
    float v[8];
    tk_ld8(X + r * ldx + c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += v[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) out[(size_t)blockIdx.y * C + c + e] = s[e];
}

__global__ void __launch_bounds__(256) k_cast_bf16(const float* __restrict__ x, long long n, bf16_t* __restrict__ y) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i + 8 <= n) {
    float v[8];
    ld8(x + i, v);
    st8(y + i, v);
  } else {
    for (long long k = i; k < n; ++k) y[k] = f2bf(x[k]);
  }
}

__global__ void __launch_bounds__(256) k_cast_f32(const bf16_t* __restrict__ x, long long n, float* __restrict__ y) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i + 8 <= n) {
    float v[8];
    ld8(x + i, v);
    *(float4*)(y + i) = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(y + i + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    for (long long k = i; k < n; ++k) y[k] = bf2f(x[k]);
  }
}

}  // namespace dmf

using namespace dmf;

static bool tk_width_ok(int E) { return E > 0 && E % 256 == 0 && E <= 256 * TK_JMAX; }

extern "C" int dmf_tok_layernorm_fwd(int x_dtype, const void* x, int ldx, long long R, int E, const float* gamma,
                                     const float* beta, float eps, int y_dtype, void* y, int ldy, float* save,
                                     void* stream) {
  DMF_CHECK_ARG(x && gamma && beta && y && R >= 0, "dmf_tok_layernorm_fwd: bad args");
  DMF_CHECK_ARG(tk_width_ok(E) && ldy % 4 == 0 && ldx % 4 == 0,
                "dmf_tok_layernorm_fwd: E (%d) must be a multiple of 256, <= %d", E, 256 * TK_JMAX);
  DMF_CHECK_ARG((x_dtype == DMF_F32 || x_dtype == DMF_BF16) && (y_dtype == DMF_F32 || y_dtype == DMF_BF16),
                "dmf_tok_layernorm_fwd: bad dtypes");
  if (R == 0) return 0;
  const dim3 grid((unsigned)((R + 3) / 4)), blk(256);
  hipStream_t st = (hipStream_t)stream;
#define DMF_LN(TX, TY) \
  hipLaunchKernelGGL((k_ln_fwd<TX, TY>), grid, blk, 0, st, (const TX*)x, ldx, R, E, gamma, beta, eps, (TY*)y, ldy, save)
  if (x_dtype == DMF_F32 && y_dtype == DMF_F32) DMF_LN(float, float);
  else if (x_dtype == DMF_F32) DMF_LN(float, bf16_t);
  else if (y_dtype == DMF_F32) DMF_LN(bf16_t, float);
  else DMF_LN(bf16_t, bf16_t);
#undef DMF_LN
  DMF_LAUNCH_CHECK("dmf_tok_layernorm_fwd");
  return 0;
}

extern "C" long long dmf_tok_bwd_ws_floats(long long R, int E) {
  return 2 * ((R + TK_ROWS - 1) / TK_ROWS) * (long long)E;
}

// the two column-sum slabs -> out0 / out1 (accumulated), rows in block order
static int tk_slab_sums(const float* ws, long long nblk, int E, float* out0, float* out1, void* stream) {
  DMF_CHECK_ARG(nblk < (1LL << 31), "token backward: too many row blocks");
  if (out0 && dmf_colsum_f32(ws, E, (int)nblk, E, out0, 1, stream)) return -2;
  if (out1 && dmf_colsum_f32(ws + nblk * E, E, (int)nblk, E, out1, 1, stream)) return -2;
  return 0;
}

extern "C" int dmf_tok_layernorm_bwd(const float* dy, int x_dtype, const void* x, int ldx, const float* save,
                                     long long R, int E, const float* gamma, const float* dres, float* dx,
                                     float* dgamma, float* dbeta, float* ws, void* stream) {
  DMF_CHECK_ARG(dy && x && save && gamma && dx && R >= 0 && (ws || !(dgamma || dbeta)),
                "dmf_tok_layernorm_bwd: bad args");
  DMF_CHECK_ARG(tk_width_ok(E) && ldx % 4 == 0, "dmf_tok_layernorm_bwd: E (%d) must be a multiple of 256, <= %d", E,
                256 * TK_JMAX);
  DMF_CHECK_ARG(x_dtype == DMF_F32 || x_dtype == DMF_BF16, "dmf_tok_layernorm_bwd: bad dtype");
  if (R == 0) return 0;
  const long long nblk = (R + TK_ROWS - 1) / TK_ROWS;
  const dim3 grid((unsigned)nblk), blk(256);
  float* s0 = dgamma ? ws : nullptr;
  float* s1 = dbeta ? ws + nblk * E : nullptr;
  if (x_dtype == DMF_F32)
    hipLaunchKernelGGL(k_ln_bwd<float>, grid, blk, 4 * E * sizeof(float), (hipStream_t)stream, dy, (const float*)x,
                       ldx, save, R, E, gamma, dres, dx, s0, s1);
  else
    hipLaunchKernelGGL(k_ln_bwd<bf16_t>, grid, blk, 4 * E * sizeof(float), (hipStream_t)stream, dy,
                       (const bf16_t*)x, ldx, save, R, E, gamma, dres, dx, s0, s1);
  DMF_LAUNCH_CHECK("dmf_tok_layernorm_bwd");
  return tk_slab_sums(ws, nblk, E, dgamma, dbeta, stream);
}

template <typename T>
static int lsdrop_launch(const char* name, const float* gout, const void* yaux, long long R, int E,
                         const float* gamma, float dropout_p, const unsigned long long* rng, int site, void* dy,
                         float* dgamma, float* dbias, float* ws, void* stream) {
  DMF_CHECK_ARG(gout && yaux && gamma && dy && R >= 0 && (ws || !(dgamma || dbias)), "%s: bad args", name);
  DMF_CHECK_ARG(tk_width_ok(E), "%s: E (%d) must be a multiple of 256, <= %d", name, E, 256 * TK_JMAX);
  DMF_CHECK_ARG(dropout_p <= 0.f || (rng && dropout_p < 1.f), "%s: dropout needs rng, p < 1", name);
  if (R == 0) return 0;
  const long long nblk = (R + TK_ROWS - 1) / TK_ROWS;
  hipLaunchKernelGGL(k_lsdrop_bwd<T>, dim3((unsigned)nblk), dim3(256),
                     4 * E * sizeof(float), (hipStream_t)stream, gout, (const T*)yaux, R, E, gamma, dropout_p, rng,
                     site, (T*)dy, dgamma ? ws : nullptr, dbias ? ws + nblk * E : nullptr);
  DMF_LAUNCH_CHECK(name);
  return tk_slab_sums(ws, nblk, E, dgamma, dbias, stream);
}

extern "C" int dmf_tok_scale_dropout_bwd(const float* gout, const void* yaux, long long R, int E, const float* gamma,
                                         float dropout_p, const unsigned long long* rng, int site, void* dy,
                                         float* dgamma, float* dbias, float* ws, void* stream) {
  return lsdrop_launch<bf16_t>("dmf_tok_scale_dropout_bwd", gout, yaux, R, E, gamma, dropout_p, rng, site, dy, dgamma,
                               dbias, ws, stream);
}

extern "C" int dmf_tok_scale_dropout_bwd_f32(const float* gout, const float* yaux, long long R, int E,
                                             const float* gamma, float dropout_p, const unsigned long long* rng,
                                             int site, float* dy, float* dgamma, float* dbias, float* ws,
                                             void* stream) {
  return lsdrop_launch<float>("dmf_tok_scale_dropout_bwd_f32", gout, yaux, R, E, gamma, dropout_p, rng, site, dy,
                              dgamma, dbias, ws, stream);
}

template <typename T>
static int colsum_launch(const char* name, const void* X, int ldx, long long R, int C, float* out, float* ws,
                         void* stream) {
  DMF_CHECK_ARG(X && out && ws && R >= 0 && C % 8 == 0 && ldx % 8 == 0 && ((uintptr_t)X % 16) == 0,
                "%s: bad args (C=%d ldx=%d)", name, C, ldx);
  if (R == 0 || C == 0) return 0;
  DMF_CHECK_ARG((R + 63) / 64 < 65536, "%s: too many rows", name);
  const int bands = (int)((R + 63) / 64);
  hipLaunchKernelGGL(k_tok_colsum<T>, dim3((unsigned)cdiv(C / 8, 256), (unsigned)bands), dim3(256), 0,
                     (hipStream_t)stream, (const T*)X, ldx, R, C, ws);
  DMF_LAUNCH_CHECK(name);
  return dmf_colsum_f32(ws, C, bands, C, out, 1, stream);  // the 64-row bands in order
}

extern "C" long long dmf_colsum_bf16_ws_floats(long long R, int C) { return ((R + 63) / 64) * (long long)C; }

extern "C" int dmf_colsum_bf16(const void* X, int ldx, long long R, int C, float* out, float* ws, void* stream) {
  return colsum_launch<bf16_t>("dmf_colsum_bf16", X, ldx, R, C, out, ws, stream);
}

extern "C" int dmf_cast_bf16(const float* x, long long n, void* y, void* stream) {
  DMF_CHECK_ARG(x && y && n >= 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0,
                "dmf_cast_bf16: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_cast_bf16, dim3((unsigned)((n + 2047) / 2048)), dim3(256), 0, (hipStream_t)stream, x, n,
                     (bf16_t*)y);
  DMF_LAUNCH_CHECK("dmf_cast_bf16");
  return 0;
}

extern "C" int dmf_cast_f32(const void* x, long long n, float* y, void* stream) {
  DMF_CHECK_ARG(x && y && n >= 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0, "dmf_cast_f32: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_cast_f32, dim3((unsigned)((n + 2047) / 2048)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)x, n, y);
  DMF_LAUNCH_CHECK("dmf_cast_f32");
  return 0;
}

// keep[i] = 1 if element i of dropout site `site` survives (the mask every
// fused dropout of the library draws: dropout_keep4 on (seed, offset, i/4, site));
// test/inspection helper, n % 4 == 0.
__global__ void k_dropout_keep_mask(const unsigned long long* rng, int site, long long n, float p,
                                    unsigned char* __restrict__ keep) {
  const unsigned long long rseed_ = rng ? rng[0] : 0ull, roff_ = rng ? rng[1] : 0ull;  // read once (see dropout_keep4v)
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= n) return;
  bool k[4];
  dropout_keep4v(rseed_, roff_, site, (unsigned long long)i, p, k);
  *(uchar4*)(keep + i) = make_uchar4(k[0], k[1], k[2], k[3]);
}

extern "C" int dmf_dropout_keep_mask(const unsigned long long* rng, int site, long long n, float p,
                                     unsigned char* keep, void* stream) {
  DMF_CHECK_ARG(rng && keep && n >= 0 && n % 4 == 0 && p >= 0.f && p < 1.f, "dmf_dropout_keep_mask: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_dropout_keep_mask, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     rng, site, n, p, keep);
  DMF_LAUNCH_CHECK("dmf_dropout_keep_mask");
  return 0;
}
