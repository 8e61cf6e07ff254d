// Token-level pieces of the DCE x DWI cross-modal fusion op
// (FusionModel.forward, model_module.py:919-1000) and the small dense layers
// around it, fp32 throughout (B x 16 tokens x 128 channels -- latency-bound):
//   - small GEMM with transposes + bias + activation (nn.Linear fwd/bwd,
//     SE excitation MLPs on pooled vectors, MHA in/out projections)
//   - LayerNorm fwd/bwd (CrossAttentionBlock.attn_ffn[0], :808)
//   - multi-head attention core for short sequences (nn.MultiheadAttention,
//     :806/:816; head-averaged weights as need_weights=True returns)
//   - adaptive average pooling of a map into Hp x Wp tokens (_to_tokens,
//     :903-917) and its transpose
//   - the gated combine fused = g0*p_dwi + g1*p_dce + bilinear_up(attn tokens)
//     (:952-973) with its backward
//   - GatingAttention (:745-780): softmax(Linear(cat(pvec_dwi, pvec_dce,
//     mean(mask_dwi), mean(mask_dce))))
#include <algorithm>

#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

static inline int gsz(long long n, int b = 256) {
  long long g = (n + b - 1) / b;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

__device__ __forceinline__ float actf(int act, float z) {
  switch (act) {
    case DMF_ACT_RELU: return fmaxf(z, 0.f);
    case DMF_ACT_GELU: return gelu_f(z);
    case DMF_ACT_SIGMOID: return sigmoid_f(z);
    default: return z;
  }
}

// C = alpha*op(A)op(B) + beta*C + bias ; then act.
// 64x64 tile, BK=16, 256 threads (4x4 outputs each). Global loads are
// coalesced along the operand's contiguous dimension and prefetched into
// registers one K-step ahead. Split-K: blockIdx.z owns K range
// [z*kchunk, (z+1)*kchunk); with gridDim.z > 1 each split stores its
// partial tile into ws[z][M][N] and k_sgemm_reduce sums the splits in a
// fixed order and applies alpha, bias and act (deterministic).
// BK = K rows staged per barrier (16; a 64-deep form measured neutral on the
// mode-A step, interleaved A/B 3108 vs 3100 vol/s, and was removed; so was a 4x4
// vector micro-tile with two 16-B LDS reads per k: 3114 vs 3108, round 4)
template <int BK>
__global__ void __launch_bounds__(256) k_sgemm(int tA, int tB, int M, int N, int K, int kchunk, float alpha,
                                               const float* __restrict__ A, int lda, const float* __restrict__ B,
                                               int ldb, float beta, float* __restrict__ C, int ldc,
                                               const float* __restrict__ bias, int act, float* __restrict__ ws) {
  constexpr int NR = BK * 64 / 256;  // staged elements per thread and operand
  __shared__ __attribute__((aligned(16))) float As[BK][68], Bs[BK][68];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
  const bool split = gridDim.z > 1;
  // load mapping: contiguous-K operands walk k fastest (16 lanes x 1 row)
  float ra[NR], rb[NR];
  auto gload = [&](int k0) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int i = threadIdx.x + 256 * r;
      int kk, mm;
      if (tA) { kk = i >> 6; mm = i & 63; } else { kk = i % BK; mm = i / BK; }
      const int m = m0 + mm, k = k0 + kk;
      ra[r] = (m < M && k < ke) ? (tA ? A[(size_t)k * lda + m] : A[(size_t)m * lda + k]) : 0.f;
      int kk2, nn;
      if (tB) { kk2 = i % BK; nn = i / BK; } else { kk2 = i >> 6; nn = i & 63; }
      const int n = n0 + nn, k2 = k0 + kk2;
      rb[r] = (n < N && k2 < ke) ? (tB ? B[(size_t)n * ldb + k2] : B[(size_t)k2 * ldb + n]) : 0.f;
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int i = threadIdx.x + 256 * r;
      if (tA) As[i >> 6][i & 63] = ra[r]; else As[i % BK][i / BK] = ra[r];
      if (tB) Bs[i % BK][i / BK] = rb[r]; else Bs[i >> 6][i & 63] = rb[r];
    }
  };
  float acc[4][4] = {};
  if (kb < ke) gload(kb);
  for (int k0 = kb; k0 < ke; k0 += BK) {
    __syncthreads();
    sstore();
    __syncthreads();
    if (k0 + BK < ke) gload(k0 + BK);
#pragma unroll
    for (int kk = 0; kk < BK; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + ty + 16 * i, n = n0 + tx + 16 * j;
      if (m < M && n < N) {
        if (split) {
          ws[((size_t)blockIdx.z * M + m) * N + n] = acc[i][j];
        } else {
          float v = alpha * acc[i][j];
          if (beta != 0.f) v += beta * C[(size_t)m * ldc + n];
          if (bias) v += bias[n];
          C[(size_t)m * ldc + n] = actf(act, v);
        }
      }
    }
}

// The small fusion GEMMs (M, N <= 512) as a grid of 16 x 16 output tiles on the exact fp32 MFMA
// (v_mfma_f32_16x16x4f32), one workgroup per tile, its K-steps split over 4 waves and the 4 partial tiles
// summed in LDS in a fixed order (deterministic, no split-K workspace or reduce launch). Lane group q
// takes k = 16 s + 4 q + e in MFMA e of step s for both operands (any op(A) / op(B) layout: element loads,
// up to SG_PF steps in flight). k_sgemm ran 12-16 us on these shapes whatever their size (a per-launch
// floor of its staged K loop, profiles/r04q_sgemm_shapes.txt).
constexpr int SG_PF = 4;
typedef __attribute__((ext_vector_type(4))) float sg_f32x4;
__global__ void __launch_bounds__(256) k_sgemm_mfma(int tA, int tB, int M, int N, int K, float alpha,
                                                    const float* __restrict__ A, int lda, const float* __restrict__ B,
                                                    int ldb, float beta, float* __restrict__ C, int ldc,
                                                    const float* __restrict__ bias, int act) {
  __shared__ __attribute__((aligned(16))) float red[4][256];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, fr = lane & 15, q = lane >> 4;
  const int tm = (M + 15) / 16;
  const int m0 = (blockIdx.x % tm) * 16, n0 = (blockIdx.x / tm) * 16;
  const int m = m0 + fr, n = n0 + fr;
  const int St = (K + 15) / 16, s0 = wv * St / 4, s1 = (wv + 1) * St / 4;
  sg_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = s0; c0 < s1; c0 += SG_PF) {
    float av[SG_PF][4], bv[SG_PF][4];
#pragma unroll
    for (int i = 0; i < SG_PF; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = (c0 + i) * 16 + 4 * q + e;
        const bool kin = c0 + i < s1 && k < K;
        av[i][e] = (kin && m < M) ? (tA ? A[(size_t)k * lda + m] : A[(size_t)m * lda + k]) : 0.f;
        bv[i][e] = (kin && n < N) ? (tB ? B[(size_t)n * ldb + k] : B[(size_t)k * ldb + n]) : 0.f;
      }
#pragma unroll
    for (int i = 0; i < SG_PF; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][e], bv[i][e], acc, 0, 0, 0);
  }
  *(float4*)(&red[wv][lane * 4]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  __syncthreads();
  // D[row 4q + r][col fr]: output row m0 + 4q + r, column n0 + fr
  const int ln = tid >> 2, r = tid & 3;
  const int mr = m0 + 4 * (ln >> 4) + r, nc = n0 + (ln & 15);
  if (mr < M && nc < N) {
    float v = alpha * (((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid]);
    if (beta != 0.f) v += beta * C[(size_t)mr * ldc + nc];
    if (bias) v += bias[nc];
    C[(size_t)mr * ldc + nc] = actf(act, v);
  }
}

__global__ void k_sgemm_reduce(int S, int M, int N, float alpha, const float* __restrict__ ws, float beta,
                               float* __restrict__ C, int ldc, const float* __restrict__ bias, int act) {
  const long long total = (long long)M * N;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(i / N), n = (int)(i % N);
    float v = 0.f;
    for (int z = 0; z < S; ++z) v += ws[(size_t)z * total + i];
    v *= alpha;
    if (beta != 0.f) v += beta * C[(size_t)m * ldc + n];
    if (bias) v += bias[n];
    C[(size_t)m * ldc + n] = actf(act, v);
  }
}

// column sums: out[n] (+)= sum_m X[m][n]
// block = 64 columns x 16 row lanes, 8 rows in flight per thread, the lanes
// combined in LDS in a fixed order (4 lanes with one load in flight took
// ~27 us over 512 rows: latency-bound)
__global__ void __launch_bounds__(1024) k_colsum(const float* __restrict__ X, int ldx, int M, int N,
                                                 float* __restrict__ out, int accumulate) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + cl;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    int m = rl;
    for (; m + 7 * 16 < M; m += 8 * 16) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += X[(size_t)(m + u * 16) * ldx + n];
    }
    for (; m < M; m += 16) a[0] += X[(size_t)m * ldx + n];
  }
  red[rl][cl] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (rl == 0 && n < N) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) v += red[i][cl];
    out[n] = accumulate ? out[n] + v : v;
  }
}

// elementwise activation backward on fp32: dx = dy * act'(z)  (z = pre-activation)
__global__ void k_act_grad_f32(const float* __restrict__ dy, const float* __restrict__ z, float* __restrict__ dx,
                               long long n, int act) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float v = z[i];
    float g;
    switch (act) {
      case DMF_ACT_RELU: g = v > 0.f ? 1.f : 0.f; break;
      case DMF_ACT_GELU: g = gelu_grad_f(v); break;
      case DMF_ACT_SIGMOID: { const float s = sigmoid_f(v); g = s * (1.f - s); break; }
      default: g = 1.f;
    }
    dx[i] = dy[i] * g;
  }
}

__global__ void k_act_f32(const float* __restrict__ x, float* __restrict__ y, long long n, int act) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] = actf(act, x[i]);
}

// dz = dg * s * (1 - s) given the sigmoid OUTPUT s
__global__ void k_sig_grad_f32(const float* __restrict__ dg, const float* __restrict__ s, float* __restrict__ dz,
                               long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    dz[i] = dg[i] * s[i] * (1.f - s[i]);
}

// F.normalize(x, dim=1) on rows (ClassificationHead, model_module.py:367-368):
// y = x / max(||x||, eps); backward dx = (dy - y (y.dy)) / ||x|| (or dy/eps)
__global__ void k_row_l2norm(const float* __restrict__ x, int R, int C, float eps, float* __restrict__ y,
                             float* __restrict__ norms) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= R) return;
  float s = 0.f;
  for (int i = lane; i < C; i += 64) s += x[(size_t)r * C + i] * x[(size_t)r * C + i];
  const float nrm = sqrtf(wave_sum(s));
  const float d = fmaxf(nrm, eps);
  for (int i = lane; i < C; i += 64) y[(size_t)r * C + i] = x[(size_t)r * C + i] / d;
  if (lane == 0 && norms) norms[r] = nrm;
}

__global__ void k_row_l2norm_bwd(const float* __restrict__ dy, const float* __restrict__ y,
                                 const float* __restrict__ norms, int R, int C, float eps, float* __restrict__ dx) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= R) return;
  const float nrm = norms[r];
  float dot = 0.f;
  for (int i = lane; i < C; i += 64) dot += y[(size_t)r * C + i] * dy[(size_t)r * C + i];
  dot = wave_sum(dot);
  const bool active = nrm > eps;
  const float d = fmaxf(nrm, eps);
  for (int i = lane; i < C; i += 64) {
    const float g = dy[(size_t)r * C + i];
    dx[(size_t)r * C + i] = active ? (g - y[(size_t)r * C + i] * dot) / d : g / d;
  }
}

// --------------------------------------------------------------- LayerNorm
__global__ void k_layernorm(const float* __restrict__ x, int R, int E, const float* __restrict__ g,
                            const float* __restrict__ b, float eps, float* __restrict__ y, float* __restrict__ save) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= R) return;
  const float* px = x + (size_t)r * E;
  float s = 0.f;
  for (int i = lane; i < E; i += 64) s += px[i];
  const float mean = wave_sum(s) / E;
  float q = 0.f;
  for (int i = lane; i < E; i += 64) { const float d = px[i] - mean; q += d * d; }
  const float rs = rsqrtf(wave_sum(q) / E + eps);
  for (int i = lane; i < E; i += 64) y[(size_t)r * E + i] = (px[i] - mean) * rs * g[i] + b[i];
  if (lane == 0 && save) { save[2 * r] = mean; save[2 * r + 1] = rs; }
}

// Blocks [0, nrb): one wave per row, dx. Blocks [nrb, ...): 64 columns each,
// dgamma / dbeta (+)= column sums over all rows in a fixed order (4 row lanes
// strided by 4, combined in LDS lane 0..3) -- deterministic, no atomics, one
// launch (nn.LayerNorm's backward reduces dgamma / dbeta in a fixed order,
// reference model_module.py:799-818).
__global__ void __launch_bounds__(256) k_layernorm_bwd(const float* __restrict__ dy, const float* __restrict__ x,
                                                       const float* __restrict__ save, int R, int E,
                                                       const float* __restrict__ g, float* __restrict__ dx, float* dg,
                                                       float* db, int nrb) {
  const int lane = threadIdx.x & 63;
  if ((int)blockIdx.x >= nrb) {
    __shared__ float red[2][4][64];
    const int c = ((int)blockIdx.x - nrb) * 64 + lane, rl = threadIdx.x >> 6;
    float ag[4] = {0.f, 0.f, 0.f, 0.f}, ab[4] = {0.f, 0.f, 0.f, 0.f};
    if (c < E) {
      int r = rl;
      for (; r + 12 < R; r += 16) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int rr = r + 4 * u;
          const float d = dy[(size_t)rr * E + c];
          ag[u] += d * ((x[(size_t)rr * E + c] - save[2 * rr]) * save[2 * rr + 1]);
          ab[u] += d;
        }
      }
      for (; r < R; r += 4) {
        const float d = dy[(size_t)r * E + c];
        ag[0] += d * ((x[(size_t)r * E + c] - save[2 * r]) * save[2 * r + 1]);
        ab[0] += d;
      }
    }
    red[0][rl][lane] = (ag[0] + ag[1]) + (ag[2] + ag[3]);
    red[1][rl][lane] = (ab[0] + ab[1]) + (ab[2] + ab[3]);
    __syncthreads();
    if (rl == 0 && c < E) {
      if (dg) dg[c] += ((red[0][0][lane] + red[0][1][lane]) + (red[0][2][lane] + red[0][3][lane]));
      if (db) db[c] += ((red[1][0][lane] + red[1][1][lane]) + (red[1][2][lane] + red[1][3][lane]));
    }
    return;
  }
  const int r = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= R) return;
  const float mean = save[2 * r], rs = save[2 * r + 1];
  const float* px = x + (size_t)r * E;
  const float* pd = dy + (size_t)r * E;
  float s1 = 0.f, s2 = 0.f;
  for (int i = lane; i < E; i += 64) {
    const float xh = (px[i] - mean) * rs;
    const float gd = pd[i] * g[i];
    s1 += gd;
    s2 += gd * xh;
  }
  s1 = wave_sum(s1) / E;
  s2 = wave_sum(s2) / E;
  for (int i = lane; i < E; i += 64) {
    const float xh = (px[i] - mean) * rs;
    dx[(size_t)r * E + i] = rs * (pd[i] * g[i] - s1 - xh * s2);
  }
}

// ------------------------------------------------------ attention (short)
// q,k,v: [B][N][ld] with head h at columns h*D..h*D+D-1. One block per (b,h);
// requires Nq,Nk <= 64, D <= 128.
__global__ void k_attn_fwd(const float* __restrict__ q, int ldq, const float* __restrict__ k, int ldk,
                           const float* __restrict__ v, int ldv, int Nq, int Nk, int H, int D, float scale,
                           float* __restrict__ o, int ldo, float* __restrict__ probs) {
  __shared__ float Ks[64][129], Vs[64][129], Ps[64][65];
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const float* qb = q + (size_t)b * Nq * ldq + h * D;
  const float* kb = k + (size_t)b * Nk * ldk + h * D;
  const float* vb = v + (size_t)b * Nk * ldv + h * D;
  for (int i = threadIdx.x; i < Nk * D; i += blockDim.x) {
    const int j = i / D, d = i % D;
    Ks[j][d] = kb[(size_t)j * ldk + d];
    Vs[j][d] = vb[(size_t)j * ldv + d];
  }
  __syncthreads();
  // scores: one thread per (i, j)
  for (int t = threadIdx.x; t < Nq * Nk; t += blockDim.x) {
    const int i = t / Nk, j = t % Nk;
    float s = 0.f;
    for (int d = 0; d < D; ++d) s += qb[(size_t)i * ldq + d] * Ks[j][d];
    Ps[i][j] = s * scale;
  }
  __syncthreads();
  // softmax per row (one thread per row; Nk <= 64)
  for (int i = threadIdx.x; i < Nq; i += blockDim.x) {
    float mx = -INFINITY;
    for (int j = 0; j < Nk; ++j) mx = fmaxf(mx, Ps[i][j]);
    float sum = 0.f;
    for (int j = 0; j < Nk; ++j) { const float e = __expf(Ps[i][j] - mx); Ps[i][j] = e; sum += e; }
    const float inv = 1.f / sum;
    for (int j = 0; j < Nk; ++j) Ps[i][j] *= inv;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < Nq * Nk; t += blockDim.x) {
    const int i = t / Nk, j = t % Nk;
    if (probs) probs[(((size_t)b * H + h) * Nq + i) * Nk + j] = Ps[i][j];
  }
  for (int t = threadIdx.x; t < Nq * D; t += blockDim.x) {
    const int i = t / D, d = t % D;
    float s = 0.f;
    for (int j = 0; j < Nk; ++j) s += Ps[i][j] * Vs[j][d];
    o[((size_t)b * Nq + i) * ldo + h * D + d] = s;
  }
}

// head-averaged attention weights (nn.MultiheadAttention average_attn_weights:
// the mean over heads of the probabilities), summed in head order
__global__ void k_head_mean(const float* __restrict__ probs, int B, int H, int NN, float* __restrict__ avgw) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * NN) return;
  const int b = t / NN, e = t - b * NN;
  float s = 0.f;
  for (int h = 0; h < H; ++h) s += probs[((size_t)b * H + h) * NN + e];
  avgw[t] = s / (float)H;
}

__global__ void k_attn_bwd(const float* __restrict__ q, int ldq, const float* __restrict__ k, int ldk,
                           const float* __restrict__ v, int ldv, const float* __restrict__ probs,
                           const float* __restrict__ dout, int lddo, int Nq, int Nk, int H, int D, float scale,
                           float* __restrict__ dq, int lddq, float* __restrict__ dk, int lddk, float* __restrict__ dv,
                           int lddv) {
  __shared__ float Ps[64][65], dS[64][65];
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const float* P = probs + ((size_t)b * H + h) * Nq * Nk;
  const float* qb = q + (size_t)b * Nq * ldq + h * D;
  const float* kb = k + (size_t)b * Nk * ldk + h * D;
  const float* vb = v + (size_t)b * Nk * ldv + h * D;
  const float* gb = dout + (size_t)b * Nq * lddo + h * D;
  for (int t = threadIdx.x; t < Nq * Nk; t += blockDim.x) Ps[t / Nk][t % Nk] = P[t];
  __syncthreads();
  // dP_ij = sum_d dO_id V_jd
  for (int t = threadIdx.x; t < Nq * Nk; t += blockDim.x) {
    const int i = t / Nk, j = t % Nk;
    float s = 0.f;
    for (int d = 0; d < D; ++d) s += gb[(size_t)i * lddo + d] * vb[(size_t)j * ldv + d];
    dS[i][j] = s;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < Nq; i += blockDim.x) {
    float r = 0.f;
    for (int j = 0; j < Nk; ++j) r += Ps[i][j] * dS[i][j];
    for (int j = 0; j < Nk; ++j) dS[i][j] = Ps[i][j] * (dS[i][j] - r);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < Nq * D; t += blockDim.x) {
    const int i = t / D, d = t % D;
    float s = 0.f;
    for (int j = 0; j < Nk; ++j) s += dS[i][j] * kb[(size_t)j * ldk + d];
    dq[((size_t)b * Nq + i) * lddq + h * D + d] = s * scale;
  }
  for (int t = threadIdx.x; t < Nk * D; t += blockDim.x) {
    const int j = t / D, d = t % D;
    float sk = 0.f, sv = 0.f;
    for (int i = 0; i < Nq; ++i) {
      sk += dS[i][j] * qb[(size_t)i * ldq + d];
      sv += Ps[i][j] * gb[(size_t)i * lddo + d];
    }
    dk[((size_t)b * Nk + j) * lddk + h * D + d] = sk * scale;
    dv[((size_t)b * Nk + j) * lddv + h * D + d] = sv;
  }
}

// --------------------------------------------------------------- tokens
// tokens[b][(i*Wp+j)][c] = mean over the (H/Hp)x(W/Wp) cell; exact division required
template <typename T>
__global__ void k_tokens_fwd(const T* __restrict__ x, int ldx, int B, int H, int W, int C, int Hp, int Wp,
                             float* __restrict__ tok) {
  const long long total = (long long)B * Hp * Wp * C;
  const int kh = H / Hp, kw = W / Wp;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    long long r = t / C;
    const int j = (int)(r % Wp); r /= Wp;
    const int i = (int)(r % Hp);
    const int b = (int)(r / Hp);
    float s = 0.f;
    for (int a = 0; a < kh; ++a)
      for (int e = 0; e < kw; ++e) s += ld(x + ((size_t)(b * H + i * kh + a) * W + j * kw + e) * ldx + c);
    tok[t] = s / (float)(kh * kw);
  }
}

template <typename T>
__global__ void k_tokens_bwd(const float* __restrict__ dtok, int B, int H, int W, int C, int Hp, int Wp,
                             T* __restrict__ dx, int lddx, int accumulate) {
  const long long total = (long long)B * H * W * C;
  const int kh = H / Hp, kw = W / Wp;
  const float inv = 1.f / (float)(kh * kw);
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    long long r = t / C;
    const int w = (int)(r % W); r /= W;
    const int h = (int)(r % H);
    const int b = (int)(r / H);
    float v = dtok[(((size_t)b * Hp + h / kh) * Wp + w / kw) * C + c] * inv;
    T* p = dx + ((size_t)(b * H + h) * W + w) * lddx + c;
    if (accumulate) v += ld(p);
    st(p, v);
  }
}

// 8-channel vector forms (C % 8 == 0, 64 % (C / 8) == 0): one wave per token,
// lanes = C/8 channel slices x PL = 64 / (C/8) pixel lanes over the cell, the
// pixel lanes combined by shuffles (the scalar form looped 64 pixels per
// channel per thread: ~18 us on a 32 x 32 x 32 x 128 map)
template <typename T>
__global__ void __launch_bounds__(256) k_tokens_fwd8(const T* __restrict__ x, int ldx, int B, int H, int W, int C,
                                                     int Hp, int Wp, float* __restrict__ tok) {
  const int CV = C >> 3, PL = 64 / CV;
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);  // token index b*Hp*Wp + i*Wp + j
  if (t >= B * Hp * Wp) return;
  const int j = t % Wp, i = (t / Wp) % Hp, b = t / (Wp * Hp);
  const int kh = H / Hp, kw = W / Wp;
  const int cv = lane % CV, pl = lane / CV;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int q = pl; q < kh * kw; q += PL) {
    const int a = q / kw, e = q - (q / kw) * kw;
    float v[8];
    ld8(x + ((size_t)(b * H + i * kh + a) * W + j * kw + e) * ldx + cv * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += v[k];
  }
  for (int o = CV; o < 64; o <<= 1)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += __shfl_xor(acc[k], o, 64);
  if (pl == 0) {
    const float inv = 1.f / (float)(kh * kw);
    float* o = tok + (size_t)t * C + cv * 8;
    *(float4*)o = make_float4(acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv);
    *(float4*)(o + 4) = make_float4(acc[4] * inv, acc[5] * inv, acc[6] * inv, acc[7] * inv);
  }
}

// thread = one pixel x 8 channels, 32-bit index math
template <typename T>
__global__ void __launch_bounds__(256) k_tokens_bwd8(const float* __restrict__ dtok, int B, int H, int W, int C, int Hp,
                                                     int Wp, T* __restrict__ dx, int lddx, int accumulate) {
  const int CV = C >> 3;
  const int total = B * H * W * CV;
  const int kh = H / Hp, kw = W / Wp;
  const float inv = 1.f / (float)(kh * kw);
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int cv = t % CV, pix = t / CV;
    const int w = pix % W, h = (pix / W) % H, b = pix / (W * H);
    const float* src = dtok + (((size_t)b * Hp + h / kh) * Wp + w / kw) * C + cv * 8;
    const float4 g0 = *(const float4*)src, g1 = *(const float4*)(src + 4);
    float v[8] = {g0.x * inv, g0.y * inv, g0.z * inv, g0.w * inv, g1.x * inv, g1.y * inv, g1.z * inv, g1.w * inv};
    T* p = dx + (size_t)pix * lddx + cv * 8;
    if (accumulate) {
      float o[8];
      ld8(p, o);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += o[k];
    }
    st8(p, v);
  }
}

// ----------------------------------------------------------- combine
__device__ __forceinline__ void lin_w(int o, int in, int out, int& i0, int& i1, float& l1) {
  const float scale = (float)in / (float)out;
  float src = (o + 0.5f) * scale - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
}

// y = g0*a + g1*b + bilinear(low) ; low: [B][Hp][Wp][C] fp32 (token layout), null -> no attention term
template <typename T>
__global__ void k_combine_fwd(const T* __restrict__ a, const T* __restrict__ bb, int ldm, const float* __restrict__ g,
                              const float* __restrict__ low, int B, int H, int W, int C, int Hp, int Wp,
                              T* __restrict__ y, int ldy) {
  const long long total = (long long)B * H * W * C;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const long long pix = t / C;
    const int n = (int)(pix / (H * W));
    const int rem = (int)(pix - (long long)n * H * W);
    const int h = rem / W, w = rem % W;
    float v = g[2 * n] * ld(a + pix * ldm + c) + g[2 * n + 1] * ld(bb + pix * ldm + c);
    if (low) {
      int h0, h1, w0, w1;
      float lh, lw;
      lin_w(h, Hp, H, h0, h1, lh);
      lin_w(w, Wp, W, w0, w1, lw);
      const float* L = low + (size_t)n * Hp * Wp * C + c;
      v += (1.f - lh) * ((1.f - lw) * L[(h0 * Wp + w0) * C] + lw * L[(h0 * Wp + w1) * C]) +
           lh * ((1.f - lw) * L[(h1 * Wp + w0) * C] + lw * L[(h1 * Wp + w1) * C]);
    }
    st(y + pix * ldy + c, v);
  }
}

// da = g0*dy, db = g1*dy (elementwise)
template <typename T>
__global__ void k_combine_bwd_maps(const T* __restrict__ dy, int lddy, const float* __restrict__ g, int HW, int C,
                                   long long total, T* __restrict__ da, T* __restrict__ db, int ldd) {
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const long long pix = t / C;
    const int n = (int)(pix / HW);
    const float d = ld(dy + pix * lddy + c);
    if (da) st(da + pix * ldd + c, g[2 * n] * d);
    if (db) st(db + pix * ldd + c, g[2 * n + 1] * d);
  }
}

// dg[n][0] = sum dy*a, dg[n][1] = sum dy*b ; block per sample
template <typename T>
__global__ void k_combine_bwd_gate(const T* __restrict__ dy, int lddy, const T* __restrict__ a,
                                   const T* __restrict__ b, int ldm, int HW, int C, float* __restrict__ dg) {
  __shared__ float red[16];
  const int n = blockIdx.x;
  float s0 = 0.f, s1 = 0.f;
  const long long base = (long long)n * HW;
  for (long long t = threadIdx.x; t < (long long)HW * C; t += blockDim.x) {
    const long long pix = base + t / C;
    const int c = (int)(t % C);
    const float d = ld(dy + pix * lddy + c);
    s0 += d * ld(a + pix * ldm + c);
    s1 += d * ld(b + pix * ldm + c);
  }
  s0 = block_sum(s0, red);
  s1 = block_sum(s1, red);
  if (threadIdx.x == 0) { dg[2 * n] = s0; dg[2 * n + 1] = s1; }
}

// dlow[n][i][j][c] = sum over output pixels of bilinear weight * dy
template <typename T>
__global__ void k_combine_bwd_low(const T* __restrict__ dy, int lddy, int B, int H, int W, int C, int Hp, int Wp,
                                  float* __restrict__ dlow) {
  const long long total = (long long)B * Hp * Wp * C;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    long long r = t / C;
    const int j = (int)(r % Wp); r /= Wp;
    const int i = (int)(r % Hp);
    const int n = (int)(r / Hp);
    float acc = 0.f;
    for (int h = 0; h < H; ++h) {
      int h0, h1;
      float lh;
      lin_w(h, Hp, H, h0, h1, lh);
      float wh = 0.f;
      if (h0 == i) wh += 1.f - lh;
      if (h1 == i) wh += lh;
      if (wh == 0.f) continue;
      for (int w = 0; w < W; ++w) {
        int w0, w1;
        float lw;
        lin_w(w, Wp, W, w0, w1, lw);
        float ww = 0.f;
        if (w0 == j) ww += 1.f - lw;
        if (w1 == j) ww += lw;
        if (ww == 0.f) continue;
        acc += wh * ww * ld(dy + ((size_t)(n * H + h) * W + w) * lddy + c);
      }
    }
    dlow[t] = acc;
  }
}

// 8-channel vector forms (C, strides multiples of 8, 16-B aligned)
// dg[n][0..1]: block of 1024 threads per sample, 16-B loads
template <typename T>
__global__ void __launch_bounds__(1024) k_combine_bwd_gate8(const T* __restrict__ dy, int lddy,
                                                            const T* __restrict__ a, const T* __restrict__ b, int ldm,
                                                            int HW, int C, float* __restrict__ dg) {
  __shared__ float red[16];
  const int n = blockIdx.x;
  const int CV = C >> 3;
  float s0 = 0.f, s1 = 0.f;
  const long long base = (long long)n * HW;
  for (long long t = threadIdx.x; t < (long long)HW * CV; t += blockDim.x) {
    const long long pix = base + t / CV;
    const int c = (int)(t % CV) * 8;
    float d[8], va[8], vb[8];
    ld8(dy + pix * lddy + c, d);
    ld8(a + pix * ldm + c, va);
    ld8(b + pix * ldm + c, vb);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s0 = fmaf(d[j], va[j], s0);
      s1 = fmaf(d[j], vb[j], s1);
    }
  }
  s0 = block_sum(s0, red);
  s1 = block_sum(s1, red);
  if (threadIdx.x == 0) {
    dg[2 * n] = s0;
    dg[2 * n + 1] = s1;
  }
}

// dlow[n][i][j][c..c+8]: loop only over the output rows/columns whose
// bilinear source interval touches (i, j)
template <typename T>
__global__ void k_combine_bwd_low8(const T* __restrict__ dy, int lddy, int B, int H, int W, int C, int Hp, int Wp,
                                   float* __restrict__ dlow) {
  const int CV = C >> 3;
  const long long total = (long long)B * Hp * Wp * CV;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int cv = (int)(t % CV);
    long long r = t / CV;
    const int j = (int)(r % Wp); r /= Wp;
    const int i = (int)(r % Hp);
    const int n = (int)(r / Hp);
    const int hl = max(0, (int)floorf(((float)i - 0.5f) * H / Hp - 0.5f) - 1);
    const int hh = min(H, (int)ceilf(((float)i + 1.5f) * H / Hp - 0.5f) + 2);
    const int wl = max(0, (int)floorf(((float)j - 0.5f) * W / Wp - 0.5f) - 1);
    const int wh = min(W, (int)ceilf(((float)j + 1.5f) * W / Wp - 0.5f) + 2);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int h = hl; h < hh; ++h) {
      int h0, h1;
      float lh;
      lin_w(h, Hp, H, h0, h1, lh);
      float wgh = 0.f;
      if (h0 == i) wgh += 1.f - lh;
      if (h1 == i) wgh += lh;
      if (wgh == 0.f) continue;
      for (int w = wl; w < wh; ++w) {
        int w0, w1;
        float lw;
        lin_w(w, Wp, W, w0, w1, lw);
        float ww = 0.f;
        if (w0 == j) ww += 1.f - lw;
        if (w1 == j) ww += lw;
        if (ww == 0.f) continue;
        float v[8];
        ld8(dy + ((size_t)(n * H + h) * W + w) * lddy + cv * 8, v);
        const float wt = wgh * ww;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(wt, v[k], acc[k]);
      }
    }
    float* o = dlow + (size_t)t * 8;
    *(float4*)o = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *(float4*)(o + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
}

// the same as one wave per low-res token: lanes = C/8 channel slices x PL pixel
// lanes over the token's bilinear support, combined by shuffles (the
// thread-per-slice form walked ~360 positions serially on 32 blocks: ~67 us)
template <typename T>
__global__ void __launch_bounds__(256) k_combine_bwd_low8w(const T* __restrict__ dy, int lddy, int B, int H, int W,
                                                           int C, int Hp, int Wp, float* __restrict__ dlow) {
  const int CV = C >> 3, PL = 64 / CV;
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= B * Hp * Wp) return;
  const int j = t % Wp, i = (t / Wp) % Hp, n = t / (Wp * Hp);
  const int cv = lane % CV, pl = lane / CV;
  const int hl = max(0, (int)floorf(((float)i - 0.5f) * H / Hp - 0.5f) - 1);
  const int hh = min(H, (int)ceilf(((float)i + 1.5f) * H / Hp - 0.5f) + 2);
  const int wl = max(0, (int)floorf(((float)j - 0.5f) * W / Wp - 0.5f) - 1);
  const int wh = min(W, (int)ceilf(((float)j + 1.5f) * W / Wp - 0.5f) + 2);
  const int nw = wh - wl, npos = (hh - hl) * nw;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int q = pl; q < npos; q += PL) {
    const int h = hl + q / nw, w = wl + (q - (q / nw) * nw);
    int h0, h1, w0, w1;
    float lh, lw;
    lin_w(h, Hp, H, h0, h1, lh);
    lin_w(w, Wp, W, w0, w1, lw);
    float wgh = 0.f, ww = 0.f;
    if (h0 == i) wgh += 1.f - lh;
    if (h1 == i) wgh += lh;
    if (w0 == j) ww += 1.f - lw;
    if (w1 == j) ww += lw;
    const float wt = wgh * ww;
    if (wt == 0.f) continue;
    float v[8];
    ld8(dy + ((size_t)(n * H + h) * W + w) * lddy + cv * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = fmaf(wt, v[k], acc[k]);
  }
  for (int o = CV; o < 64; o <<= 1)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += __shfl_xor(acc[k], o, 64);
  if (pl == 0) {
    float* o = dlow + (size_t)t * C + cv * 8;
    *(float4*)o = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *(float4*)(o + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
}

// ---------------------------------------------------------------- gating
// x = [pv_dwi (C), pv_dce (C), conf_dwi, conf_dce]; g = softmax(W x + b), 2 outputs
__global__ void k_gate_fwd(const float* __restrict__ pa, const float* __restrict__ pb, const float* __restrict__ ca,
                           const float* __restrict__ cb, int C, const float* __restrict__ Wt,
                           const float* __restrict__ bias, float* __restrict__ g) {
  __shared__ float red[16];
  const int n = blockIdx.x;
  const int In = 2 * C + (ca ? 2 : 0);
  float z0 = 0.f, z1 = 0.f;
  for (int i = threadIdx.x; i < In; i += blockDim.x) {
    float x;
    if (i < C) x = pa[n * C + i];
    else if (i < 2 * C) x = pb[n * C + i - C];
    else if (i == 2 * C) x = ca[n];
    else x = cb[n];
    z0 += Wt[i] * x;
    z1 += Wt[In + i] * x;
  }
  z0 = block_sum(z0, red) + bias[0];
  z1 = block_sum(z1, red) + bias[1];
  if (threadIdx.x == 0) {
    const float m = fmaxf(z0, z1);
    const float e0 = __expf(z0 - m), e1 = __expf(z1 - m);
    g[2 * n] = e0 / (e0 + e1);
    g[2 * n + 1] = e1 / (e0 + e1);
  }
}

// dz = softmax backward; dW (+)=, db (+)=, dpa/dpb/dca/dcb written (nullable).
// Blocks [0, B): one item each, the input gradients. Blocks [B, ...): 256
// weight columns each, dW / db summed over the items in item order
// (deterministic, no atomics; nn.Linear's backward, reference
// model_module.py:745-780).
__device__ __forceinline__ void gate_dz(const float* g, const float* dg, int n, float& dz0, float& dz1) {
  const float g0 = g[2 * n], g1 = g[2 * n + 1];
  const float s = dg[2 * n] * g0 + dg[2 * n + 1] * g1;
  dz0 = g0 * (dg[2 * n] - s);
  dz1 = g1 * (dg[2 * n + 1] - s);
}

__global__ void k_gate_bwd(const float* __restrict__ pa, const float* __restrict__ pb, const float* __restrict__ ca,
                           const float* __restrict__ cb, int C, const float* __restrict__ Wt,
                           const float* __restrict__ g, const float* __restrict__ dg, float* dW, float* db,
                           float* __restrict__ dpa, float* __restrict__ dpb, float* __restrict__ dca,
                           float* __restrict__ dcb, int B) {
  const int In = 2 * C + (ca ? 2 : 0);
  if ((int)blockIdx.x >= B) {
    const int i = ((int)blockIdx.x - B) * blockDim.x + threadIdx.x;
    if (i < In && dW) {
      float a0 = 0.f, a1 = 0.f;
      for (int n = 0; n < B; ++n) {
        float dz0, dz1;
        gate_dz(g, dg, n, dz0, dz1);
        const float x = i < C ? pa[n * C + i] : (i < 2 * C ? pb[n * C + i - C] : (i == 2 * C ? ca[n] : cb[n]));
        a0 += dz0 * x;
        a1 += dz1 * x;
      }
      dW[i] += a0;
      dW[In + i] += a1;
    }
    if (i == 0 && db) {
      float b0 = 0.f, b1 = 0.f;
      for (int n = 0; n < B; ++n) {
        float dz0, dz1;
        gate_dz(g, dg, n, dz0, dz1);
        b0 += dz0;
        b1 += dz1;
      }
      db[0] += b0;
      db[1] += b1;
    }
    return;
  }
  const int n = blockIdx.x;
  float dz0, dz1;
  gate_dz(g, dg, n, dz0, dz1);
  for (int i = threadIdx.x; i < In; i += blockDim.x) {
    const float dx = dz0 * Wt[i] + dz1 * Wt[In + i];
    if (i < C) { if (dpa) dpa[n * C + i] = dx; }
    else if (i < 2 * C) { if (dpb) dpb[n * C + i - C] = dx; }
    else if (i == 2 * C) { if (dca) dca[n] = dx; }
    else { if (dcb) dcb[n] = dx; }
  }
}


// ------------------------------------------------ SE / excitation MLP
// The excitation of an SEBlock (model_module.py:25-43) or of the input
// modality attention: hpre = pooled W1^T + b1, hact = gelu(hpre), gate =
// sigmoid(hact W2^T + b2), as two launches of one small dense-layer kernel
// (was 2 x (GEMM + split reduce + activation)). Each wave owns ONE output
// column j for every row: its weight row is held in registers (float4 slices,
// lanes stride K), the block's input rows are staged once in LDS, and each
// (row, j) dot product ends in one wave sum. Outputs are spread over J/4
// workgroups so the weight rows stream from L2 in parallel (a one-workgroup-
// per-row form ran ~57 us, latency-bound on its weight reads).
constexpr int DR_LDS = 64 * 1024;  // input-row staging per block
constexpr int DR_TMAX = 8;         // K <= 8 * 256

template <int ACT>
__global__ void __launch_bounds__(256) k_dense_rows(const float* __restrict__ in, int N, int K,
                                                    const float* __restrict__ W, const float* __restrict__ b, int J,
                                                    float* __restrict__ pre, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = blockIdx.x * 4 + wv;
  const int K4 = (K + 3) & ~3;
  const int T = (K4 + 255) / 256;
  const int NC = max(1, min(N, DR_LDS / (K4 * 4)));
  const bool v4 = (K & 3) == 0;
  float4 wr[DR_TMAX];
#pragma unroll
  for (int t = 0; t < DR_TMAX; ++t) {
    const int k = lane * 4 + t * 256;
    wr[t] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < T && j < J && k < K) {
      if (v4) {
        wr[t] = *(const float4*)(W + (size_t)j * K + k);
      } else {
        const float* wp = W + (size_t)j * K;
        wr[t].x = wp[k];
        if (k + 1 < K) wr[t].y = wp[k + 1];
        if (k + 2 < K) wr[t].z = wp[k + 2];
        if (k + 3 < K) wr[t].w = wp[k + 3];
      }
    }
  }
  const float bj = (b && j < J) ? b[j] : 0.f;
  for (int n0 = 0; n0 < N; n0 += NC) {
    const int nn = min(NC, N - n0);
    __syncthreads();
    if (v4) {
      // all of a thread's staging loads in flight before its LDS stores (a load -> store
      // chain per element serialises on the L2 latency)
      const int kv = K >> 2, tot = nn * kv;
      for (int e0 = 0; e0 < tot; e0 += 256 * 8) {
        float4 t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int e = e0 + u * 256 + threadIdx.x;
          if (e < tot) {
            const int r = e / kv, k = (e - r * kv) * 4;
            t[u] = *(const float4*)(in + (size_t)(n0 + r) * K + k);
          }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int e = e0 + u * 256 + threadIdx.x;
          if (e < tot) {
            const int r = e / kv, k = (e - r * kv) * 4;
            *(float4*)(xs + r * K4 + k) = t[u];
          }
        }
      }
    } else {
      for (int e = threadIdx.x; e < nn * K4; e += 256) {
        const int r = e / K4, k = e - r * K4;
        xs[r * K4 + k] = k < K ? in[(size_t)(n0 + r) * K + k] : 0.f;
      }
    }
    __syncthreads();
    if (j >= J) continue;
    for (int r0 = 0; r0 < nn; r0 += 4) {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = min(r0 + u, nn - 1);
#pragma unroll
        for (int t = 0; t < DR_TMAX; ++t) {
          const int k = lane * 4 + t * 256;
          if (t < T && k < K4) {
            const float4 x = *(const float4*)(xs + r * K4 + k);
            acc[u] = fmaf(wr[t].x, x.x, fmaf(wr[t].y, x.y, fmaf(wr[t].z, x.z, fmaf(wr[t].w, x.w, acc[u]))));
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = wave_sum(acc[u]);
      if (lane < 4 && r0 + lane < nn) {
        const float a = lane == 0 ? acc[0] : lane == 1 ? acc[1] : lane == 2 ? acc[2] : acc[3];
        const float z = a + bj;
        const size_t o = (size_t)(n0 + r0 + lane) * J + j;
        if (pre) pre[o] = z;
        out[o] = ACT == DMF_ACT_GELU ? gelu_f(z) : sigmoid_f(z);
      }
    }
  }
}

// The whole excitation in ONE workgroup for the small SEs of the path (N <= 64 rows, C and mid multiples
// of 4, both layers' activations in LDS): squeeze sum -> fc1 + GELU -> fc2 + sigmoid with 16 waves of
// 16 x 16 output tiles on the exact fp32 MFMA (v_mfma_f32_16x16x4f32). K runs in 16-wide steps whose
// lanes load float4 slices of the activation row (LDS) and of the weight row (global, 64 contiguous
// bytes per row per step): lane group q takes k = 16 s + 4 q + e in MFMA e of step s, the same order for
// both operands. The three launches (partial-plane sum, two dense-row passes, ~30 us with their gaps
// on the step's serial tail) become one of a few microseconds.
typedef __attribute__((ext_vector_type(4))) float se_f32x4;
constexpr int SE1_THREADS = 1024;
constexpr int SE1_PF = 4;  // K-steps whose weight loads a wave issues together

// One layer act(X W^T + b) over 16 x 16 output tiles, X [N][K] in LDS (row stride K), W [J][K] global.
// With fewer tiles than waves each tile's K-steps are split over P waves (P a power of two): every wave
// is busy and its weight loads are a few steps long, not a chain of K/16 dependent L2 round trips; the
// P partial tiles meet in LDS (`red`, 16 x 256 floats) and are summed in a fixed order.
template <int ACT>
__device__ __forceinline__ void se_layer(const float* X, int N, int K, const float* __restrict__ W,
                                         const float* __restrict__ b, int J, float* pre, float* out_g, float* out_l,
                                         float* red, int tid) {
  constexpr int NWV = SE1_THREADS / 64;
  const int lane = tid & 63, wv = tid >> 6, fr = lane & 15, q = lane >> 4;
  const int tn = (N + 15) / 16, T = tn * ((J + 15) / 16), S = (K + 15) / 16;
  int P = 1;
  while (P * 2 * T <= NWV && P * 2 <= S) P *= 2;
  const int G = NWV / P;  // tiles per round
  for (int base = 0; base < T; base += G) {
    const int t = base + wv / P, p = wv % P;
    se_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (t < T) {
      const int n = (t % tn) * 16 + fr, j = (t / tn) * 16 + fr;
      const int s0 = p * S / P, s1 = (p + 1) * S / P;
      // the weight slices of up to SE1_PF K-steps in flight together (one L2 round trip per chunk)
      for (int c0 = s0; c0 < s1; c0 += SE1_PF) {
        float4 wb[SE1_PF];
#pragma unroll
        for (int i = 0; i < SE1_PF; ++i) {
          const int k = (c0 + i) * 16 + 4 * q;  // K % 4 == 0: a float4 is wholly in or out
          wb[i] = (c0 + i < s1 && k < K && j < J) ? *(const float4*)(W + (size_t)j * K + k)
                                                   : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < SE1_PF; ++i) {
          if (c0 + i >= s1) break;
          const int k = (c0 + i) * 16 + 4 * q;
          const float4 a = (k < K && n < N) ? *(const float4*)(X + n * K + k) : make_float4(0.f, 0.f, 0.f, 0.f);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, wb[i].x, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, wb[i].y, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, wb[i].z, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, wb[i].w, acc, 0, 0, 0);
        }
      }
    }
    *(float4*)(red + wv * 256 + lane * 4) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    __syncthreads();
    // D[row 4q + r][col fr] of each tile: output row n0 + 4q + r, column j0 + fr
    for (int i = tid; i < G * 256; i += SE1_THREADS) {
      const int tl = i >> 8, e = i & 255, tt = base + tl;
      if (tt >= T) continue;
      float v = 0.f;
      for (int pp = 0; pp < P; ++pp) v += red[(tl * P + pp) * 256 + e];
      const int ln = e >> 2, r = e & 3;
      const int nr = (tt % tn) * 16 + 4 * (ln >> 4) + r, jc = (tt / tn) * 16 + (ln & 15);
      if (nr >= N || jc >= J) continue;
      const float z = v + (b ? b[jc] : 0.f);
      if (pre) pre[(size_t)nr * J + jc] = z;
      const float o = ACT == DMF_ACT_GELU ? gelu_f(z) : sigmoid_f(z);
      out_g[(size_t)nr * J + jc] = o;
      if (out_l) out_l[nr * J + jc] = o;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(SE1_THREADS) k_se_mlp1(const float* __restrict__ ws, int S, int N, int C, float scale,
                                                         const float* __restrict__ w1, const float* __restrict__ b1,
                                                         int mid, const float* __restrict__ w2,
                                                         const float* __restrict__ b2, float* __restrict__ pooled,
                                                         float* __restrict__ hpre, float* __restrict__ hact,
                                                         float* __restrict__ gate) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* red = sm;                  // [16 waves][256]
  float* xs = sm + 16 * 256;        // [N][C]
  float* hs = xs + N * C;           // [N][mid]
  const int tid = threadIdx.x;
  const int NC = N * C;
  for (int i = tid; i < NC; i += SE1_THREADS) {
    float v = 0.f;
    for (int z = 0; z < S; ++z) v += ws[(size_t)z * NC + i];
    v *= scale;
    xs[i] = v;
    if (pooled) pooled[i] = v;
  }
  __syncthreads();
  se_layer<DMF_ACT_GELU>(xs, N, C, w1, b1, mid, hpre, hact, hs, red, tid);
  se_layer<DMF_ACT_SIGMOID>(hs, N, mid, w2, b2, C, nullptr, gate, nullptr, red, tid);
}

// One dense layer of a larger SE as a grid of 16 x 16 output tiles, one workgroup (4 waves) per tile with
// its K-steps split over the waves (partials summed in LDS in a fixed order), on the fp32 MFMA as
// se_layer. The fc1 launch (S > 0) squeezes on the fly: X[n][k] = scale * sum_z ws[z][n][k], and the
// workgroups of the first column tile write `pooled`. Two launches in place of k_sum_planes + two
// k_dense_rows passes (whose per-column wave sums made them latency chains: ~17 + 14 us at C = 256).
template <int ACT>
__global__ void __launch_bounds__(256) k_se_dense(const float* __restrict__ X, int S, float scale, int N, int K,
                                                  const float* __restrict__ W, const float* __restrict__ b, int J,
                                                  float* __restrict__ pooled, float* __restrict__ pre,
                                                  float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float red[4][256];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, fr = lane & 15, q = lane >> 4;
  const int tn = (N + 15) / 16;
  const int n0 = (blockIdx.x % tn) * 16, j0 = (blockIdx.x / tn) * 16;
  const int n = n0 + fr, j = j0 + fr;
  const int St = (K + 15) / 16, s0 = wv * St / 4, s1 = (wv + 1) * St / 4;
  const bool wpool = pooled && j0 == 0;
  const long long NK = (long long)N * K;
  se_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = s0; c0 < s1; c0 += SE1_PF) {
    float4 wb[SE1_PF], xb[SE1_PF];
#pragma unroll
    for (int i = 0; i < SE1_PF; ++i) {
      const int k = (c0 + i) * 16 + 4 * q;  // K % 4 == 0: a float4 is wholly in or out
      const bool kin = c0 + i < s1 && k < K;
      wb[i] = (kin && j < J) ? *(const float4*)(W + (size_t)j * K + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      if (kin && n < N) {
        if (S > 0) {
          for (int z = 0; z < S; ++z) {
            const float4 v = *(const float4*)(X + z * NK + (size_t)n * K + k);
            a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
          }
          a.x *= scale; a.y *= scale; a.z *= scale; a.w *= scale;
          if (wpool) *(float4*)(pooled + (size_t)n * K + k) = a;
        } else {
          a = *(const float4*)(X + (size_t)n * K + k);
        }
      }
      xb[i] = a;
    }
#pragma unroll
    for (int i = 0; i < SE1_PF; ++i) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[i].x, wb[i].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[i].y, wb[i].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[i].z, wb[i].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[i].w, wb[i].w, acc, 0, 0, 0);
    }
  }
  *(float4*)(&red[wv][lane * 4]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  __syncthreads();
  // D[row 4q + r][col fr]: output row n0 + 4q + r, column j0 + fr
  const int e = tid, ln = e >> 2, r = e & 3;
  const float v = red[0][e] + red[1][e] + red[2][e] + red[3][e];
  const int nr = n0 + 4 * (ln >> 4) + r, jc = j0 + (ln & 15);
  if (nr < N && jc < J) {
    const float z = v + (b ? b[jc] : 0.f);
    if (pre) pre[(size_t)nr * J + jc] = z;
    out[(size_t)nr * J + jc] = ACT == DMF_ACT_GELU ? gelu_f(z) : sigmoid_f(z);
  }
}

// pooled[n][c] = scale * sum_z ws[z][n][c] (the squeeze's stage-1 partial planes)
__global__ void k_sum_planes(const float* __restrict__ ws, int S, long long NC, float scale, float* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < NC; i += (long long)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int z = 0; z < S; ++z) v += ws[(size_t)z * NC + i];
    out[i] = v * scale;
  }
}

}  // namespace dmf

using namespace dmf;

// K splits used for an (M, N, K) problem: enough blocks to cover the chip,
// >= 128 K per split (1 = no split)
static int sgemm_splits(int M, int N, int K) {
  const int tiles = cdiv(N, 64) * cdiv(M, 64);
  // >= 128 K per split: a split of a short K (the fusion's 128-wide token linears) costs a reduce
  // launch for less than it saves
  int S = std::max(1, std::min(cdiv(512, tiles), K / 128));
  if (S <= 1) return 1;
  const int kchunk = cdiv(cdiv(K, S), 16) * 16;
  return std::max(1, cdiv(K, kchunk));
}


// 1 (default): the small GEMMs (M * N <= 512^2, K <= 8192) on k_sgemm_mfma; 0: always k_sgemm
static int g_sgemm_mfma = 1;
extern "C" int dmf_sgemm_tune(int mfma) {
  g_sgemm_mfma = mfma != 0;
  return 0;
}

extern "C" int dmf_sgemm_ws_size(int M, int N, int K) {
  const int S = sgemm_splits(M, N, K);
  return S > 1 ? S * M * N : 0;
}

extern "C" int dmf_sgemm(int transA, int transB, int M, int N, int K, float alpha, const float* A, int lda,
                         const float* B, int ldb, float beta, float* C, int ldc, const float* bias, int act,
                         float* workspace, void* stream) {
  DMF_CHECK_ARG(A && B && C && M >= 0 && N >= 0 && K >= 0, "dmf_sgemm: bad args");
  if (M == 0 || N == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (g_sgemm_mfma && (long long)M * N <= 512LL * 512 && K <= 8192) {
    hipLaunchKernelGGL(k_sgemm_mfma, dim3((unsigned)(cdiv(M, 16) * cdiv(N, 16))), dim3(256), 0, st, transA, transB, M,
                       N, K, alpha, A, lda, B, ldb, beta, C, ldc, bias, act);
    DMF_LAUNCH_CHECK("dmf_sgemm");
    return 0;
  }
  // (beta != 0 -- an accumulating weight gradient -- splits too: the ordered reduce adds beta * C)
  int S = workspace ? sgemm_splits(M, N, K) : 1;
  const int kchunk = S > 1 ? cdiv(cdiv(K, S), 16) * 16 : std::max(K, 1);
  S = S > 1 ? cdiv(K, kchunk) : 1;
  dim3 grid(cdiv(N, 64), cdiv(M, 64), S);
  hipLaunchKernelGGL((k_sgemm<16>), grid, dim3(256), 0, st, transA, transB, M, N, K, kchunk, alpha, A, lda, B, ldb,
                     beta, C, ldc, bias, act, workspace);
  if (S > 1)
    hipLaunchKernelGGL(k_sgemm_reduce, dim3(gsz((long long)M * N)), dim3(256), 0, st, S, M, N, alpha, workspace, beta,
                       C, ldc, bias, act);
  DMF_LAUNCH_CHECK("dmf_sgemm");
  return 0;
}

extern "C" int dmf_colsum_f32(const float* X, int ldx, int M, int N, float* out, int accumulate, void* stream) {
  DMF_CHECK_ARG(X && out, "dmf_colsum_f32: bad args");
  if (N == 0) return 0;
  hipLaunchKernelGGL(k_colsum, dim3(cdiv(N, 64)), dim3(1024), 0, (hipStream_t)stream, X, ldx, M, N, out, accumulate);
  DMF_LAUNCH_CHECK("dmf_colsum_f32");
  return 0;
}

extern "C" int dmf_act_grad_f32(const float* dy, const float* z, float* dx, long long n, int act, void* stream) {
  DMF_CHECK_ARG(dy && z && dx, "dmf_act_grad_f32: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_act_grad_f32, dim3(gsz(n)), dim3(256), 0, (hipStream_t)stream, dy, z, dx, n, act);
  DMF_LAUNCH_CHECK("dmf_act_grad_f32");
  return 0;
}

extern "C" int dmf_act_f32(const float* x, float* y, long long n, int act, void* stream) {
  DMF_CHECK_ARG(x && y, "dmf_act_f32: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_act_f32, dim3(gsz(n)), dim3(256), 0, (hipStream_t)stream, x, y, n, act);
  DMF_LAUNCH_CHECK("dmf_act_f32");
  return 0;
}

extern "C" int dmf_sig_grad_f32(const float* dg, const float* s, float* dz, long long n, void* stream) {
  DMF_CHECK_ARG(dg && s && dz, "dmf_sig_grad_f32: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_sig_grad_f32, dim3(gsz(n)), dim3(256), 0, (hipStream_t)stream, dg, s, dz, n);
  DMF_LAUNCH_CHECK("dmf_sig_grad_f32");
  return 0;
}

extern "C" int dmf_row_l2norm(const float* x, int R, int C, float eps, float* y, float* norms, void* stream) {
  DMF_CHECK_ARG(x && y && R > 0 && C > 0, "dmf_row_l2norm: bad args");
  hipLaunchKernelGGL(k_row_l2norm, dim3(cdiv(R, 4)), dim3(256), 0, (hipStream_t)stream, x, R, C, eps, y, norms);
  DMF_LAUNCH_CHECK("dmf_row_l2norm");
  return 0;
}

extern "C" int dmf_row_l2norm_bwd(const float* dy, const float* y, const float* norms, int R, int C, float eps,
                                  float* dx, void* stream) {
  DMF_CHECK_ARG(dy && y && norms && dx, "dmf_row_l2norm_bwd: bad args");
  hipLaunchKernelGGL(k_row_l2norm_bwd, dim3(cdiv(R, 4)), dim3(256), 0, (hipStream_t)stream, dy, y, norms, R, C, eps,
                     dx);
  DMF_LAUNCH_CHECK("dmf_row_l2norm_bwd");
  return 0;
}

extern "C" int dmf_layernorm_fwd(const float* x, int R, int E, const float* gamma, const float* beta, float eps,
                                 float* y, float* save, void* stream) {
  DMF_CHECK_ARG(x && gamma && beta && y && R > 0 && E > 0, "dmf_layernorm_fwd: bad args");
  hipLaunchKernelGGL(k_layernorm, dim3(cdiv(R, 4)), dim3(256), 0, (hipStream_t)stream, x, R, E, gamma, beta, eps, y,
                     save);
  DMF_LAUNCH_CHECK("dmf_layernorm_fwd");
  return 0;
}

extern "C" int dmf_layernorm_bwd(const float* dy, const float* x, const float* save, int R, int E, const float* gamma,
                                 float* dx, float* dgamma, float* dbeta, void* stream) {
  DMF_CHECK_ARG(dy && x && save && gamma && dx && R > 0 && E > 0, "dmf_layernorm_bwd: bad args");
  const int nrb = cdiv(R, 4), ncb = (dgamma || dbeta) ? cdiv(E, 64) : 0;
  hipLaunchKernelGGL(k_layernorm_bwd, dim3(nrb + ncb), dim3(256), 0, (hipStream_t)stream, dy, x, save, R, E, gamma,
                     dx, dgamma, dbeta, nrb);
  DMF_LAUNCH_CHECK("dmf_layernorm_bwd");
  return 0;
}

extern "C" int dmf_attn_fwd(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv, int B, int Nq,
                            int Nk, int H, int D, float scale, float* out, int ldo, float* probs, float* avg_weights,
                            void* stream) {
  DMF_CHECK_ARG(q && k && v && out && Nq <= 64 && Nk <= 64 && D <= 128,
                "dmf_attn_fwd: short-sequence kernel needs Nq,Nk<=64, D<=128 (got %d,%d,%d)", Nq, Nk, D);
  DMF_CHECK_ARG(!avg_weights || probs, "dmf_attn_fwd: avg_weights needs the probs buffer");
  hipLaunchKernelGGL(k_attn_fwd, dim3(B * H), dim3(256), 0, (hipStream_t)stream, q, ldq, k, ldk, v, ldv, Nq, Nk, H, D,
                     scale, out, ldo, probs);
  if (avg_weights)
    hipLaunchKernelGGL(k_head_mean, dim3(cdiv((long long)B * Nq * Nk, 256)), dim3(256), 0, (hipStream_t)stream, probs,
                       B, H, Nq * Nk, avg_weights);
  DMF_LAUNCH_CHECK("dmf_attn_fwd");
  return 0;
}

extern "C" int dmf_attn_bwd(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv,
                            const float* probs, const float* dout, int lddo, int B, int Nq, int Nk, int H, int D,
                            float scale, float* dq, int lddq, float* dk, int lddk, float* dv, int lddv, void* stream) {
  DMF_CHECK_ARG(q && k && v && probs && dout && dq && dk && dv && Nq <= 64 && Nk <= 64,
                "dmf_attn_bwd: bad args");
  hipLaunchKernelGGL(k_attn_bwd, dim3(B * H), dim3(256), 0, (hipStream_t)stream, q, ldq, k, ldk, v, ldv, probs, dout,
                     lddo, Nq, Nk, H, D, scale, dq, lddq, dk, lddk, dv, lddv);
  DMF_LAUNCH_CHECK("dmf_attn_bwd");
  return 0;
}

extern "C" int dmf_tokens_fwd(int dtype, const void* x, int ldx, int B, int H, int W, int C, int Hp, int Wp,
                              float* tokens, void* stream) {
  DMF_CHECK_ARG(x && tokens && Hp > 0 && Wp > 0 && H % Hp == 0 && W % Wp == 0,
                "dmf_tokens_fwd: map %dx%d must divide into %dx%d tokens", H, W, Hp, Wp);
  const long long total = (long long)B * Hp * Wp * C;
  const int CV = C / 8;
  if (C % 8 == 0 && CV <= 64 && 64 % CV == 0 && ldx % 8 == 0 && ((uintptr_t)x % 16) == 0 &&
      ((uintptr_t)tokens % 16) == 0 && (long long)B * H * W * ldx < (1LL << 31)) {
    const dim3 g(cdiv((long long)B * Hp * Wp, 4));
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_tokens_fwd8<T>, g, dim3(256), 0, (hipStream_t)stream, (const T*)x, ldx, B, H, W, C,
                         Hp, Wp, tokens));
    DMF_LAUNCH_CHECK("dmf_tokens_fwd");
    return 0;
  }
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_tokens_fwd<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, (const T*)x,
                       ldx, B, H, W, C, Hp, Wp, tokens));
  DMF_LAUNCH_CHECK("dmf_tokens_fwd");
  return 0;
}

extern "C" int dmf_tokens_bwd(int dtype, const float* dtokens, int B, int H, int W, int C, int Hp, int Wp, void* dx,
                              int lddx, int accumulate, void* stream) {
  DMF_CHECK_ARG(dtokens && dx && H % Hp == 0 && W % Wp == 0, "dmf_tokens_bwd: bad args");
  const long long total = (long long)B * H * W * C;
  if (C % 8 == 0 && lddx % 8 == 0 && ((uintptr_t)dx % 16) == 0 && ((uintptr_t)dtokens % 16) == 0 &&
      (long long)B * H * W * lddx < (1LL << 31)) {
    const long long t8 = total / 8;
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_tokens_bwd8<T>, dim3(gsz(t8)), dim3(256), 0, (hipStream_t)stream, dtokens, B, H, W, C,
                         Hp, Wp, (T*)dx, lddx, accumulate));
    DMF_LAUNCH_CHECK("dmf_tokens_bwd");
    return 0;
  }
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_tokens_bwd<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, dtokens, B, H, W, C,
                       Hp, Wp, (T*)dx, lddx, accumulate));
  DMF_LAUNCH_CHECK("dmf_tokens_bwd");
  return 0;
}

extern "C" int dmf_fusion_combine_fwd(int dtype, const void* p_dwi, const void* p_dce, int ld, const float* gates,
                                      const float* lowres, int B, int H, int W, int C, int Hp, int Wp, void* y,
                                      int ldy, void* stream) {
  DMF_CHECK_ARG(p_dwi && p_dce && gates && y, "dmf_fusion_combine_fwd: bad args");
  const long long total = (long long)B * H * W * C;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_combine_fwd<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream,
                       (const T*)p_dwi, (const T*)p_dce, ld, gates, lowres, B, H, W, C, Hp, Wp, (T*)y,
                       ldy));
  DMF_LAUNCH_CHECK("dmf_fusion_combine_fwd");
  return 0;
}

extern "C" int dmf_fusion_combine_bwd(int dtype, const void* dy, int lddy, const void* p_dwi, const void* p_dce,
                                      int ld, const float* gates, int B, int H, int W, int C, int Hp, int Wp,
                                      void* dp_dwi, void* dp_dce, int ldd, float* dgates, float* dlowres,
                                      void* stream) {
  DMF_CHECK_ARG(dy && p_dwi && p_dce && gates, "dmf_fusion_combine_bwd: bad args");
  const long long total = (long long)B * H * W * C;
  hipStream_t st_ = (hipStream_t)stream;
  const bool v8 = C % 8 == 0 && C / 8 <= 64 && 64 % (C / 8) == 0 && lddy % 8 == 0 && ld % 8 == 0 &&
                  ((uintptr_t)dy % 16) == 0 && (!dlowres || ((uintptr_t)dlowres % 16) == 0) &&
                  ((uintptr_t)p_dwi % 16) == 0 && ((uintptr_t)p_dce % 16) == 0;
  if (v8) {
    DMF_DISPATCH_DTYPE(dtype, T,
      if (dp_dwi || dp_dce)
        hipLaunchKernelGGL(k_combine_bwd_maps<T>, dim3(gsz(total)), dim3(256), 0, st_, (const T*)dy, lddy,
                           gates, H * W, C, total, (T*)dp_dwi, (T*)dp_dce, ldd);
      if (dgates)
        hipLaunchKernelGGL(k_combine_bwd_gate8<T>, dim3(B), dim3(1024), 0, st_, (const T*)dy, lddy,
                           (const T*)p_dwi, (const T*)p_dce, ld, H * W, C, dgates);
      if (dlowres)
        hipLaunchKernelGGL(k_combine_bwd_low8w<T>, dim3(cdiv((long long)B * Hp * Wp, 4)), dim3(256), 0, st_,
                           (const T*)dy, lddy, B, H, W, C, Hp, Wp, dlowres));
  } else DMF_DISPATCH_DTYPE(dtype, T, if (dp_dwi || dp_dce)
      hipLaunchKernelGGL(k_combine_bwd_maps<T>, dim3(gsz(total)), dim3(256), 0, st_, (const T*)dy, lddy,
                         gates, H * W, C, total, (T*)dp_dwi, (T*)dp_dce, ldd);
    if (dgates)
      hipLaunchKernelGGL(k_combine_bwd_gate<T>, dim3(B), dim3(256), 0, st_, (const T*)dy, lddy,
                         (const T*)p_dwi, (const T*)p_dce, ld, H * W, C, dgates);
    if (dlowres)
      hipLaunchKernelGGL(k_combine_bwd_low<T>, dim3(gsz((long long)B * Hp * Wp * C)), dim3(256), 0, st_,
                         (const T*)dy, lddy, B, H, W, C, Hp, Wp, dlowres));
  DMF_LAUNCH_CHECK("dmf_fusion_combine_bwd");
  return 0;
}

extern "C" int dmf_gate_fwd(const float* pv_dwi, const float* pv_dce, const float* conf_dwi, const float* conf_dce,
                            int B, int C, const float* W, const float* b, float* gates, void* stream) {
  DMF_CHECK_ARG(pv_dwi && pv_dce && W && b && gates && ((conf_dwi == nullptr) == (conf_dce == nullptr)),
                "dmf_gate_fwd: bad args");
  hipLaunchKernelGGL(k_gate_fwd, dim3(B), dim3(256), 0, (hipStream_t)stream, pv_dwi, pv_dce, conf_dwi, conf_dce, C, W,
                     b, gates);
  DMF_LAUNCH_CHECK("dmf_gate_fwd");
  return 0;
}

extern "C" int dmf_gate_bwd(const float* pv_dwi, const float* pv_dce, const float* conf_dwi, const float* conf_dce,
                            int B, int C, const float* W, const float* gates, const float* dgates, float* dW,
                            float* db, float* dpv_dwi, float* dpv_dce, float* dconf_dwi, float* dconf_dce,
                            void* stream) {
  DMF_CHECK_ARG(pv_dwi && pv_dce && W && gates && dgates, "dmf_gate_bwd: bad args");
  const int In = 2 * C + (conf_dwi ? 2 : 0);
  const int ncb = (dW || db) ? cdiv(In, 256) : 0;
  hipLaunchKernelGGL(k_gate_bwd, dim3(B + ncb), dim3(256), 0, (hipStream_t)stream, pv_dwi, pv_dce, conf_dwi, conf_dce,
                     C, W, gates, dgates, dW, db, dpv_dwi, dpv_dce, dconf_dwi, dconf_dce, B);
  DMF_LAUNCH_CHECK("dmf_gate_bwd");
  return 0;
}

// 1 (default): two launches of fp32-MFMA tiles (k_se_dense); 2: the one-workgroup form (k_se_mlp1) where it
// fits, else as 1; 0: the three-launch form (k_sum_planes + two k_dense_rows). tools/se_bench.py, N = 32:
// C = 128: 25.8 (0) / 10.6 (2) us; C = 256: 28.7 (0) / 6.8 (1) us; C = 512: 35.8 (0) / 11.8 (1) us
static int g_se_one_launch = 1;
extern "C" int dmf_se_mlp_tune(int mode) {
  DMF_CHECK_ARG(mode >= 0 && mode <= 2, "dmf_se_mlp_tune: mode %d (0..2)", mode);
  g_se_one_launch = mode;
  return 0;
}

extern "C" int dmf_se_mlp(const float* ws, int S, int N, int C, float scale, const float* w1, const float* b1,
                          int mid, const float* w2, const float* b2, float* pooled, float* hpre, float* hact,
                          float* gate, void* stream) {
  DMF_CHECK_ARG(ws && w1 && w2 && hact && gate && S >= 1 && N >= 1 && C >= 1 && mid >= 1, "dmf_se_mlp: bad args");
  DMF_CHECK_ARG(C <= DR_TMAX * 256 && mid <= DR_TMAX * 256, "dmf_se_mlp: C and mid must be <= 2048");
  DMF_CHECK_ARG(((uintptr_t)w1 & 15) == 0 && ((uintptr_t)w2 & 15) == 0 && ((uintptr_t)ws & 15) == 0 &&
                    ((uintptr_t)hact & 15) == 0 && (!pooled || ((uintptr_t)pooled & 15) == 0),
                "dmf_se_mlp: weights and vectors must be 16-B aligned");
  DMF_CHECK_ARG(pooled || (S == 1 && scale == 1.f), "dmf_se_mlp: a split / scaled squeeze needs `pooled`");
  hipStream_t st = (hipStream_t)stream;
  const size_t lds1 = (size_t)N * (C + mid) * 4 + 16 * 256 * 4;
  // (one CU runs both layers on the fp32 MFMA, 2*N*C*mid FMAs each: it wins up to the C = 128 SEs --
  // 11.8 vs 26.0 us at N = 32, C = 128 -- and ties at C = 256, tools/se_bench.py)
  if (g_se_one_launch == 2 && N <= 64 && C % 4 == 0 && mid % 4 == 0 && lds1 <= 96 * 1024 &&
      (long long)N * C * mid <= 32LL * 128 * 64 &&
      (!pooled || pooled != ws || S == 1)) {
    // (pooled == ws with S == 1: the squeeze read and its write touch the same element in one thread)
    hipLaunchKernelGGL(k_se_mlp1, dim3(1), dim3(SE1_THREADS), lds1, st, ws, S, N, C, scale, w1, b1, mid, w2, b2,
                       pooled, hpre, hact, gate);
    DMF_LAUNCH_CHECK("dmf_se_mlp");
    return 0;
  }
  if (g_se_one_launch && C % 4 == 0 && mid % 4 == 0 && (!pooled || pooled != ws)) {
    // two launches of MFMA tiles (k_se_dense); fc1 squeezes the partial planes on the fly, up to 2 of them
    // (every column tile re-reads the planes: beyond that one k_sum_planes pass first is cheaper)
    const int tn = cdiv(N, 16);
    const float* xs = ws;
    int S1 = S;
    float sc1 = scale;
    float* pool1 = pooled;
    if (S > 2) {
      const long long nc = (long long)N * C;
      hipLaunchKernelGGL(k_sum_planes, dim3(gsz(nc)), dim3(256), 0, st, ws, S, nc, scale, pooled);
      xs = pooled;
      S1 = 0;
      sc1 = 1.f;
      pool1 = nullptr;
    }
    hipLaunchKernelGGL(k_se_dense<DMF_ACT_GELU>, dim3((unsigned)(tn * cdiv(mid, 16))), dim3(256), 0, st, xs, S1, sc1,
                       N, C, w1, b1, mid, pool1, hpre, hact);
    hipLaunchKernelGGL(k_se_dense<DMF_ACT_SIGMOID>, dim3((unsigned)(tn * cdiv(C, 16))), dim3(256), 0, st,
                       (const float*)hact, 0, 1.f, N, mid, w2, b2, C, (float*)nullptr, (float*)nullptr, gate);
    DMF_LAUNCH_CHECK("dmf_se_mlp");
    return 0;
  }
  const float* x = ws;
  if (pooled && (S > 1 || scale != 1.f || pooled != ws)) {
    const long long nc = (long long)N * C;
    hipLaunchKernelGGL(k_sum_planes, dim3(gsz(nc)), dim3(256), 0, st, ws, S, nc, scale, pooled);
    x = pooled;
  }
  hipLaunchKernelGGL(k_dense_rows<DMF_ACT_GELU>, dim3(cdiv(mid, 4)), dim3(256), DR_LDS, st, x, N, C, w1, b1, mid, hpre,
                     hact);
  hipLaunchKernelGGL(k_dense_rows<DMF_ACT_SIGMOID>, dim3(cdiv(C, 4)), dim3(256), DR_LDS, st, (const float*)hact, N,
                     mid, w2, b2, C, (float*)nullptr, gate);
  DMF_LAUNCH_CHECK("dmf_se_mlp");
  return 0;
}
