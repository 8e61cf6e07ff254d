// Batch-norm (train/eval), fused affine + residual + activation + dropout,
// and their backward, on NHWC tensors. Semantics follow torch BatchNorm2d as
// used everywhere on the hot path (timm Bottleneck bn1..bn3, adapter necks
// model_module.py:440-447, ResNetLite :259-280, heads, projectors):
//   train: mean/biased var over (N,H,W); running_mean/var updated with
//          momentum and the unbiased (n/(n-1)) variance; eval: running stats.
// Dropout (model_module.py:263, :273, nn.Dropout element-wise) uses a Philox
// counter stream keyed by (seed, per-step offset from device memory, site id,
// element index) so the backward regenerates the same mask.
#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

__device__ __forceinline__ float act_fwd(int act, float z) {
  switch (act) {
    case DMF_ACT_RELU: return fmaxf(z, 0.f);
    case DMF_ACT_GELU: return gelu_f(z);
    case DMF_ACT_SIGMOID: return sigmoid_f(z);
    default: return z;
  }
}
__device__ __forceinline__ float act_grad(int act, float z) {
  switch (act) {
    case DMF_ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case DMF_ACT_GELU: return gelu_grad_f(z);
    case DMF_ACT_SIGMOID: { const float s = sigmoid_f(z); return s * (1.f - s); }
    default: return 1.f;
  }
}

// ---------------------------------------------------------- bn finalize
// partials [T][C][2] -> mean/invstd, per-channel affine (scale, shift), and
// running-stat update. Block: 64 channels x 4 tile lanes.
// stage 1 (large T): block (channel group, tile chunk) -> double partials [S][C][2]
__global__ void k_bn_stage1(const float* __restrict__ part, int T, int C, int chunk, double* __restrict__ out) {
  __shared__ double red[4][64][2];
  const int cl = threadIdx.x & 63, tl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int t0 = blockIdx.y * chunk, t1 = min(T, t0 + chunk);
  double s = 0.0, q = 0.0;
  if (c < C)
    for (int t = t0 + tl; t < t1; t += 4) {
      const float2 v = *(const float2*)(part + ((size_t)t * C + c) * 2);
      s += v.x;
      q += v.y;
    }
  red[tl][cl][0] = s;
  red[tl][cl][1] = q;
  __syncthreads();
  if (tl == 0 && c < C) {
    out[((size_t)blockIdx.y * C + c) * 2] = red[0][cl][0] + red[1][cl][0] + red[2][cl][0] + red[3][cl][0];
    out[((size_t)blockIdx.y * C + c) * 2 + 1] = red[0][cl][1] + red[1][cl][1] + red[2][cl][1] + red[3][cl][1];
  }
}

template <typename PT>
__global__ void k_bn_finalize(const PT* __restrict__ part, int T, int C, BnFin f) {
  __shared__ double red[4][64][2];
  const int cl = threadIdx.x & 63, tl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s = 0.0, q = 0.0;
  if (f.training && c < C) {
    for (int t = tl; t < T; t += 4) {
      s += (double)part[((size_t)t * C + c) * 2];
      q += (double)part[((size_t)t * C + c) * 2 + 1];
    }
  }
  red[tl][cl][0] = s;
  red[tl][cl][1] = q;
  __syncthreads();
  if (tl == 0 && c < C) {
    s = red[0][cl][0] + red[1][cl][0] + red[2][cl][0] + red[3][cl][0];
    q = red[0][cl][1] + red[1][cl][1] + red[2][cl][1] + red[3][cl][1];
    bn_fin_channel(f, c, C, s, q);
  }
  if (f.training && f.nbt && blockIdx.x == 0 && threadIdx.x == 0) *f.nbt += 1;
}

// single-launch finalize for T <= 1024 tiles: block of 1024 threads =
// 16 channels x 64 tile lanes (T/64 independent loads per lane, then a
// fixed-order LDS tree in double) -- C/16 blocks, so even C = 64 spreads
// over 4 CUs and a lane waits for at most a few loads (latency-bound launch)
__global__ void __launch_bounds__(1024) k_bn_finalize_wide(const float* __restrict__ part, int T, int C, BnFin f) {
  __shared__ double red[64][16][2];
  const int cl = threadIdx.x & 15, tl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double s = 0.0, q = 0.0;
  if (c < C) {
    int t = tl;
    for (; t + 64 < T; t += 128) {
      const float2 v0 = *(const float2*)(part + ((size_t)t * C + c) * 2);
      const float2 v1 = *(const float2*)(part + ((size_t)(t + 64) * C + c) * 2);
      s += (double)v0.x + (double)v1.x;
      q += (double)v0.y + (double)v1.y;
    }
    if (t < T) {
      const float2 v = *(const float2*)(part + ((size_t)t * C + c) * 2);
      s += (double)v.x;
      q += (double)v.y;
    }
  }
  red[tl][cl][0] = s;
  red[tl][cl][1] = q;
  __syncthreads();
#pragma unroll
  for (int w = 32; w > 0; w >>= 1) {
    if (tl < w) {
      red[tl][cl][0] += red[tl + w][cl][0];
      red[tl][cl][1] += red[tl + w][cl][1];
    }
    __syncthreads();
  }
  if (tl == 0 && c < C) bn_fin_channel(f, c, C, red[0][cl][0], red[0][cl][1]);
  if (f.nbt && blockIdx.x == 0 && threadIdx.x == 0) *f.nbt += 1;
}

// ------------------------------------------------------ fused affine/act
// y = drop(act(x*sa + ba + [res*sr + br | res]))
template <typename T>
__global__ void k_affine_act(const T* __restrict__ x, int ldx, const float* __restrict__ ssa,
                             const T* __restrict__ res, int ldr, const float* __restrict__ ssr, int act,
                             float p, const unsigned long long* rng, int site, T* __restrict__ y, int ldy,
                             long long M, int C) {
  const unsigned long long rseed_ = rng ? rng[0] : 0ull, roff_ = rng ? rng[1] : 0ull;  // read once (see dropout_keep4v)
  constexpr int V = 4;
  const int cv = C / V;
  const long long total = M * cv;
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long m = i / cv;
    const int c0 = (int)(i - m * cv) * V;
    float v[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float z = ld(x + m * ldx + c0 + k);
      if (ssa) z = z * ssa[c0 + k] + ssa[C + c0 + k];
      if (res) {
        float r = ld(res + m * ldr + c0 + k);
        if (ssr) r = r * ssr[c0 + k] + ssr[C + c0 + k];
        z += r;
      }
      v[k] = act_fwd(act, z);
    }
    if (p > 0.f) {
      bool keep[4];
      dropout_keep4v(rseed_, roff_, site, (unsigned long long)(m * C + c0), p, keep);
#pragma unroll
      for (int k = 0; k < V; ++k) v[k] = keep[k] ? v[k] * sc : 0.f;
    }
#pragma unroll
    for (int k = 0; k < V; ++k) st(y + m * ldy + c0 + k, v[k]);
  }
}

// 8-channel vectorised variant (C, strides multiple of 8; 16-B bf16 accesses)
template <typename T, int ACT>
__global__ void k_affine_act8(const T* __restrict__ x, int ldx, const float* __restrict__ ssa,
                              const T* __restrict__ res, int ldr, const float* __restrict__ ssr, float p,
                              const unsigned long long* rng, int site, T* __restrict__ y, int ldy, long long M,
                              int C) {
  const unsigned long long rseed_ = rng ? rng[0] : 0ull, roff_ = rng ? rng[1] : 0ull;  // read once (see dropout_keep4v)
  // 32-bit index math (the host routes M*C/8 >= 2^31 to k_affine_act)
  const unsigned cv = (unsigned)C >> 3;
  const unsigned total = (unsigned)(M * cv);
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const unsigned m = i / cv;
    const int c0 = (int)(i - m * cv) << 3;
    float v[8], r[8];
    ld8(x + (size_t)m * ldx + c0, v);
    if (ssa) {
      const float4 s0 = *(const float4*)(ssa + c0), s1 = *(const float4*)(ssa + c0 + 4);
      const float4 b0 = *(const float4*)(ssa + C + c0), b1 = *(const float4*)(ssa + C + c0 + 4);
      v[0] = v[0] * s0.x + b0.x; v[1] = v[1] * s0.y + b0.y; v[2] = v[2] * s0.z + b0.z; v[3] = v[3] * s0.w + b0.w;
      v[4] = v[4] * s1.x + b1.x; v[5] = v[5] * s1.y + b1.y; v[6] = v[6] * s1.z + b1.z; v[7] = v[7] * s1.w + b1.w;
    }
    if (res) {
      ld8(res + (size_t)m * ldr + c0, r);
      if (ssr) {
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = r[k] * ssr[c0 + k] + ssr[C + c0 + k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += r[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (ACT == DMF_ACT_RELU) v[k] = fmaxf(v[k], 0.f);
      else if (ACT == DMF_ACT_GELU) v[k] = gelu_f(v[k]);
      else if (ACT == DMF_ACT_SIGMOID) v[k] = sigmoid_f(v[k]);
    }
    if (p > 0.f) {
      bool keep[4];
      dropout_keep4v(rseed_, roff_, site, (unsigned long long)m * C + c0, p, keep);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = keep[k] ? v[k] * sc : 0.f;
      dropout_keep4v(rseed_, roff_, site, (unsigned long long)m * C + c0 + 4, p, keep);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[4 + k] = keep[k] ? v[4 + k] * sc : 0.f;
    }
    st8(y + (size_t)m * ldy + c0, v);
  }
}

// ------------------------------------------- BN apply with the finalize folded in
// One affine source: batch statistics accumulated by the producing conv
// (dmf_conv2d_fwd_acc, [C][2] sums) finalized here, or a precomputed
// scale/shift, or none.
struct BnApplySrc {
  const double* acc;  // [replicas][C][2]
  const float* ss;
  BnFin fin;
  int replicas;
};

// (scale, shift) of channel c; `write`: this block also publishes
// scale_shift / save_mean_invstd and updates the running statistics
// (exactly what dmf_bn_finalize does for a slab)
__device__ __forceinline__ void bn_src_affine(const BnApplySrc& s, int c, int C, bool write, float& sc, float& sh) {
  if (s.acc) {
    double sum = 0.0, sq = 0.0;
    for (int r = 0; r < s.replicas; ++r) {  // fixed order
      sum += s.acc[((size_t)r * C + c) * 2];
      sq += s.acc[((size_t)r * C + c) * 2 + 1];
    }
    if (write) {
      bn_fin_channel(s.fin, c, C, sum, sq);
    }
    const double m = sum / s.fin.count;
    double v = sq / s.fin.count - m * m;
    if (v < 0.0) v = 0.0;
    const float inv = rsqrtf((float)v + s.fin.eps);
    const float g = s.fin.gamma ? s.fin.gamma[c] : 1.f, b = s.fin.beta ? s.fin.beta[c] : 0.f;
    sc = g * inv;
    sh = b - (float)m * g * inv;
  } else if (s.ss) {
    sc = s.ss[c];
    sh = s.ss[C + c];
  } else {
    sc = 1.f;
    sh = 0.f;
  }
}

// y = drop(act(x*sa + ba [+ res*sr + br | + res])). Block = 64 channels
// (blockIdx.x, fastest, so the resident blocks stream whole rows) x rows_per_blk pixels (blockIdx.y);
// 256 threads = 8 16-B
// channel chunks x 32 rows; the block's 64 (scale, shift) pairs are
// finalized once into LDS. Dropout elements are indexed m*C + c exactly as
// k_affine_act8 / k_act_bwd, so backward regenerates the same masks.
template <typename T, int ACT, int RES, int U>
__global__ void __launch_bounds__(256) k_bn_apply(const T* __restrict__ x, int ldx, BnApplySrc A,
                                                   const T* __restrict__ res, int ldr, BnApplySrc R, float p,
                                                   const unsigned long long* rng, int site, T* __restrict__ y, int ldy,
                                                   int M, int C, int rows_per_blk) {
  const unsigned long long rseed_ = rng ? rng[0] : 0ull, roff_ = rng ? rng[1] : 0ull;  // read once (see dropout_keep4v)
  __shared__ float sa[2][64], sr[2][64];
  const int tid = threadIdx.x;
  const int cg = blockIdx.x * 64;
  const bool first = blockIdx.y == 0;
  const int cl = (tid & 7) * 8, c0 = cg + cl;
  const int mbeg = blockIdx.y * rows_per_blk;
  const int mend = min(M, mbeg + rows_per_blk);
  // U rows per thread in flight: all U (x, res) loads issue before the first conversion; the first
  // group's loads go out before the finalize prologue, so its arena reads hide under them
  Vec8<T> xr[U], rr[U];
  auto load = [&](int mu) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = mu + 32 * u;
      xr[u] = zero8<T>();
      rr[u] = zero8<T>();
      if (m < mend) {
        xr[u] = ldv8(x + (size_t)m * ldx + c0);
        if (RES != 0) rr[u] = ldv8(res + (size_t)m * ldr + c0);
      }
    }
  };
  int mu = mbeg + (tid >> 3);
  if (c0 < C) load(mu);
  if (tid < 64) {
    const int c = cg + tid;
    float sc = 1.f, sh = 0.f;
    if (c < C) bn_src_affine(A, c, C, first, sc, sh);
    sa[0][tid] = sc;
    sa[1][tid] = sh;
  } else if (RES == 2 && tid < 128) {
    const int c = cg + tid - 64;
    float sc = 1.f, sh = 0.f;
    if (c < C) bn_src_affine(R, c, C, first, sc, sh);
    sr[0][tid - 64] = sc;
    sr[1][tid - 64] = sh;
  }
  if (first && blockIdx.x == 0 && tid == 0) {
    if (A.acc && A.fin.nbt) *A.fin.nbt += 1;
    if (RES == 2 && R.acc && R.fin.nbt) *R.fin.nbt += 1;
  }
  __syncthreads();
  if (c0 >= C) return;
  float s8[8], h8[8], rs8[8], rh8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s8[k] = sa[0][cl + k];
    h8[k] = sa[1][cl + k];
    if (RES == 2) {
      rs8[k] = sr[0][cl + k];
      rh8[k] = sr[1][cl + k];
    }
  }
  const float dsc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (; mu < mend; mu += 32 * U) {
    if (mu != mbeg + (tid >> 3)) load(mu);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = mu + 32 * u;
      if (m >= mend) break;
      float v[8];
      unpack8(xr[u], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = v[k] * s8[k] + h8[k];
      if (RES != 0) {
        float r[8];
        unpack8(rr[u], r);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += RES == 2 ? r[k] * rs8[k] + rh8[k] : r[k];
      }
      if constexpr (ACT == DMF_ACT_GELU) {
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
          const dmf_f2 g = gelu_f2(dmf_f2{v[k], v[k + 1]});
          v[k] = g.x;
          v[k + 1] = g.y;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (ACT == DMF_ACT_RELU) v[k] = fmaxf(v[k], 0.f);
          else if (ACT == DMF_ACT_SIGMOID) v[k] = sigmoid_f(v[k]);
        }
      }
      if (p > 0.f) {
        bool keep[4];
        dropout_keep4v(rseed_, roff_, site, (unsigned long long)m * C + c0, p, keep);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = keep[k] ? v[k] * dsc : 0.f;
        dropout_keep4v(rseed_, roff_, site, (unsigned long long)m * C + c0 + 4, p, keep);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[4 + k] = keep[k] ? v[4 + k] * dsc : 0.f;
      }
      st8(y + (size_t)m * ldy + c0, v);
    }
  }
}

// dz = dy * drop' * act'(z), z recomputed exactly as in k_affine_act
template <typename T>
__global__ void k_act_bwd(const T* __restrict__ dy, int lddy, const T* __restrict__ x, int ldx,
                          const float* __restrict__ ssa, const T* __restrict__ res, int ldr,
                          const float* __restrict__ ssr, int act, float p, const unsigned long long* rng, int site,
                          T* __restrict__ dz, int lddz, long long M, int C) {
  const unsigned long long rseed_ = rng ? rng[0] : 0ull, roff_ = rng ? rng[1] : 0ull;  // read once (see dropout_keep4v)
  constexpr int V = 4;
  const int cv = C / V;
  const long long total = M * cv;
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long m = i / cv;
    const int c0 = (int)(i - m * cv) * V;
    bool keep[4] = {true, true, true, true};
    if (p > 0.f) dropout_keep4v(rseed_, roff_, site, (unsigned long long)(m * C + c0), p, keep);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float g = ld(dy + m * lddy + c0 + k);
      if (p > 0.f) g = keep[k] ? g * sc : 0.f;
      if (act != DMF_ACT_NONE) {
        float z = ld(x + m * ldx + c0 + k);
        if (ssa) z = z * ssa[c0 + k] + ssa[C + c0 + k];
        if (res) {
          float r = ld(res + m * ldr + c0 + k);
          if (ssr) r = r * ssr[c0 + k] + ssr[C + c0 + k];
          z += r;
        }
        g *= act_grad(act, z);
      }
      st(dz + m * lddz + c0 + k, g);
    }
  }
}

// per-tile column sums of dz and dz*xhat: part[tile][c] = (sum dz, sum dz*(x-mean)*inv)
// block = 256 threads = 64 channel lanes x 4 row lanes, tile = 256 rows
template <typename T>
__global__ void k_bn_bwd_reduce(const T* __restrict__ dz, int lddz, const T* __restrict__ x, int ldx,
                                const float* __restrict__ save, long long M, int C, float* __restrict__ part) {
  __shared__ float red[4][64][2];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  const long long r0 = (long long)blockIdx.x * 256;
  float s = 0.f, q = 0.f;
  if (c < C) {
    const float mean = x ? save[c] : 0.f, inv = x ? save[C + c] : 0.f;
    for (int r = rl; r < 256; r += 4) {
      const long long m = r0 + r;
      if (m >= M) break;
      const float g = ld(dz + m * lddz + c);
      s += g;
      if (x) q += g * (ld(x + m * ldx + c) - mean) * inv;
    }
  }
  red[rl][cl][0] = s;
  red[rl][cl][1] = q;
  __syncthreads();
  if (rl == 0 && c < C) {
    s = red[0][cl][0] + red[1][cl][0] + red[2][cl][0] + red[3][cl][0];
    q = red[0][cl][1] + red[1][cl][1] + red[2][cl][1] + red[3][cl][1];
    *(float2*)(part + ((size_t)blockIdx.x * C + c) * 2) = make_float2(s, q);
  }
}

// k_bn_bwd_reduce on 8-channel vectors: block = 32 row lanes x 8 channel lanes of
// 8 channels (64 channels), 16-B loads (the scalar form moves 2 B per lane per
// load: ~3 TB/s on the 1024-channel shortcut BatchNorms); same tile = 256 rows
// and the same partial slab
template <typename T>
__global__ void __launch_bounds__(256) k_bn_bwd_reduce8(const T* __restrict__ dz, int lddz, const T* __restrict__ x,
                                                        int ldx, const float* __restrict__ save, long long M, int C,
                                                        float* __restrict__ part) {
  __shared__ float red[32][65 * 2];
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.y * 64 + cl * 8;
  const long long r0 = (long long)blockIdx.x * 256;
  float s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s[e] = 0.f; q[e] = 0.f; }
  if (c0 < C) {
    float mean[8], inv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mean[e] = x ? save[c0 + e] : 0.f;
      inv[e] = x ? save[C + c0 + e] : 0.f;
    }
    for (int r = rl; r < 256; r += 32) {
      const long long m = r0 + r;
      if (m >= M) break;
      float g[8];
      ld8(dz + m * lddz + c0, g);
      if (x) {
        float xv[8];
        ld8(x + m * ldx + c0, xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) q[e] += g[e] * (xv[e] - mean[e]) * inv[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += g[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[rl][(cl * 8 + e) * 2] = s[e];
    red[rl][(cl * 8 + e) * 2 + 1] = q[e];
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int c = threadIdx.x >> 1, w = threadIdx.x & 1;
    float t = 0.f;
#pragma unroll 8
    for (int r = 0; r < 32; ++r) t += red[r][c * 2 + w];
    const int cg = blockIdx.y * 64 + c;
    if (cg < C) part[((size_t)blockIdx.x * C + cg) * 2 + w] = t;
  }
}

// sum tiles -> dbeta (=sum dz), dgamma (=sum dz*xhat) (accumulated into the
// fp32 grads if given) and dx coefficients coef[3][C]: dx = A*dz + Cc*x + B
__global__ void k_bn_bwd_finalize(const float* __restrict__ part, int T, int C, double count, int training,
                                  const float* __restrict__ gamma, const float* __restrict__ save,
                                  float* dgamma, float* dbeta, float* __restrict__ coef) {
  __shared__ double red[4][64][2];
  const int cl = threadIdx.x & 63, tl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s = 0.0, q = 0.0;
  if (c < C)
    for (int t = tl; t < T; t += 4) {
      const float2 v = *(const float2*)(part + ((size_t)t * C + c) * 2);
      s += v.x;
      q += v.y;
    }
  red[tl][cl][0] = s;
  red[tl][cl][1] = q;
  __syncthreads();
  if (tl == 0 && c < C) {
    s = red[0][cl][0] + red[1][cl][0] + red[2][cl][0] + red[3][cl][0];
    q = red[0][cl][1] + red[1][cl][1] + red[2][cl][1] + red[3][cl][1];
    if (dbeta) dbeta[c] += (float)s;
    if (dgamma) dgamma[c] += (float)q;
    if (coef) {
      const double g = gamma ? gamma[c] : 1.0;
      const double mean = save[c], inv = save[C + c];
      const double A = g * inv;
      // eval-mode BN (running stats) is a per-channel affine: dx = A*dz
      const double Cc = training ? -g * inv * inv * q / count : 0.0;
      const double B = training ? -g * inv * s / count - Cc * mean : 0.0;
      coef[c] = (float)A;
      coef[C + c] = (float)Cc;
      coef[2 * C + c] = (float)B;
    }
  }
}

template <typename T>
__global__ void k_bn_bwd_apply(const T* __restrict__ dz, int lddz, const T* __restrict__ x, int ldx,
                               const float* __restrict__ coef, T* __restrict__ dx, int lddx, long long M, int C) {
  const long long total = M * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long m = i / C;
    const int c = (int)(i - m * C);
    const float v = coef[c] * ld(dz + m * lddz + c) + coef[C + c] * ld(x + m * ldx + c) + coef[2 * C + c];
    st(dx + m * lddx + c, v);
  }
}

// Fused activation/dropout backward + BatchNorm backward column reduction:
// dz (= k_act_bwd's output) is written once and the per-tile BN partials
// (sum dz, sum dz*xhat) of the same 256-row tile come out of the same pass
// (k_bn_bwd_reduce would re-read dz and x). Block = 32 row lanes x 8 channel
// lanes of 8 channels (64 channels), 16-B accesses; x is the BN input (the
// raw conv output), z = x*ssa + shift (+ residual) recomputed for act'.
// F: which optional operands the instance handles (bit 0 residual, bit 1 second gradient, bit 2 dropout),
// so the common plain-ReLU instance holds no registers for the others (occupancy: ~180 VGPRs for all)
template <typename T, int ACT, int F>
__global__ void __launch_bounds__(256, (F & 5) ? 1 : 4) k_act_bwd_bnred8(const T* __restrict__ dy, int lddy,
                                                        const T* __restrict__ dy2, int lddy2, const T* __restrict__ x,
                                                        int ldx, const float* __restrict__ ssa,
                                                        const T* __restrict__ res, int ldr,
                                                        const float* __restrict__ ssr, float p,
                                                        const unsigned long long* rng, int site,
                                                        const float* __restrict__ save, T* __restrict__ dz, int lddz,
                                                        long long M, int C, float* __restrict__ part,
                                                        double* __restrict__ acc, int replicas) {
  const unsigned long long rseed_ = rng ? rng[0] : 0ull, roff_ = rng ? rng[1] : 0ull;  // read once (see dropout_keep4v)
  constexpr bool HR = (F & 1) && ACT != DMF_ACT_NONE, HD = F & 2, HP = F & 4;
  __shared__ float red[32][65 * 2];
  __shared__ __attribute__((aligned(16))) float rss[2][64];  // the residual's BN scale / shift (HR): read per row
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * 64 + cl * 8;
  const long long r0 = (long long)blockIdx.y * 256;
  const float sc = HP && p > 0.f ? 1.f / (1.f - p) : 1.f;
  float s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s[e] = 0.f; q[e] = 0.f; }
  if constexpr (HR) {
    if (threadIdx.x < 128) {
      const int c = blockIdx.x * 64 + (threadIdx.x & 63), w = threadIdx.x >> 6;
      rss[w][threadIdx.x & 63] = c < C && ssr ? ssr[w * C + c] : (w == 0 ? 1.f : 0.f);
    }
    __syncthreads();
  }
  if (c0 < C) {
    float mean[8], inv[8], a[8], b[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mean[e] = save[c0 + e];
      inv[e] = save[C + c0 + e];
      a[e] = ssa[c0 + e];
      b[e] = ssa[C + c0 + e];
    }
    // 8 rows per thread in two batches of 4, every load of a batch issued before any row is
    // converted: one row at a time left each thread with 2 loads in flight and the kernel
    // latency-bound at ~2.5 TB/s
    constexpr int RB = (HR || HD) ? 2 : 4;  // rows per batch: keep the 3- and 4-operand forms near 128 VGPRs
#pragma unroll 1
    for (int jb = 0; jb < 8; jb += RB) {
      Vec8<T> vg[RB], vg2[RB], vx[RB], vr[RB];
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        const long long m = r0 + rl + 32 * (jb + j);
        const bool in = m < M;
        vg[j] = in ? ldv8(dy + m * lddy + c0) : zero8<T>();
        if constexpr (HD) vg2[j] = in && dy2 ? ldv8(dy2 + m * lddy2 + c0) : zero8<T>();
        vx[j] = in ? ldv8(x + m * ldx + c0) : zero8<T>();
        if constexpr (HR) vr[j] = in && res ? ldv8(res + m * ldr + c0) : zero8<T>();
      }
#pragma unroll
      for (int j = 0; j < RB; ++j) {
      const long long m = r0 + rl + 32 * (jb + j);
      if (m >= M) break;
      float g[8], xv[8];
      unpack8(vg[j], g);
      if constexpr (HD) {
        // a second gradient of the same output (the next block's shortcut), summed here in fp32
        // instead of by a separate add pass
        float g2[8];
        unpack8(vg2[j], g2);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] += g2[e];
      }
      unpack8(vx[j], xv);
      if (HP && p > 0.f) {
        bool keep[4];
        dropout_keep4v(rseed_, roff_, site, (unsigned long long)m * C + c0, p, keep);
#pragma unroll
        for (int k = 0; k < 4; ++k) g[k] = keep[k] ? g[k] * sc : 0.f;
        dropout_keep4v(rseed_, roff_, site, (unsigned long long)m * C + c0 + 4, p, keep);
#pragma unroll
        for (int k = 0; k < 4; ++k) g[4 + k] = keep[k] ? g[4 + k] * sc : 0.f;
      }
      if (ACT != DMF_ACT_NONE) {
        float z[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) z[e] = xv[e] * a[e] + b[e];
        if constexpr (HR) {
          float rv[8];
          unpack8(vr[j], rv);
          const float4 ra0 = *(const float4*)&rss[0][cl * 8], ra1 = *(const float4*)&rss[0][cl * 8 + 4];
          const float4 rb0 = *(const float4*)&rss[1][cl * 8], rb1 = *(const float4*)&rss[1][cl * 8 + 4];
          const float ra[8] = {ra0.x, ra0.y, ra0.z, ra0.w, ra1.x, ra1.y, ra1.z, ra1.w};
          const float rb[8] = {rb0.x, rb0.y, rb0.z, rb0.w, rb1.x, rb1.y, rb1.z, rb1.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) z[e] += rv[e] * ra[e] + rb[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] *= act_grad(ACT, z[e]);
      }
      st8(dz + m * lddz + c0, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s[e] += g[e];
        q[e] += g[e] * (xv[e] - mean[e]) * inv[e];
      }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[rl][(cl * 8 + e) * 2] = s[e];
    red[rl][(cl * 8 + e) * 2 + 1] = q[e];
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int c = threadIdx.x >> 1, w = threadIdx.x & 1;
    float t = 0.f;
#pragma unroll 8
    for (int r = 0; r < 32; ++r) t += red[r][c * 2 + w];
    const int cg = blockIdx.x * 64 + c;
    if (cg < C) {
      if (acc) unsafeAtomicAdd(acc + ((size_t)(blockIdx.y % (unsigned)replicas) * C + cg) * 2 + w, (double)t);
      else part[((size_t)blockIdx.y * C + cg) * 2 + w] = t;
    }
  }
}

// BN backward apply, 8 channels per thread: dx = A*dz + Cc*x + B
template <typename T>
__global__ void k_bn_bwd_apply8(const T* __restrict__ dz, int lddz, const T* __restrict__ x, int ldx,
                                const float* __restrict__ coef, T* __restrict__ dx, int lddx, long long M, int C) {
  const unsigned cv = (unsigned)C >> 3;
  const unsigned total = (unsigned)(M * cv);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const unsigned m = i / cv;
    const int c0 = (int)(i - m * cv) << 3;
    float g[8], xv[8];
    ld8(dz + (size_t)m * lddz + c0, g);
    ld8(x + (size_t)m * ldx + c0, xv);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = coef[c0 + e] * g[e] + coef[C + c0 + e] * xv[e] + coef[2 * C + c0 + e];
    st8(dx + (size_t)m * lddx + c0, g);
  }
}

// BN backward apply with the finalize folded in (dmf_bn_bwd_apply_acc): block =
// 64 channels (blockIdx.x) x rows_per_blk pixels (blockIdx.y); its 64 (A, Cc, B) come from the
// column sums accumulated by dmf_act_bwd_bn_reduce_acc into [replicas][C][2]
// doubles (summed in a fixed order, the arithmetic of k_bn_bwd_finalize_wide);
// the blockIdx.x == 0 blocks also add dgamma / dbeta. dx = A*dz + Cc*x + B.
template <typename T, int U = 1>
__global__ void __launch_bounds__(256) k_bn_bwd_apply_acc(const T* __restrict__ dz, int lddz, const T* __restrict__ x,
                                                          int ldx, const double* __restrict__ acc, int replicas,
                                                          double count, int training, const float* __restrict__ gamma,
                                                          const float* __restrict__ save, float* dgamma, float* dbeta,
                                                          T* __restrict__ dx, int lddx, int M, int C,
                                                          int rows_per_blk) {
  __shared__ float sco[3][64];
  const int tid = threadIdx.x;
  const int cg = blockIdx.x * 64;
  const int cl = (tid & 7) * 8, c0 = cg + cl;
  const int mbeg = blockIdx.y * rows_per_blk;
  const int mend = min(M, mbeg + rows_per_blk);
  // U rows per thread per round, every load of the round issued before any row is converted; the
  // first round's loads go out before the finalize prologue (its arena reads hide under them)
  Vec8<T> vg[U], vx[U];
  auto load = [&](int m) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int mu = m + 32 * u;
      vg[u] = mu < mend ? ldv8(dz + (size_t)mu * lddz + c0) : zero8<T>();
      vx[u] = mu < mend ? ldv8(x + (size_t)mu * ldx + c0) : zero8<T>();
    }
  };
  int m = mbeg + (tid >> 3);
  if (c0 < C) load(m);
  if (tid < 64) {
    const int c = cg + tid;
    float A = 0.f, Cc = 0.f, B = 0.f;
    if (c < C) {
      double s = 0.0, q = 0.0;
      for (int r = 0; r < replicas; ++r) {  // fixed order
        s += acc[((size_t)r * C + c) * 2];
        q += acc[((size_t)r * C + c) * 2 + 1];
      }
      if (blockIdx.y == 0) {
        if (dbeta) dbeta[c] += (float)s;
        if (dgamma) dgamma[c] += (float)q;
      }
      const double g = gamma ? gamma[c] : 1.0;
      const double mean = save[c], inv = save[C + c];
      const double a = g * inv;
      const double cc = training ? -g * inv * inv * q / count : 0.0;
      const double b = training ? -g * inv * s / count - cc * mean : 0.0;
      A = (float)a;
      Cc = (float)cc;
      B = (float)b;
    }
    sco[0][tid] = A;
    sco[1][tid] = Cc;
    sco[2][tid] = B;
  }
  __syncthreads();
  if (c0 >= C) return;
  float a8[8], c8[8], b8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a8[k] = sco[0][cl + k];
    c8[k] = sco[1][cl + k];
    b8[k] = sco[2][cl + k];
  }
  for (; m < mend; m += 32 * U) {
    if (m != mbeg + (tid >> 3)) load(m);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int mu = m + 32 * u;
      if (mu >= mend) break;
      float g[8], xv[8];
      unpack8(vg[u], g);
      unpack8(vx[u], xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = a8[e] * g[e] + c8[e] * xv[e] + b8[e];
      st8(dx + (size_t)mu * lddx + c0, g);
    }
  }
}


// dmf_bn_bwd_finalize for many tiles: 16 channels x 64 tile lanes per block
__global__ void __launch_bounds__(1024) k_bn_bwd_finalize_wide(const float* __restrict__ part, int T, int C,
                                                               double count, int training,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ save, float* dgamma,
                                                               float* dbeta, float* __restrict__ coef) {
  __shared__ double red[64][16][2];
  const int cl = threadIdx.x & 15, tl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double s = 0.0, q = 0.0;
  if (c < C)
    for (int t = tl; t < T; t += 64) {
      const float2 v = *(const float2*)(part + ((size_t)t * C + c) * 2);
      s += v.x;
      q += v.y;
    }
  red[tl][cl][0] = s;
  red[tl][cl][1] = q;
  __syncthreads();
  for (int o = 32; o > 0; o >>= 1) {
    if (tl < o) {
      red[tl][cl][0] += red[tl + o][cl][0];
      red[tl][cl][1] += red[tl + o][cl][1];
    }
    __syncthreads();
  }
  if (tl == 0 && c < C) {
    s = red[0][cl][0];
    q = red[0][cl][1];
    if (dbeta) dbeta[c] += (float)s;
    if (dgamma) dgamma[c] += (float)q;
    if (coef) {
      const double g = gamma ? gamma[c] : 1.0;
      const double mean = save[c], inv = save[C + c];
      const double A = g * inv;
      const double Cc = training ? -g * inv * inv * q / count : 0.0;
      const double B = training ? -g * inv * s / count - Cc * mean : 0.0;
      coef[c] = (float)A;
      coef[C + c] = (float)Cc;
      coef[2 * C + c] = (float)B;
    }
  }
}

static inline int grid_for(long long n, int block = 256) {
  long long g = (n + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace dmf

using namespace dmf;

extern "C" int dmf_bn_finalize_ws_size(int ntiles, int C) {
  return ntiles <= 1024 ? 0 : ((ntiles + 31) / 32) * C * 2;
}

extern "C" int dmf_bn_finalize(const float* partials, int ntiles, int C, double count, double unbias_count,
                               const float* gamma, const float* beta, float* running_mean, float* running_var,
                               long long* num_batches_tracked, float momentum, float eps, int training,
                               float* scale_shift, float* save_mean_invstd, double* workspace, void* stream) {
  DMF_CHECK_ARG(C > 0 && scale_shift, "dmf_bn_finalize: bad args");
  DMF_CHECK_ARG(!training || (partials && ntiles > 0 && count > 0), "dmf_bn_finalize: training needs partials");
  DMF_CHECK_ARG(training || (running_mean && running_var), "dmf_bn_finalize: eval needs running stats");
  hipStream_t st_ = (hipStream_t)stream;
  BnFin f{gamma, beta, running_mean, running_var, num_batches_tracked, momentum, eps, count, unbias_count, training,
          scale_shift, save_mean_invstd};
  if (training && ntiles > 64 && ntiles <= 1024) {
    hipLaunchKernelGGL(k_bn_finalize_wide, dim3(cdiv(C, 16)), dim3(1024), 0, st_, partials, ntiles, C, f);
  } else if (training && ntiles > 64) {
    DMF_CHECK_ARG(workspace, "dmf_bn_finalize: %d tiles need a workspace (dmf_bn_finalize_ws_size)", ntiles);
    const int S = (ntiles + 31) / 32;
    hipLaunchKernelGGL(k_bn_stage1, dim3(cdiv(C, 64), S), dim3(256), 0, st_, partials, ntiles, C, 32, workspace);
    hipLaunchKernelGGL(k_bn_finalize<double>, dim3(cdiv(C, 64)), dim3(256), 0, st_, (const double*)workspace, S, C,
                       f);
  } else {
    hipLaunchKernelGGL(k_bn_finalize<float>, dim3(cdiv(C, 64)), dim3(256), 0, st_, partials, ntiles, C, f);
  }
  DMF_LAUNCH_CHECK("dmf_bn_finalize");
  return 0;
}

extern "C" int dmf_bn_finalize_acc(const double* acc, int replicas, int C, double count, double unbias_count,
                                   const float* gamma, const float* beta, float* running_mean, float* running_var,
                                   long long* num_batches_tracked, float momentum, float eps, float* scale_shift,
                                   float* save_mean_invstd, void* stream) {
  DMF_CHECK_ARG(acc && replicas >= 1 && replicas <= 64 && C > 0 && count > 0 && scale_shift,
                "dmf_bn_finalize_acc: bad args");
  BnFin f{gamma, beta, running_mean, running_var, num_batches_tracked, momentum, eps, count, unbias_count, 1,
          scale_shift, save_mean_invstd};
  hipLaunchKernelGGL(k_bn_finalize<double>, dim3(cdiv(C, 64)), dim3(256), 0, (hipStream_t)stream, acc, replicas, C,
                     f);
  DMF_LAUNCH_CHECK("dmf_bn_finalize_acc");
  return 0;
}

extern "C" int dmf_affine_act(int dtype, const void* x, int ldx, const float* scale_shift, const void* res, int ldr,
                              const float* res_scale_shift, int act, float dropout_p,
                              const unsigned long long* rng, int site, void* y, int ldy, long long M, int C,
                              void* stream) {
  DMF_CHECK_ARG(C % 4 == 0, "dmf_affine_act: C=%d must be a multiple of 4", C);
  DMF_CHECK_ARG(dropout_p <= 0.f || rng, "dmf_affine_act: dropout needs rng state");
  DMF_CHECK_ARG(dropout_p < 1.f, "dmf_affine_act: dropout p must be < 1");
  if (M == 0) return 0;
  const bool vec8 = C % 8 == 0 && M * (C / 8) < (1LL << 31) && ldx % 8 == 0 && ldy % 8 == 0 && (!res || ldr % 8 == 0) &&
                    ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0 && (!res || ((uintptr_t)res % 16) == 0) &&
                    (!scale_shift || ((uintptr_t)scale_shift % 16) == 0);
  if (vec8) {
    const int g8 = grid_for(M * (C / 8));
    hipStream_t s = (hipStream_t)stream;
#define DMF_AA8(TT, A)                                                                                          \
  hipLaunchKernelGGL((k_affine_act8<TT, A>), dim3(g8), dim3(256), 0, s, (const TT*)x, ldx, scale_shift,          \
                     (const TT*)res, ldr, res_scale_shift, dropout_p, rng, site, (TT*)y, ldy, M, C)
    DMF_DISPATCH_DTYPE(dtype, T, switch (act) {
        case DMF_ACT_RELU: DMF_AA8(T, DMF_ACT_RELU); break;
        case DMF_ACT_GELU: DMF_AA8(T, DMF_ACT_GELU); break;
        case DMF_ACT_SIGMOID: DMF_AA8(T, DMF_ACT_SIGMOID); break;
        default: DMF_AA8(T, DMF_ACT_NONE);
      });
#undef DMF_AA8
    DMF_LAUNCH_CHECK("dmf_affine_act");
    return 0;
  }
  const int g = grid_for(M * (C / 4));
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_affine_act<T>, dim3(g), dim3(256), 0, (hipStream_t)stream, (const T*)x, ldx,
                       scale_shift, (const T*)res, ldr, res_scale_shift, act, dropout_p, rng, site, (T*)y,
                       ldy, M, C));
  DMF_LAUNCH_CHECK("dmf_affine_act");
  return 0;
}


static BnApplySrc bn_src(const dmf_bn_desc* d, const float* ss) {
  BnApplySrc s{};
  if (d) {
    s.acc = d->acc;
    s.fin = BnFin{d->gamma, d->beta, d->running_mean, d->running_var, d->num_batches_tracked, d->momentum, d->eps,
                  d->count, d->unbias_count, 1, d->scale_shift, d->save_mean_invstd};
    s.replicas = d->replicas;
  } else {
    s.ss = ss;
  }
  return s;
}

extern "C" int dmf_bn_apply(int dtype, const void* x, int ldx, const dmf_bn_desc* bn, const float* scale_shift,
                            const void* res, int ldr, const dmf_bn_desc* res_bn, const float* res_scale_shift, int act,
                            float dropout_p, const unsigned long long* rng, int site, void* y, int ldy, long long M,
                            int C, void* stream) {
  DMF_CHECK_ARG(dtype == DMF_F32 || is16(dtype), "dmf_bn_apply: bad dtype %d", dtype);
  DMF_CHECK_ARG(C > 0 && C % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 && (!res || ldr % 8 == 0),
                "dmf_bn_apply: C=%d and strides must be multiples of 8", C);
  DMF_CHECK_ARG(M < (1LL << 31), "dmf_bn_apply: M=%lld too large", M);
  DMF_CHECK_ARG(((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0 && (!res || ((uintptr_t)res % 16) == 0),
                "dmf_bn_apply: pointers must be 16-byte aligned");
  DMF_CHECK_ARG(!bn || (bn->acc && bn->scale_shift && bn->count > 0 && bn->replicas >= 1 && bn->replicas <= 64),
                "dmf_bn_apply: bad batch-norm descriptor");
  DMF_CHECK_ARG(!res_bn || (res && res_bn->acc && res_bn->scale_shift && res_bn->count > 0 && res_bn->replicas >= 1 &&
                            res_bn->replicas <= 64),
                "dmf_bn_apply: bad residual batch-norm descriptor");
  DMF_CHECK_ARG(dropout_p <= 0.f || rng, "dmf_bn_apply: dropout needs rng state");
  DMF_CHECK_ARG(dropout_p < 1.f, "dmf_bn_apply: dropout p must be < 1");
  if (M == 0) return 0;
  const BnApplySrc A = bn_src(bn, scale_shift);
  const BnApplySrc R = bn_src(res_bn, res_scale_shift);
  const int gy = cdiv(C, 64);
  // ~8 row iterations per thread, but at least ~1024 blocks in flight
  int rows = 256;
  while (rows > 32 && (long long)cdiv(M, rows) * gy < 1024) rows >>= 1;
  // (gridDim.y <= 65535: beyond 16.7 M rows each block walks more rows)
  if (cdiv(M, rows) > 65535) rows = (int)(cdiv(cdiv(M, 65535), 32) * 32);
  const dim3 g((unsigned)gy, (unsigned)cdiv(M, rows));  // channel groups fastest: resident blocks cover whole rows
  const int resk = res == nullptr ? 0 : ((res_bn || res_scale_shift) ? 2 : 1);
  hipStream_t s = (hipStream_t)stream;
#define DMF_BA_U(TT, AC, RK, UU)                                                                             \
  hipLaunchKernelGGL((k_bn_apply<TT, AC, RK, UU>), g, dim3(256), 0, s, (const TT*)x, ldx, A, (const TT*)res, ldr, \
                     R, dropout_p, rng, site, (TT*)y, ldy, (int)M, C, rows)
// (2 or 4 rows of loads in flight per thread computed the same bits and measured within noise or slower,
// round 5: profiles/r05fb_apply_rows{1,2,4}.txt, r05fb_modeA_apply_rows_ab.txt; the launch path is U = 1)
#define DMF_BA(TT, AC, RK) DMF_BA_U(TT, AC, RK, 1)
#define DMF_BA_R(TT, AC)                 \
  do {                                   \
    if (resk == 0) DMF_BA(TT, AC, 0);     \
    else if (resk == 1) DMF_BA(TT, AC, 1); \
    else DMF_BA(TT, AC, 2);               \
  } while (0)
#define DMF_BA_A(TT)                                      \
  do {                                                    \
    switch (act) {                                        \
      case DMF_ACT_RELU: DMF_BA_R(TT, DMF_ACT_RELU); break; \
      case DMF_ACT_GELU: DMF_BA_R(TT, DMF_ACT_GELU); break; \
      case DMF_ACT_SIGMOID: DMF_BA_R(TT, DMF_ACT_SIGMOID); break; \
      default: DMF_BA_R(TT, DMF_ACT_NONE);                \
    }                                                     \
  } while (0)
  DMF_DISPATCH_DTYPE(dtype, T, DMF_BA_A(T));
#undef DMF_BA_A
#undef DMF_BA_R
#undef DMF_BA
#undef DMF_BA_U
  DMF_LAUNCH_CHECK("dmf_bn_apply");
  return 0;
}

extern "C" int dmf_act_bwd(int dtype, const void* dy, int lddy, const void* x, int ldx, const float* scale_shift,
                           const void* res, int ldr, const float* res_scale_shift, int act, float dropout_p,
                           const unsigned long long* rng, int site, void* dz, int lddz, long long M, int C,
                           void* stream) {
  DMF_CHECK_ARG(C % 4 == 0, "dmf_act_bwd: C=%d must be a multiple of 4", C);
  DMF_CHECK_ARG(dropout_p <= 0.f || rng, "dmf_act_bwd: dropout needs rng state");
  DMF_CHECK_ARG(act == DMF_ACT_NONE || x, "dmf_act_bwd: activation backward needs x");
  if (M == 0) return 0;
  const int g = grid_for(M * (C / 4));
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_act_bwd<T>, dim3(g), dim3(256), 0, (hipStream_t)stream, (const T*)dy, lddy,
                       (const T*)x, ldx, scale_shift, (const T*)res, ldr, res_scale_shift, act, dropout_p,
                       rng, site, (T*)dz, lddz, M, C));
  DMF_LAUNCH_CHECK("dmf_act_bwd");
  return 0;
}

extern "C" int dmf_bn_bwd_tiles(long long M) { return (int)((M + 255) / 256); }

extern "C" int dmf_bn_bwd_reduce(int dtype, const void* dz, int lddz, const void* x, int ldx,
                                 const float* save_mean_invstd, long long M, int C, float* partials, void* stream) {
  DMF_CHECK_ARG(M > 0 && C > 0 && partials, "dmf_bn_bwd_reduce: bad args");
  DMF_CHECK_ARG(!x || save_mean_invstd, "dmf_bn_bwd_reduce: x given without saved stats");
  const long long tiles = (M + 255) / 256;
  DMF_CHECK_ARG(tiles < 65536LL * 32768LL, "dmf_bn_bwd_reduce: too many rows");
  dim3 grid((unsigned)tiles, (unsigned)cdiv(C, 64));
  if (C % 8 == 0 && lddz % 8 == 0 && (!x || ldx % 8 == 0) &&
      ((uintptr_t)dz | (uintptr_t)(x ? x : dz)) % 16 == 0) {
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_bn_bwd_reduce8<T>, grid, dim3(256), 0, (hipStream_t)stream, (const T*)dz, lddz,
                         (const T*)x, ldx, save_mean_invstd, M, C, partials));
  } else DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_bn_bwd_reduce<T>, grid, dim3(256), 0, (hipStream_t)stream, (const T*)dz, lddz,
                       (const T*)x, ldx, save_mean_invstd, M, C, partials));
  DMF_LAUNCH_CHECK("dmf_bn_bwd_reduce");
  return 0;
}

extern "C" int dmf_bn_bwd_finalize(const float* partials, int ntiles, int C, double count, int training,
                                   const float* gamma, const float* save_mean_invstd, float* dgamma, float* dbeta,
                                   float* coef, void* stream) {
  DMF_CHECK_ARG(partials && ntiles > 0 && C > 0, "dmf_bn_bwd_finalize: bad args");
  DMF_CHECK_ARG(!coef || save_mean_invstd, "dmf_bn_bwd_finalize: coef needs saved stats");
  if (ntiles > 64)
    hipLaunchKernelGGL(k_bn_bwd_finalize_wide, dim3(cdiv(C, 16)), dim3(1024), 0, (hipStream_t)stream, partials, ntiles,
                       C, count, training, gamma, save_mean_invstd, dgamma, dbeta, coef);
  else
    hipLaunchKernelGGL(k_bn_bwd_finalize, dim3(cdiv(C, 64)), dim3(256), 0, (hipStream_t)stream, partials, ntiles, C,
                       count, training, gamma, save_mean_invstd, dgamma, dbeta, coef);
  DMF_LAUNCH_CHECK("dmf_bn_bwd_finalize");
  return 0;
}

extern "C" int dmf_bn_bwd_apply(int dtype, const void* dz, int lddz, const void* x, int ldx, const float* coef,
                                void* dx, int lddx, long long M, int C, void* stream) {
  DMF_CHECK_ARG(dz && x && coef && dx, "dmf_bn_bwd_apply: bad args");
  if (M == 0) return 0;
  if (C % 8 == 0 && ldx % 8 == 0 && lddz % 8 == 0 && lddx % 8 == 0 && M * (C / 8) < (1LL << 31) &&
      ((uintptr_t)dz | (uintptr_t)x | (uintptr_t)dx) % 16 == 0) {
    const int g8 = grid_for(M * (C / 8));
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_bn_bwd_apply8<T>, dim3(g8), dim3(256), 0, (hipStream_t)stream, (const T*)dz,
                         lddz, (const T*)x, ldx, coef, (T*)dx, lddx, M, C));
    DMF_LAUNCH_CHECK("dmf_bn_bwd_apply");
    return 0;
  }
  const int g = grid_for(M * C);
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_bn_bwd_apply<T>, dim3(g), dim3(256), 0, (hipStream_t)stream, (const T*)dz, lddz,
                       (const T*)x, ldx, coef, (T*)dx, lddx, M, C));
  DMF_LAUNCH_CHECK("dmf_bn_bwd_apply");
  return 0;
}

static int act_bwd_bn_reduce_impl(int dtype, const void* dy, int lddy, const void* dy2, int lddy2, const void* x,
                                  int ldx, const float* scale_shift, const void* res, int ldr,
                                  const float* res_scale_shift, int act, float dropout_p,
                                  const unsigned long long* rng, int site, const float* save_mean_invstd, void* dz,
                                  int lddz, long long M, int C, float* partials, double* acc, int replicas,
                                  void* stream);

extern "C" int dmf_act_bwd_bn_reduce(int dtype, const void* dy, int lddy, const void* dy2, int lddy2, const void* x,
                                     int ldx, const float* scale_shift, const void* res, int ldr,
                                     const float* res_scale_shift, int act, float dropout_p,
                                     const unsigned long long* rng, int site, const float* save_mean_invstd, void* dz,
                                     int lddz, long long M, int C, float* partials, void* stream) {
  DMF_CHECK_ARG(partials, "dmf_act_bwd_bn_reduce: bad args");
  return act_bwd_bn_reduce_impl(dtype, dy, lddy, dy2, lddy2, x, ldx, scale_shift, res, ldr, res_scale_shift, act,
                                dropout_p, rng, site, save_mean_invstd, dz, lddz, M, C, partials, nullptr, 0, stream);
}

extern "C" int dmf_act_bwd_bn_reduce_acc(int dtype, const void* dy, int lddy, const void* dy2, int lddy2,
                                         const void* x, int ldx, const float* scale_shift, const void* res, int ldr,
                                         const float* res_scale_shift, int act, float dropout_p,
                                         const unsigned long long* rng, int site, const float* save_mean_invstd,
                                         void* dz, int lddz, long long M, int C, double* acc, int replicas,
                                         void* stream) {
  DMF_CHECK_ARG(acc && ((uintptr_t)acc % 8) == 0 && replicas >= 1 && replicas <= 64,
                "dmf_act_bwd_bn_reduce_acc: bad statistics arena");
  DMF_CHECK_ARG(C % 8 == 0 && lddy % 8 == 0 && ldx % 8 == 0 && lddz % 8 == 0 && (!res || ldr % 8 == 0) &&
                    ((uintptr_t)dy | (uintptr_t)x | (uintptr_t)dz | (uintptr_t)(res ? res : dz)) % 16 == 0,
                "dmf_act_bwd_bn_reduce_acc: needs 8-channel vectors (C=%d)", C);
  return act_bwd_bn_reduce_impl(dtype, dy, lddy, dy2, lddy2, x, ldx, scale_shift, res, ldr, res_scale_shift, act,
                                dropout_p, rng, site, save_mean_invstd, dz, lddz, M, C, nullptr, acc, replicas, stream);
}

extern "C" int dmf_bn_bwd_apply_acc(int dtype, const void* dz, int lddz, const void* x, int ldx, const double* acc,
                                    int replicas, double count, int training, const float* gamma,
                                    const float* save_mean_invstd, float* dgamma, float* dbeta, void* dx, int lddx,
                                    long long M, int C, void* stream) {
  DMF_CHECK_ARG(dz && x && acc && save_mean_invstd && dx && count > 0 && replicas >= 1 && replicas <= 64,
                "dmf_bn_bwd_apply_acc: bad args");
  DMF_CHECK_ARG(C % 8 == 0 && lddz % 8 == 0 && ldx % 8 == 0 && lddx % 8 == 0 && M < (1LL << 31) &&
                    ((uintptr_t)dz | (uintptr_t)x | (uintptr_t)dx) % 16 == 0,
                "dmf_bn_bwd_apply_acc: needs 8-channel vectors (C=%d)", C);
  if (M == 0) return 0;
  const int gy = cdiv(C, 64);
  int rows = 256;
  while (rows > 32 && (long long)cdiv(M, rows) * gy < 1024) rows >>= 1;
  if (cdiv(M, rows) > 65535) rows = (int)(cdiv(cdiv(M, 65535), 32) * 32);  // (gridDim.y <= 65535)
  const dim3 g((unsigned)gy, (unsigned)cdiv(M, rows));  // channel groups fastest: resident blocks cover whole rows
#define DMF_BBA(U)                                                                                          \
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((k_bn_bwd_apply_acc<T, U>), g, dim3(256), 0, (hipStream_t)stream, \
                                                  (const T*)dz, lddz, (const T*)x, ldx, acc, replicas, count,     \
                                                  training, gamma, save_mean_invstd, dgamma, dbeta, (T*)dx, lddx, \
                                                  (int)M, C, rows))
  DMF_BBA(1);  // (2 / 4 rows in flight: within noise, profiles/r05aa_bwd_apply_rows_modeB_ab.txt)
#undef DMF_BBA
  DMF_LAUNCH_CHECK("dmf_bn_bwd_apply_acc");
  return 0;
}

static int act_bwd_bn_reduce_impl(int dtype, const void* dy, int lddy, const void* dy2, int lddy2, const void* x,
                                  int ldx, const float* scale_shift, const void* res, int ldr,
                                  const float* res_scale_shift, int act, float dropout_p,
                                  const unsigned long long* rng, int site, const float* save_mean_invstd, void* dz,
                                  int lddz, long long M, int C, float* partials, double* acc, int replicas,
                                  void* stream) {
  DMF_CHECK_ARG(dy && x && scale_shift && save_mean_invstd && dz && (partials || acc) && M > 0 && C > 0,
                "dmf_act_bwd_bn_reduce: bad args");
  DMF_CHECK_ARG(dropout_p <= 0.f || rng, "dmf_act_bwd_bn_reduce: dropout needs rng state");
  // (the vector kernel's residual term is compiled in per specialisation: a shortcut BatchNorm without
  // its shortcut would add the shift alone)
  DMF_CHECK_ARG(!res_scale_shift || res, "dmf_act_bwd_bn_reduce: res_scale_shift needs res");
  const bool vec8 = C % 8 == 0 && lddy % 8 == 0 && ldx % 8 == 0 && lddz % 8 == 0 && (!res || ldr % 8 == 0) &&
                    (!dy2 || lddy2 % 8 == 0) &&
                    ((uintptr_t)dy | (uintptr_t)x | (uintptr_t)dz | (uintptr_t)(res ? res : dz) |
                     (uintptr_t)(dy2 ? dy2 : dz)) % 16 == 0;
  DMF_CHECK_ARG(vec8 || !dy2, "dmf_act_bwd_bn_reduce: a second gradient needs 8-channel vectors (C=%d)", C);
  if (!vec8) {
    int rc = dmf_act_bwd(dtype, dy, lddy, x, ldx, scale_shift, res, ldr, res_scale_shift, act, dropout_p, rng, site,
                         dz, lddz, M, C, stream);
    if (rc) return rc;
    return dmf_bn_bwd_reduce(dtype, dz, lddz, x, ldx, save_mean_invstd, M, C, partials, stream);
  }
  const long long tiles = (M + 255) / 256;
  DMF_CHECK_ARG(tiles < 65536LL, "dmf_act_bwd_bn_reduce: too many rows");
  dim3 grid((unsigned)cdiv(C, 64), (unsigned)tiles);  // channel groups fastest: resident blocks cover whole rows
  hipStream_t s = (hipStream_t)stream;
  // residual / second-gradient / dropout specialisations (k_act_bwd_bnred8's F); any dropout takes
  // the all-operands instance
  const int F = dropout_p > 0.f ? 7 : ((res && act != DMF_ACT_NONE) ? 1 : 0) | (dy2 ? 2 : 0);
#define DMF_ABR(TT, A, FF)                                                                                   \
  hipLaunchKernelGGL((k_act_bwd_bnred8<TT, A, FF>), grid, dim3(256), 0, s, (const TT*)dy, lddy, (const TT*)dy2, \
                     lddy2, (const TT*)x, ldx, scale_shift, (const TT*)res, ldr, res_scale_shift, dropout_p, rng, \
                     site, save_mean_invstd, (TT*)dz, lddz, M, C, partials, acc, replicas)
#define DMF_ABR_F(TT, A)                 \
  switch (F) {                           \
    case 0: DMF_ABR(TT, A, 0); break;    \
    case 1: DMF_ABR(TT, A, 1); break;    \
    case 2: DMF_ABR(TT, A, 2); break;    \
    case 3: DMF_ABR(TT, A, 3); break;    \
    default: DMF_ABR(TT, A, 7); break;   \
  }
  DMF_DISPATCH_DTYPE(dtype, T, switch (act) {
      case DMF_ACT_RELU: DMF_ABR_F(T, DMF_ACT_RELU); break;
      case DMF_ACT_GELU: DMF_ABR_F(T, DMF_ACT_GELU); break;
      case DMF_ACT_SIGMOID: DMF_ABR(T, DMF_ACT_SIGMOID, 7); break;
      default: DMF_ABR(T, DMF_ACT_NONE, 7);
    });
#undef DMF_ABR_F
#undef DMF_ABR
  DMF_LAUNCH_CHECK("dmf_act_bwd_bn_reduce");
  return 0;
}
