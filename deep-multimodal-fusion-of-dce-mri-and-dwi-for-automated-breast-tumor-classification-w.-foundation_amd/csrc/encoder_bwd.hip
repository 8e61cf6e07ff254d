// Backward kernels that only the all-trainable (unfrozen encoder) step needs:
//   - gated mix z = sig(w)*a + (1-sig(w))*b (model_module.py:674-675,
//     :689-690): da, db, dw
//   - MaskGuidedSpatialAttention (model_module.py:75-97): df, dmask and the
//     parameter grads, recomputing the per-pixel 16-channel mask processor
//     from the mask and the closed-form GroupNorm(1,16) statistics.
#include <algorithm>

#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

template <typename T>
__global__ void k_mix_bwd(const T* __restrict__ dz, int lddz, const T* __restrict__ a, int lda,
                          const T* __restrict__ b, int ldb, const float* __restrict__ wlogit, T* __restrict__ da,
                          T* __restrict__ db, int ldd, float* __restrict__ part, long long M, int C) {
  __shared__ float red[16];
  const float al = 1.f / (1.f + __expf(-wlogit[0]));
  float acc = 0.f;
  const long long total = M * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long m = i / C;
    const int c = (int)(i - m * C);
    const float g = ld(dz + m * lddz + c);
    const float av = ld(a + m * lda + c), bv = ld(b + m * ldb + c);
    st(da + m * ldd + c, al * g);
    st(db + m * ldd + c, (1.f - al) * g);
    acc += g * (av - bv);
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc * al * (1.f - al);
}

// 8-channel vector form (16-B accesses, 32-bit index math): the scalar form's
// per-element 64-bit divisions ran ~60 us on a 32k x 256 map
template <typename T>
__global__ void __launch_bounds__(256) k_mix_bwd8(const T* __restrict__ dz, int lddz, const T* __restrict__ a,
                                                  int lda, const T* __restrict__ b, int ldb,
                                                  const float* __restrict__ wlogit, T* __restrict__ da,
                                                  T* __restrict__ db, int ldd, float* __restrict__ part, int M, int C) {
  __shared__ float red[16];
  const float al = 1.f / (1.f + __expf(-wlogit[0]));
  const int CV = C >> 3;
  const int total = M * CV;
  float acc = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV, m = i / CV;
    float g[8], av[8], bv[8], o1[8], o2[8];
    ld8(dz + (size_t)m * lddz + cv * 8, g);
    ld8(a + (size_t)m * lda + cv * 8, av);
    ld8(b + (size_t)m * ldb + cv * 8, bv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o1[k] = al * g[k];
      o2[k] = (1.f - al) * g[k];
      acc = fmaf(g[k], av[k] - bv[k], acc);
    }
    st8(da + (size_t)m * ldd + cv * 8, o1);
    st8(db + (size_t)m * ldd + cv * 8, o2);
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc * al * (1.f - al);
}

struct MaskAttnB {
  const float* w1;
  const float* g;
  const float* b;
  const float* w2;
  const float* b2;
  const float* gamma;
  float eps;
  int hid;
};

__device__ __forceinline__ void ma_stats(const MaskAttnB& P, const float* stats, int n, int HW, float& mu, float& rs) {
  float mw = 0.f, mw2 = 0.f;
  for (int c = 0; c < P.hid; ++c) { mw += P.w1[c]; mw2 += P.w1[c] * P.w1[c]; }
  mw /= P.hid;
  mw2 /= P.hid;
  const float mm = stats[2 * n] / HW, mm2 = stats[2 * n + 1] / HW;
  mu = mw * mm;
  rs = rsqrtf(fmaxf(mw2 * mm2 - mu * mu, 0.f) + P.eps);
}

// pass 1: grid (sample, 64-pixel slice), one wave per pixel at a time.
// grads layout: [hid] dw1, [hid] dgn_w, [hid] dgn_b, [hid] dw2, [1] db2, [1] dgamma
// ws: dhh [N][HW][hid], then S [N][slices][2] (per-slice partial sums, summed
// in order by pass 2)
constexpr int MA_PIX = 64;
template <typename T>
__global__ void k_mask_attn_bwd1(const T* __restrict__ dout, int lddo, const T* __restrict__ f, int ldf,
                                 const T* __restrict__ m, MaskAttnB P, const float* __restrict__ stats, int HW, int C,
                                 T* __restrict__ df, int lddf, float* __restrict__ dhh, float* __restrict__ S,
                                 float* __restrict__ slab) {
  __shared__ float sacc[4][64];  // per-wave accumulators for lanes < hid: [gn_w, gn_b, w2] + [db2, dgamma, S1, S2]
  __shared__ float sw[4][8];
  const int n = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float mu, rs;
  ma_stats(P, stats, n, HW, mu, rs);
  float a_gw = 0.f, a_gb = 0.f, a_w2 = 0.f;  // lane c < hid
  float a_db2 = 0.f, a_dgam = 0.f, a_s1 = 0.f, a_s2 = 0.f;
  const int p_end = min(HW, (int)(blockIdx.y + 1) * MA_PIX);
  for (int p = blockIdx.y * MA_PIX + wid; p < p_end; p += 4) {
    const long long pix = (long long)n * HW + p;
    const float mv = ld(m + pix);
    // recompute forward for this pixel (every lane computes the scalar z)
    float z = P.b2[0];
    for (int c = 0; c < P.hid; ++c) z += P.w2[c] * gelu_f((P.w1[c] * mv - mu) * rs * P.g[c] + P.b[c]);
    const float s = sigmoid_f(z);
    const float A = fminf(fmaxf(s, 1e-4f), 1.f - 1e-4f);
    const float gam = P.gamma[0];
    float gsum = 0.f;
    if (sizeof(T) == 2 && (C & 7) == 0 && ((lddo | ldf | lddf) & 7) == 0) {
      for (int c = lane * 8; c < C; c += 512) {
        float d[8], fv[8];
        ld8(dout + pix * lddo + c, d);
        ld8(f + pix * ldf + c, fv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          gsum += d[e] * fv[e];
          d[e] *= 1.f + gam * A;
        }
        st8(df + pix * lddf + c, d);
      }
    } else {
      for (int c = lane; c < C; c += 64) {
        const float d = ld(dout + pix * lddo + c);
        const float fv = ld(f + pix * ldf + c);
        gsum += d * fv;
        st(df + pix * lddf + c, d * (1.f + gam * A));
      }
    }
    gsum = wave_sum(gsum);
    const float dA = gsum * gam;
    if (lane == 0) a_dgam += gsum * A;
    const float ds = (s >= 1e-4f && s <= 1.f - 1e-4f) ? dA : 0.f;
    const float dzv = ds * s * (1.f - s);
    if (lane == 0) a_db2 += dzv;
    if (lane < P.hid) {
      const int c = lane;
      const float hh = (P.w1[c] * mv - mu) * rs;
      const float v = hh * P.g[c] + P.b[c];
      const float u = gelu_f(v);
      a_w2 += dzv * u;
      const float dv = dzv * P.w2[c] * gelu_grad_f(v);
      a_gw += dv * hh;
      a_gb += dv;
      const float dh = dv * P.g[c];
      dhh[pix * P.hid + c] = dh;
      a_s1 += dh;
      a_s2 += dh * hh;
    }
  }
  // reduce over the 4 waves into this block's slab row (grads layout; summed over the rows in
  // row order after pass 2: deterministic, no atomics)
  float* row = slab + ((size_t)n * gridDim.y + blockIdx.y) * (4 * P.hid + 2);
  a_s1 = wave_sum(a_s1);
  a_s2 = wave_sum(a_s2);
  sacc[wid][lane] = a_gw;
  __syncthreads();
  if (wid == 0 && lane < P.hid) row[P.hid + lane] = (sacc[0][lane] + sacc[1][lane]) + (sacc[2][lane] + sacc[3][lane]);
  __syncthreads();
  sacc[wid][lane] = a_gb;
  __syncthreads();
  if (wid == 0 && lane < P.hid) row[2 * P.hid + lane] = (sacc[0][lane] + sacc[1][lane]) + (sacc[2][lane] + sacc[3][lane]);
  __syncthreads();
  sacc[wid][lane] = a_w2;
  __syncthreads();
  if (wid == 0 && lane < P.hid) row[3 * P.hid + lane] = (sacc[0][lane] + sacc[1][lane]) + (sacc[2][lane] + sacc[3][lane]);
  if (lane == 0) {
    sw[wid][0] = a_db2;
    sw[wid][1] = a_dgam;
    sw[wid][2] = a_s1;
    sw[wid][3] = a_s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t[4] = {0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < 4; ++w)
      for (int k = 0; k < 4; ++k) t[k] += sw[w][k];
    row[4 * P.hid] = t[0];
    row[4 * P.hid + 1] = t[1];
    S[2 * ((size_t)n * gridDim.y + blockIdx.y)] = t[2];
    S[2 * ((size_t)n * gridDim.y + blockIdx.y) + 1] = t[3];
  }
}

// pass 2: GroupNorm(1,hid) backward + 1x1 conv (1 -> hid) backward
template <typename T>
__global__ void k_mask_attn_bwd2(const T* __restrict__ m, MaskAttnB P, const float* __restrict__ stats, int HW,
                                 const float* __restrict__ dhh, const float* __restrict__ S, T* __restrict__ dm,
                                 float* __restrict__ slab) {
  __shared__ float sacc[4][64];
  const int n = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float mu, rs;
  ma_stats(P, stats, n, HW, mu, rs);
  const float G = (float)P.hid * HW;
  float s1 = 0.f, s2 = 0.f;
  for (int j = 0; j < (int)gridDim.y; ++j) {
    s1 += S[2 * ((size_t)n * gridDim.y + j)];
    s2 += S[2 * ((size_t)n * gridDim.y + j) + 1];
  }
  const float m1 = s1 / G, m2 = s2 / G;
  float a_w1 = 0.f;
  const int p_end = min(HW, (int)(blockIdx.y + 1) * MA_PIX);
  for (int p = blockIdx.y * MA_PIX + wid; p < p_end; p += 4) {
    const long long pix = (long long)n * HW + p;
    const float mv = ld(m + pix);
    float contrib = 0.f;
    if (lane < P.hid) {
      const int c = lane;
      const float hh = (P.w1[c] * mv - mu) * rs;
      const float dh = rs * (dhh[pix * P.hid + c] - m1 - hh * m2);
      a_w1 += dh * mv;
      contrib = dh * P.w1[c];
    }
    contrib = wave_sum(contrib);
    if (lane == 0) st(dm + pix, contrib);
  }
  sacc[wid][lane] = a_w1;
  __syncthreads();
  if (wid == 0 && lane < P.hid)
    slab[((size_t)n * gridDim.y + blockIdx.y) * (4 * P.hid + 2) + lane] =
        (sacc[0][lane] + sacc[1][lane]) + (sacc[2][lane] + sacc[3][lane]);
}

}  // namespace dmf

using namespace dmf;

extern "C" int dmf_mix_bwd(int dtype, const void* dz, int lddz, const void* a, int lda, const void* b, int ldb,
                           const float* wlogit, void* da, void* db, int ldd, float* dw, long long M, int C,
                           float* ws, void* stream) {
  DMF_CHECK_ARG(dz && a && b && wlogit && da && db && dw && ws && M > 0 && C > 0, "dmf_mix_bwd: bad args");
  const int es = is16(dtype) ? 2 : 4;
  if (C % 8 == 0 && lddz % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldd % 8 == 0 && M * std::max(ldd, lddz) < (1LL << 31) &&
      ((uintptr_t)dz | (uintptr_t)a | (uintptr_t)b | (uintptr_t)da | (uintptr_t)db) % (8 * es) == 0) {
    long long g8 = (M * C / 8 + 255) / 256;
    if (g8 > 2048) g8 = 2048;
    if (g8 < 1) g8 = 1;
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_mix_bwd8<T>, dim3((unsigned)g8), dim3(256), 0, (hipStream_t)stream, (const T*)dz,
                         lddz, (const T*)a, lda, (const T*)b, ldb, wlogit, (T*)da, (T*)db, ldd, ws,
                         (int)M, C));
    DMF_LAUNCH_CHECK("dmf_mix_bwd");
    return dmf_colsum_f32(ws, 1, (int)g8, 1, dw, 1, stream);  // dw += the block partials in block order
  }
  long long g = (M * C + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_mix_bwd<T>, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, (const T*)dz,
                       lddz, (const T*)a, lda, (const T*)b, ldb, wlogit, (T*)da, (T*)db, ldd, ws,
                       M, C));
  DMF_LAUNCH_CHECK("dmf_mix_bwd");
  return dmf_colsum_f32(ws, 1, (int)g, 1, dw, 1, stream);
}

extern "C" int dmf_mask_attn_bwd_ws_size(int N, int HW, int hidden) {
  const long long rows = (long long)N * cdiv(HW, MA_PIX);
  return (int)((long long)N * HW * hidden + 2LL * rows + rows * (4LL * hidden + 2));
}

extern "C" int dmf_mask_attn_bwd(int dtype, const void* dout, int lddo, const void* f, int ldf, const void* m, int N,
                                 int HW, int C, const float* w1, const float* gn_w, const float* gn_b, const float* w2,
                                 const float* b2, const float* gamma, int hidden, float eps, const float* stats,
                                 void* df, int lddf, void* dm, float* workspace, float* grads, void* stream) {
  DMF_CHECK_ARG(dout && f && m && w1 && gn_w && gn_b && w2 && b2 && gamma && stats && df && dm && workspace && grads &&
                    hidden > 0 && hidden <= 64,
                "dmf_mask_attn_bwd: bad args");
  MaskAttnB P{w1, gn_w, gn_b, w2, b2, gamma, eps, hidden};
  float* dhh = workspace;
  const int rows = N * cdiv(HW, MA_PIX);
  float* S = workspace + (size_t)N * HW * hidden;
  float* slab = S + 2 * (size_t)rows;  // [rows][4 * hidden + 2] per-block parameter-gradient partials
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(N, cdiv(HW, MA_PIX));
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_mask_attn_bwd1<T>, grid, dim3(256), 0, s, (const T*)dout, lddo, (const T*)f,
                       ldf, (const T*)m, P, stats, HW, C, (T*)df, lddf, dhh, S, slab);
    hipLaunchKernelGGL(k_mask_attn_bwd2<T>, grid, dim3(256), 0, s, (const T*)m, P, stats, HW, dhh, S,
                       (T*)dm, slab));
  DMF_LAUNCH_CHECK("dmf_mask_attn_bwd");
  // grads (+)= the slab's column sums in row order
  return dmf_colsum_f32(slab, 4 * hidden + 2, rows, 4 * hidden + 2, grads, 1, stream);
}
