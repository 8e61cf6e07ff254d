// Batched bf16 GEMM on MFMA (gfx950) and the long-sequence attention pieces
// of the hybrid TransformerStage (configuration 5: transformer_model.py
// :68-134 -- qkv / proj / fc1 / fc2 linears, softmax(q k^T * scale) with
// attention dropout, P v -- and their backward).
//
//   t = alpha * op(A[z]) op(B[z]) + bias[n]            (f32 accumulation)
//   aux[m][n] = bf16(t)                                  (optional: pre-activation kept for backward)
//   forward epilogue : t = dropout(act(t))
//   gradient epilogue: t = dropout_mask(t) * act'(pre[m][n])   (when `pre` is given)
//   t *= colscale[n]; t += res[m][n]; C[m][n] = t; dbias[n] += t (column sums, atomics)
//   op(A)[m][k] = TA ? A[k*lda + m] : A[m*lda + k]
//   op(B)[k][n] = TB ? B[k*ldb + n] : B[n*ldb + k]      ("NT": weights [N][K])
//   batch z = z1*H + z2 (blockIdx.z), element offsets z1*s1 + z2*s2 per operand
//   (the attention heads are column slices of the packed qkv rows).
//
// Tile 128x128x64, 256 threads (2x2 waves of 64x64 = 4x4 16x16x32 bf16 MFMA
// fragments, fp32 accumulation), register-staged 16-B loads one K-step ahead,
// LDS rows of 128 B (64 k) XOR-swizzled (chunk ^ row&7). A K-contiguous
// operand is staged as whole 16-B chunks; a transposed operand (M- or
// N-contiguous) is loaded as 16-B runs along M/N and scattered into the same
// k-contiguous LDS image (8 x ds_write_b16 per chunk). Epilogue through LDS,
// 16-B stores.
#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

typedef __attribute__((ext_vector_type(8))) short g_bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float g_f32x4_t;

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  const float* bias;
  int M, N, K, lda, ldb, ldc;
  int H;                     // inner batch count
  long long sA1, sA2, sB1, sB2, sC1, sC2;
  float alpha;
  int act;
  int ntiles;
  const float* colscale;     // [N] LayerScale gamma or null
  const float* res;          // f32 residual [m*ldr + n] (may alias C) or null
  int ldr;
  bf16_t* aux;               // bf16 copy of t before act/dropout or null
  int ldaux;
  const bf16_t* pre;         // gradient epilogue: saved pre-activation or null
  int ldpre;
  float dp;                  // dropout probability (0: none)
  const unsigned long long* rng;
  int site;
  float* dbias;              // column sums of the final t (accumulated) or null
};

constexpr int GBM = 128, GBN = 128, GBK = 64, GTHREADS = 256;
constexpr int GSTAGE = (GBM + GBN) * 128;

__device__ __forceinline__ float g_act(int act, float v) {
  switch (act) {
    case DMF_ACT_RELU: return fmaxf(v, 0.f);
    case DMF_ACT_GELU: return gelu_f(v);
    case DMF_ACT_SIGMOID: return sigmoid_f(v);
    default: return v;
  }
}
__device__ __forceinline__ float g_act_grad(int act, float z) {
  switch (act) {
    case DMF_ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case DMF_ACT_GELU: return gelu_grad_f(z);
    case DMF_ACT_SIGMOID: { const float s = sigmoid_f(z); return s * (1.f - s); }
    default: return 1.f;
  }
}

// Loader of one 128-row operand tile (rows = M or N index, 64 k) for K-step k0.
// TR: operand stored transposed (k-major, rows contiguous).
template <bool TR>
struct TileLoad {
  uint4 v[4];
  __device__ __forceinline__ void load(const bf16_t* base, int ld, int rows, int K, int r0, int k0, int tid) {
    if (!TR) {
      // 128 rows x 8 chunks: thread -> chunk (tid & 7) of rows (tid >> 3) + 32 i
      const int q = tid & 7, rb = tid >> 3;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + rb + 32 * i, k = k0 + q * 8;
        v[i] = (r < rows && k < K) ? *(const uint4*)(base + (size_t)r * ld + k) : make_uint4(0, 0, 0, 0);
      }
    } else {
      // 64 k x 16 runs of 8 rows: thread -> run (tid & 15) of k (tid >> 4) + 16 i
      const int q = tid & 15, kb = tid >> 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + kb + 16 * i, r = r0 + q * 8;
        v[i] = (k < K && r < rows) ? *(const uint4*)(base + (size_t)k * ld + r) : make_uint4(0, 0, 0, 0);
      }
    }
  }
  __device__ __forceinline__ void store(char* S, int tid) const {
    if (!TR) {
      const int q = tid & 7, rb = tid >> 3;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = rb + 32 * i;
        *(uint4*)(S + row * 128 + ((q ^ (row & 7)) << 4)) = v[i];
      }
    } else {
      const int q = tid & 15, kb = tid >> 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kl = kb + 16 * i;
        const int ch = kl >> 3, w = kl & 7;
        const uint32_t u[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int row = q * 8 + e;
          *(bf16_t*)(S + row * 128 + ((ch ^ (row & 7)) << 4) + w * 2) = (bf16_t)(u[e >> 1] >> ((e & 1) * 16));
        }
      }
    }
  }
};

template <typename OutT, bool TA, bool TB>
__global__ void __launch_bounds__(GTHREADS, 2) k_gemm_bf16(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int mt = blockIdx.x / g.ntiles, nt = blockIdx.x % g.ntiles;
  const int m0 = mt * GBM, n0 = nt * GBN;
  const int z = blockIdx.z, z1 = z / g.H, z2 = z - (z / g.H) * g.H;
  const bf16_t* A = g.A + z1 * g.sA1 + z2 * g.sA2;
  const bf16_t* B = g.B + z1 * g.sB1 + z2 * g.sB2;

  TileLoad<TA> la;
  TileLoad<TB> lb;
  g_f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = g_f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + GBK - 1) / GBK;
  la.load(A, g.lda, g.M, g.K, m0, 0, tid);
  lb.load(B, g.ldb, g.N, g.K, n0, 0, tid);
  la.store(smem, tid);
  lb.store(smem + GBM * 128, tid);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * GSTAGE;
    if (kt + 1 < nk) {
      la.load(A, g.lda, g.M, g.K, m0, (kt + 1) * GBK, tid);
      lb.load(B, g.ldb, g.N, g.K, n0, (kt + 1) * GBK, tid);
    }
    const char* As = cur;
    const char* Bs = cur + GBM * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + fg;
      uint4 av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + fr;
        av[i] = *(const uint4*)(As + row * 128 + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + fr;
        bv[j] = *(const uint4*)(Bs + col * 128 + ((ch ^ (col & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(g_bf16x8_t*)&av[i], *(g_bf16x8_t*)&bv[j], acc[i][j],
                                                              0, 0, 0);
    }
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * GSTAGE;
      la.store(nxt, tid);
      lb.store(nxt + GBM * 128, tid);
    }
    __syncthreads();
  }

  // epilogue through an f32 LDS image of the tile, 16-B stores
  float* Cs = (float*)smem;  // [128][128 + 4]
  constexpr int FST = GBN + 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + i * 16 + fg * 4 + r;
        const int col = wn * 64 + j * 16 + fr;
        Cs[row * FST + col] = acc[i][j][r];
      }
  __syncthreads();
  constexpr int EPC = 16 / sizeof(OutT);
  constexpr int CPR = GBN / EPC;  // chunks per row; a thread always owns chunk column tid % CPR
  OutT* C = (OutT*)g.C + z1 * g.sC1 + z2 * g.sC2;
  const float ks = g.dp > 0.f ? 1.f / (1.f - g.dp) : 1.f;
  const unsigned long long ebase = (unsigned long long)z * g.M * g.N;
  float csum[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) csum[e] = 0.f;
  const int chn = tid % CPR;
  const int n = n0 + chn * EPC;
  for (int row = tid / CPR; row < GBM; row += GTHREADS / CPR) {
    const int m = m0 + row;
    if (m >= g.M || n >= g.N) continue;
    float v[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      v[e] = Cs[row * FST + chn * EPC + e] * g.alpha;
      if (g.bias) v[e] += g.bias[n + e];
    }
    if (g.aux) {
      bf16_t* ap = g.aux + z1 * g.sC1 + z2 * g.sC2 + (size_t)m * g.ldaux + n;
#pragma unroll
      for (int e = 0; e < EPC; e += 4) {
        uint2 u;
        u.x = (uint32_t)f2bf(v[e]) | ((uint32_t)f2bf(v[e + 1]) << 16);
        u.y = (uint32_t)f2bf(v[e + 2]) | ((uint32_t)f2bf(v[e + 3]) << 16);
        *(uint2*)(ap + e) = u;
      }
    }
    if (!g.pre) {
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[e] = g_act(g.act, v[e]);
    }
    if (g.dp > 0.f) {
#pragma unroll
      for (int e = 0; e < EPC; e += 4) {
        bool keep[4];
        dropout_keep4(g.rng, g.site, ebase + (unsigned long long)m * g.N + n + e, g.dp, keep);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[e + q] = keep[q] ? v[e + q] * ks : 0.f;
      }
    }
    if (g.pre) {
      const bf16_t* pp = g.pre + z1 * g.sC1 + z2 * g.sC2 + (size_t)m * g.ldpre + n;
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[e] *= g_act_grad(g.act, bf2f(pp[e]));
    }
    if (g.colscale) {
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[e] *= g.colscale[n + e];
    }
    if (g.res) {
      const float* rp = g.res + (size_t)m * g.ldr + n;
#pragma unroll
      for (int e = 0; e < EPC; e += 4) {
        const float4 c = *(const float4*)(rp + e);
        v[e] += c.x; v[e + 1] += c.y; v[e + 2] += c.z; v[e + 3] += c.w;
      }
    }
    if (g.dbias) {
#pragma unroll
      for (int e = 0; e < EPC; ++e) csum[e] += v[e];
    }
    OutT* dst = C + (size_t)m * g.ldc + n;
    if constexpr (sizeof(OutT) == 4) {
      *(float4*)dst = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      uint4 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
      o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
      *(uint4*)dst = o;
    }
  }
  if (g.dbias) {
    // threads sharing a chunk column: tid % CPR; reduce through LDS, one atomic per column
    __syncthreads();
#pragma unroll
    for (int e = 0; e < EPC; ++e) Cs[tid * EPC + e] = csum[e];
    __syncthreads();
    if (tid < GBN) {
      const int c = tid, cc = c / EPC, ce = c % EPC;
      float s = 0.f;
      for (int t = cc; t < GTHREADS; t += CPR) s += Cs[t * EPC + ce];
      if (n0 + c < g.N) atomicAdd(g.dbias + n0 + c, s);
    }
  }
}

// ----------------------------------------------------- softmax + dropout
// One wave per row of length L (fp32 scores S): p = softmax(scale * s);
// Ps (bf16) = p (kept for backward); Pd (bf16) = dropout(p) / (1 - dp) (the
// operand of P v). Dropout element index = row * L + col (site `site`).
__global__ void __launch_bounds__(256) k_softmax_drop(const float* __restrict__ S, int lds_, long long rows, int L,
                                                      float scale, float dp, const unsigned long long* rng, int site,
                                                      bf16_t* __restrict__ Ps, bf16_t* __restrict__ Pd, int ldp) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* s = S + row * lds_;
  float mx = -INFINITY;
  for (int c = lane * 4; c < L; c += 256) {
    const float4 v = *(const float4*)(s + c);
    mx = fmaxf(mx, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float sum = 0.f;
  for (int c = lane * 4; c < L; c += 256) {
    const float4 v = *(const float4*)(s + c);
    sum += __expf((v.x - mx) * scale) + __expf((v.y - mx) * scale) + __expf((v.z - mx) * scale) +
           __expf((v.w - mx) * scale);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  const float inv = 1.f / sum;
  const float ks = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  for (int c = lane * 4; c < L; c += 256) {
    const float4 v = *(const float4*)(s + c);
    float p[4] = {__expf((v.x - mx) * scale) * inv, __expf((v.y - mx) * scale) * inv,
                  __expf((v.z - mx) * scale) * inv, __expf((v.w - mx) * scale) * inv};
    uint2 u;
    u.x = (uint32_t)f2bf(p[0]) | ((uint32_t)f2bf(p[1]) << 16);
    u.y = (uint32_t)f2bf(p[2]) | ((uint32_t)f2bf(p[3]) << 16);
    *(uint2*)(Ps + row * ldp + c) = u;
    if (dp > 0.f) {
      bool keep[4];
      dropout_keep4(rng, site, (unsigned long long)(row * L + c), dp, keep);
#pragma unroll
      for (int e = 0; e < 4; ++e) p[e] = keep[e] ? p[e] * ks : 0.f;
      u.x = (uint32_t)f2bf(p[0]) | ((uint32_t)f2bf(p[1]) << 16);
      u.y = (uint32_t)f2bf(p[2]) | ((uint32_t)f2bf(p[3]) << 16);
    }
    *(uint2*)(Pd + row * ldp + c) = u;
  }
}

// dS = scale * P * (g - sum_j P g), g = dPd * keep / (1 - dp)   (bf16 out)
__global__ void __launch_bounds__(256) k_softmax_drop_bwd(const bf16_t* __restrict__ Ps, int ldp,
                                                          const float* __restrict__ dPd, int ldg, long long rows,
                                                          int L, float scale, float dp,
                                                          const unsigned long long* rng, int site,
                                                          bf16_t* __restrict__ dS, int lds_) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float ks = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  float dot = 0.f;
  for (int c = lane * 4; c < L; c += 256) {
    const uint2 u = *(const uint2*)(Ps + row * ldp + c);
    const float4 gv = *(const float4*)(dPd + row * ldg + c);
    float gg[4] = {gv.x, gv.y, gv.z, gv.w};
    if (dp > 0.f) {
      bool keep[4];
      dropout_keep4(rng, site, (unsigned long long)(row * L + c), dp, keep);
#pragma unroll
      for (int e = 0; e < 4; ++e) gg[e] = keep[e] ? gg[e] * ks : 0.f;
    }
    dot += bf2f((bf16_t)(u.x & 0xffff)) * gg[0] + bf2f((bf16_t)(u.x >> 16)) * gg[1] +
           bf2f((bf16_t)(u.y & 0xffff)) * gg[2] + bf2f((bf16_t)(u.y >> 16)) * gg[3];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
  for (int c = lane * 4; c < L; c += 256) {
    const uint2 u = *(const uint2*)(Ps + row * ldp + c);
    const float4 gv = *(const float4*)(dPd + row * ldg + c);
    float gg[4] = {gv.x, gv.y, gv.z, gv.w};
    if (dp > 0.f) {
      bool keep[4];
      dropout_keep4(rng, site, (unsigned long long)(row * L + c), dp, keep);
#pragma unroll
      for (int e = 0; e < 4; ++e) gg[e] = keep[e] ? gg[e] * ks : 0.f;
    }
    const float p[4] = {bf2f((bf16_t)(u.x & 0xffff)), bf2f((bf16_t)(u.x >> 16)), bf2f((bf16_t)(u.y & 0xffff)),
                        bf2f((bf16_t)(u.y >> 16))};
    uint2 o;
    o.x = (uint32_t)f2bf(scale * p[0] * (gg[0] - dot)) | ((uint32_t)f2bf(scale * p[1] * (gg[1] - dot)) << 16);
    o.y = (uint32_t)f2bf(scale * p[2] * (gg[2] - dot)) | ((uint32_t)f2bf(scale * p[3] * (gg[3] - dot)) << 16);
    *(uint2*)(dS + row * lds_ + c) = o;
  }
}

}  // namespace dmf

using namespace dmf;

extern "C" int dmf_gemm_bf16(int out_dtype, int ta, int tb, int M, int N, int K, float alpha, const void* A, int lda,
                             long long sA1, long long sA2, const void* B, int ldb, long long sB1, long long sB2,
                             void* C, int ldc, long long sC1, long long sC2, int batch1, int batch2,
                             const float* bias, int act, const float* colscale, const float* res, int ldr, void* aux,
                             int ldaux, const void* pre, int ldpre, float dropout_p,
                             const unsigned long long* rng, int site, float* dbias, void* stream) {
  DMF_CHECK_ARG(out_dtype == DMF_F32 || out_dtype == DMF_BF16, "dmf_gemm_bf16: bad out dtype %d", out_dtype);
  DMF_CHECK_ARG(M > 0 && N > 0 && K > 0 && batch1 > 0 && batch2 > 0, "dmf_gemm_bf16: empty problem");
  DMF_CHECK_ARG(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0, "dmf_gemm_bf16: K (%d) and lda/ldb must be multiples of 8", K);
  DMF_CHECK_ARG(!ta || M % 8 == 0, "dmf_gemm_bf16: transposed A needs M %% 8 == 0");
  DMF_CHECK_ARG(!tb || N % 8 == 0, "dmf_gemm_bf16: transposed B needs N %% 8 == 0");
  const int epc = out_dtype == DMF_F32 ? 4 : 8;
  DMF_CHECK_ARG(N % epc == 0 && ldc % epc == 0, "dmf_gemm_bf16: N (%d) and ldc must be multiples of %d", N, epc);
  DMF_CHECK_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0 && ((uintptr_t)C % 16) == 0 &&
                    sA1 % 8 == 0 && sA2 % 8 == 0 && sB1 % 8 == 0 && sB2 % 8 == 0 && sC1 % epc == 0 &&
                    sC2 % epc == 0,
                "dmf_gemm_bf16: operands and batch strides must be 16-byte aligned");
  DMF_CHECK_ARG(!res || (batch1 * batch2 == 1 && ldr % 4 == 0 && ((uintptr_t)res % 16) == 0),
                "dmf_gemm_bf16: residual needs an unbatched, 16-byte aligned f32 operand");
  DMF_CHECK_ARG(!aux || (ldaux % 4 == 0 && ((uintptr_t)aux % 8) == 0), "dmf_gemm_bf16: aux must be 8-byte aligned");
  DMF_CHECK_ARG(dropout_p <= 0.f || (rng && dropout_p < 1.f), "dmf_gemm_bf16: dropout needs rng state and p < 1");
  GemmArgs g{(const bf16_t*)A, (const bf16_t*)B, C, bias, M, N, K, lda, ldb, ldc, batch2,
             sA1, sA2, sB1, sB2, sC1, sC2, alpha, act, cdiv(N, GBN), colscale, res, ldr, (bf16_t*)aux, ldaux,
             (const bf16_t*)pre, ldpre, dropout_p, rng, site, dbias};
  const dim3 grid((unsigned)(cdiv(M, GBM) * g.ntiles), 1, (unsigned)(batch1 * batch2));
  DMF_CHECK_ARG((long long)cdiv(M, GBM) * g.ntiles < (1LL << 31) && batch1 * batch2 < 65536,
                "dmf_gemm_bf16: grid too large");
  const size_t lds = 2 * GSTAGE > GBM * (GBN + 4) * 4 ? 2 * GSTAGE : GBM * (GBN + 4) * 4;
  hipStream_t st = (hipStream_t)stream;
#define DMF_G(OT, TA_, TB_) hipLaunchKernelGGL((k_gemm_bf16<OT, TA_, TB_>), grid, dim3(GTHREADS), lds, st, g)
  if (out_dtype == DMF_F32) {
    if (!ta && !tb) DMF_G(float, false, false);
    else if (!ta && tb) DMF_G(float, false, true);
    else if (ta && !tb) DMF_G(float, true, false);
    else DMF_G(float, true, true);
  } else {
    if (!ta && !tb) DMF_G(bf16_t, false, false);
    else if (!ta && tb) DMF_G(bf16_t, false, true);
    else if (ta && !tb) DMF_G(bf16_t, true, false);
    else DMF_G(bf16_t, true, true);
  }
#undef DMF_G
  DMF_LAUNCH_CHECK("dmf_gemm_bf16");
  return 0;
}

extern "C" int dmf_softmax_dropout(const float* S, int lds, long long rows, int L, float scale, float dropout_p,
                                   const unsigned long long* rng, int site, void* probs, void* probs_dropped, int ldp,
                                   void* stream) {
  DMF_CHECK_ARG(L % 4 == 0 && lds % 4 == 0 && ldp % 4 == 0, "dmf_softmax_dropout: L and strides must be multiples of 4");
  DMF_CHECK_ARG(dropout_p <= 0.f || rng, "dmf_softmax_dropout: dropout needs rng state");
  DMF_CHECK_ARG(dropout_p < 1.f, "dmf_softmax_dropout: p must be < 1");
  if (rows == 0) return 0;
  hipLaunchKernelGGL(k_softmax_drop, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, S, lds, rows,
                     L, scale, dropout_p, rng, site, (bf16_t*)probs, (bf16_t*)probs_dropped, ldp);
  DMF_LAUNCH_CHECK("dmf_softmax_dropout");
  return 0;
}

extern "C" int dmf_softmax_dropout_bwd(const void* probs, int ldp, const float* dprobs_dropped, int ldg,
                                       long long rows, int L, float scale, float dropout_p,
                                       const unsigned long long* rng, int site, void* dscores, int lds,
                                       void* stream) {
  DMF_CHECK_ARG(L % 4 == 0 && ldp % 4 == 0 && ldg % 4 == 0 && lds % 4 == 0,
                "dmf_softmax_dropout_bwd: L and strides must be multiples of 4");
  DMF_CHECK_ARG(dropout_p <= 0.f || rng, "dmf_softmax_dropout_bwd: dropout needs rng state");
  if (rows == 0) return 0;
  hipLaunchKernelGGL(k_softmax_drop_bwd, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)probs, ldp, dprobs_dropped, ldg, rows, L, scale, dropout_p, rng, site,
                     (bf16_t*)dscores, lds);
  DMF_LAUNCH_CHECK("dmf_softmax_dropout_bwd");
  return 0;
}
