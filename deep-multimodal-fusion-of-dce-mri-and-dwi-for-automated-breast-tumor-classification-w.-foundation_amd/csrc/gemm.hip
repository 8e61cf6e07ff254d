// Batched GEMM on MFMA (gfx950) and the long-sequence attention pieces of the
// hybrid TransformerStage (configuration 5: transformer_model.py :68-134 --
// qkv / proj / fc1 / fc2 linears, softmax(q k^T * scale) with attention
// dropout, P v -- and their backward).
//
//   t = alpha * op(A[z]) op(B[z]) + bias[n]            (f32 accumulation)
//   aux[m][n] = IT(t)                                    (optional: pre-activation kept for backward)
//   forward epilogue : t = dropout(act(t))
//   gradient epilogue: t = dropout_mask(t) * act'(pre[m][n])   (when `pre` is given)
//   t *= colscale[n]; t += res[m][n]; C[m][n] = t; dbias[n] += t (column sums: per-tile slab rows, then
//   an ordered sum over the tiles)
//   op(A)[m][k] = TA ? A[k*lda + m] : A[m*lda + k]
//   op(B)[k][n] = TB ? B[k*ldb + n] : B[n*ldb + k]      ("NT": weights [N][K])
//   batch z = z1*H + z2 (blockIdx.z), element offsets z1*s1 + z2*s2 per operand
//   (the attention heads are column slices of the packed qkv rows).
//
// Two operand types IT share one kernel body: bf16 (throughput mode,
// 16x16x32 bf16 MFMA) and f32 (the parity mode, 16x16x4 f32 MFMA -- exact
// f32 products, the conv engine's f32 path). Tile 128x128 by 128 BYTES of k
// (64 bf16 / 32 f32), 256 threads (2x2 waves of 64x64 = 4x4 16x16 MFMA
// fragments, fp32 accumulation), register-staged 16-B loads one K-step
// ahead, LDS rows of 128 B XOR-swizzled (chunk ^ row&7). A K-contiguous
// operand is staged as whole 16-B chunks; a transposed operand (M- or
// N-contiguous) is loaded as 16-B runs along M/N and scattered into the same
// k-contiguous LDS image. In the f32 mode a lane's 16-B chunk holds 4
// consecutive k: 4 MFMAs take element e of the chunks of all 4 lane groups,
// the same k permutation on A and B. Epilogue through LDS, 16-B stores.
#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

typedef __attribute__((ext_vector_type(8))) short g_bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float g_f32x4_t;

struct GemmArgs {
  const void* A;
  const void* B;
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
  void* aux;                 // IT copy of t before act/dropout or null
  int ldaux;
  const void* pre;           // gradient epilogue: saved pre-activation (IT) or null
  int ldpre;
  float dp;                  // dropout probability (0: none)
  const unsigned long long* rng;
  int site;
  float* dbias;              // column sums of the final t (accumulated) or null
  float* dbias_ws;           // [M tiles][N] per-tile column sums (dbias: summed in tile order after the launch)
};

constexpr int GBM = 128, GBN = 128, GTHREADS = 256;   // k per step: 128 bytes of IT
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

// Loader of one 128-row operand tile (rows = M or N index, 128 bytes of k)
// for K-step k0. TR: operand stored transposed (k-major, rows contiguous).
template <bool TR, typename IT>
struct TileLoad {
  static constexpr int EPC = 16 / sizeof(IT);    // elements per 16-B chunk
  static constexpr int RUNS = GBM / EPC;         // TR: 16-B runs per k row
  static constexpr int KPP = GTHREADS / RUNS;    // TR: k rows per pass
  uint4 v[4];
  __device__ __forceinline__ void load(const IT* base, int ld, int rows, int K, int r0, int k0, int tid) {
    if (!TR) {
      // 128 rows x 8 chunks: thread -> chunk (tid & 7) of rows (tid >> 3) + 32 i
      const int q = tid & 7, rb = tid >> 3;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + rb + 32 * i, k = k0 + q * EPC;
        v[i] = (r < rows && k < K) ? *(const uint4*)(base + (size_t)r * ld + k) : make_uint4(0, 0, 0, 0);
      }
    } else {
      // 4 * KPP k x RUNS runs of EPC rows: thread -> run (tid % RUNS) of k (tid / RUNS) + KPP i
      const int q = tid % RUNS, kb = tid / RUNS;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + kb + KPP * i, r = r0 + q * EPC;
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
      const int q = tid % RUNS, kb = tid / RUNS;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kl = kb + KPP * i;
        const int ch = kl / EPC, w = kl % EPC;
        const uint32_t u[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          const int row = q * EPC + e;
          char* dst = S + row * 128 + ((ch ^ (row & 7)) << 4) + w * (int)sizeof(IT);
          if constexpr (sizeof(IT) == 2)
            *(bf16_t*)dst = (bf16_t)(u[e >> 1] >> ((e & 1) * 16));
          else
            *(uint32_t*)dst = u[e];
        }
      }
    }
  }
};

__device__ __forceinline__ void g_store_aux(bf16_t* ap, const float* v) {
  uint2 u;
  u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  *(uint2*)ap = u;
}
__device__ __forceinline__ void g_store_aux(float* ap, const float* v) {
  *(float4*)ap = make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ float g_ld(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ float g_ld(const float* p) { return *p; }

// k_gemm's epilogue on an f32 LDS image Cs[BM][BN + 4] of the finished tile (bias, aux copy, activation or
// its gradient, dropout, LayerScale, f32 residual, column sums), 16-B stores; NTH threads. A thread owns
// one EPC-wide column chunk (its bias / LayerScale values stay in registers) and walks its rows RB at a
// time with every row's LDS and global loads issued before the first store: with the per-column loads
// inside the row loop (and C possibly aliasing them) each row paid a full global-load latency, which
// made the epilogue ~2x the K loop (18432x1536x512: 108 -> 64 us; config 5 step 1150 -> 1227 vol/s).
template <typename IT, typename OutT, int BM, int BN, int NTH, int ACT>
__device__ __forceinline__ void gemm_epilogue_act(const GemmArgs& g, const float* Cs, int tid, int m0, int n0, int z,
                                                  float (&csum)[16 / sizeof(OutT)]) {
  constexpr int FST = BN + 4;
  constexpr int EPC = 16 / sizeof(OutT);
  constexpr int CPR = BN / EPC;        // chunks per row; a thread always owns chunk column tid % CPR
  constexpr int RPP = NTH / CPR;       // rows per pass
  constexpr int NR = BM / RPP;         // passes
  constexpr int RB = NR >= 4 ? 4 : NR;  // rows in flight per thread
  static_assert(NR % RB == 0, "gemm_epilogue rows");
  const int z1 = z / g.H, z2 = z - (z / g.H) * g.H;
  OutT* __restrict__ C = (OutT*)g.C + z1 * g.sC1 + z2 * g.sC2;
  const float ks = g.dp > 0.f ? 1.f / (1.f - g.dp) : 1.f;
  // Philox (seed, offset) read once: the epilogue's stores would otherwise force a reload per mask
  const unsigned long long rseed = g.dp > 0.f ? g.rng[0] : 0ull, roff = g.dp > 0.f ? g.rng[1] : 0ull;
  const unsigned long long ebase = (unsigned long long)z * g.M * g.N;
  const int chn = tid % CPR, r0 = tid / CPR;
  const int n = n0 + chn * EPC;
  if (n >= g.N) return;
  float bv[EPC], sv[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) {
    bv[e] = g.bias ? g.bias[n + e] : 0.f;
    sv[e] = g.colscale ? g.colscale[n + e] : 1.f;
  }
  const float* __restrict__ res = g.res;
  const IT* __restrict__ pre = g.pre ? (const IT*)g.pre + z1 * g.sC1 + z2 * g.sC2 : nullptr;
  IT* __restrict__ aux = g.aux ? (IT*)g.aux + z1 * g.sC1 + z2 * g.sC2 : nullptr;
  for (int pb = 0; pb < NR; pb += RB) {
    float v[RB][EPC];
    float rv[RB][EPC];
    float pv[RB][EPC];
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int row = r0 + (pb + q) * RPP, m = m0 + row;
      const bool ok = m < g.M;
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[q][e] = Cs[row * FST + chn * EPC + e];
      if (res) {
#pragma unroll
        for (int e = 0; e < EPC; e += 4) {
          const float4 c = ok ? *(const float4*)(res + (size_t)m * g.ldr + n + e) : make_float4(0.f, 0.f, 0.f, 0.f);
          rv[q][e] = c.x; rv[q][e + 1] = c.y; rv[q][e + 2] = c.z; rv[q][e + 3] = c.w;
        }
      }
      if (pre) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) pv[q][e] = ok ? g_ld(pre + (size_t)m * g.ldpre + n + e) : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int row = r0 + (pb + q) * RPP, m = m0 + row;
      if (m >= g.M) continue;
      float* w = v[q];
#pragma unroll
      for (int e = 0; e < EPC; ++e) w[e] = w[e] * g.alpha + bv[e];
      if (aux) {
        IT* ap = aux + (size_t)m * g.ldaux + n;
#pragma unroll
        for (int e = 0; e < EPC; e += 4) g_store_aux(ap + e, w + e);
      }
      if (!pre) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) w[e] = g_act(ACT, w[e]);
      }
      if (g.dp > 0.f) {
#pragma unroll
        for (int e = 0; e < EPC; e += 4) {
          bool keep[4];
          dropout_keep4v(rseed, roff, g.site, ebase + (unsigned long long)m * g.N + n + e, g.dp, keep);
#pragma unroll
          for (int t = 0; t < 4; ++t) w[e + t] = keep[t] ? w[e + t] * ks : 0.f;
        }
      }
      if (pre) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) w[e] *= g_act_grad(ACT, pv[q][e]);
      }
#pragma unroll
      for (int e = 0; e < EPC; ++e) w[e] *= sv[e];
      if (res) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) w[e] += rv[q][e];
      }
      if (g.dbias) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) csum[e] += w[e];
      }
      OutT* dst = C + (size_t)m * g.ldc + n;
      if constexpr (sizeof(OutT) == 4) {
        *(float4*)dst = make_float4(w[0], w[1], w[2], w[3]);
      } else {
        uint4 o;
        o.x = (uint32_t)f2bf(w[0]) | ((uint32_t)f2bf(w[1]) << 16);
        o.y = (uint32_t)f2bf(w[2]) | ((uint32_t)f2bf(w[3]) << 16);
        o.z = (uint32_t)f2bf(w[4]) | ((uint32_t)f2bf(w[5]) << 16);
        o.w = (uint32_t)f2bf(w[6]) | ((uint32_t)f2bf(w[7]) << 16);
        *(uint4*)dst = o;
      }
    }
  }
}

template <typename IT, typename OutT, int BM, int BN, int NTH>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& g, float* Cs, int tid, int m0, int n0, int z) {
  constexpr int EPC = 16 / sizeof(OutT);
  constexpr int CPR = BN / EPC;
  float csum[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) csum[e] = 0.f;
  // the activation as a compile-time choice: a runtime switch per element was if-converted
  switch (g.act) {
    case DMF_ACT_RELU: gemm_epilogue_act<IT, OutT, BM, BN, NTH, DMF_ACT_RELU>(g, Cs, tid, m0, n0, z, csum); break;
    case DMF_ACT_GELU: gemm_epilogue_act<IT, OutT, BM, BN, NTH, DMF_ACT_GELU>(g, Cs, tid, m0, n0, z, csum); break;
    case DMF_ACT_SIGMOID: gemm_epilogue_act<IT, OutT, BM, BN, NTH, DMF_ACT_SIGMOID>(g, Cs, tid, m0, n0, z, csum); break;
    default: gemm_epilogue_act<IT, OutT, BM, BN, NTH, DMF_ACT_NONE>(g, Cs, tid, m0, n0, z, csum); break;
  }
  if (g.dbias) {
    // threads sharing a chunk column: tid % CPR; reduce through LDS into this M tile's slab row
    // (dbias = the slab's column sums in tile order, after the launch: deterministic)
    __syncthreads();
#pragma unroll
    for (int e = 0; e < EPC; ++e) Cs[tid * EPC + e] = csum[e];
    __syncthreads();
    if (tid < BN) {
      const int c = tid, cc = c / EPC, ce = c % EPC;
      float s = 0.f;
      for (int t = cc; t < NTH; t += CPR) s += Cs[t * EPC + ce];
      if (n0 + c < g.N) g.dbias_ws[(size_t)(m0 / BM) * g.N + n0 + c] = s;
    }
  }
}

template <typename IT, typename OutT, bool TA, bool TB>
__global__ void __launch_bounds__(GTHREADS, 2) k_gemm(GemmArgs g) {
  constexpr int GBK = 128 / sizeof(IT);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int mt = blockIdx.x / g.ntiles, nt = blockIdx.x % g.ntiles;
  const int m0 = mt * GBM, n0 = nt * GBN;
  const int z = blockIdx.z, z1 = z / g.H, z2 = z - (z / g.H) * g.H;
  const IT* A = (const IT*)g.A + z1 * g.sA1 + z2 * g.sA2;
  const IT* B = (const IT*)g.B + z1 * g.sB1 + z2 * g.sB2;

  TileLoad<TA, IT> la;
  TileLoad<TB, IT> lb;
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
      if constexpr (sizeof(IT) == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(g_bf16x8_t*)&av[i], *(g_bf16x8_t*)&bv[j],
                                                                acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(((const uint32_t*)&av[i])[e]),
                                                               __uint_as_float(((const uint32_t*)&bv[j])[e]),
                                                               acc[i][j], 0, 0, 0);
      }
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
  gemm_epilogue<IT, OutT, GBM, GBN, GTHREADS>(g, Cs, tid, m0, n0, z);
}


// ----------------------------------------------------- softmax + dropout
// One wave per row of length L (fp32 scores S): p = softmax(scale * s);
// Ps (PT: bf16, or f32 in the parity mode) = p (kept for backward);
// Pd = dropout(p) / (1 - dp) (the operand of P v). Dropout element index =
// row * L + col (site `site`). Columns >= Lv are key padding (a token count
// rounded up to the GEMM granule): excluded from the max / sum, p = 0 there.
__device__ __forceinline__ float4 g_ld4(const bf16_t* p) {
  const uint2 u = *(const uint2*)p;
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ float4 g_ld4(const float* p) { return *(const float4*)p; }

template <typename PT>
__global__ void __launch_bounds__(256) k_softmax_drop(const float* __restrict__ S, int lds_, long long rows, int L,
                                                      int Lv, float scale, float dp, const unsigned long long* rng,
                                                      int site, PT* __restrict__ Ps, PT* __restrict__ Pd, int ldp) {
  const unsigned long long rseed_ = rng ? rng[0] : 0ull, roff_ = rng ? rng[1] : 0ull;  // read once (see dropout_keep4v)
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* s = S + row * lds_;
  auto ld = [&](int c) {  // 4 scores, key padding at -inf
    float4 v = *(const float4*)(s + c);
    if (c + 3 >= Lv) {
      if (c >= Lv) v.x = -INFINITY;
      if (c + 1 >= Lv) v.y = -INFINITY;
      if (c + 2 >= Lv) v.z = -INFINITY;
      v.w = -INFINITY;
    }
    return v;
  };
  float mx = -INFINITY;
  for (int c = lane * 4; c < L; c += 256) {
    const float4 v = ld(c);
    mx = fmaxf(mx, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float sum = 0.f;
  for (int c = lane * 4; c < L; c += 256) {
    const float4 v = ld(c);
    sum += __expf((v.x - mx) * scale) + __expf((v.y - mx) * scale) + __expf((v.z - mx) * scale) +
           __expf((v.w - mx) * scale);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  const float inv = 1.f / sum;
  const float ks = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  for (int c = lane * 4; c < L; c += 256) {
    const float4 v = ld(c);
    float p[4] = {__expf((v.x - mx) * scale) * inv, __expf((v.y - mx) * scale) * inv,
                  __expf((v.z - mx) * scale) * inv, __expf((v.w - mx) * scale) * inv};
    g_store_aux(Ps + row * ldp + c, p);
    if (dp > 0.f) {
      bool keep[4];
      dropout_keep4v(rseed_, roff_, site, (unsigned long long)(row * L + c), dp, keep);
#pragma unroll
      for (int e = 0; e < 4; ++e) p[e] = keep[e] ? p[e] * ks : 0.f;
    }
    g_store_aux(Pd + row * ldp + c, p);
  }
}

// dS = scale * P * (g - sum_j P g), g = dPd * keep / (1 - dp)   (PT out)
template <typename PT>
__global__ void __launch_bounds__(256) k_softmax_drop_bwd(const PT* __restrict__ Ps, int ldp,
                                                          const float* __restrict__ dPd, int ldg, long long rows,
                                                          int L, float scale, float dp,
                                                          const unsigned long long* rng, int site,
                                                          PT* __restrict__ dS, int lds_) {
  const unsigned long long rseed_ = rng ? rng[0] : 0ull, roff_ = rng ? rng[1] : 0ull;  // read once (see dropout_keep4v)
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float ks = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  float dot = 0.f;
  for (int c = lane * 4; c < L; c += 256) {
    const float4 pv = g_ld4(Ps + row * ldp + c);
    const float4 gv = *(const float4*)(dPd + row * ldg + c);
    float gg[4] = {gv.x, gv.y, gv.z, gv.w};
    if (dp > 0.f) {
      bool keep[4];
      dropout_keep4v(rseed_, roff_, site, (unsigned long long)(row * L + c), dp, keep);
#pragma unroll
      for (int e = 0; e < 4; ++e) gg[e] = keep[e] ? gg[e] * ks : 0.f;
    }
    dot += pv.x * gg[0] + pv.y * gg[1] + pv.z * gg[2] + pv.w * gg[3];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
  for (int c = lane * 4; c < L; c += 256) {
    const float4 pv = g_ld4(Ps + row * ldp + c);
    const float4 gv = *(const float4*)(dPd + row * ldg + c);
    float gg[4] = {gv.x, gv.y, gv.z, gv.w};
    if (dp > 0.f) {
      bool keep[4];
      dropout_keep4v(rseed_, roff_, site, (unsigned long long)(row * L + c), dp, keep);
#pragma unroll
      for (int e = 0; e < 4; ++e) gg[e] = keep[e] ? gg[e] * ks : 0.f;
    }
    const float o[4] = {scale * pv.x * (gg[0] - dot), scale * pv.y * (gg[1] - dot), scale * pv.z * (gg[2] - dot),
                        scale * pv.w * (gg[3] - dot)};
    g_store_aux(dS + row * lds_ + c, o);
  }
}

}  // namespace dmf

using namespace dmf;

template <typename IT>
static int gemm_launch(const char* name, int out_dtype, int ta, int tb, int M, int N, int K, float alpha,
                       const void* A, int lda, long long sA1, long long sA2, const void* B, int ldb, long long sB1,
                       long long sB2, void* C, int ldc, long long sC1, long long sC2, int batch1, int batch2,
                       const float* bias, int act, const float* colscale, const float* res, int ldr, void* aux,
                       int ldaux, const void* pre, int ldpre, float dropout_p, const unsigned long long* rng,
                       int site, float* dbias, float* dbias_ws, void* stream) {
  constexpr int ie = 16 / sizeof(IT);  // operand elements per 16 bytes
  DMF_CHECK_ARG(out_dtype == DMF_F32 || out_dtype == DMF_BF16, "%s: bad out dtype %d", name, out_dtype);
  DMF_CHECK_ARG(M > 0 && N > 0 && K > 0 && batch1 > 0 && batch2 > 0, "%s: empty problem", name);
  DMF_CHECK_ARG(K % ie == 0 && lda % ie == 0 && ldb % ie == 0, "%s: K (%d) and lda/ldb must be multiples of %d",
                name, K, ie);
  DMF_CHECK_ARG(!ta || M % ie == 0, "%s: transposed A needs M %% %d == 0", name, ie);
  DMF_CHECK_ARG(!tb || N % ie == 0, "%s: transposed B needs N %% %d == 0", name, ie);
  const int epc = out_dtype == DMF_F32 ? 4 : 8;
  DMF_CHECK_ARG(N % epc == 0 && ldc % epc == 0, "%s: N (%d) and ldc must be multiples of %d", name, N, epc);
  DMF_CHECK_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0 && ((uintptr_t)C % 16) == 0 &&
                    sA1 % ie == 0 && sA2 % ie == 0 && sB1 % ie == 0 && sB2 % ie == 0 && sC1 % epc == 0 &&
                    sC2 % epc == 0,
                "%s: operands and batch strides must be 16-byte aligned", name);
  DMF_CHECK_ARG(!res || (batch1 * batch2 == 1 && ldr % 4 == 0 && ((uintptr_t)res % 16) == 0),
                "%s: residual needs an unbatched, 16-byte aligned f32 operand", name);
  DMF_CHECK_ARG(!aux || (ldaux % 4 == 0 && ((uintptr_t)aux % (4 * sizeof(IT))) == 0),
                "%s: aux rows must hold whole, aligned groups of 4", name);
  DMF_CHECK_ARG(dropout_p <= 0.f || (rng && dropout_p < 1.f), "%s: dropout needs rng state and p < 1", name);
  DMF_CHECK_ARG(!dbias || (dbias_ws && batch1 * batch2 == 1), "%s: dbias needs an unbatched problem and its "
                "workspace (cdiv(M, 128) * N floats)", name);
  GemmArgs g{A, B, C, bias, M, N, K, lda, ldb, ldc, batch2,
             sA1, sA2, sB1, sB2, sC1, sC2, alpha, act, cdiv(N, GBN), colscale, res, ldr, aux, ldaux,
             pre, ldpre, dropout_p, rng, site, dbias, dbias_ws};
  const dim3 grid((unsigned)(cdiv(M, GBM) * g.ntiles), 1, (unsigned)(batch1 * batch2));
  DMF_CHECK_ARG((long long)cdiv(M, GBM) * g.ntiles < (1LL << 31) && batch1 * batch2 < 65536, "%s: grid too large",
                name);
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = 2 * GSTAGE > GBM * (GBN + 4) * 4 ? 2 * GSTAGE : GBM * (GBN + 4) * 4;
#define DMF_G(OT, TA_, TB_) hipLaunchKernelGGL((k_gemm<IT, OT, TA_, TB_>), grid, dim3(GTHREADS), lds, st, g)
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
  DMF_LAUNCH_CHECK(name);
  if (dbias) return dmf_colsum_f32(dbias_ws, N, cdiv(M, GBM), N, dbias, 1, stream);
  return 0;
}

extern "C" int dmf_gemm_bf16(int out_dtype, int ta, int tb, int M, int N, int K, float alpha, const void* A, int lda,
                             long long sA1, long long sA2, const void* B, int ldb, long long sB1, long long sB2,
                             void* C, int ldc, long long sC1, long long sC2, int batch1, int batch2,
                             const float* bias, int act, const float* colscale, const float* res, int ldr, void* aux,
                             int ldaux, const void* pre, int ldpre, float dropout_p,
                             const unsigned long long* rng, int site, float* dbias, float* dbias_ws, void* stream) {
  return gemm_launch<bf16_t>("dmf_gemm_bf16", out_dtype, ta, tb, M, N, K, alpha, A, lda, sA1, sA2, B, ldb, sB1, sB2,
                             C, ldc, sC1, sC2, batch1, batch2, bias, act, colscale, res, ldr, aux, ldaux, pre, ldpre,
                             dropout_p, rng, site, dbias, dbias_ws, stream);
}

extern "C" int dmf_gemm_f32(int out_dtype, int ta, int tb, int M, int N, int K, float alpha, const float* A, int lda,
                            long long sA1, long long sA2, const float* B, int ldb, long long sB1, long long sB2,
                            void* C, int ldc, long long sC1, long long sC2, int batch1, int batch2,
                            const float* bias, int act, const float* colscale, const float* res, int ldr, float* aux,
                            int ldaux, const float* pre, int ldpre, float dropout_p,
                            const unsigned long long* rng, int site, float* dbias, float* dbias_ws, void* stream) {
  return gemm_launch<float>("dmf_gemm_f32", out_dtype, ta, tb, M, N, K, alpha, A, lda, sA1, sA2, B, ldb, sB1, sB2,
                            C, ldc, sC1, sC2, batch1, batch2, bias, act, colscale, res, ldr, aux, ldaux, pre, ldpre,
                            dropout_p, rng, site, dbias, dbias_ws, stream);
}

template <typename PT>
static int softmax_launch(const char* name, const float* S, int lds, long long rows, int L, int Lv, float scale,
                          float dropout_p, const unsigned long long* rng, int site, void* probs, void* probs_dropped,
                          int ldp, void* stream) {
  DMF_CHECK_ARG(L % 4 == 0 && lds % 4 == 0 && ldp % 4 == 0, "%s: L and strides must be multiples of 4", name);
  DMF_CHECK_ARG(Lv > 0 && Lv <= L, "%s: valid length %d must be in [1, L=%d]", name, Lv, L);
  DMF_CHECK_ARG(dropout_p <= 0.f || rng, "%s: dropout needs rng state", name);
  DMF_CHECK_ARG(dropout_p < 1.f, "%s: p must be < 1", name);
  if (rows == 0) return 0;
  hipLaunchKernelGGL(k_softmax_drop<PT>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, S, lds,
                     rows, L, Lv, scale, dropout_p, rng, site, (PT*)probs, (PT*)probs_dropped, ldp);
  DMF_LAUNCH_CHECK(name);
  return 0;
}

template <typename PT>
static int softmax_bwd_launch(const char* name, const void* probs, int ldp, const float* dprobs_dropped, int ldg,
                              long long rows, int L, float scale, float dropout_p, const unsigned long long* rng,
                              int site, void* dscores, int lds, void* stream) {
  DMF_CHECK_ARG(L % 4 == 0 && ldp % 4 == 0 && ldg % 4 == 0 && lds % 4 == 0, "%s: L and strides must be multiples of 4",
                name);
  DMF_CHECK_ARG(dropout_p <= 0.f || rng, "%s: dropout needs rng state", name);
  if (rows == 0) return 0;
  hipLaunchKernelGGL(k_softmax_drop_bwd<PT>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     (const PT*)probs, ldp, dprobs_dropped, ldg, rows, L, scale, dropout_p, rng, site, (PT*)dscores,
                     lds);
  DMF_LAUNCH_CHECK(name);
  return 0;
}

extern "C" int dmf_softmax_dropout(const float* S, int lds, long long rows, int L, int Lv, float scale,
                                   float dropout_p, const unsigned long long* rng, int site, void* probs,
                                   void* probs_dropped, int ldp, void* stream) {
  return softmax_launch<bf16_t>("dmf_softmax_dropout", S, lds, rows, L, Lv, scale, dropout_p, rng, site, probs,
                                probs_dropped, ldp, stream);
}

extern "C" int dmf_softmax_dropout_f32(const float* S, int lds, long long rows, int L, int Lv, float scale,
                                       float dropout_p, const unsigned long long* rng, int site, float* probs,
                                       float* probs_dropped, int ldp, void* stream) {
  return softmax_launch<float>("dmf_softmax_dropout_f32", S, lds, rows, L, Lv, scale, dropout_p, rng, site, probs,
                               probs_dropped, ldp, stream);
}

extern "C" int dmf_softmax_dropout_bwd(const void* probs, int ldp, const float* dprobs_dropped, int ldg,
                                       long long rows, int L, float scale, float dropout_p,
                                       const unsigned long long* rng, int site, void* dscores, int lds,
                                       void* stream) {
  return softmax_bwd_launch<bf16_t>("dmf_softmax_dropout_bwd", probs, ldp, dprobs_dropped, ldg, rows, L, scale,
                                    dropout_p, rng, site, dscores, lds, stream);
}

extern "C" int dmf_softmax_dropout_bwd_f32(const float* probs, int ldp, const float* dprobs_dropped, int ldg,
                                           long long rows, int L, float scale, float dropout_p,
                                           const unsigned long long* rng, int site, float* dscores, int lds,
                                           void* stream) {
  return softmax_bwd_launch<float>("dmf_softmax_dropout_bwd_f32", probs, ldp, dprobs_dropped, ldg, rows, L, scale,
                                   dropout_p, rng, site, dscores, lds, stream);
}
