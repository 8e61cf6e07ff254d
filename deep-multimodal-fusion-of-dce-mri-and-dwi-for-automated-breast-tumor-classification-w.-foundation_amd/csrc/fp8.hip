// fp8 (OCP e4m3fn) patch-embed GEMM of configuration 5: PatchEmbed.proj, a
// conv with kernel = stride = patch (transformer_model.py:7-32), as
//   tokens[m][e] = rs[m] * ws[e] * sum_k q8(x)[m][k] * q8(W)[e][k] + bias[e]
// m = (n, ho, wo) token, k = (r, s, c) patch element (the conv engine's
// [Cout][KH][KW][CinP] order). Activations are scaled per token row and the
// weights per output channel so each row's max maps to 448 (e4m3 max), then
// packed with v_cvt_pk_fp8_f32; the GEMM runs v_mfma_f32_16x16x32_fp8_fp8
// (fp32 accumulation) and the scales are applied in the epilogue. The
// backward stays bf16 (the straight-through estimate through the
// quantisation, like fp8 training recipes keep it).
#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

typedef __attribute__((ext_vector_type(4))) float f8_f32x4;

__device__ __forceinline__ uint2 pack8_e4m3(const float v[8]) {
  int w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
  w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], w0, true);
  int w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], 0, false);
  w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], w1, true);
  return make_uint2((unsigned)w0, (unsigned)w1);
}

// one wave per token row: gather the P x P patch from NHWC bf16, row amax,
// scale, pack (8 elements per lane per pass; C % 8 == 0 so a chunk never
// crosses a tap)
__global__ void __launch_bounds__(256) k_patch_quant(const bf16_t* __restrict__ x, int H, int W, int C, int ldx, int P,
                                                     int Ho, int Wo, uint8_t* __restrict__ q, int ldq,
                                                     float* __restrict__ rscale, long long M) {
  const int lane = threadIdx.x & 63;
  const long long m = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;  // wave-uniform
  const int K = P * P * C;
  const int hw = Ho * Wo;
  const int n = (int)(m / hw), rem = (int)(m - (long long)n * hw);
  const int ho = rem / Wo, wo = rem - ho * Wo;
  auto src = [&](int k) {
    const int tap = k / C, c = k - tap * C;
    const int r = tap / P, s = tap - (tap / P) * P;
    return x + ((size_t)(n * H + ho * P + r) * W + wo * P + s) * ldx + c;
  };
  float amax = 0.f;
  for (int k = lane * 8; k < K; k += 512) {
    float v[8];
    ld8(src(k), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
  }
  amax = wave_max(amax);
  const float sc = amax > 0.f ? 448.f / amax : 1.f;
  for (int k = lane * 8; k < K; k += 512) {
    float v[8];
    ld8(src(k), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= sc;
    *(uint2*)(q + (size_t)m * ldq + k) = pack8_e4m3(v);
  }
  if (lane == 0) rscale[m] = amax > 0.f ? amax / 448.f : 1.f;
}

// one wave per output channel: torch conv weight [E][C][P][P] (fp32) ->
// e4m3 rows [E][(r,s,c)], per-channel scale
__global__ void __launch_bounds__(256) k_weight_quant(const float* __restrict__ w, int E, int C, int P,
                                                      uint8_t* __restrict__ q, float* __restrict__ cscale) {
  const int lane = threadIdx.x & 63;
  const int e_ = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e_ >= E) return;
  const int K = P * P * C;
  auto at = [&](int k) {
    const int tap = k / C, c = k - tap * C;
    const int r = tap / P, s = tap - (tap / P) * P;
    return w[(((size_t)e_ * C + c) * P + r) * P + s];
  };
  float amax = 0.f;
  for (int k = lane; k < K; k += 64) amax = fmaxf(amax, fabsf(at(k)));
  amax = wave_max(amax);
  const float sc = amax > 0.f ? 448.f / amax : 1.f;
  for (int k = lane * 8; k < K; k += 512) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = at(k + e) * sc;
    *(uint2*)(q + (size_t)e_ * K + k) = pack8_e4m3(v);
  }
  if (lane == 0) cscale[e_] = amax > 0.f ? amax / 448.f : 1.f;
}

// C[m][n] (bf16) = as[m] * bs[n] * sum_k A[m][k] B[n][k] + bias[n]; A, B e4m3
// K-contiguous rows. 128x128 tile, 256 threads (2x2 waves of 64x64 = 4x4
// 16x16x32 fragments), K-step 128 (one 128-B LDS row per operand row, 16-B
// chunks XOR-swizzled by row&7), register-staged double buffer.
constexpr int F8BM = 128, F8BN = 128, F8BK = 128;
constexpr int F8STAGE = (F8BM + F8BN) * F8BK;

__global__ void __launch_bounds__(256, 2) k_gemm_fp8(const uint8_t* __restrict__ A, int lda,
                                                     const float* __restrict__ as, const uint8_t* __restrict__ B,
                                                     int ldb, const float* __restrict__ bs,
                                                     const float* __restrict__ bias, bf16_t* __restrict__ Cm, int ldc,
                                                     int M, int N, int K, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int mt = blockIdx.x / ntiles, nt = blockIdx.x % ntiles;
  const int m0 = mt * F8BM, n0 = nt * F8BN;
  // loader: 128 rows x 8 chunks per operand; thread -> chunk tid&7 of rows tid>>3 + 32i
  const int lq = tid & 7, lr = tid >> 3;
  uint4 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = lr + 32 * i, k = k0 + lq * 16;
      ra[i] = (m0 + r < M && k < K) ? *(const uint4*)(A + (size_t)(m0 + r) * lda + k) : make_uint4(0, 0, 0, 0);
      rb[i] = (n0 + r < N && k < K) ? *(const uint4*)(B + (size_t)(n0 + r) * ldb + k) : make_uint4(0, 0, 0, 0);
    }
  };
  auto lstore = [&](char* S) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = lr + 32 * i;
      *(uint4*)(S + row * 128 + ((lq ^ (row & 7)) << 4)) = ra[i];
      *(uint4*)(S + F8BM * 128 + row * 128 + ((lq ^ (row & 7)) << 4)) = rb[i];
    }
  };
  f8_f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f8_f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (K + F8BK - 1) / F8BK;
  gload(0);
  lstore(smem);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const char* S = smem + (kt & 1) * F8STAGE;
    if (kt + 1 < nk) gload((kt + 1) * F8BK);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int ch = kk * 2 + (fg >> 1), half = (fg & 1) * 8;
      long av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + fr;
        av[i] = *(const long*)(S + row * 128 + ((ch ^ (row & 7)) << 4) + half);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + fr;
        bv[j] = *(const long*)(S + F8BM * 128 + col * 128 + ((ch ^ (col & 7)) << 4) + half);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(smem + ((kt + 1) & 1) * F8STAGE);
    __syncthreads();
  }
  // epilogue: D[4*fg + e][fr] of each 16x16 fragment, scaled and packed into a bf16 LDS image of the
  // tile, then written as whole 16-B row chunks (a lane's fragment values are one column of 4 rows:
  // stored straight, every wave instruction was 64 two-byte pieces scattered over 16 rows)
  constexpr int CST = F8BN + 8;  // bf16 elements per LDS row (16 B pad)
  bf16_t* Cs = (bf16_t*)smem;
  float rsc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + wm * 64 + i * 16 + fg * 4 + e;
      rsc[i][e] = m < M ? as[m] : 0.f;
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cl = wn * 64 + j * 16 + fr, n = n0 + cl;
    const float sb = n < N ? bs[n] : 0.f, bb = (bias && n < N) ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Cs[(wm * 64 + i * 16 + fg * 4 + e) * CST + cl] = f2bf(acc[i][j][e] * rsc[i][e] * sb + bb);
  }
  __syncthreads();
  for (int idx = tid; idx < F8BM * (F8BN / 8); idx += 256) {
    const int row = idx / (F8BN / 8), ch = idx - row * (F8BN / 8);
    const int m = m0 + row, n = n0 + ch * 8;
    if (m < M && n < N) *(uint4*)(Cm + (size_t)m * ldc + n) = *(const uint4*)(Cs + row * CST + ch * 8);
  }
}

// The same product on the block-scaled MFMA: v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 operands
// and unit E8M0 block scales (127 = 2^0) is the plain e4m3 dot product at twice the clock rate of
// the non-scaled form (MI355X_MICROARCH.md, MFMA table); the per-row / per-channel scales stay in
// the epilogue. Tile (16*FM) x 256 with 4 waves of (16*FM) x 64 (one wave per SIMD, FM x 4
// fragments, one MFMA per fragment per 128-B K-step). FM = 9 puts configuration 5's 18432 x 512
// patch-embed GEMM on exactly 256 workgroups (the 128x128 form ran 576 = 1.125 rounds of two per
// CU). A and B rows go global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) into a 3-stage ring,
// two K-steps in flight, the conv engine's source-side XOR swizzle (k_conv_fwd_wide); rows past
// M / N and K-chunks past K read zeros from the buffer range check. A lane's 32 K-bytes are the
// two 16-B chunks 2*(lane>>4), +1 of its row, for A and B alike (the sum over K is the same for
// any K order shared by both operands).
typedef __attribute__((ext_vector_type(8))) int f8_v8i;
constexpr int F8S_BN = 256, F8S_NST = 3;
__host__ __device__ constexpr int f8s_stage(int fm) { return (16 * fm + F8S_BN) * 128; }
__host__ __device__ constexpr int f8s_lds(int fm) {
  return F8S_NST * f8s_stage(fm) > 16 * fm * (F8S_BN + 8) * 2 ? F8S_NST * f8s_stage(fm) : 16 * fm * (F8S_BN + 8) * 2;
}

template <int FM>
__global__ void __launch_bounds__(256, 1) k_gemm_fp8_dma(const uint8_t* __restrict__ A, int lda,
                                                         const float* __restrict__ as, const uint8_t* __restrict__ B,
                                                         int ldb, const float* __restrict__ bs,
                                                         const float* __restrict__ bias, bf16_t* __restrict__ Cm,
                                                         int ldc, int M, int N, int K, int ntiles) {
  constexpr int TBM = 16 * FM, GA = TBM / 8, G = GA + F8S_BN / 8, NGW = (G + 3) / 4;
  constexpr int STAGE = f8s_stage(FM);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lin / ntiles, nt = lin % ntiles;
  const int m0 = mt * TBM, n0 = nt * F8S_BN;
  const int lr = lane >> 3, lc = (lane & 7) ^ lr;
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  const v4i_t ra = buf_rsrc(A, (long long)M * lda), rb = buf_rsrc(B, (long long)N * ldb);

  // this wave's 8-row groups g = wid + 4t: A rows m0 + 8g + lr for g < GA, B rows n0 + 8(g - GA) + lr
  const int ng = (G - wid + 3) / 4;
  unsigned vo[NGW];
#pragma unroll
  for (int t = 0; t < NGW; ++t) {
    const int g = wid + 4 * t;
    if (g < GA) {
      const int r = m0 + 8 * g + lr;
      vo[t] = r < M ? (unsigned)(r * lda + lc * 16) : BUF_OOB;
    } else {
      const int r = n0 + 8 * (g - GA) + lr;
      vo[t] = r < N ? (unsigned)(r * ldb + lc * 16) : BUF_OOB;
    }
  }
  const int nk = (K + 127) / 128;
  auto issue = [&](int kt, int stage) {
    const int k0 = kt * 128;
    const bool kok = k0 + lc * 16 < K;
#pragma unroll
    for (int t = 0; t < NGW; ++t) {
      if (t < ng) {
        const int g = wid + 4 * t;
        dma16(g < GA ? ra : rb, kok ? vo[t] : BUF_OOB, (unsigned)k0, lds0 + stage * STAGE + g * 1024);
      }
    }
  };

  f8_f32x4 acc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f8_f32x4{0.f, 0.f, 0.f, 0.f};
  const int c0 = ((2 * fg) ^ (fr & 7)) * 16, c1 = ((2 * fg + 1) ^ (fr & 7)) * 16;

  issue(0, 0);
  if (nk > 1) issue(1, 1);
  int st = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // retire this wave's DMA of K-step kt (kt+1's stay in flight), then the barrier publishes every
    // wave's part and orders the refill of stage (kt+2)%3 after all reads of kt-1 (see k_conv_fwd_wide)
    if (kt + 1 < nk) {
      if (ng == NGW) asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(NGW) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(NGW - 1) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (kt + 2 < nk) issue(kt + 2, st == 0 ? 2 : st - 1);
    const char* S = smem + st * STAGE;
    f8_v8i bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const char* p = S + (TBM + wid * 64 + j * 16 + fr) * 128;
      const int4 lo = *(const int4*)(p + c0), hi = *(const int4*)(p + c1);
      bv[j] = f8_v8i{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const char* p = S + (i * 16 + fr) * 128;
      const int4 lo = *(const int4*)(p + c0), hi = *(const int4*)(p + c1);
      const f8_v8i av = f8_v8i{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv[j], acc[i][j], 0, 0, 0, 127, 0, 127);
    }
    st = st == 2 ? 0 : st + 1;
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  // epilogue as k_gemm_fp8: scales + bias into a bf16 LDS image, then 16-B row stores
  constexpr int CST = F8S_BN + 8;
  bf16_t* Cs = (bf16_t*)smem;
  float rsc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + i * 16 + fg * 4 + e;
      rsc[i][e] = m < M ? as[m] : 0.f;
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cl = wid * 64 + j * 16 + fr, n = n0 + cl;
    const float sb = n < N ? bs[n] : 0.f, bb = (bias && n < N) ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) Cs[(i * 16 + fg * 4 + e) * CST + cl] = f2bf(acc[i][j][e] * rsc[i][e] * sb + bb);
  }
  __syncthreads();
  for (int idx = tid; idx < TBM * (F8S_BN / 8); idx += 256) {
    const int row = idx / (F8S_BN / 8), ch = idx - row * (F8S_BN / 8);
    const int m = m0 + row, n = n0 + ch * 8;
    if (m < M && n < N) *(uint4*)(Cm + (size_t)m * ldc + n) = *(const uint4*)(Cs + row * CST + ch * 8);
  }
}

// 0: the 128x128 non-scaled form; 1 (default): the block-scaled 144x256 LDS-DMA form where it applies
static int g_fp8_var = 1, g_fp8_last = -1;

}  // namespace dmf

using namespace dmf;

extern "C" int dmf_gemm_fp8_tune(int var) {
  DMF_CHECK_ARG(var == 0 || var == 1, "dmf_gemm_fp8_tune: var %d (0 or 1)", var);
  g_fp8_var = var;
  return 0;
}
extern "C" int dmf_gemm_fp8_last_form(void) { return g_fp8_last; }

extern "C" int dmf_patch_quant_fp8(const void* x, int N, int H, int W, int C, int ldx, int P, void* q, int ldq,
                                   float* row_scale, void* stream) {
  DMF_CHECK_ARG(x && q && row_scale && N > 0 && P > 0 && C % 8 == 0 && ldx % 8 == 0 && ((uintptr_t)x % 16) == 0,
                "dmf_patch_quant_fp8: bad args (C=%d ldx=%d)", C, ldx);
  DMF_CHECK_ARG(H % P == 0 && W % P == 0 && ldq >= P * P * C && ldq % 8 == 0 && ((uintptr_t)q % 8) == 0,
                "dmf_patch_quant_fp8: bad geometry (H=%d W=%d P=%d ldq=%d)", H, W, P, ldq);
  const int Ho = H / P, Wo = W / P;
  const long long M = (long long)N * Ho * Wo;
  hipLaunchKernelGGL(k_patch_quant, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)x, H, W, C, ldx, P, Ho, Wo, (uint8_t*)q, ldq, row_scale, M);
  DMF_LAUNCH_CHECK("dmf_patch_quant_fp8");
  return 0;
}

extern "C" int dmf_weight_quant_fp8(const float* w, int E, int C, int P, void* q, float* col_scale, void* stream) {
  DMF_CHECK_ARG(w && q && col_scale && E > 0 && C > 0 && P > 0 && (P * P * C) % 8 == 0,
                "dmf_weight_quant_fp8: bad args");
  hipLaunchKernelGGL(k_weight_quant, dim3((unsigned)((E + 3) / 4)), dim3(256), 0, (hipStream_t)stream, w, E, C, P,
                     (uint8_t*)q, col_scale);
  DMF_LAUNCH_CHECK("dmf_weight_quant_fp8");
  return 0;
}

extern "C" int dmf_gemm_fp8(int M, int N, int K, const void* A, int lda, const float* a_scale, const void* B, int ldb,
                            const float* b_scale, const float* bias, void* C, int ldc, void* stream) {
  DMF_CHECK_ARG(A && B && C && a_scale && b_scale && M > 0 && N > 0 && K > 0, "dmf_gemm_fp8: bad args");
  DMF_CHECK_ARG(K % 16 == 0 && lda % 16 == 0 && ldb % 16 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0,
                "dmf_gemm_fp8: K (%d) and row strides must be multiples of 16 bytes", K);
  DMF_CHECK_ARG(N % 8 == 0 && ldc % 8 == 0 && ((uintptr_t)C % 16) == 0,
                "dmf_gemm_fp8: N (%d) and ldc must be multiples of 8, C 16-byte aligned (16-B row stores)", N);
  // block-scaled form: 32-bit buffer offsets; at least one chip-filling round of its tiles
  if (g_fp8_var == 1 && N >= F8S_BN && (long long)M * lda < (1LL << 31) && (long long)N * ldb < (1LL << 31) &&
      (long long)cdiv(M, 144) * cdiv(N, F8S_BN) >= 256) {
    const int nt = cdiv(N, F8S_BN);
    hipLaunchKernelGGL(k_gemm_fp8_dma<9>, dim3((unsigned)(cdiv(M, 144) * nt)), dim3(256), (size_t)f8s_lds(9),
                       (hipStream_t)stream, (const uint8_t*)A, lda, a_scale, (const uint8_t*)B, ldb, b_scale, bias,
                       (bf16_t*)C, ldc, M, N, K, nt);
    DMF_LAUNCH_CHECK("dmf_gemm_fp8");
    g_fp8_last = 1;
    return 0;
  }
  const int ntiles = cdiv(N, F8BN);
  const long long blocks = (long long)cdiv(M, F8BM) * ntiles;
  DMF_CHECK_ARG(blocks < (1LL << 31), "dmf_gemm_fp8: grid too large");
  hipLaunchKernelGGL(k_gemm_fp8, dim3((unsigned)blocks), dim3(256), (size_t)2 * F8STAGE, (hipStream_t)stream,
                     (const uint8_t*)A, lda, a_scale, (const uint8_t*)B, ldb, b_scale, bias, (bf16_t*)C, ldc, M, N, K,
                     ntiles);
  DMF_LAUNCH_CHECK("dmf_gemm_fp8");
  g_fp8_last = 0;
  return 0;
}
