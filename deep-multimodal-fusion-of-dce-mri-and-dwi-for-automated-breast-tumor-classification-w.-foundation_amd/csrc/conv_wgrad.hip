// Weight gradient of the implicit-GEMM convolution (NHWC), split over the
// pixel (reduction) axis into fp32 slabs that dmf_conv2d_wgrad_reduce sums
// deterministically into the torch-layout [Cout][Cin][KH][KW] gradient.
//   dW[co][(r,s,ci)] = sum_{m=(n,ho,wo)} dY[m][co] * X[n, ho*st-pad+r*dil, wo*st-pad+s*dil, ci]
// GEMM: M' = Cout, N' = KH*KW*Cin, K' = pixels. Both operands are
// pixel-major in HBM, so tiles are loaded along channels (16-B vectors,
// coalesced) and transposed into K'-contiguous LDS rows on the way in; the
// MFMA core is the same 128x128 / 4-wave / 16x16 fragment layout as conv.hip.
// Also: small-shape convolution kernels for the single-channel heads
// (ReconHead's 3x3 conv to recon_ch=1, MaskHeadResize.out 1x1 to 1 channel,
// model_module.py:117, :187) and the 1-input-channel 1x1 convs
// (MaskGuidedSpatialAttention.mask_processor[0], Projector on r1/r2,
// model_module.py:68, :639-640).
#include <algorithm>

#include "dmf_common.h"
#include "../../include/dmf_hip.h"

namespace dmf {

typedef __attribute__((ext_vector_type(8))) short bf16x8_w;
typedef __attribute__((ext_vector_type(4))) float f32x4_w;

struct WgArgs {
  const void* x;   // input NHWC [N][H][W][ldx]
  const void* dy;  // grad out NHWC [N][Ho][Wo][lddy]
  float* ws;       // slabs [splits][Cout][Ktot]
  int N, H, W, Cin, ldx;  // Cin = total channels over both sources
  const void* x2;         // optional channel-concat second source
  int C1, ldx2;
  int Ho, Wo, Cout, lddy;
  int KH, KW, stride, pad, dil;
  int Ktot, M;  // Ktot = KH*KW*Cin, M = N*Ho*Wo
  int mtiles, ntiles, splits, pix_per_split;
};

// (tile, split) of this block. (Ordering the blocks split-major per XCD, so the tiles of one pixel split
// share one L2, was measured within noise -- profiles/r05n_wgrad_xcd_ab.txt -- and removed in round 6.)
__device__ __forceinline__ int2 wg_block(const WgArgs&) { return make_int2(blockIdx.x, blockIdx.y); }

template <typename T>
__global__ void __launch_bounds__(256, 2) k_conv_wgrad(WgArgs a) {
  constexpr int EPC = 16 / sizeof(T);
  constexpr int BK = 8 * EPC;  // pixels per k-step
  constexpr int ROWB = 128;    // bytes per LDS row (BK elements)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tile = blockIdx.x;
  const int mt = tile / a.ntiles, nt = tile % a.ntiles;
  const int split = blockIdx.y;
  const int co0 = mt * 128, k0 = nt * 128;
  const int p_begin = split * a.pix_per_split;
  const int p_end = min(a.M, p_begin + a.pix_per_split);
  const T* __restrict__ X = (const T*)a.x;
  const T* __restrict__ DY = (const T*)a.dy;

  // loader: 128 channels = 128/EPC chunks per pixel row; BK pixel rows
  constexpr int CPR = 128 / EPC;            // chunks per pixel (16 bf16, 32 f32)
  constexpr int LOADS = BK * CPR / 256;     // per thread per operand (4 both)
  const int chunk = tid % CPR;
  const int prow = tid / CPR;               // 0 .. 256/CPR-1
  constexpr int PSTEP = 256 / CPR;

  // B' column chunk -> tap, ci (fixed per thread)
  const int kcol = k0 + chunk * EPC;
  const bool kok = kcol < a.Ktot;
  const int tap = kok ? kcol / a.Cin : 0;
  int ci = kcol - tap * a.Cin;
  const T* xsrc = X;
  int ldxs = a.ldx;
  if (ci >= a.C1) {
    xsrc = (const T*)a.x2;
    ci -= a.C1;
    ldxs = a.ldx2;
  }
  const int r = tap / a.KW, s = tap % a.KW;
  const int cocol = co0 + chunk * EPC;
  const bool cook = cocol < a.Cout;

  T ra[LOADS][EPC], rb[LOADS][EPC];
  auto gload = [&](int p0) {
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int p = p0 + prow + PSTEP * i;
      uint4 va = make_uint4(0, 0, 0, 0), vb = make_uint4(0, 0, 0, 0);
      if (p < p_end) {
        if (cook) va = *(const uint4*)(DY + (size_t)p * a.lddy + cocol);
        if (kok) {
          const int hw = a.Ho * a.Wo;
          const int n = p / hw, rem = p - n * hw;
          const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
          const int hi = ho * a.stride - a.pad + r * a.dil, wi = wo * a.stride - a.pad + s * a.dil;
          if (hi >= 0 && hi < a.H && wi >= 0 && wi < a.W)
            vb = *(const uint4*)(xsrc + ((size_t)(n * a.H + hi) * a.W + wi) * ldxs + ci);
        }
      }
      *(uint4*)ra[i] = va;
      *(uint4*)rb[i] = vb;
    }
  };
  // transpose store: element (channel row cr, pixel col pc) at
  // row*128 + ((pc/EPC) ^ (row&7))*16 + (pc%EPC)*sizeof(T)
  auto lds_store = [&](int stage) {
    char* As = smem + stage * 2 * 128 * ROWB;
    char* Bs = As + 128 * ROWB;
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int pc = prow + PSTEP * i;
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        const int row = chunk * EPC + e;
        const int off = row * ROWB + (((pc / EPC) ^ (row & 7)) << 4) + (pc % EPC) * (int)sizeof(T);
        *(T*)(As + off) = ra[i][e];
        *(T*)(Bs + off) = rb[i][e];
      }
    }
  };

  f32x4_w acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_w{0.f, 0.f, 0.f, 0.f};

  const int nk = (p_end - p_begin + BK - 1) / BK;
  if (nk > 0) {
    gload(p_begin);
    lds_store(0);
  }
  __syncthreads();
  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(p_begin + (kt + 1) * BK);
    const char* As = smem + cur * 2 * 128 * ROWB;
    const char* Bs = As + 128 * ROWB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + fg;
      uint4 av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + fr;
        av[i] = *(const uint4*)(As + row * ROWB + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + fr;
        bv[j] = *(const uint4*)(Bs + col * ROWB + ((ch ^ (col & 7)) << 4));
      }
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = mfma16<T>(av[i], bv[j], acc[i][j]);
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
    if (kt + 1 < nk) lds_store(cur ^ 1);
    __syncthreads();
  }
  // store slab: rows = co, cols = k
  float* slab = a.ws + (size_t)split * a.Cout * a.Ktot;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = co0 + wm * 64 + i * 16 + fg * 4 + q;
        const int k = k0 + wn * 64 + j * 16 + fr;
        if (co < a.Cout && k < a.Ktot) slab[(size_t)co * a.Ktot + k] = acc[i][j][q];
      }
}

// bf16 weight gradient on transposed LDS reads. Both operands stay pixel-major
// in LDS exactly as they arrive from HBM (16-B channel vectors, one 256-B row
// per pixel per 128-channel sub-image), and the MFMA fragments, which want 8
// consecutive pixels per lane, are gathered with ds_read_b64_tr_b16 (two
// 4-pixel x 16-channel blocks per fragment). Sub-image byte layout: 256-B rows
// with the 16-B chunk XOR (((row&3)<<2)|((row>>2)&3)), conflict-free for the
// 16x16x32 transposed reads. Register-staged double buffer, one barrier per
// 64-pixel K-step; each thread walks its gather rows' (n,ho,wo) incrementally.
typedef short v4s_w __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_w lds_v4s_w;

__device__ __forceinline__ int wtr_off(int row, int ch) {
  return (row << 8) + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

template <int WM, int WN, typename ET = bf16_t>
__global__ void __launch_bounds__(64 * WM * WN, (WM * WN <= 4) ? 2 : 1) k_conv_wgrad_tr(WgArgs a) {
  constexpr int T = 64 * WM * WN;
  constexpr int BM = 64 * WM, BN = 64 * WN, BK = 64;
  constexpr int SUB = BK * 256;                      // one 128-channel sub-image
  constexpr int STAGE = (BM / 128 + BN / 128) * SUB;  // A sub-images, then B
  constexpr int CPRA = BM / 8, RPPA = T / CPRA, PA = BK / RPPA;
  constexpr int CPRB = BN / 8, RPPB = T / CPRB, PB = BK / RPPB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int2 tb = wg_block(a);
  const int mt = tb.x / a.ntiles, nt = tb.x % a.ntiles;
  const int co0 = mt * BM, k0 = nt * BN;
  const int p_begin = tb.y * a.pix_per_split;
  const int p_end = min(a.M, p_begin + a.pix_per_split);
  const bf16_t* __restrict__ DY = (const bf16_t*)a.dy;

  // A loader: chunk of dY row (channels co0 + 8*ca ..)
  const int ca = tid % CPRA, ra = tid / CPRA;
  const int cocol = co0 + ca * 8;
  const bool cook = cocol < a.Cout;
  // B loader: chunk column -> (tap, ci, source), fixed per thread
  const int cb = tid % CPRB, rb = tid / CPRB;
  const int kcol = k0 + cb * 8;
  const bool kok = kcol < a.Ktot;
  const int tap = kok ? kcol / a.Cin : 0;
  int ci = kcol - tap * a.Cin;
  const bf16_t* xsrc = (const bf16_t*)a.x;
  int ldxs = a.ldx;
  if (ci >= a.C1) {
    xsrc = (const bf16_t*)a.x2;
    ci -= a.C1;
    ldxs = a.ldx2;
  }
  const int roff = (tap / a.KW) * a.dil - a.pad, soff = (tap % a.KW) * a.dil - a.pad;
  // gather-row cursors (n, ho, wo) of this thread's B rows at the current K-step
  int bn_[PB], bho[PB], bwo[PB];
  {
    const int hw = a.Ho * a.Wo;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int p = p_begin + rb + i * RPPB;
      bn_[i] = p / hw;
      const int rem = p - bn_[i] * hw;
      bho[i] = rem / a.Wo;
      bwo[i] = rem - bho[i] * a.Wo;
    }
  }
  const int dho = BK / a.Wo, dwo = BK % a.Wo;

  uint4 sa[PA], sb[PB];
  auto gload = [&](int kb) {
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int p = kb + ra + i * RPPA;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (cook && p < p_end) v = *(const uint4*)(DY + (size_t)p * a.lddy + cocol);
      sa[i] = v;
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int p = kb + rb + i * RPPB;
      const int hi = bho[i] * a.stride + roff, wi = bwo[i] * a.stride + soff;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (kok && p < p_end && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W)
        v = *(const uint4*)(xsrc + ((size_t)(bn_[i] * a.H + hi) * a.W + wi) * ldxs + ci);
      sb[i] = v;
      // advance this row's cursor by one K-step
      int wo = bwo[i] + dwo, ho = bho[i] + dho, n = bn_[i];
      if (wo >= a.Wo) { wo -= a.Wo; ++ho; }
      while (ho >= a.Ho) { ho -= a.Ho; ++n; }
      bwo[i] = wo; bho[i] = ho; bn_[i] = n;
    }
  };
  auto lds_store = [&](int stage) {
    char* S = smem + stage * STAGE;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int cc = ca * 8;
      *(uint4*)(S + (cc >> 7) * SUB + wtr_off(ra + i * RPPA, (cc & 127) >> 3)) = sa[i];
    }
    char* SB = S + (BM / 128) * SUB;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int cc = cb * 8;
      *(uint4*)(SB + (cc >> 7) * SUB + wtr_off(rb + i * RPPB, (cc & 127) >> 3)) = sb[i];
    }
  };

  f32x4_w acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_w{0.f, 0.f, 0.f, 0.f};

  const int nk = (p_end - p_begin + BK - 1) / BK;
  if (nk > 0) {
    gload(p_begin);
    lds_store(0);
  }
  __syncthreads();
  // transposed-read lane roles: group g, block row q, 4-column quarter p4
  const int g = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(p_begin + (kt + 1) * BK);
    const char* SA = smem + cur * STAGE;
    const char* SB = SA + (BM / 128) * SUB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_w af[4], bfr[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = kk * 32 + 8 * g + 4 * h + q;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int cl = wm * 64 + i * 16;
          const char* pa = SA + (cl >> 7) * SUB + wtr_off(row, ((cl & 127) >> 3) + (p4 >> 1)) + 8 * (p4 & 1);
          const v4s_w v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_w*)pa);
#pragma unroll
          for (int e = 0; e < 4; ++e) af[i][4 * h + e] = v[e];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cl = wn * 64 + j * 16;
          const char* pb = SB + (cl >> 7) * SUB + wtr_off(row, ((cl & 127) >> 3) + (p4 >> 1)) + 8 * (p4 & 1);
          const v4s_w v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_w*)pb);
#pragma unroll
          for (int e = 0; e < 4; ++e) bfr[j][4 * h + e] = v[e];
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = mfma16<ET>(__builtin_bit_cast(uint4, af[i]), __builtin_bit_cast(uint4, bfr[j]), acc[i][j]);
    }
    if (kt + 1 < nk) lds_store(cur ^ 1);
    __syncthreads();
  }
  float* slab = a.ws + (size_t)tb.y * a.Cout * a.Ktot;
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + wm * 64 + i * 16 + fg * 4 + e;
        const int k = k0 + wn * 64 + j * 16 + fr;
        if (co < a.Cout && k < a.Ktot) slab[(size_t)co * a.Ktot + k] = acc[i][j][e];
      }
}

// k_conv_wgrad_tr<2, 2> with both operands staged by LDS-DMA (buffer_load ...
// lds) instead of global -> VGPR -> ds_write_b128: the register-staged form
// spends 8 ds_write_b128 per thread per K-step (13 LDS-transfer cycles each,
// ~830 cycles per 64-pixel step at two workgroups per CU against ~1024 MFMA
// cycles), which the DMA path does not pay. Same 128x128 tile, 64-pixel
// K-steps, sub-image layout (wtr_off) and transposed fragment reads; the XOR
// swizzle is applied on the source side: DMA piece p of wave w lands rows
// 16w + 4p .. +3 (lane -> row 16w + 4p + lane/16, slot lane%16), so the lane
// loads chunk slot ^ (((lane/16) << 2) | p). Zero padding, pixel tails and
// channel tails read zeros from the buffer range check. Two stages, the next
// step's 8 pieces per wave issued right after the barrier that frees them.
// DUAL (channel-concat input): each 128-column tile must lie in one tap of
// one source (Cin % 128 == 0, C1 % 128 == 0), so the source is wave-uniform.
// FMW: 16-row output-channel fragments per wave (4: a 64x64 wave tile; 8: 128x64, the 256x256 tile of
// 8 waves, half the operand staging per MFMA of the 128x128 / 128x256 forms)
template <bool DUAL, int WM, int WN, int FMW = 4, typename ET = bf16_t>
__global__ void __launch_bounds__(64 * WM * WN, (WM * WN <= 4) ? 2 : 1) k_conv_wgrad_dma(WgArgs a) {
  constexpr int NW = WM * WN;
  constexpr int BM = 16 * FMW * WM, BN = 64 * WN, BK = 64, SUB = BK * 256;
  constexpr int SA_N = BM / 128, SB_N = BN / 128, STAGE = (SA_N + SB_N) * SUB;
  constexpr int PA = SA_N * 16 / NW, PB = SB_N * 16 / NW;  // 1 KiB DMA pieces per wave per operand
  static_assert(PA >= 1 && PB >= 1 && PA * NW == SA_N * 16 && PB * NW == SB_N * 16, "piece split");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int2 tb = wg_block(a);
  const int mt = tb.x / a.ntiles, nt = tb.x % a.ntiles;
  const int co0 = mt * BM, k0 = nt * BN;
  const int p_begin = tb.y * a.pix_per_split;
  const int p_end = min(a.M, p_begin + a.pix_per_split);
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem);

  const v4i_t rdy = buf_rsrc(a.dy, (long long)a.M * a.lddy * 2);
  // B source of this tile (one tap, one source when DUAL)
  const int tap0 = k0 / a.Cin;
  const bool hi_src = DUAL && (k0 - tap0 * a.Cin) >= a.C1;
  const v4i_t rx = hi_src ? buf_rsrc(a.x2, (long long)a.N * a.H * a.W * a.ldx2 * 2)
                          : buf_rsrc(a.x, (long long)a.N * a.H * a.W * a.ldx * 2);
  const int ldxs = hi_src ? a.ldx2 : a.ldx;

  // A piece i of this wave: global piece P = wid*PA + i -> sub-image P/16, rows 4*(P%16) .. +3
  // (lane row 4*(P%16) + lane/16); the lane stages chunk (lane%16) ^ ((lane/16 << 2) | (P & 3))
  int ach[PA], arow[PA];
  unsigned alds[PA];
  bool aok[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int P = wid * PA + i;
    const int ch = (lane & 15) ^ (((lane >> 4) << 2) | (P & 3));
    ach[i] = co0 + (P >> 4) * 128 + ch * 8;
    aok[i] = ach[i] < a.Cout;
    arow[i] = (P & 15) * 4;
    alds[i] = (unsigned)((P >> 4) * SUB + (P & 15) * 4 * 256);
  }
  int bci[PB], roff[PB], soff[PB], cn[PB], cho[PB], cwo[PB], brow[PB];
  unsigned blds[PB];
  bool bok[PB];
  const int hw = a.Ho * a.Wo;
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int P = wid * PB + i;
    const int ch = (lane & 15) ^ (((lane >> 4) << 2) | (P & 3));
    const int kcol = k0 + (P >> 4) * 128 + ch * 8;
    bok[i] = kcol < a.Ktot;
    const int tap = bok[i] ? kcol / a.Cin : 0;
    int ci = kcol - tap * a.Cin;
    if (hi_src) ci -= a.C1;
    bci[i] = ci;
    roff[i] = (tap / a.KW) * a.dil - a.pad;
    soff[i] = (tap % a.KW) * a.dil - a.pad;
    brow[i] = (P & 15) * 4;
    blds[i] = (unsigned)(SA_N * SUB + (P >> 4) * SUB + (P & 15) * 4 * 256);
    const int pix = p_begin + brow[i] + (lane >> 4);
    cn[i] = pix / hw;
    const int rem = pix - cn[i] * hw;
    cho[i] = rem / a.Wo;
    cwo[i] = rem - cho[i] * a.Wo;
  }
  const int dho = BK / a.Wo, dwo = BK % a.Wo;
  auto issue = [&](int stage, int kb) {
    const unsigned S = lds0 + stage * STAGE;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int pix = kb + arow[i] + (lane >> 4);
      const unsigned ao = (pix < p_end && aok[i]) ? (unsigned)(((long long)pix * a.lddy + ach[i]) * 2) : BUF_OOB;
      dma16(rdy, ao, 0, S + alds[i]);
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int pix = kb + brow[i] + (lane >> 4);
      const int hi = cho[i] * a.stride + roff[i], wi = cwo[i] * a.stride + soff[i];
      const bool ok = pix < p_end && bok[i] && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
      const unsigned bo = ok ? (unsigned)((((long long)(cn[i] * a.H + hi) * a.W + wi) * ldxs + bci[i]) * 2) : BUF_OOB;
      dma16(rx, bo, 0, S + blds[i]);
      int wo = cwo[i] + dwo, ho = cho[i] + dho, n = cn[i];
      if (wo >= a.Wo) { wo -= a.Wo; ++ho; }
      while (ho >= a.Ho) { ho -= a.Ho; ++n; }
      cwo[i] = wo; cho[i] = ho; cn[i] = n;
    }
  };

  f32x4_w acc[FMW][4];
#pragma unroll
  for (int i = 0; i < FMW; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_w{0.f, 0.f, 0.f, 0.f};

  const int nk = (p_end - p_begin + BK - 1) / BK;
  if (nk > 0) issue(0, p_begin);
  const int g = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt is the only DMA in flight: retire it; the barrier publishes every wave's
    // pieces and orders the refill of the other stage after every wave's reads of step kt-1
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + 1 < nk) issue((kt + 1) & 1, p_begin + (kt + 1) * BK);
    const char* SA = smem + (kt & 1) * STAGE;
    const char* SB = SA + SA_N * SUB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_w af[FMW], bfr[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = kk * 32 + 8 * g + 4 * h + q;
#pragma unroll
        for (int i = 0; i < FMW; ++i) {
          const int cl = wm * (16 * FMW) + i * 16;
          const char* pa = SA + (cl >> 7) * SUB + wtr_off(row, ((cl & 127) >> 3) + (p4 >> 1)) + 8 * (p4 & 1);
          const v4s_w v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_w*)pa);
#pragma unroll
          for (int e = 0; e < 4; ++e) af[i][4 * h + e] = v[e];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cl = wn * 64 + j * 16;
          const char* pb = SB + (cl >> 7) * SUB + wtr_off(row, ((cl & 127) >> 3) + (p4 >> 1)) + 8 * (p4 & 1);
          const v4s_w v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_w*)pb);
#pragma unroll
          for (int e = 0; e < 4; ++e) bfr[j][4 * h + e] = v[e];
        }
      }
#pragma unroll
      for (int i = 0; i < FMW; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = mfma16<ET>(__builtin_bit_cast(uint4, af[i]), __builtin_bit_cast(uint4, bfr[j]), acc[i][j]);
    }
  }
  float* slab = a.ws + (size_t)tb.y * a.Cout * a.Ktot;
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int i = 0; i < FMW; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + wm * (16 * FMW) + i * 16 + fg * 4 + e;
        const int k = k0 + wn * 64 + j * 16 + fr;
        if (co < a.Cout && k < a.Ktot) slab[(size_t)co * a.Ktot + k] = acc[i][j][e];
      }
}

// Gate gradient of a channel-gated conv input y = x * gate[n][c] (the SE
// block in front of the backbone stem, model_module.py:584-591) from the
// per-sample weight-gradient slabs G_n = sum_{pixels of n} dY (x) im2col(y):
//   sum_hw dL/dy[n,c,h,w] * y[n,c,h,w] = sum_{co,r,s} W[co][c][r][s] * G_n[co][(r,s,c)]
// so dgate[n][c] = that / gate[n][c]; the stem's input gradient is never formed.
__global__ void k_gate_grad_wslab(const float* __restrict__ ws, int Cout, int C, int CinP, int KK,
                                  const float* __restrict__ w, const float* __restrict__ gate,
                                  float* __restrict__ dgate) {
  __shared__ float red[16];
  const int c = blockIdx.x, n = blockIdx.y;
  const float* slab = ws + (size_t)n * Cout * KK * CinP;
  float acc = 0.f;
  for (int i = threadIdx.x; i < Cout * KK; i += blockDim.x) {
    const int co = i / KK, t = i - co * KK;
    acc += w[((size_t)co * C + c) * KK + t] * slab[((size_t)co * KK + t) * CinP + c];
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) dgate[(size_t)n * C + c] = acc / gate[(size_t)n * C + c];
}

// sum slabs, reorder [Cout][KH][KW][CinP] -> torch [Cout][Cin][KH][KW], accumulate.
// Threads walk the SLAB order (ci fastest: every split's read is coalesced),
// 32-bit index math, four splits' loads in flight; the torch-layout store is
// KH*KW-strided for 3x3 (1/splits of the traffic). The split sum keeps its
// fixed order (deterministic).
__global__ void __launch_bounds__(256) k_wgrad_reduce(const float* __restrict__ ws, int splits, int Cout, int Cin,
                                                      int CinP, int KH, int KW, float* __restrict__ dw,
                                                      int accumulate) {
  const int KK = KH * KW;
  const int total = Cout * KK * Cin;  // slab elements that map to a torch element
  const long long slab = (long long)Cout * KK * CinP;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int ci = i % Cin, t = i / Cin;  // t = co * KK + rs
    const int co = t / KK, rs = t - co * KK;
    const float* src = ws + (long long)t * CinP + ci;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
    int sp = 0;
    for (; sp + 4 <= splits; sp += 4) {
      v0 += src[(sp + 0) * slab];
      v1 += src[(sp + 1) * slab];
      v2 += src[(sp + 2) * slab];
      v3 += src[(sp + 3) * slab];
    }
    for (; sp < splits; ++sp) v0 += src[sp * slab];
    const float v = (v0 + v1) + (v2 + v3);
    float* d = dw + ((long long)co * Cin + ci) * KK + rs;
    *d = accumulate ? *d + v : v;
  }
}

// The same sum for small weights with many splits (a 64x64 1x1 weight runs ~128-512 splits): one
// thread per element walked `splits` slabs in a chain of dependent load rounds (4096 weights x 512
// splits: 28 us). Here SL split lanes per element each sum every SL-th slab (four in flight), then
// the lanes are added in lane order through LDS (fixed order: deterministic). Block = 256/SL
// consecutive elements (slab order, coalesced) x SL split lanes.
template <int SL>
__global__ void __launch_bounds__(256) k_wgrad_reduce_sl(const float* __restrict__ ws, int splits, int Cout, int Cin,
                                                         int CinP, int KH, int KW, float* __restrict__ dw,
                                                         int accumulate) {
  constexpr int EL = 256 / SL;
  __shared__ float red[SL][EL + 1];
  const int el = threadIdx.x % EL, sl = threadIdx.x / EL;
  const int KK = KH * KW;
  const int total = Cout * KK * Cin;
  const long long slab = (long long)Cout * KK * CinP;
  const int i = blockIdx.x * EL + el;
  float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
  int ci = 0, t = 0;
  if (i < total) {
    ci = i % Cin;
    t = i / Cin;
    const float* src = ws + (long long)t * CinP + ci;
    int sp = sl;
    for (; sp + 3 * SL < splits; sp += 4 * SL) {
      v0 += src[(sp + 0 * SL) * slab];
      v1 += src[(sp + 1 * SL) * slab];
      v2 += src[(sp + 2 * SL) * slab];
      v3 += src[(sp + 3 * SL) * slab];
    }
    for (; sp < splits; sp += SL) v0 += src[sp * slab];
  }
  red[sl][el] = (v0 + v1) + (v2 + v3);
  __syncthreads();
  if (sl == 0 && i < total) {
    float v = red[0][el];
#pragma unroll
    for (int s = 1; s < SL; ++s) v += red[s][el];
    const int co = t / KK, rs = t - co * KK;
    float* d = dw + ((long long)co * Cin + ci) * KK + rs;
    *d = accumulate ? *d + v : v;
  }
}

// --------------------------------------------------- single-output-channel
// y[m] = sum_{r,s,ci} x[n, ho*st-pad+r*dil, wo*st-pad+s*dil, ci] * w[(r,s,ci)] + b
// one 16-lane group per output pixel
template <typename T>
__global__ void k_conv_cout1(const T* __restrict__ x, int N, int H, int W, int Cin, int ldx,
                             const float* __restrict__ w, const float* __restrict__ bias, int KH, int KW, int stride,
                             int pad, int dil, T* __restrict__ y, int Ho, int Wo, int ldy, int act) {
  const int g = threadIdx.x & 15;
  const long long m = (long long)blockIdx.x * (blockDim.x / 16) + (threadIdx.x >> 4);
  const long long M = (long long)N * Ho * Wo;
  float acc = 0.f;
  if (m < M) {
    const int n = (int)(m / (Ho * Wo));
    const int rem = (int)(m - (long long)n * Ho * Wo);
    const int ho = rem / Wo, wo = rem % Wo;
    for (int r = 0; r < KH; ++r) {
      const int hi = ho * stride - pad + r * dil;
      if (hi < 0 || hi >= H) continue;
      for (int s = 0; s < KW; ++s) {
        const int wi = wo * stride - pad + s * dil;
        if (wi < 0 || wi >= W) continue;
        const T* px = x + ((size_t)(n * H + hi) * W + wi) * ldx;
        const float* pw = w + (size_t)(r * KW + s) * Cin;
        for (int c = g; c < Cin; c += 16) acc += ld(px + c) * pw[c];
      }
    }
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 16);
  if (m < M && g == 0) {
    float v = acc + (bias ? bias[0] : 0.f);
    if (act == DMF_ACT_GELU) v = gelu_f(v);
    else if (act == DMF_ACT_SIGMOID) v = sigmoid_f(v);
    else if (act == DMF_ACT_RELU) v = fmaxf(v, 0.f);
    st(y + m * ldy, v);
  }
}

// dx[n,h,w,ci] = sum_{r,s} dy[n,(h+pad-r*dil)/st,(w+pad-s*dil)/st] * w[(r,s,ci)]
template <typename T>
__global__ void k_conv_cout1_dgrad(const T* __restrict__ dy, int lddy, const float* __restrict__ w, int N, int H,
                                   int W, int Cin, int KH, int KW, int stride, int pad, int dil, int Ho, int Wo,
                                   T* __restrict__ dx, int lddx) {
  const long long total = (long long)N * H * W * Cin;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % Cin);
    const long long pix = i / Cin;
    const int n = (int)(pix / (H * W));
    const int rem = (int)(pix - (long long)n * H * W);
    const int h = rem / W, wq = rem % W;
    float acc = 0.f;
    for (int r = 0; r < KH; ++r) {
      const int hn = h + pad - r * dil;
      if (hn < 0 || hn % stride) continue;
      const int ho = hn / stride;
      if (ho >= Ho) continue;
      for (int s = 0; s < KW; ++s) {
        const int wn = wq + pad - s * dil;
        if (wn < 0 || wn % stride) continue;
        const int wo = wn / stride;
        if (wo >= Wo) continue;
        acc += ld(dy + ((size_t)(n * Ho + ho) * Wo + wo) * lddy) * w[(size_t)(r * KW + s) * Cin + ci];
      }
    }
    st(dx + pix * lddx + ci, acc);
  }
}

// 8-channel vector form of the same: thread = one pixel x 8 input channels,
// 32-bit index math (the scalar form's 64-bit divisions per element cost
// ~50 us on a 32k x 128 map), the 8 weights of every tap from L1
template <typename T>
__global__ void __launch_bounds__(256) k_conv_cout1_dgrad8(const T* __restrict__ dy, int lddy,
                                                           const float* __restrict__ w, int N, int H, int W, int Cin,
                                                           int KH, int KW, int stride, int pad, int dil, int Ho, int Wo,
                                                           T* __restrict__ dx, int lddx) {
  const int CV = Cin >> 3;
  const int total = N * H * W * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV, pix = i / CV;
    const int n = pix / (H * W), rem = pix - n * (H * W);
    const int h = rem / W, wq = rem - (rem / W) * W;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < KH; ++r) {
      const int hn = h + pad - r * dil;
      if (hn < 0 || hn % stride) continue;
      const int ho = hn / stride;
      if (ho >= Ho) continue;
      for (int s2 = 0; s2 < KW; ++s2) {
        const int wn = wq + pad - s2 * dil;
        if (wn < 0 || wn % stride) continue;
        const int wo = wn / stride;
        if (wo >= Wo) continue;
        const float g = ld(dy + ((n * Ho + ho) * Wo + wo) * lddy);
        const float4* wp = (const float4*)(w + (r * KW + s2) * Cin + cv * 8);
        const float4 a = wp[0], b = wp[1];
        acc[0] = fmaf(g, a.x, acc[0]);
        acc[1] = fmaf(g, a.y, acc[1]);
        acc[2] = fmaf(g, a.z, acc[2]);
        acc[3] = fmaf(g, a.w, acc[3]);
        acc[4] = fmaf(g, b.x, acc[4]);
        acc[5] = fmaf(g, b.y, acc[5]);
        acc[6] = fmaf(g, b.z, acc[6]);
        acc[7] = fmaf(g, b.w, acc[7]);
      }
    }
    st8(dx + (size_t)pix * lddx + cv * 8, acc);
  }
}

// dw[(r,s,ci)] partial over a pixel chunk: block = (tap-chunk of 256 columns, split)
template <typename T>
__global__ void k_conv_cout1_wgrad(const T* __restrict__ x, int N, int H, int W, int Cin, int ldx,
                                   const T* __restrict__ dy, int lddy, int KH, int KW, int stride, int pad, int dil,
                                   int Ho, int Wo, int ppsplit, float* __restrict__ ws, float* __restrict__ dbias_ws) {
  const int K = KH * KW * Cin;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const long long M = (long long)N * Ho * Wo;
  const long long p0 = (long long)blockIdx.y * ppsplit;
  const long long p1 = min(M, p0 + ppsplit);
  float acc = 0.f, accb = 0.f;
  const bool kok = k < K;
  const int tap = kok ? k / Cin : 0, ci = k - tap * Cin, r = tap / KW, s = tap % KW;
  for (long long p = p0; p < p1; ++p) {
    const int n = (int)(p / (Ho * Wo));
    const int rem = (int)(p - (long long)n * Ho * Wo);
    const int ho = rem / Wo, wo = rem % Wo;
    const float g = ld(dy + p * lddy);
    accb += g;
    if (kok) {
      const int hi = ho * stride - pad + r * dil, wi = wo * stride - pad + s * dil;
      if (hi >= 0 && hi < H && wi >= 0 && wi < W) acc += g * ld(x + ((size_t)(n * H + hi) * W + wi) * ldx + ci);
    }
  }
  if (kok) ws[(size_t)blockIdx.y * K + k] = acc;
  if (dbias_ws && blockIdx.x == 0 && threadIdx.x == 0) dbias_ws[blockIdx.y] = accb;
}

// 8-channel vector form (Cin, ldx multiples of 8): thread = one 8-channel
// slice of one tap, positions walked incrementally (no divisions in the
// loop), 16-B loads, several positions in flight.
template <typename T>
__global__ void __launch_bounds__(256) k_conv_cout1_wgrad8(const T* __restrict__ x, int N, int H, int W, int Cin,
                                                           int ldx, const T* __restrict__ dy, int lddy, int KH, int KW,
                                                           int stride, int pad, int dil, int Ho, int Wo, int ppsplit,
                                                           float* __restrict__ ws, float* __restrict__ dbias_ws) {
  const int CV = Cin >> 3;
  const int KV = KH * KW * CV;
  const int kv = blockIdx.x * blockDim.x + threadIdx.x;
  const bool kok = kv < KV;
  const int tap = kok ? kv / CV : 0, cv = kv - tap * CV, r = tap / KW, s = tap - (tap / KW) * KW;
  const long long M = (long long)N * Ho * Wo;
  const long long p0 = (long long)blockIdx.y * ppsplit;
  const long long p1 = min(M, p0 + ppsplit);
  int n = (int)(p0 / ((long long)Ho * Wo));
  const int rem = (int)(p0 - (long long)n * Ho * Wo);
  int ho = rem / Wo, wo = rem - (rem / Wo) * Wo;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float accb = 0.f;
#pragma unroll 4
  for (long long p = p0; p < p1; ++p) {
    const float g = ld(dy + p * lddy);
    accb += g;
    const int hi = ho * stride - pad + r * dil, wi = wo * stride - pad + s * dil;
    if (kok && hi >= 0 && hi < H && wi >= 0 && wi < W) {
      float v[8];
      ld8(x + ((size_t)(n * H + hi) * W + wi) * ldx + cv * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(g, v[j], acc[j]);
    }
    if (++wo == Wo) {
      wo = 0;
      if (++ho == Ho) {
        ho = 0;
        ++n;
      }
    }
  }
  if (kok) {
    float* o = ws + (size_t)blockIdx.y * KV * 8 + (size_t)kv * 8;
    *(float4*)o = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *(float4*)(o + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
  if (dbias_ws && blockIdx.x == 0 && threadIdx.x == 0) dbias_ws[blockIdx.y] = accb;
}

// pixel-lane form for 1-output-channel weight gradients: block = CVt 8-channel
// slices (of all KH*KW*Cin/8) x R = 256 / CVt pixel lanes, so a short K (a
// 1x1 head over 64 channels: 8 slices) still fills the block; each split's
// partial is reduced over the R lanes in LDS (fixed order). Writes
// ws[split][K] and the bias partials wsb[split].
template <typename T>
__global__ void __launch_bounds__(256) k_conv_cout1_wgrad8r(const T* __restrict__ x, int N, int H, int W, int Cin,
                                                            int ldx, const T* __restrict__ dy, int lddy, int KH, int KW,
                                                            int stride, int pad, int dil, int Ho, int Wo, int ppsplit,
                                                            int CVt, float* __restrict__ ws,
                                                            float* __restrict__ dbias_ws) {
  __shared__ float red[256 * 9];
  const int CV = Cin >> 3;
  const int KV = KH * KW * CV;
  const int R = 256 / CVt;
  const int cl = threadIdx.x % CVt, rl = threadIdx.x / CVt;
  const int kv = blockIdx.x * CVt + cl;
  const bool kok = kv < KV && rl < R;
  const int tap = kok ? kv / CV : 0, cv = kv - tap * CV, r = tap / KW, s = tap - (tap / KW) * KW;
  const int M = N * Ho * Wo;
  const int p0 = blockIdx.y * ppsplit, p1 = min(M, p0 + ppsplit);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float accb = 0.f;
  if (rl < R) {
#pragma unroll 2
    for (int p = p0 + rl; p < p1; p += R) {
      const int n = p / (Ho * Wo), rem = p - n * (Ho * Wo);
      const int ho = rem / Wo, wo = rem - (rem / Wo) * Wo;
      const float g = ld(dy + p * lddy);
      accb += g;
      const int hi = ho * stride - pad + r * dil, wi = wo * stride - pad + s * dil;
      if (kok && hi >= 0 && hi < H && wi >= 0 && wi < W) {
        float v[8];
        ld8(x + ((size_t)(n * H + hi) * W + wi) * ldx + cv * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(g, v[j], acc[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x * 9 + j] = acc[j];
  red[threadIdx.x * 9 + 8] = accb;
  __syncthreads();
  for (int t = threadIdx.x; t < CVt * 8; t += 256) {
    const int c = t >> 3, j = t & 7;
    float v = 0.f;
    for (int q = 0; q < R; ++q) v += red[(q * CVt + c) * 9 + j];
    if (blockIdx.x * CVt + c < KV) ws[(size_t)blockIdx.y * KV * 8 + (size_t)(blockIdx.x * CVt + c) * 8 + j] = v;
  }
  if (dbias_ws && blockIdx.x == 0 && threadIdx.x == 0) {
    float v = 0.f;  // every pixel lane of the first slice saw its pixels' dy once
    for (int q = 0; q < R; ++q) v += red[(q * CVt) * 9 + 8];
    dbias_ws[blockIdx.y] = v;
  }
}

// out[k] (+)= sum over splits of ws[s][k]: block = 64 columns x 16 split lanes,
// 8 loads in flight per thread, the 16 lanes combined in LDS in a fixed order
// (the one-thread-per-column form ran 40 us over 512 splits)
// cin > 0: column k = tap * cin + ci lands at out[ci * (K / cin) + tap] (torch [Cin][KH][KW])
__global__ void __launch_bounds__(1024) k_sum_splits16(const float* __restrict__ ws, int splits, int K,
                                                       float* __restrict__ out, int accumulate, int cin) {
  __shared__ float red[16][64];
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + c;
  float v = 0.f;
  if (k < K) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int s = q;
    for (; s + 7 * 16 < splits; s += 8 * 16) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += ws[(size_t)(s + u * 16) * K + k];
    }
    for (; s < splits; s += 16) a[0] += ws[(size_t)s * K + k];
    v = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  }
  red[q][c] = v;
  __syncthreads();
  if (q == 0 && k < K) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][c];
    const int o = cin > 0 ? (k % cin) * (K / cin) + k / cin : k;
    out[o] = accumulate ? out[o] + t : t;
  }
}

__global__ void k_sum_splits(const float* __restrict__ ws, int splits, int K, float* __restrict__ out, int accumulate) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
  int s = 0;
  for (; s + 3 < splits; s += 4) {
    v0 += ws[(size_t)s * K + k];
    v1 += ws[(size_t)(s + 1) * K + k];
    v2 += ws[(size_t)(s + 2) * K + k];
    v3 += ws[(size_t)(s + 3) * K + k];
  }
  for (; s < splits; ++s) v0 += ws[(size_t)s * K + k];
  const float v = (v0 + v1) + (v2 + v3);
  out[k] = accumulate ? out[k] + v : v;
}

// ----------------------------------------------------- single input channel
// y[m][co] = x[m] * w[co] + b[co] (optionally with activation)
template <typename T>
__global__ void k_conv_cin1(const T* __restrict__ x, int ldx, const float* __restrict__ w, const float* __restrict__ b,
                            T* __restrict__ y, int ldy, long long M, int Cout, int act) {
  const long long total = M * Cout;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long m = i / Cout;
    const int c = (int)(i - m * Cout);
    float v = ld(x + m * ldx) * w[c] + (b ? b[c] : 0.f);
    if (act == DMF_ACT_GELU) v = gelu_f(v);
    else if (act == DMF_ACT_RELU) v = fmaxf(v, 0.f);
    else if (act == DMF_ACT_SIGMOID) v = sigmoid_f(v);
    st(y + m * ldy + c, v);
  }
}

// dx[m] = sum_c dy[m][c] w[c]; one 64-lane wave per row
template <typename T>
__global__ void k_conv_cin1_dgrad(const T* __restrict__ dy, int lddy, const float* __restrict__ w, T* __restrict__ dx,
                                  int lddx, long long M, int Cout) {
  const int lane = threadIdx.x & 63;
  const long long m = (long long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (m >= M) return;
  float acc = 0.f;
  for (int c = lane; c < Cout; c += 64) acc += ld(dy + m * lddy + c) * w[c];
  acc = wave_sum(acc);
  if (lane == 0) st(dx + m * lddx, acc);
}

// dw partial per row-tile: ws[tile][c] = sum_{m in tile} dy[m][c]*x[m]; db similarly
template <typename T>
__global__ void k_conv_cin1_wgrad(const T* __restrict__ x, int ldx, const T* __restrict__ dy, int lddy, long long M,
                                  int Cout, float* __restrict__ ws, float* __restrict__ wsb) {
  const int c = threadIdx.x;
  const long long m0 = (long long)blockIdx.x * 256;
  if (c >= Cout) return;
  float a = 0.f, b = 0.f;
  for (int r = 0; r < 256; ++r) {
    const long long m = m0 + r;
    if (m >= M) break;
    const float g = ld(dy + m * lddy + c);
    a += g * ld(x + m * ldx);
    b += g;
  }
  ws[(size_t)blockIdx.x * Cout + c] = a;
  if (wsb) wsb[(size_t)blockIdx.x * Cout + c] = b;
}

static inline int gsz(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

}  // namespace dmf

using namespace dmf;

// bf16 weight-gradient forms (dmf_conv_wgrad_tune): key 2 = transposed-read kernels on (1, default: the
// LDS-DMA form below), 2 = its 128 x 256 register-staged variant, 0 = the plain gather kernel; key 0 = LDS-DMA
// staging (k_conv_wgrad_dma, default) vs register-staged k_conv_wgrad_tr; key 1 = the 128 x 256 LDS-DMA tile
// for 1x1 convs with K <= 1024 (default on)
static int g_wgrad_tr = 1;
static int wgrad_tr_enabled() { return g_wgrad_tr; }
static int g_wgrad_dma = 1;
static int wgrad_dma_enabled() { return g_wgrad_dma; }
static int g_wgrad_wide = 1;
// key 3: the 256x256 LDS-DMA tile (8 waves of 128x64, one workgroup per CU): 0 off, 1 (default) where
// legal and the weight has >= 2^18 entries, 2 wherever legal. Measured on the encoder pair's 39 shapes
// (tools/wgrad_bench.py --sq, profiles/r04e_wgrad_sq.txt): 9.40 -> 7.66 ms per step; the only losers are
// the small 1x1 weights (256x256, 256x512: 1.5-2 us each, too few 256-wide tiles to fill the chip)
static int g_wgrad_sq = 1;
// the 256x256 form takes a launch (and sizes its pixel splits for it): bf16/f16, 256-row and -column
// tiles whole (Cout % 256 == 0, Ktot % 256 == 0); a dual-source input also needs Cin, C1 % 256 == 0
// (checked at launch, which otherwise keeps the 128-wide forms with the same split count)
static bool wgrad_sq_ok(int dtype, int Cout, long long Ktot) {
  if (!is16(dtype) || !g_wgrad_sq || Cout % 256 != 0 || Ktot % 256 != 0) return false;
  return g_wgrad_sq == 2 || (long long)Cout * Ktot >= (1LL << 18);
}

// key 4: split-lane reducers for many-split sums (k_wgrad_reduce_sl): 0 off, 1 (default) on
static int g_reduce_sl = 1;
// key 5: the block count the pixel splits aim for, in percent of one chip-filling wave. Default 50:
// a weight gradient runs beside the other encoder's backward (and its own dX chain), and a launch
// sized to fill the chip alone holds CUs those need -- mode B, interleaved A/B: 20 % 944, 30 % 992,
// 40 % 1010, 50 % 1011-1015, 65 % 1010, 100 % 988, 200 % 975 vol/s
static int g_wgrad_fill = 50;

extern "C" int dmf_conv_wgrad_tune(int key, int value) {
  DMF_CHECK_ARG(key >= 0 && key <= 5, "dmf_conv_wgrad_tune: unknown key %d", key);
  if (key == 5) {
    DMF_CHECK_ARG(value >= 10 && value <= 400, "dmf_conv_wgrad_tune: fill %d%%", value);
    g_wgrad_fill = value;
  } else if (key == 4) g_reduce_sl = value != 0;
  else if (key == 0) g_wgrad_dma = value != 0;
  else if (key == 1) g_wgrad_wide = value != 0;
  else if (key == 3) {
    DMF_CHECK_ARG(value >= 0 && value <= 2, "dmf_conv_wgrad_tune: 256x256 tile mode %d", value);
    g_wgrad_sq = value;
  }
  else {
    DMF_CHECK_ARG(value >= 0 && value <= 2, "dmf_conv_wgrad_tune: transposed-read mode %d", value);
    g_wgrad_tr = value;
  }
  return 0;
}

extern "C" int dmf_conv2d_wgrad_splits(int dtype, int Cout, int Cin, int KH, int KW, long long M) {
  const bool sq = wgrad_sq_ok(dtype, Cout, (long long)KH * KW * Cin) && wgrad_tr_enabled() && wgrad_dma_enabled();
  const long long tiles = sq ? (long long)(Cout / 256) * (((long long)KH * KW * Cin) / 256)
                             : (long long)cdiv(Cout, 128) * cdiv((long long)KH * KW * Cin, 128);
  // transposed-read kernel: ~2 resident blocks per CU, and every split costs
  // a Cout x K fp32 slab round trip, so aim for one wave of 512 blocks (256 of the 256x256 form)
  long long target = sq ? 256 : (is16(dtype) && wgrad_tr_enabled()) ? 512 : 1024;
  target = std::max(1LL, target * g_wgrad_fill / 100);
  long long want = (target + tiles - 1) / tiles;
  // >= 256 pixels (4 K-steps) per split, and at most 64 MiB of fp32 slabs: a small
  // weight (64x64 1x1: one tile) then runs 128 splits of 4 K-steps instead of 32
  // latency-bound splits of 16 (~20 us -> a few us), a large one keeps its split count
  long long maxs = (M + 255) / 256;
  const long long slab = (long long)Cout * KH * KW * Cin;
  const long long maxb = std::max(1LL, (16LL << 20) / std::max(1LL, slab));
  if (maxs > maxb) maxs = maxb;
  if (want > maxs) want = maxs;
  if (want < 1) want = 1;
  if (want > 512) want = 512;
  return (int)want;
}

extern "C" int dmf_conv2d_wgrad_pixel_step(int dtype) {
  return is16(dtype) ? 64 : 32;
}

extern "C" int dmf_conv2d_wgrad(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* x2,
                                int Cin2, int ldx2, const void* dy, int Ho, int Wo, int Cout, int lddy, int KH, int KW,
                                int stride, int pad, int dil, int splits, float* workspace, void* stream) {
  const int epc = is16(dtype) ? 8 : 4;
  DMF_CHECK_ARG(dtype == DMF_F32 || is16(dtype), "dmf_conv2d_wgrad: bad dtype");
  DMF_CHECK_ARG(Cin % epc == 0 && ldx % epc == 0 && Cout % epc == 0 && lddy % epc == 0,
                "dmf_conv2d_wgrad: channel counts/strides must be multiples of %d (Cin=%d Cout=%d)", epc, Cin, Cout);
  DMF_CHECK_ARG(splits >= 1 && workspace, "dmf_conv2d_wgrad: bad workspace");
  DMF_CHECK_ARG(Ho == (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1 && Wo == (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1,
                "dmf_conv2d_wgrad: geometry mismatch");
  WgArgs a{};
  a.x = x; a.dy = dy; a.ws = workspace;
  DMF_CHECK_ARG(!x2 || (Cin2 % epc == 0 && ldx2 % epc == 0), "dmf_conv2d_wgrad: bad second source");
  a.N = N; a.H = H; a.W = W; a.Cin = Cin + (x2 ? Cin2 : 0); a.ldx = ldx;
  a.x2 = x2; a.C1 = x2 ? Cin : a.Cin; a.ldx2 = ldx2;
  a.Ho = Ho; a.Wo = Wo; a.Cout = Cout; a.lddy = lddy;
  a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad; a.dil = dil;
  a.Ktot = KH * KW * a.Cin;
  a.M = N * Ho * Wo;
  a.mtiles = cdiv(Cout, 128);
  a.ntiles = cdiv(a.Ktot, 128);
  a.splits = splits;
  const int bk = is16(dtype) ? 64 : 8 * epc;
  a.pix_per_split = cdiv(cdiv(a.M, splits), bk) * bk;
  dim3 grid(a.mtiles * a.ntiles, splits);
  const size_t lds = 2 * 2 * 128 * 128;
  DMF_CHECK_ARG((uintptr_t)x % 16 == 0 && (uintptr_t)dy % 16 == 0 && (!x2 || (uintptr_t)x2 % 16 == 0),
                "dmf_conv2d_wgrad: pointers must be 16-byte aligned");
  auto launch16 = [&](auto tag) {
    using ET = decltype(tag);
    if (wgrad_tr_enabled() == 2 && a.Ktot >= 256) {
      // 128 x 256 tile, 8 waves: half the operand re-reads per flop
      a.ntiles = cdiv(a.Ktot, 256);
      grid = dim3(a.mtiles * a.ntiles, splits);
      hipLaunchKernelGGL((k_conv_wgrad_tr<2, 4, ET>), grid, dim3(512), (size_t)2 * 3 * 64 * 256, (hipStream_t)stream, a);
    } else if (wgrad_tr_enabled() && wgrad_dma_enabled() &&
               (long long)a.N * a.H * a.W * std::max(a.ldx, x2 ? a.ldx2 : 0) * 2 < (1LL << 31) &&
               (long long)a.M * a.lddy * 2 < (1LL << 31) && (!x2 || (a.Cin % 128 == 0 && a.C1 % 128 == 0))) {
      // 128x256 tiles (8 waves, one workgroup per CU, 96 KiB): a third less operand staging per
      // flop than 128x128 at two workgroups per CU. Measured (tools/wgrad_bench.py): faster on the
      // 1x1 convs up to K = 1024 (512->2048: 96.9 -> 87.0 us), slower on the 3x3s and K = 2048
      const bool wide = g_wgrad_wide && a.KH * a.KW == 1 && a.Ktot >= 256 && a.Ktot <= 1024 && a.Cout >= 128 &&
                        (!x2 || (a.Cin % 256 == 0 && a.C1 % 256 == 0));
      if (wgrad_sq_ok(dtype, a.Cout, a.Ktot) && (!x2 || (a.Cin % 256 == 0 && a.C1 % 256 == 0))) {
        a.mtiles = a.Cout / 256;
        a.ntiles = a.Ktot / 256;
        grid = dim3(a.mtiles * a.ntiles, splits);
        if (x2) hipLaunchKernelGGL((k_conv_wgrad_dma<true, 2, 4, 8, ET>), grid, dim3(512), (size_t)2 * 4 * 64 * 256, (hipStream_t)stream, a);
        else hipLaunchKernelGGL((k_conv_wgrad_dma<false, 2, 4, 8, ET>), grid, dim3(512), (size_t)2 * 4 * 64 * 256, (hipStream_t)stream, a);
      } else if (wide) {
        a.ntiles = cdiv(a.Ktot, 256);
        grid = dim3(a.mtiles * a.ntiles, splits);
        if (x2) hipLaunchKernelGGL((k_conv_wgrad_dma<true, 2, 4, 4, ET>), grid, dim3(512), (size_t)2 * 3 * 64 * 256, (hipStream_t)stream, a);
        else hipLaunchKernelGGL((k_conv_wgrad_dma<false, 2, 4, 4, ET>), grid, dim3(512), (size_t)2 * 3 * 64 * 256, (hipStream_t)stream, a);
      } else if (x2) {
        hipLaunchKernelGGL((k_conv_wgrad_dma<true, 2, 2, 4, ET>), grid, dim3(256), (size_t)2 * 2 * 64 * 256, (hipStream_t)stream, a);
      } else {
        hipLaunchKernelGGL((k_conv_wgrad_dma<false, 2, 2, 4, ET>), grid, dim3(256), (size_t)2 * 2 * 64 * 256, (hipStream_t)stream, a);
      }
    } else if (wgrad_tr_enabled()) {
      hipLaunchKernelGGL((k_conv_wgrad_tr<2, 2, ET>), grid, dim3(256), (size_t)2 * 2 * 64 * 256, (hipStream_t)stream, a);
    } else {
      hipLaunchKernelGGL(k_conv_wgrad<ET>, grid, dim3(256), lds, (hipStream_t)stream, a);
    }
  };
  if (dtype == DMF_BF16) launch16(bf16_t{});
  else if (dtype == DMF_F16) launch16(f16_t{});
  else hipLaunchKernelGGL(k_conv_wgrad<float>, grid, dim3(256), lds, (hipStream_t)stream, a);
  DMF_LAUNCH_CHECK("dmf_conv2d_wgrad");
  return 0;
}

extern "C" int dmf_conv2d_wgrad_reduce(const float* workspace, int splits, int Cout, int Cin, int CinP, int KH, int KW,
                                       float* dw, int accumulate, void* stream) {
  DMF_CHECK_ARG(workspace && dw && splits >= 1 && CinP >= Cin, "dmf_conv2d_wgrad_reduce: bad args");
  const long long total = (long long)Cout * Cin * KH * KW;
  DMF_CHECK_ARG(total < (1LL << 31) && (long long)Cout * KH * KW * CinP < (1LL << 31),
                "dmf_conv2d_wgrad_reduce: %lld weights exceed the 32-bit walk", total);
  // split-lane forms where they measured faster (tools/wgrad_bench.py --reduce, profiles/r04i_wgrad_reduce.txt):
  // small weights with many splits (4096 x 512 splits: 18.6 -> 5.5 us); above ~48K weights at >= 64 splits
  // the 64-B segments per slab row lose to the one-lane walk (262144 x 64: 13.8 -> 24.9 us)
  if (g_reduce_sl && splits >= 64 && total <= 49152) {
    hipLaunchKernelGGL(k_wgrad_reduce_sl<16>, dim3((unsigned)cdiv(total, 16LL)), dim3(256), 0, (hipStream_t)stream,
                       workspace, splits, Cout, Cin, CinP, KH, KW, dw, accumulate);
    DMF_LAUNCH_CHECK("dmf_conv2d_wgrad_reduce");
    return 0;
  }
  if (g_reduce_sl && splits >= 24 && splits < 64 && total <= (1LL << 20)) {
    hipLaunchKernelGGL(k_wgrad_reduce_sl<4>, dim3((unsigned)cdiv(total, 64LL)), dim3(256), 0, (hipStream_t)stream,
                       workspace, splits, Cout, Cin, CinP, KH, KW, dw, accumulate);
    DMF_LAUNCH_CHECK("dmf_conv2d_wgrad_reduce");
    return 0;
  }
  hipLaunchKernelGGL(k_wgrad_reduce, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream, workspace, splits, Cout, Cin,
                     CinP, KH, KW, dw, accumulate);
  DMF_LAUNCH_CHECK("dmf_conv2d_wgrad_reduce");
  return 0;
}

extern "C" int dmf_conv2d_wgrad_gate(const float* workspace, int N, int Cout, int Cin, int CinP, int KH, int KW,
                                     const float* w, const float* gate, float* dgate, void* stream) {
  DMF_CHECK_ARG(workspace && w && gate && dgate && N > 0 && Cin > 0 && CinP >= Cin,
                "dmf_conv2d_wgrad_gate: bad args");
  hipLaunchKernelGGL(k_gate_grad_wslab, dim3(Cin, N), dim3(256), 0, (hipStream_t)stream, workspace, Cout, Cin, CinP,
                     KH * KW, w, gate, dgate);
  DMF_LAUNCH_CHECK("dmf_conv2d_wgrad_gate");
  return 0;
}

// The same with 8-channel (16-B) vectors: G lanes per output pixel, lane g takes the channel chunks
// 8g, 8g + 8G, ... of every tap (k_conv_cout1 moved 2-B elements, 16 lanes x 2 B = 32 B per pixel per
// load instruction). Needs Cin % 8 == 0, ldx % 8 == 0 and a 16-B aligned x.
namespace dmf {
template <typename T, int G>
__global__ void __launch_bounds__(256) k_conv_cout1_v8(const T* __restrict__ x, int N, int H, int W, int Cin, int ldx,
                                                       const float* __restrict__ w, const float* __restrict__ bias,
                                                       int KH, int KW, int stride, int pad, int dil,
                                                       T* __restrict__ y, int Ho, int Wo, int ldy, int act) {
  const int g = threadIdx.x & (G - 1);
  const long long m = (long long)blockIdx.x * (256 / G) + (threadIdx.x / G);
  const long long M = (long long)N * Ho * Wo;
  float acc = 0.f;
  if (m < M) {
    const int n = (int)(m / (Ho * Wo));
    const int rem = (int)(m - (long long)n * Ho * Wo);
    const int ho = rem / Wo, wo = rem - (rem / Wo) * Wo;
    for (int r = 0; r < KH; ++r) {
      const int hi = ho * stride - pad + r * dil;
      if (hi < 0 || hi >= H) continue;
      for (int s = 0; s < KW; ++s) {
        const int wi = wo * stride - pad + s * dil;
        if (wi < 0 || wi >= W) continue;
        const T* px = x + ((size_t)(n * H + hi) * W + wi) * ldx;
        const float* pw = w + (size_t)(r * KW + s) * Cin;
        for (int c = g * 8; c < Cin; c += G * 8) {
          float v[8];
          unpack8(ldv8(px + c), v);
          const float4 w0 = *(const float4*)(pw + c), w1 = *(const float4*)(pw + c + 4);
          acc = fmaf(v[0], w0.x, fmaf(v[1], w0.y, fmaf(v[2], w0.z, fmaf(v[3], w0.w, acc))));
          acc = fmaf(v[4], w1.x, fmaf(v[5], w1.y, fmaf(v[6], w1.z, fmaf(v[7], w1.w, acc))));
        }
      }
    }
  }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, G);
  if (m < M && g == 0) {
    float v = acc + (bias ? bias[0] : 0.f);
    if (act == DMF_ACT_GELU) v = gelu_f(v);
    else if (act == DMF_ACT_SIGMOID) v = sigmoid_f(v);
    else if (act == DMF_ACT_RELU) v = fmaxf(v, 0.f);
    st(y + m * ldy, v);
  }
}
}  // namespace dmf

extern "C" int dmf_conv_cout1_fwd(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const float* w,
                                  const float* bias, int KH, int KW, int stride, int pad, int dil, void* y, int Ho,
                                  int Wo, int ldy, int act, void* stream) {
  DMF_CHECK_ARG(x && w && y, "dmf_conv_cout1_fwd: null pointer");
  const long long M = (long long)N * Ho * Wo;
  if (M == 0) return 0;
  if (Cin % 8 == 0 && ldx % 8 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)w % 16) == 0) {
    if (Cin <= 64) {
      DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((k_conv_cout1_v8<T, 8>), dim3((unsigned)cdiv(M, 32)), dim3(256), 0,
                                                      (hipStream_t)stream, (const T*)x, N, H, W, Cin, ldx, w, bias, KH,
                                                      KW, stride, pad, dil, (T*)y, Ho, Wo, ldy, act));
    } else {
      DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((k_conv_cout1_v8<T, 16>), dim3((unsigned)cdiv(M, 16)), dim3(256), 0,
                                                      (hipStream_t)stream, (const T*)x, N, H, W, Cin, ldx, w, bias, KH,
                                                      KW, stride, pad, dil, (T*)y, Ho, Wo, ldy, act));
    }
    DMF_LAUNCH_CHECK("dmf_conv_cout1_fwd");
    return 0;
  }
  const int grid = (int)((M + 15) / 16);
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_conv_cout1<T>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const T*)x, N, H, W,
                       Cin, ldx, w, bias, KH, KW, stride, pad, dil, (T*)y, Ho, Wo, ldy, act));
  DMF_LAUNCH_CHECK("dmf_conv_cout1_fwd");
  return 0;
}

extern "C" int dmf_conv_cout1_dgrad(int dtype, const void* dy, int lddy, const float* w, int N, int H, int W, int Cin,
                                    int KH, int KW, int stride, int pad, int dil, int Ho, int Wo, void* dx, int lddx,
                                    void* stream) {
  DMF_CHECK_ARG(dy && w && dx, "dmf_conv_cout1_dgrad: null pointer");
  const long long total = (long long)N * H * W * Cin;
  if (total == 0) return 0;
  if (Cin % 8 == 0 && lddx % 8 == 0 && ((uintptr_t)dx % 16) == 0 && ((uintptr_t)w % 16) == 0 && total < (1LL << 31)) {
    const long long t8 = total / 8;
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_conv_cout1_dgrad8<T>, dim3(gsz(t8)), dim3(256), 0, (hipStream_t)stream,
                         (const T*)dy, lddy, w, N, H, W, Cin, KH, KW, stride, pad, dil, Ho, Wo, (T*)dx, lddx));
    DMF_LAUNCH_CHECK("dmf_conv_cout1_dgrad");
    return 0;
  }
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_conv_cout1_dgrad<T>, dim3(gsz(total)), dim3(256), 0, (hipStream_t)stream,
                       (const T*)dy, lddy, w, N, H, W, Cin, KH, KW, stride, pad, dil, Ho, Wo, (T*)dx, lddx));
  DMF_LAUNCH_CHECK("dmf_conv_cout1_dgrad");
  return 0;
}

extern "C" int dmf_conv_cout1_wgrad_splits(long long M) {
  // 128 pixels per split (the pixel-lane form walks them with 256 / CVt lanes), at most 512
  long long s = (M + 127) / 128;
  if (s > 512) s = 512;
  return (int)(s < 1 ? 1 : s);
}

// ws: [splits][KH*KW*Cin] + [splits] (bias partials); dw (layout [KH][KW][Cin]) and db accumulate
static int cout1_wgrad(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* dy, int lddy,
                       int KH, int KW, int stride, int pad, int dil, int Ho, int Wo, int splits, float* workspace,
                       float* dw, float* db, bool torch_layout, void* stream);

extern "C" int dmf_conv_cout1_wgrad(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* dy,
                                    int lddy, int KH, int KW, int stride, int pad, int dil, int Ho, int Wo, int splits,
                                    float* workspace, float* dw, float* db, void* stream) {
  return cout1_wgrad(dtype, x, N, H, W, Cin, ldx, dy, lddy, KH, KW, stride, pad, dil, Ho, Wo, splits, workspace, dw, db,
                     false, stream);
}

extern "C" int dmf_conv_cout1_wgrad_torch(int dtype, const void* x, int N, int H, int W, int Cin, int ldx,
                                          const void* dy, int lddy, int KH, int KW, int stride, int pad, int dil, int Ho,
                                          int Wo, int splits, float* workspace, float* dw, float* db, void* stream) {
  return cout1_wgrad(dtype, x, N, H, W, Cin, ldx, dy, lddy, KH, KW, stride, pad, dil, Ho, Wo, splits, workspace, dw, db,
                     true, stream);
}

static int cout1_wgrad(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* dy, int lddy,
                       int KH, int KW, int stride, int pad, int dil, int Ho, int Wo, int splits, float* workspace,
                       float* dw, float* db, bool torch_layout, void* stream) {
  DMF_CHECK_ARG(x && dy && workspace && splits >= 1, "dmf_conv_cout1_wgrad: bad args");
  const long long M = (long long)N * Ho * Wo;
  const int K = KH * KW * Cin;
  const int pps = (int)((M + splits - 1) / splits);
  dim3 grid(cdiv(K, 256), splits);
  float* wsb = workspace + (size_t)splits * K;
  if (Cin % 8 == 0 && ldx % 8 == 0 && ((uintptr_t)x % 16) == 0 && M < (1LL << 31)) {
    const int KV = K / 8;
    const int CVt = KV >= 64 ? 64 : (KV >= 32 ? 32 : (KV >= 16 ? 16 : (KV >= 8 ? 8 : (KV >= 4 ? 4 : (KV >= 2 ? 2 : 1)))));
    const dim3 g8(cdiv(KV, CVt), splits);
    DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_conv_cout1_wgrad8r<T>, g8, dim3(256), 0, (hipStream_t)stream, (const T*)x, N, H,
                         W, Cin, ldx, (const T*)dy, lddy, KH, KW, stride, pad, dil, Ho, Wo, pps, CVt, workspace,
                         wsb));
  } else DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_conv_cout1_wgrad<T>, grid, dim3(256), 0, (hipStream_t)stream, (const T*)x, N, H, W,
                       Cin, ldx, (const T*)dy, lddy, KH, KW, stride, pad, dil, Ho, Wo, pps, workspace, wsb));
  DMF_LAUNCH_CHECK("dmf_conv_cout1_wgrad");
  if (dw)
    hipLaunchKernelGGL(k_sum_splits16, dim3(cdiv(K, 64)), dim3(1024), 0, (hipStream_t)stream, workspace, splits, K, dw,
                       1, torch_layout ? Cin : 0);
  if (db) hipLaunchKernelGGL(k_sum_splits16, dim3(1), dim3(1024), 0, (hipStream_t)stream, wsb, splits, 1, db, 1, 0);
  DMF_LAUNCH_CHECK("dmf_conv_cout1_wgrad(reduce)");
  return 0;
}

extern "C" int dmf_conv_cin1_fwd(int dtype, const void* x, int ldx, const float* w, const float* bias, void* y, int ldy,
                                 long long M, int Cout, int act, void* stream) {
  DMF_CHECK_ARG(x && w && y, "dmf_conv_cin1_fwd: null pointer");
  if (M == 0) return 0;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_conv_cin1<T>, dim3(gsz(M * Cout)), dim3(256), 0, (hipStream_t)stream, (const T*)x,
                       ldx, w, bias, (T*)y, ldy, M, Cout, act));
  DMF_LAUNCH_CHECK("dmf_conv_cin1_fwd");
  return 0;
}

extern "C" int dmf_conv_cin1_dgrad(int dtype, const void* dy, int lddy, const float* w, void* dx, int lddx, long long M,
                                   int Cout, void* stream) {
  DMF_CHECK_ARG(dy && w && dx, "dmf_conv_cin1_dgrad: null pointer");
  if (M == 0) return 0;
  const int grid = (int)((M + 3) / 4);
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_conv_cin1_dgrad<T>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const T*)dy,
                       lddy, w, (T*)dx, lddx, M, Cout));
  DMF_LAUNCH_CHECK("dmf_conv_cin1_dgrad");
  return 0;
}

extern "C" int dmf_conv_cin1_wgrad_tiles(long long M) { return (int)((M + 255) / 256); }

// ws: [tiles][Cout] (+[tiles][Cout] for bias); dw/db accumulate
extern "C" int dmf_conv_cin1_wgrad(int dtype, const void* x, int ldx, const void* dy, int lddy, long long M, int Cout,
                                   float* workspace, float* dw, float* db, void* stream) {
  DMF_CHECK_ARG(x && dy && workspace && Cout <= 256, "dmf_conv_cin1_wgrad: bad args (Cout<=256)");
  const int tiles = (int)((M + 255) / 256);
  float* wsb = db ? workspace + (size_t)tiles * Cout : nullptr;
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_conv_cin1_wgrad<T>, dim3(tiles), dim3(256), 0, (hipStream_t)stream, (const T*)x,
                       ldx, (const T*)dy, lddy, M, Cout, workspace, wsb));
  DMF_LAUNCH_CHECK("dmf_conv_cin1_wgrad");
  // reduce tiles: treat [tiles][Cout] as splits x K
  if (dw) hipLaunchKernelGGL(k_sum_splits16, dim3(cdiv(Cout, 64)), dim3(1024), 0, (hipStream_t)stream, workspace, tiles, Cout, dw, 1, 0);
  if (db) hipLaunchKernelGGL(k_sum_splits16, dim3(cdiv(Cout, 64)), dim3(1024), 0, (hipStream_t)stream, wsb, tiles, Cout, db, 1, 0);
  DMF_LAUNCH_CHECK("dmf_conv_cin1_wgrad(reduce)");
  return 0;
}
