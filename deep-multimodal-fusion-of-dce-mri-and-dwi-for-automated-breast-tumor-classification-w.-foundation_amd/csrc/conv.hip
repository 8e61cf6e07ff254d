// Implicit-GEMM 2-D convolution on MFMA (gfx950), NHWC activations.
//
// One engine serves every conv of the hot path (timm ResNet-50 OS8 at
// foundation_model.py:260-267, the adapter necks model_module.py:440-447,
// the ResNetLite blocks :259-280, heads :113-118/:150-187/:337-345 and the
// fusion projections :857-862) in two roles:
//   FWD  : Y[m = (n,ho,wo)][co] = sum_{(r,s,ci)} X[n, ho*st-pad+r*dil, wo*st-pad+s*dil, ci] * W[co][r][s][ci]
//   DGRAD: dX[m = (n,h,w)][ci]  = sum_{(r,s,co)} dY[n, (h+pad-r*dil)/st, (w+pad-s*dil)/st, co] * Wt[ci][r][s][co]
//          (terms whose division is inexact or out of range are zero)
// GEMM view: M = output pixels, N = output channels, K = taps x input
// channels; A gathered on the fly from the NHWC source (zero padding by
// predicate), B = weights stored K-contiguous.
//
// Tiling (bf16): 128x128 block tile, BK = 64, 4 waves in 2x2, each wave a
// 64x64 sub-tile of 4x4 v_mfma_f32_16x16x32_bf16 fragments, fp32
// accumulation. f32 parity mode: same geometry with BK = 32 floats and
// v_mfma_f32_16x16x4_f32 (exact f32 FMA chains).
// LDS: double-buffered A/B stages of [128 rows][8 x 16-B chunks] with an XOR
// swizzle chunk ^ (row & 7) (conflict-free ds_read_b128 fragment reads).
// Epilogue: + bias, optional activation, optional per-channel batch-norm
// partial statistics (sum, sum^2 over the tile's valid rows -> slab
// partials[mtile][co][2], reduced deterministically by dmf_bn_finalize), then
// an LDS-staged, 16-B coalesced store with an output channel stride (so
// producers can write straight into a channel slice of a concat buffer).
#include <algorithm>
#include <vector>

#include "conv_core.h"

namespace dmf {


template <int ACT>
__device__ __forceinline__ float in_act_f(float v) {
  if (ACT == DMF_ACT_RELU) return fmaxf(v, 0.f);
  if (ACT == DMF_ACT_GELU) return gelu_f(v);
  return v;
}

// x <- act(x*sc + sh) on one 16-B chunk (8 bf16 or 4 f32)
template <typename T, int INA>
__device__ __forceinline__ void chunk_affine(uint4& u, const float* sc, const float* sh) {
  if constexpr (sizeof(T) == 2) {
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float lo = B16<T>::lo(w[i]), hi = B16<T>::hi(w[i]);
      lo = in_act_f<INA>(lo * sc[2 * i] + sh[2 * i]);
      hi = in_act_f<INA>(hi * sc[2 * i + 1] + sh[2 * i + 1]);
      w[i] = B16<T>::pack(lo, hi);
    }
    u = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    float f[4] = {__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = in_act_f<INA>(f[i] * sc[i] + sh[i]);
    u = make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
  }
}

// one LDS stage of A/B fragments -> (BM/32)x(BN/32) MFMA fragments per wave
// (2x2 waves, each a (BM/2)x(BN/2) sub-tile)
template <typename T, int BM = CBM, int BN = CBN, int WMW = 2, int WNW = 2, bool PRIO = false>
__device__ __forceinline__ void conv_mma(const char* As, f32x4_t (&acc)[BM / (16 * WMW)][BN / (16 * WNW)], int wm,
                                         int wn, int lane) {
  constexpr int FM = BM / (16 * WMW), FN = BN / (16 * WNW);
  const char* Bs = As + BM * 128;
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int ch = kk * 4 + fg;
    uint4 av[FM], bv[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * (BM / WMW) + i * 16 + fr;
      av[i] = *(const uint4*)(As + row * 128 + ((ch ^ (row & 7)) << 4));
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wn * (BN / WNW) + j * 16 + fr;
      bv[j] = *(const uint4*)(Bs + col * 128 + ((ch ^ (col & 7)) << 4));
    }
    if constexpr (sizeof(T) == 2) {
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = mfma16<T>(av[i], bv[j], acc[i][j]);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const float fa = __uint_as_float(((const uint32_t*)&av[i])[e]);
            const float fb = __uint_as_float(((const uint32_t*)&bv[j])[e]);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, acc[i][j], 0, 0, 0);
          }
    }
  }
}


// bias / activation or BN partial statistics, LDS-staged 16-B stores
template <typename T, int BM = CBM, int BN = CBN, int WMW = 2, int WNW = 2>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x4_t (&acc)[BM / (16 * WMW)][BN / (16 * WNW)],
                                              char* smem, int tid, int mt, int nt, int m0, int n0) {
  constexpr int FM = BM / (16 * WMW), FN = BN / (16 * WNW);
  constexpr int NT = 64 * WMW * WNW;
  constexpr int EPC = 16 / sizeof(T);
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WNW, wn = wid % WNW;
  const int fr = lane & 15, fg = lane >> 4;
  const bool has_bias = a.bias != nullptr;
  const bool stats = a.partials != nullptr;
  float* red = (float*)smem;  // [2 wm][BN cols][2] floats
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = n0 + wn * (BN / WNW) + j * 16 + fr;
    const float bsv = (has_bias && col < a.Nout) ? a.bias[col] : 0.f;
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * (BM / WMW) + i * 16 + fg * 4 + r;
        float v = acc[i][j][r] + bsv;
        if (stats && row < a.M) { s += v; ss += v * v; }
        acc[i][j][r] = v;
      }
    }
    if (!stats && !a.res_add) apply_act_col(a.act, acc, j);  // (with a residual: after its add, below)
    if (stats) {
      s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
      ss += __shfl_xor(ss, 16, 64); ss += __shfl_xor(ss, 32, 64);
      if (fg == 0) {
        const int lc = wn * (BN / WNW) + j * 16 + fr;
        red[(wm * BN + lc) * 2 + 0] = s;
        red[(wm * BN + lc) * 2 + 1] = ss;
      }
    }
  }
  if (stats) {
    __syncthreads();
    if (tid < BN) {
      const int col = n0 + tid;
      if (col < a.Nout) {
        float2 v = make_float2(0.f, 0.f);
#pragma unroll
        for (int q = 0; q < WMW; ++q) {
          v.x += red[(q * BN + tid) * 2 + 0];
          v.y += red[(q * BN + tid) * 2 + 1];
        }
        float2* dst = (float2*)(a.partials + ((size_t)mt * a.Nout + col) * 2);
        if (a.stat_acc) {
          acc_stats(a, mt, col, v);
        } else if (a.tickets) {
          // write-through (sc1) slab store: visible to the reducer on any XCD without a release fence
          __hip_atomic_store((unsigned long long*)dst, *(unsigned long long*)&v, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        } else {
          *dst = v;
        }
      }
    }
  }
  __syncthreads();
  // stage C tile through LDS: [128 rows][128 + pad] of T
  constexpr int CPAD = 16 / sizeof(T);
  constexpr int CST = BN + CPAD;
  T* Cs = (T*)smem;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * (BM / WMW) + i * 16 + fg * 4 + r;
        const int col = wn * (BN / WNW) + j * 16 + fr;
        Cs[row * CST + col] = Cvt<T>::store(acc[i][j][r]);
      }
  __syncthreads();
  // scratch past the C staging area: [0] last-arriver flag, [64..] reducer doubles
  char* xtra = smem + conv_lds_main(sizeof(T), BM, BN);
  if (a.tickets) {
    // the slab stores (issued before the C staging) drain; then one ticket per block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned prev = __hip_atomic_fetch_add(a.tickets + nt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *(int*)xtra = prev == (unsigned)(a.mtiles - 1);
    }
    __syncthreads();
  }
  T* Y = (T*)a.y;
  constexpr int CPR = BN / EPC;  // chunks per row
  for (int idx = tid; idx < BM * CPR; idx += NT) {
    const int row = idx / CPR, chn = idx - (idx / CPR) * CPR;
    const int m = m0 + row, n = n0 + chn * EPC;
    if (m < a.M && n < a.Nout) {
      uint4 v = *(const uint4*)(Cs + row * CST + chn * EPC);
      if (a.res_add) {
        // act(y + residual) on the 16-B chunk (the staged y already holds the folded bias)
        const uint4 r = *(const uint4*)((const T*)a.res + (size_t)m * a.ldr + n);
        T yv[EPC], rv[EPC];
        __builtin_memcpy(yv, &v, 16);
        __builtin_memcpy(rv, &r, 16);
        float f[EPC];
#pragma unroll
        for (int e = 0; e < EPC; ++e) f[e] = Cvt<T>::load(yv[e]) + Cvt<T>::load(rv[e]);
        apply_act_arr(a.act, f);
#pragma unroll
        for (int e = 0; e < EPC; ++e) yv[e] = Cvt<T>::store(f[e]);
        __builtin_memcpy(&v, yv, 16);
      }
      *(uint4*)(Y + (size_t)m * a.ldy + n) = v;
    }
  }
  if (a.tickets && *(const int*)xtra) {
    // last block of this column tile: reduce the slab (sc1 loads, fixed order, double)
    constexpr int NP = NT / BN;  // tile-row lanes per column
    const int cl = tid % BN, part = tid / BN;
    const int col = n0 + cl;
    double s = 0.0, q = 0.0;
    if (col < a.Nout) {
      // sc1 buffer loads (the slab was stored write-through), 8 independent
      // loads in flight per batch; fixed summation order (deterministic)
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          a.partials, 0, (int)((long long)a.mtiles * a.Nout * 8), BUF_FLAGS_EP);
      const unsigned stride = (unsigned)(NP * a.Nout * 8);
      unsigned off = (unsigned)((part * a.Nout + col) * 8);
      int t = part;
      for (; t + 7 * NP < a.mtiles; t += 8 * NP) {
        uint2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          v[u] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rp, off + u * stride, 0, 16));
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          s += (double)__uint_as_float(v[u].x);
          q += (double)__uint_as_float(v[u].y);
        }
        off += 8 * stride;
      }
      for (; t < a.mtiles; t += NP, off += stride) {
        const uint2 v = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rp, off, 0, 16));
        s += (double)__uint_as_float(v.x);
        q += (double)__uint_as_float(v.y);
      }
    }
    double* dred = (double*)(xtra + 64);
    dred[(part * BN + cl) * 2] = s;
    dred[(part * BN + cl) * 2 + 1] = q;
    __syncthreads();
    if (part == 0 && col < a.Nout) {
      for (int pp = 1; pp < NP; ++pp) {
        s += dred[(pp * BN + cl) * 2];
        q += dred[(pp * BN + cl) * 2 + 1];
      }
      bn_fin_channel(a.fin, col, a.Nout, s, q);
    }
    if (tid == 0) {
      if (nt == 0 && a.fin.training && a.fin.nbt) *a.fin.nbt += 1;
      __hip_atomic_store(a.tickets + nt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------ forward, buffer-load form
// FWD with C (and C1) multiples of BK and no input prologue. Every load is a
// raw buffer load with a 32-bit per-lane offset: out-of-range lanes (M/N
// edges, zero padding) get an offset past the buffer and read zeros from the
// range check -- no branches, no 64-bit address math. The K-step's tap and
// channel offsets are block-uniform (SGPR soffset). PADCHK = false for 1x1,
// stride-1, pad-0 convs (no per-row bounds at all).

// INA >= 0 (plain 1x1 only, PADCHK = DUAL = false): the producer's BN apply
// + activation x <- act(x*scale + shift) runs on each A chunk between its
// load and its LDS write (ConvArgs::in_ss = [scale C][shift C]); the
// activated tensor is never written to HBM.
template <typename T, bool PADCHK, bool DUAL, int BM, int BN, int INA = -1>
__global__ void __launch_bounds__(CTHREADS, (BM * BN <= 64 * 64) ? 4 : ((BM * BN <= 64 * 128) ? 3 : 2)) k_conv_fwd_buf(ConvArgs a) {
  const StampScope stamp_scope_(a.stamp);  // (null unless tools/stream_stamps.py armed it)
  constexpr int RA = BM / 32, RB = BN / 32;  // 16-B chunks per thread per K-step
  constexpr int SB = (BM + BN) * 128;        // LDS stage bytes
  constexpr int ES = sizeof(T);
  constexpr int EPC = 16 / ES;
  constexpr int BK = 8 * EPC;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int nblk = gridDim.x;
  const int lin = xcd_remap(blockIdx.x, nblk);
  const int mt = lin / a.ntiles, nt = lin % a.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int q = tid & 7, rbase = tid >> 3;

  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.x), 0, (int)((long long)a.N * a.H * a.W * a.ldx * ES), BUF_FLAGS);
  const __amdgpu_buffer_rsrc_t rx2 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.x2 ? a.x2 : a.x), 0, (int)((long long)a.N * a.H * a.W * (a.x2 ? a.ldx2 : a.ldx) * ES),
      BUF_FLAGS);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.w), 0, (int)((long long)a.Nout * a.Ktot * ES), BUF_FLAGS);

  // per-row origin (element offsets; may be negative for padded rows)
  int h0[RA], w0[RA], b1[RA], b2[RA];
  bool mok[RA];
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    const int m = m0 + rbase + 32 * i;
    mok[i] = m < a.M;
    const int mm = mok[i] ? m : 0;
    const int hw = a.Ho * a.Wo;
    const int n = mm / hw, rem = mm - (mm / hw) * hw;
    const int ho = rem / a.Wo, wo = rem - (rem / a.Wo) * a.Wo;
    h0[i] = ho * a.stride - a.pad;
    w0[i] = wo * a.stride - a.pad;
    const int pix = (n * a.H + h0[i]) * a.W + w0[i];
    b1[i] = pix * a.ldx + q * EPC;
    b2[i] = pix * a.ldx2 + q * EPC;
  }
  unsigned vb[RB];
#pragma unroll
  for (int i = 0; i < RB; ++i) {
    const int n = n0 + rbase + 32 * i;
    vb[i] = n < a.Nout ? (unsigned)((n * a.Ktot + q * EPC) * ES) : BUF_OOB;
  }
  const int nk = a.Ktot / BK;
  // input affine: the whole [scale C][shift C] vector staged once in LDS past
  // the stage ring + epilogue scratch, so the per-K-step reads are ds_read_b128
  float* ss_lds = (float*)(smem + conv_lds_main(ES, BM, BN) + CONV_LDS_EXTRA);
  if constexpr (INA >= 0) {
    for (int i = tid * 4; i < 2 * a.C; i += CTHREADS * 4) *(float4*)(ss_lds + i) = *(const float4*)(a.in_ss + i);
    __syncthreads();
  } else {
    (void)ss_lds;
  }

  // two register sets: tile kt+1 is in flight while tile kt+2 is issued
  uint4 ra0[RA], rb0[RB], ra1[RA], rb1[RB];
  // K cursor (filter row, column, channel): gload() runs in K order (the
  // clamped tail re-issues only feed registers that are never stored)
  // Channel chunk outer, filter tap inner: the KH*KW consecutive K-steps of
  // one 64-channel chunk re-read the same input rows (shifted by a tap), so
  // the im2col gather hits L2 instead of re-streaming the input per tap.
  int cr = 0, cs = 0, cc = 0;
  auto gload = [&](int kt, uint4 (&ra)[RA], uint4 (&rb)[RB]) {
    (void)kt;
    const int c0 = cc, rd = cr * a.dil, sd = cs * a.dil;
    const int k0 = (cr * a.KW + cs) * a.C + c0;  // uniform
    if (++cs == a.KW) {
      cs = 0;
      if (++cr == a.KH) { cr = 0; cc += BK; }
    }
    // block-uniform source choice as a branch, so each path keeps its descriptor in SGPRs
    if (DUAL && c0 >= a.C1) {
      const int toff = (rd * a.W + sd) * a.ldx2 + (c0 - a.C1);
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        bool ok = mok[i];
        if (PADCHK) ok = ok && (unsigned)(h0[i] + rd) < (unsigned)a.H && (unsigned)(w0[i] + sd) < (unsigned)a.W;
        const unsigned vo = ok ? (unsigned)((b2[i] + toff) * ES) : BUF_OOB;
        ra[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rx2, vo, 0, 0));
      }
    } else {
      const int toff = (rd * a.W + sd) * a.ldx + c0;
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        bool ok = mok[i];
        if (PADCHK) ok = ok && (unsigned)(h0[i] + rd) < (unsigned)a.H && (unsigned)(w0[i] + sd) < (unsigned)a.W;
        const unsigned vo = ok ? (unsigned)((b1[i] + toff) * ES) : BUF_OOB;
        ra[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, vo, 0, 0));
      }
    }
#pragma unroll
    for (int i = 0; i < RB; ++i)
      rb[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rw, vb[i], k0 * ES, 0));
  };
  auto lds_store = [&](int stage, uint4 (&ra)[RA], const uint4 (&rb)[RB], int tile) {
    char* base = smem + stage * SB;
    if constexpr (INA >= 0) {
      // plain 1x1: tile t covers channels t*BK .. t*BK+BK-1; this thread's 16-B chunk q
      const int c = tile * BK + q * EPC;
      float sc[EPC], sh[EPC];
#pragma unroll
      for (int e = 0; e < EPC; e += 4) {
        *(float4*)(sc + e) = *(const float4*)(ss_lds + c + e);
        *(float4*)(sh + e) = *(const float4*)(ss_lds + a.C + c + e);
      }
#pragma unroll
      for (int i = 0; i < RA; ++i) chunk_affine<T, INA>(ra[i], sc, sh);
    } else {
      (void)tile;
    }
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int row = rbase + 32 * i;
      *(uint4*)(base + row * 128 + ((q ^ (row & 7)) << 4)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int row = rbase + 32 * i;
      *(uint4*)(base + BM * 128 + row * 128 + ((q ^ (row & 7)) << 4)) = rb[i];
    }
  };

  f32x4_t acc[RA][RB];
#pragma unroll
  for (int i = 0; i < RA; ++i)
#pragma unroll
    for (int j = 0; j < RB; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // Loads are issued unconditionally (tile index clamped at the tail) so the
  // loop body has no branches around them: the compiler's vmcnt then counts
  // exactly one tile still in flight at each LDS write.
  if (nk <= 2) {  // short K (1x1 over <= 128 channels): no pipeline to fill
    gload(0, ra0, rb0);
    if (nk == 2) gload(1, ra1, rb1);
    lds_store(0, ra0, rb0, 0);
    if (nk == 2) lds_store(1, ra1, rb1, 1);
    __syncthreads();
    conv_mma<T, BM, BN>(smem, acc, wm, wn, lane);
    if (nk == 2) conv_mma<T, BM, BN>(smem + SB, acc, wm, wn, lane);
    __syncthreads();
    conv_epilogue<T, BM, BN>(a, acc, smem, tid, mt, nt, m0, n0);
    return;
  }
  gload(0, ra0, rb0);
  gload(1, ra1, rb1);
  lds_store(0, ra0, rb0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 2) {
    // even step: LDS stage 0 holds tile kt, ra1/rb1 carry tile kt+1
    gload(min(kt + 2, nk - 1), ra0, rb0);
    conv_mma<T, BM, BN>(smem, acc, wm, wn, lane);
    lds_store(1, ra1, rb1, min(kt + 1, nk - 1));
    __syncthreads();
    if (kt + 1 >= nk) break;
    // odd step: stage 1 holds tile kt+1, ra0/rb0 carry tile kt+2
    gload(min(kt + 3, nk - 1), ra1, rb1);
    conv_mma<T, BM, BN>(smem + SB, acc, wm, wn, lane);
    lds_store(0, ra0, rb0, min(kt + 2, nk - 1));
    __syncthreads();
  }
  conv_epilogue<T, BM, BN>(a, acc, smem, tid, mt, nt, m0, n0);
}

// ------------------------------------------- forward, LDS-DMA wide form (bf16)
// 256x128 block tile, 8 waves (4x2) of 64x64 each (4x4 MFMA fragments, 32
// v_mfma_f32_16x16x32_bf16 per wave per K-step, two waves per SIMD), BK = 64,
// one workgroup per CU. A and B tiles go global -> LDS directly (buffer_load_dwordx4 ... lds:
// no VGPR staging, no ds_write pass) into a 3-deep ring of [256+128 rows][128
// B] stages, two tiles in flight across the single raw s_barrier of each
// K-step (counted vmcnt, never 0 in the loop). The LDS-DMA writes each wave-
// instruction's 64 x 16 B linearly (8 rows x 128 B), so the conv_mma XOR
// swizzle (chunk ^ row&7) is applied on the SOURCE side: lane l fetches
// logical chunk (l&7) ^ (l>>3) of its row. Zero padding and the M tail are
// buffer range-check zeros (offset past the buffer). Requires C (and C1) %
// 64 == 0, Nout % 128 == 0, no input prologue.
constexpr int WBM = 256, WBN = 128, WSTAGE = (WBM + WBN) * 128, WNSTAGE = 3;
constexpr int WWM = 4, WWN = 2, WTHREADS = 64 * WWM * WWN;  // 8 waves of 64x64: two per SIMD
constexpr int WLDS = WNSTAGE * WSTAGE;  // 147456 B: also holds the C staging tile

template <bool PADCHK, bool DUAL, typename T = bf16_t>
__global__ void __launch_bounds__(WTHREADS, 1) k_conv_fwd_wide(ConvArgs a) {
  const StampScope stamp_scope_(a.stamp);  // (null unless tools/stream_stamps.py armed it)
  constexpr int ES = 2, EPC = 8, BK = 64;
  constexpr int NW = WTHREADS / 64;
  constexpr int NA = WBM / 8 / NW;  // A row-groups (8 rows) per wave: 4
  constexpr int NB = WBN / 8 / NW;  // B row-groups per wave: 2
  static_assert(NA + NB == 6, "vmcnt counts below assume 6 DMA per wave per K-step");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WWN, wn = wid % WWN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lin / a.ntiles, nt = lin % a.ntiles;
  const int m0 = mt * WBM, n0 = nt * WBN;
  const int lr = lane >> 3;        // row within an 8-row group
  const int lc = (lane & 7) ^ lr;  // logical 16-B chunk this lane fetches (source-side swizzle)
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem);

  const v4i_t rx = buf_rsrc(a.x, (long long)a.N * a.H * a.W * a.ldx * ES);
  const v4i_t rx2 = buf_rsrc(DUAL ? a.x2 : a.x, (long long)a.N * a.H * a.W * (DUAL ? a.ldx2 : a.ldx) * ES);
  const v4i_t rw = buf_rsrc(a.w, (long long)a.Nout * a.Ktot * ES);

  // this lane's A rows: wid*(NA*8) + i*8 + lr
  int h0[NA], w0[NA], b1[NA], b2[NA];
  bool mok[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = m0 + wid * (NA * 8) + i * 8 + lr;
    mok[i] = m < a.M;
    const int mm = mok[i] ? m : 0;
    const int hw = a.Ho * a.Wo;
    const int n = mm / hw, rem = mm - (mm / hw) * hw;
    const int ho = rem / a.Wo, wo = rem - (rem / a.Wo) * a.Wo;
    h0[i] = ho * a.stride - a.pad;
    w0[i] = wo * a.stride - a.pad;
    const int pix = (n * a.H + h0[i]) * a.W + w0[i];
    b1[i] = pix * a.ldx + lc * EPC;
    b2[i] = DUAL ? pix * a.ldx2 + lc * EPC : 0;
  }
  unsigned vb[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int n = n0 + wid * (NB * 8) + i * 8 + lr;  // Nout % 128 == 0: always in range
    vb[i] = (unsigned)((n * a.Ktot + lc * EPC) * ES);
  }
  const int nk = a.Ktot / BK;

  // K cursor (filter row r, column s, channel c0) advanced without divisions: issue() runs in K order
  // channel chunk outer, tap inner (see k_conv_fwd_buf): L2 reuse of the gather
  int cr = 0, cs = 0, cc = 0;
  auto issue = [&](int kt, int stage) {
    (void)kt;
    const unsigned As = lds0 + stage * WSTAGE;
    const unsigned Bs = As + WBM * 128;
    const int c0 = cc, rd = cr * a.dil, sd = cs * a.dil;
    const int k0 = (cr * a.KW + cs) * a.C + c0;  // uniform
    if (++cs == a.KW) {
      cs = 0;
      if (++cr == a.KH) { cr = 0; cc += BK; }
    }
    if (DUAL && c0 >= a.C1) {
      const int toff = (rd * a.W + sd) * a.ldx2 + (c0 - a.C1);
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        bool ok = mok[i];
        if (PADCHK) ok = ok && (unsigned)(h0[i] + rd) < (unsigned)a.H && (unsigned)(w0[i] + sd) < (unsigned)a.W;
        const unsigned vo = ok ? (unsigned)((b2[i] + toff) * ES) : BUF_OOB;
        dma16(rx2, vo, 0, As + (wid * (NA * 8) + i * 8) * 128);
      }
    } else {
      const int toff = (rd * a.W + sd) * a.ldx + c0;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        bool ok = mok[i];
        if (PADCHK) ok = ok && (unsigned)(h0[i] + rd) < (unsigned)a.H && (unsigned)(w0[i] + sd) < (unsigned)a.W;
        const unsigned vo = ok ? (unsigned)((b1[i] + toff) * ES) : BUF_OOB;
        dma16(rx, vo, 0, As + (wid * (NA * 8) + i * 8) * 128);
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) dma16(rw, vb[i], (unsigned)(k0 * ES), Bs + (wid * (NB * 8) + i * 8) * 128);
  };

  f32x4_t acc[WBM / (16 * WWM)][WBN / (16 * WWN)];
#pragma unroll
  for (int i = 0; i < WBM / (16 * WWM); ++i)
#pragma unroll
    for (int j = 0; j < WBN / (16 * WWN); ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // ring: tile kt lives in stage kt % 3; tiles kt+1 and kt+2 in flight while kt is computed
  issue(0, 0);
  if (nk > 1) issue(1, 1);
  int st = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // retire this wave's DMA of tile kt (tile kt+1's 6 may stay in flight); the barrier then
    // publishes every wave's part of tile kt and orders the refill of stage (kt+2)%3 after
    // every wave's reads of tile kt-1 (retired by lgkmcnt(0))
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(6)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + 2 < nk) issue(kt + 2, st == 0 ? 2 : st - 1);
    conv_mma<T, WBM, WBN, WWM, WWN>(smem + st * WSTAGE, acc, wm, wn, lane);
    st = st == 2 ? 0 : st + 1;
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  conv_epilogue<T, WBM, WBN, WWM, WWN>(a, acc, smem, tid, mt, nt, m0, n0);
}

// --------------------------------------- forward, LDS-DMA square form (bf16)
// 256x256 block tile, 8 waves (2 M x 4 N) of 128x64 each (8x4 MFMA
// fragments, 64 v_mfma_f32_16x16x32_bf16 per wave per K-step), BK = 64, one
// workgroup per CU, two 64 KiB LDS stages. A K-step stages 64 KiB per CU for
// twice the MFMA work of the 256x128 form (32 B per MFMA-cycle instead of
// 47): on the 256x128 form the per-CU load path, not the matrix pipe, was the
// bound (SQ PMC: 43 % MFMA busy, 36 % of wave time parked in waitcnt /
// barrier). The next tile's 8 LDS-DMA pieces per wave are issued between
// the current tile's MFMA groups, right after the one barrier per K-step
// that retires the current tile (vmcnt(0): only it is in flight) and frees
// the other stage. Requires Nout % 256 == 0 plus the wide form's conditions.

// VAR bit 0: waves 4-7 at static priority 1; bit 1: s_setprio around each MFMA group.
// WM_ x WN_ waves: launched as 2 x 4 (8 waves, 128x64 each, two per SIMD). The 2 x 2 split (4 waves,
// one per SIMD, 128x128 each, accumulators in the AGPR half of the register file) computes the same bits
// and was measured slower on every hot shape (round 5, profiles/r05c_sq_4wave_ab.txt); its launch path
// was removed in round 6.
template <bool PADCHK, bool DUAL, int VAR, typename T = bf16_t, int WM_ = QWM, int WN_ = QWN>
__global__ void __launch_bounds__(64 * WM_ * WN_, 1) k_conv_fwd_sq(ConvArgs a) {
  const StampScope stamp_scope_(a.stamp);  // (null unless tools/stream_stamps.py armed it)
  constexpr int ES = 2, EPC = 8, BK = 64;
  constexpr int NW = WM_ * WN_;
  constexpr int NA = QBM / 8 / NW;  // A row-groups (8 rows) per wave: 4 (8 waves) / 8 (4 waves)
  constexpr int NB = QBN / 8 / NW;  // B row-groups per wave
  constexpr int FM = QBM / (16 * WM_), FN = QBN / (16 * WN_);
  constexpr int PPK = (NA + NB) / 2;  // DMA pieces per k-half
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN_, wn = wid % WN_;
  if constexpr (VAR & 1) {
    if (wid >= 4) __builtin_amdgcn_s_setprio(1);
  }
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lin / a.ntiles, nt = lin % a.ntiles;
  const int m0 = mt * QBM, n0 = nt * QBN;
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;  // source-side swizzle (see k_conv_fwd_wide)
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem);

  const v4i_t rx = buf_rsrc(a.x, (long long)a.N * a.H * a.W * a.ldx * ES);
  const v4i_t rx2 = buf_rsrc(DUAL ? a.x2 : a.x, (long long)a.N * a.H * a.W * (DUAL ? a.ldx2 : a.ldx) * ES);
  const v4i_t rw = buf_rsrc(a.w, (long long)a.Nout * a.Ktot * ES);

  int h0[NA], w0[NA], b1[NA], b2[NA];
  bool mok[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = m0 + wid * (NA * 8) + i * 8 + lr;
    mok[i] = m < a.M;
    const int mm = mok[i] ? m : 0;
    const int hw = a.Ho * a.Wo;
    const int n = mm / hw, rem = mm - (mm / hw) * hw;
    const int ho = rem / a.Wo, wo = rem - (rem / a.Wo) * a.Wo;
    h0[i] = ho * a.stride - a.pad;
    w0[i] = wo * a.stride - a.pad;
    const int pix = (n * a.H + h0[i]) * a.W + w0[i];
    b1[i] = pix * a.ldx + lc * EPC;
    b2[i] = DUAL ? pix * a.ldx2 + lc * EPC : 0;
  }
  unsigned vb[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int n = n0 + wid * (NB * 8) + i * 8 + lr;  // Nout % 256 == 0: always in range
    vb[i] = (unsigned)((n * a.Ktot + lc * EPC) * ES);
  }
  const int nk = a.Ktot / BK;

  // K cursor: channel chunk outer, tap inner. prep() fixes one K-step's
  // source, tap offset and weight offset; piece(p) issues DMA piece p of it.
  int cr = 0, cs = 0, cc = 0;
  bool p_hi = false;
  int p_toff = 0, p_rd = 0, p_sd = 0;
  unsigned p_koff = 0, p_As = 0, p_Bs = 0;
  auto prep = [&](int stage) {
    const int c0 = cc, rd = cr * a.dil, sd = cs * a.dil;
    p_koff = (unsigned)(((cr * a.KW + cs) * a.C + c0) * ES);
    if (++cs == a.KW) {
      cs = 0;
      if (++cr == a.KH) { cr = 0; cc += BK; }
    }
    p_hi = DUAL && c0 >= a.C1;
    p_toff = p_hi ? (rd * a.W + sd) * a.ldx2 + (c0 - a.C1) : (rd * a.W + sd) * a.ldx + c0;
    p_rd = rd;
    p_sd = sd;
    p_As = lds0 + stage * QSTAGE;
    p_Bs = p_As + QBM * 128;
  };
  auto piece = [&](int p) {
    if (p < NA) {
      bool ok = mok[p];
      if (PADCHK) ok = ok && (unsigned)(h0[p] + p_rd) < (unsigned)a.H && (unsigned)(w0[p] + p_sd) < (unsigned)a.W;
      const unsigned vo = ok ? (unsigned)(((p_hi ? b2[p] : b1[p]) + p_toff) * ES) : BUF_OOB;
      dma16(p_hi ? rx2 : rx, vo, 0, p_As + (wid * (NA * 8) + p * 8) * 128);
    } else {
      const int i = p - NA;
      dma16(rw, vb[i], p_koff, p_Bs + (wid * (NB * 8) + i * 8) * 128);
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  prep(0);
#pragma unroll
  for (int p = 0; p < NA + NB; ++p) piece(p);
  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt is the only DMA in flight: retire it; the barrier publishes every wave's part
    // and orders the refill of the other stage after every wave's reads of tile kt-1
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const bool more = kt + 1 < nk;
    if (more) prep((kt + 1) & 1);
    const char* As = smem + (kt & 1) * QSTAGE;
    const char* Bs = As + QBM * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + fg;
      uint4 av[FM], bv[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * (QBN / WN_) + j * 16 + fr;
        bv[j] = *(const uint4*)(Bs + col * 128 + ((ch ^ (col & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * (QBM / WM_) + i * 16 + fr;
        av[i] = *(const uint4*)(As + row * 128 + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if constexpr (PPK >= FM) {
          if (more)
#pragma unroll
            for (int q = 0; q < PPK / FM; ++q) piece(kk * PPK + i * (PPK / FM) + q);
        } else {
          if (more && i % (FM / PPK) == 0) piece(kk * PPK + i / (FM / PPK));
        }
        if constexpr ((VAR & 2) != 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = mfma16<T>(av[i], bv[j], acc[i][j]);
        if constexpr ((VAR & 2) != 0) __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  conv_epilogue<T, QBM, QBN, WM_, WN_>(a, acc, smem, tid, mt, nt, m0, n0);
}

// ------------------------------- forward, persistent LDS-DMA square form (bf16)
// The 256x256 / BK=64 LDS-DMA tile of k_conv_fwd_sq as a PERSISTENT kernel:
// gridDim = min(tiles, CUs), each block walks its tiles (xcd-remapped
// linear order, stride gridDim) as ONE flat stream of K-steps, so the next
// tile's first K-step is already in flight while the current tile's
// epilogue runs -- the per-tile fill and drain that dominate short-K convs
// (1x1 over 256..1024 channels: 4..16 K-steps per tile) overlap.
// The epilogue needs no LDS: the MFMA operands are swapped (weights are the
// row operand, pixels the column operand) and the weight rows of each
// wave's 64-channel slab are loaded in a permuted order, so after the K loop
// lane (g = lane>>4, p = lane&15) holds output channels 8g..8g+7 and
// 32+8g..32+8g+7 (of the wave's 64) of pixel p of every pixel fragment: two
// 16-B bf16 stores per pixel row, in each of which the 4 lanes of a pixel
// write one contiguous 64-B run (whole half-lines, not interleaved 16-B
// pieces of two stores),
// straight from the accumulators (no C staging, the stage ring stays free
// for the next tile's DMA). BN statistics: per-lane sums over the lane's
// pixels, a 16-lane shuffle reduction, then the 2 pixel-half waves combine
// in a 4 KiB LDS slot (slab mode) or each add (stat_acc mode).

// EPI: the epilogue, fixed at compile time so only its path is in the code
// (a runtime switch per tile inflated the kernel to ~13 k instructions of
// activation variants): 0 = BN partial statistics (no activation), 1 + act =
// bias + DMF_ACT_* activation. The next K-step's DMA pieces are spread over
// both k-halves (pieces 0-3 in the first, 4-7 in the second; "all 8 in one
// half" or "all 8 after the barrier" measured no better).
template <bool PADCHK, bool DUAL, int EPI, int TBM = QBM, int TBN = QBN, int TWN = QWN, typename T = bf16_t>
__global__ void __launch_bounds__(64 * 2 * TWN, TWN == 4 ? 1 : 2) k_conv_fwd_ps(ConvArgs a) {
  const StampScope stamp_scope_(a.stamp);  // (null unless tools/stream_stamps.py armed it)
  constexpr int ES = 2, BK = 64;
  constexpr int TWM = 2;  // two pixel-half waves per 64-channel slab (ps_epilogue)
  constexpr int NTH = 64 * TWM * TWN, NW = TWM * TWN;
  constexpr int STG = (TBM + TBN) * 128;  // one K-step stage: TBM pixel rows + TBN weight rows of 128 B
  constexpr int NA = TBM / 8 / NW;  // pixel row-groups (8 rows) per wave: 4
  constexpr int NB = TBN / 8 / NW;  // weight row-groups per wave: 4
  constexpr int FM = TBM / (16 * TWM), FN = TBN / (16 * TWN);  // 8 (256x256) or 4 (128x128) pixel x 4 channel fragments
  static_assert(NA == 4 && NB == 4 && FN == 4, "k_conv_fwd_ps geometry");
  // an epilogue's stores per wave (+2 float64 atomics, pixel-half 0, stat_acc); the statistics-only
  // epilogue (12) stores nothing, so nothing younger than the in-flight DMA may be waited out
  constexpr int EPI_VM = EPI == 12 ? 0 : EPI == 15 ? 4 * FM : 2 * FM;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / TWN, wn = wid % TWN;
  // (no static priority split between the wave halves here: measured -0.4 % encoder forward
  // without it, interleaved A/B; k_conv_fwd_sq keeps its VAR 1)
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;  // source-side swizzle (see k_conv_fwd_wide)
  const int fr = lane & 15, fg = lane >> 4;
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  float* sred = (float*)(smem + 2 * STG);

  const v4i_t rx = buf_rsrc(a.x, (long long)a.N * a.H * a.W * a.ldx * ES);
  const v4i_t rx2 = buf_rsrc(DUAL ? a.x2 : a.x, (long long)a.N * a.H * a.W * (DUAL ? a.ldx2 : a.ldx) * ES);
  const v4i_t rw = buf_rsrc(a.w, (long long)a.Nout * a.Ktot * ES);
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(a.y, 0, (int)((long long)a.M * a.ldy * ES), BUF_FLAGS);
  const int nk = a.Ktot / BK;
  const int ntile = a.mtiles * a.ntiles;
  const int hw = a.Ho * a.Wo;
  // bias (heads / projections with bias) staged once: the epilogue must issue no vmem load
  // (a compiler-visible load would be waited for behind the in-flight DMA)
  float* sbias = sred + 2 * TBN * 2;
  if constexpr (EPI == 8 || EPI == 11) {
    // the known BatchNorm(s) of the affine epilogue: [scale | shift (+ the shortcut's shift) | shortcut scale]
    // (aff_acc: the BatchNorm finalized here from the float64 arena, dmf_conv2d_fwd_affine_acc; block 0
    // also moves the running statistics)
    for (int i = tid; i < a.Nout; i += NTH) {
      const float2 ss = a.aff_acc ? arena_bn_channel(a, i, blockIdx.x == 0) : make_float2(a.out_ss[i], a.out_ss[a.Nout + i]);
      sbias[i] = ss.x;
      sbias[a.Nout + i] = ss.y + (EPI == 11 ? a.res_ss[a.Nout + i] : 0.f);
      if (EPI == 11) sbias[2 * a.Nout + i] = a.res_ss[i];
    }
    if (a.aff_acc && blockIdx.x == 0 && tid == 0 && a.fin.nbt) *a.fin.nbt += 1;
    __syncthreads();
  } else if constexpr (EPI == 15) {
    // the token residual epilogue: [bias | colscale] x Nout
    for (int i = tid; i < a.Nout; i += NTH) {
      sbias[i] = a.bias ? a.bias[i] : 0.f;
      sbias[a.Nout + i] = a.colscale ? a.colscale[i] : 1.f;
    }
    __syncthreads();
  } else if (a.bias) {
    for (int i = tid; i < a.Nout; i += NTH) sbias[i] = a.bias[i];
    __syncthreads();
  }

  // DMA row state of the tile being STAGED (may run one tile ahead of the tile being computed)
  int h0[NA], w0[NA], b1[NA], b2[NA];
  bool mok[NA];
  unsigned vb[NB];
  auto rows_for = [&](int lin) {
    const int mt = lin / a.ntiles, nt = lin - (lin / a.ntiles) * a.ntiles;
    const int m0 = mt * TBM, n0 = nt * TBN;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = m0 + wid * (NA * 8) + i * 8 + lr;
      mok[i] = m < a.M;
      const int mm = mok[i] ? m : 0;
      const int n = mm / hw, rem = mm - (mm / hw) * hw;
      const int ho = rem / a.Wo, wo = rem - (rem / a.Wo) * a.Wo;
      h0[i] = ho * a.stride - a.pad;
      w0[i] = wo * a.stride - a.pad;
      const int pix = (n * a.H + h0[i]) * a.W + w0[i];
      b1[i] = pix * a.ldx + lc * 8;
      b2[i] = DUAL ? pix * a.ldx2 + lc * 8 : 0;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int n = n0 + ps_perm(wid * (NB * 8) + i * 8 + lr);  // Nout % 256 == 0: in range
      vb[i] = (unsigned)((n * a.Ktot + lc * 8) * ES);
    }
  };

  // K cursor of the staged stream: channel chunk outer, tap inner
  int cr = 0, cs = 0, cc = 0;
  bool p_hi = false;
  int p_toff = 0, p_rd = 0, p_sd = 0;
  unsigned p_koff = 0, p_As = 0, p_Bs = 0;
  auto prep = [&](int stage) {
    const int c0 = cc, rd = cr * a.dil, sd = cs * a.dil;
    p_koff = (unsigned)(((cr * a.KW + cs) * a.C + c0) * ES);
    if (++cs == a.KW) {
      cs = 0;
      if (++cr == a.KH) { cr = 0; cc += BK; }
    }
    p_hi = DUAL && c0 >= a.C1;
    p_toff = p_hi ? (rd * a.W + sd) * a.ldx2 + (c0 - a.C1) : (rd * a.W + sd) * a.ldx + c0;
    p_rd = rd;
    p_sd = sd;
    p_As = lds0 + stage * STG;
    p_Bs = p_As + TBM * 128;
  };
  auto piece = [&](int p) {
    if (p < NA) {
      bool ok = mok[p];
      if (PADCHK) ok = ok && (unsigned)(h0[p] + p_rd) < (unsigned)a.H && (unsigned)(w0[p] + p_sd) < (unsigned)a.W;
      const unsigned vo = ok ? (unsigned)(((p_hi ? b2[p] : b1[p]) + p_toff) * ES) : BUF_OOB;
      dma16(p_hi ? rx2 : rx, vo, 0, p_As + (wid * (NA * 8) + p * 8) * 128);
    } else {
      const int i = p - NA;
      dma16(rw, vb[i], p_koff, p_Bs + (wid * (NB * 8) + i * 8) * 128);
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  int t = blockIdx.x;  // position in this block's tile sequence (stride gridDim)
  if (t >= ntile) return;
  int lin = xcd_remap(t, ntile);
  rows_for(lin);
  prep(0);
#pragma unroll
  for (int p = 0; p < NA + NB; ++p) piece(p);
  int kt = 0, st = 0;
  bool epi = false;  // the previous iteration ran an epilogue (its stores may stay in flight)
  for (;;) {
    // retire the staged step's DMA (the oldest vmem ops of this wave); the barrier publishes every
    // wave's part and orders the refill of the other stage after every wave's reads of the previous
    // step. After an epilogue its 16 stores (+2 atomics) are younger: leave them in flight.
    if (epi) {
      // (EPI 8 / 11 with aff_acc carry an arena in stat_acc but issue no statistics atomics)
      if ((EPI == 0 || EPI == 5 || EPI == 12) && (a.stat_acc > 0 || a.stat_acc == -1) && wm == 0)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(EPI_VM + 2) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(EPI_VM) : "memory");
      epi = false;
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const bool last = kt + 1 == nk;
    const int tnext = t + (int)gridDim.x;
    bool more = true;
    if (!last) {
      prep(st ^ 1);
    } else if (tnext < ntile) {
      // first K-step of this block's next tile goes in flight under this step and the epilogue
      rows_for(xcd_remap(tnext, ntile));
      cr = 0; cs = 0; cc = 0;
      prep(st ^ 1);
    } else {
      more = false;
    }
    const char* Ps = smem + st * STG;  // pixel rows
    const char* Ws = Ps + TBM * 128;   // weight rows (permuted)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + fg;
      uint4 pv[FM], wv[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * (TBN / TWN) + j * 16 + fr;
        wv[j] = *(const uint4*)(Ws + row * 128 + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * (TBM / TWM) + i * 16 + fr;
        pv[i] = *(const uint4*)(Ps + row * 128 + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        // the next K-step's 8 pieces, 4 per k-half, spread over the FM fragment rows
        if (more && i % (FM / 4) == 0 && !(a.dbg & 2)) piece(kk * 4 + i / (FM / 4));
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = mfma16<T>(wv[j], pv[i], acc[i][j]);
      }
    }
    st ^= 1;
    if (!last) {
      ++kt;
      continue;
    }
    // ---------------- epilogue of tile `lin` (the next tile's step 0 is in flight)
    if constexpr (EPI == 15) ps_epilogue_tokres<TBN, FM, TBM>(a, acc, lin, sbias, wm, wn, fr, fg);
    else if (!(a.dbg & 4)) ps_epilogue<EPI, TBN, FM, TBM, T>(a, acc, lin, ry, sred, sbias, tid, wm, wn, fr, fg);
    epi = !(a.dbg & 4);
    if (!more) break;
    t = tnext;
    lin = xcd_remap(t, ntile);
    kt = 0;
  }
}

// INA: A-prologue activation (-1 = no prologue, else DMF_ACT_*)
// FASTC: C (and the concat split C1) are multiples of BK, so every K-step
// lies inside one filter tap: the tap/channel decode is block-uniform
// (scalar) instead of two integer divisions per lane and step.
template <typename T, bool DGRAD, int INA, bool FASTC>
__global__ void __launch_bounds__(CTHREADS, 2) k_conv_igemm(ConvArgs a) {
  const StampScope stamp_scope_(a.stamp);  // (null unless tools/stream_stamps.py armed it)
  constexpr int EPC = 16 / sizeof(T);  // elements per 16-B chunk
  constexpr int BK = 8 * EPC;          // 8 chunks per LDS row
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int nblk = gridDim.x;
  const int lin = xcd_remap(blockIdx.x, nblk);
  const int mt = lin / a.ntiles, nt = lin % a.ntiles;
  const int m0 = mt * CBM, n0 = nt * CBN;

  const T* __restrict__ X = (const T*)a.x;
  const T* __restrict__ Wt = (const T*)a.w;

  // ---- per-thread load assignment: chunk q of rows (tid>>3) + 32*i
  const int q = tid & 7;
  const int rbase = tid >> 3;
  // A rows: decode output pixel once
  int a_n[4], a_h[4], a_w[4];
  bool a_ok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + rbase + 32 * i;
    a_ok[i] = m < a.M;
    const int mm = a_ok[i] ? m : 0;
    const int hw = a.Ho * a.Wo;
    a_n[i] = mm / hw;
    const int rem = mm - a_n[i] * hw;
    a_h[i] = rem / a.Wo;
    a_w[i] = rem - a_h[i] * a.Wo;
  }
  const int nk = (a.Ktot + BK - 1) / BK;

  uint4 ra[4], rb[4];
  auto gload = [&](int kt) {
    const int k = kt * BK + q * EPC;
    bool kok;
    int tap, c;
    if constexpr (FASTC) {
      const int k0 = kt * BK;  // uniform
      tap = k0 / a.C;
      c = k0 - tap * a.C + q * EPC;
      kok = true;
    } else {
      kok = k < a.Ktot;
      tap = kok ? k / a.C : 0;
      c = k - tap * a.C;
    }
    const int r = tap / a.KW, s = tap - (tap / a.KW) * a.KW;
    const T* src = X;
    int ldsrc = a.ldx;
    if (!DGRAD && c >= a.C1) {  // channel-concat second source (BackboneAdapter chain [2,3])
      src = (const T*)a.x2;
      c -= a.C1;
      ldsrc = a.ldx2;
    }
    float sc[EPC], sh[EPC];
    if constexpr (INA >= 0) {
#pragma unroll
      for (int e = 0; e < EPC; e += 4) {
        const float4 s4 = *(const float4*)(a.in_ss + c + e), h4 = *(const float4*)(a.in_ss + a.C + c + e);
        sc[e] = s4.x; sc[e + 1] = s4.y; sc[e + 2] = s4.z; sc[e + 3] = s4.w;
        sh[e] = h4.x; sh[e + 1] = h4.y; sh[e + 2] = h4.z; sh[e + 3] = h4.w;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool ok = kok && a_ok[i];
      int hi, wi;
      if (!DGRAD) {
        hi = a_h[i] * a.stride - a.pad + r * a.dil;
        wi = a_w[i] * a.stride - a.pad + s * a.dil;
      } else {
        const int hn = a_h[i] + a.pad - r * a.dil, wn_ = a_w[i] + a.pad - s * a.dil;
        if (a.stride == 1) {  // uniform branch: no integer division on the common path
          hi = hn;
          wi = wn_;
        } else {
          ok = ok && hn >= 0 && wn_ >= 0 && (hn % a.stride) == 0 && (wn_ % a.stride) == 0;
          hi = hn / a.stride;
          wi = wn_ / a.stride;
        }
      }
      ok = ok && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
      if (ok) {
        const size_t off = ((size_t)(a_n[i] * a.H + hi) * a.W + wi) * ldsrc + c;
        ra[i] = *(const uint4*)(src + off);
        if constexpr (INA >= 0) chunk_affine<T, INA>(ra[i], sc, sh);
      } else {
        ra[i] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + rbase + 32 * i;
      if (kok && n < a.Nout) {
        rb[i] = *(const uint4*)(Wt + (size_t)n * a.Ktot + k);
      } else {
        rb[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto lds_store = [&](int stage) {
    char* base = smem + stage * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = rbase + 32 * i;
      *(uint4*)(base + row * 128 + ((q ^ (row & 7)) << 4)) = ra[i];
      *(uint4*)(base + CBM * 128 + row * 128 + ((q ^ (row & 7)) << 4)) = rb[i];
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  gload(0);
  lds_store(0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    conv_mma<T>(smem + cur * STAGE_BYTES, acc, wm, wn, lane);
    if (kt + 1 < nk) lds_store(cur ^ 1);
    __syncthreads();
  }
  conv_epilogue<T>(a, acc, smem, tid, mt, nt, m0, n0);
}

// Which kernel/tile a forward launch uses. The buffer-load kernel needs C
// (and C1) multiples of BK, no input prologue and < 2 GiB operands. Tile:
// BN = 64 when Cout <= 64 (no wasted MFMA columns), BM = 64 when 128-row
// tiles would leave fewer than ~2 blocks per CU.
struct ConvPlan {
  bool buf;
  bool wide;  // k_conv_fwd_wide (LDS-DMA, 256x128)
  bool sq;    // k_conv_fwd_sq (LDS-DMA, 256x256)
  int bm, bn;
  bool ps;    // k_conv_fwd_ps (persistent LDS-DMA 256x256, register epilogue)
  bool pp;    // k_conv_fwd_pp (conv_pp.hip: ping-pong 8-phase 256x256, register epilogue)
  bool stem;  // k_conv_stem (conv_stem.hip): 7x7 / 2 over 8 or 16 channels, 64 out
};
// 7 = ping-pong 256x256 form (conv_pp.hip): 0 off, 1 (default) for 3x3 and K >= 1024 (where it beats the
// persistent form: tools/conv_bench.py --tunes, profiles/r03h_conv_ab.txt), 2 for every legal shape
static int g_pp_mode = 1;
// 10 = the dedicated 7x7 stem kernel (conv_stem.hip) on (1, default) / off
static int g_stem_enable = 1;
// 11 = the statistics epilogue without bias adds / row masks for whole-tile launches (EPI 5) on / off
static int g_fast_epi = 1;
// runtime knobs (dmf_conv_tune): 0 = square tile on/off, 1 = square-tile VAR
static int g_sq_enable = 1, g_sq_var = 1;
// 2 = forced forward tile for A/B sweeps: 0 auto, 1 buf 128x128, 2 buf 64x128,
// 3 buf 128x64, 4 buf 64x64, 5 wide 256x128, 6 square 256x256 (only where legal)
static int g_force = 0;
// 3 = dmf_conv2d_fwd_acc accumulation mode (benchmarking; see acc_stats): 0 default
static int g_stat_mode = 0;
// 4 = persistent square form (k_conv_fwd_ps) on (1, default) / off
static int g_ps_enable = 1;
// benchmarking bits of k_conv_fwd_ps (skip DMA / epilogue / stores / statistics): set only through
// dmf_conv_tune key 6 by the A/B tools (a stray setting would silently corrupt outputs)
static int g_ps_dbg = 0;
// 16 = k_conv_fwd_ps output stores nontemporal (streaming) for outputs of at least this many MiB; 0 off.
// Default 100 (the 512->2048 / S=384 expansions): mode A +0.3 %, config 5 +0.6 %, mode B / config 2
// +0.2 % (profiles/r06o_nt_store_ab.txt); at 60 (the 64 MiB outputs too) mode A lost 0.3 %
static int g_ps_nt_mb = 100;
// 14 / 15 = tiles a launch needs before the wide (256x128) / square (256x256) forms take it: one per
// CU. At 128 (half a tile per CU, the other encoder stream filling the rest) the two-stream
// mode-A step measured -1.2 %, but every single-stream launch runs on half the GPU: config 2
// (one stream) -14 %, conv-forward roofline fraction 0.27 -> 0.23 (profiles/r02s_bench.json)
static long long g_wide_min_tiles = 256;
static long long g_min_tiles = 256;
static int cu_count() {
  static int cached = 0;
  if (!cached) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cached, hipDeviceAttributeMultiprocessorCount, dev);
    if (cached <= 0) cached = 256;
  }
  return cached;
}

static ConvPlan conv_plan(int dtype, bool dgrad, const ConvArgs& a) {
  ConvPlan p{false, false, false, CBM, CBN, false, false, false};
  if (g_stem_enable && conv_stem_ok(dtype, dgrad, a)) {
    p.stem = true;
    p.bm = conv_stem_m_tile(a);
    p.bn = 64;
    return p;
  }
  const bool plain = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0;
  // an input affine runs on the buffer-load kernel for plain 1x1 convs, else on k_conv_igemm
  if (dgrad || (a.in_ss != nullptr && !(plain && a.x2 == nullptr)))
    return p;
  const int es = is16(dtype) ? 2 : 4;
  const int bk = is16(dtype) ? 64 : 32;
  const bool fastc = a.C % bk == 0 && (a.x2 == nullptr || a.C1 % bk == 0);
  const long long xbytes = (long long)a.N * a.H * a.W * a.ldx * es;
  const long long x2bytes = a.x2 ? (long long)a.N * a.H * a.W * a.ldx2 * es : 0;
  const long long wbytes = (long long)a.Nout * a.Ktot * es;
  p.buf = fastc && xbytes < (1LL << 31) && x2bytes < (1LL << 31) && wbytes < (1LL << 31);
  if (!p.buf) return p;
  if (a.in_ss != nullptr) {
    p.bn = a.Nout <= 64 ? 64 : 128;
    p.bm = (long long)cdiv(a.M, 128) * cdiv(a.Nout, p.bn) < 512 ? 64 : 128;
    return p;
  }
  if (g_force) {
    const bool wide_ok = is16(dtype) && a.Nout % WBN == 0 && a.Ktot >= 512;
    const bool sq_ok = is16(dtype) && a.Nout % QBN == 0 && a.Ktot >= 512;
    if (g_force == 6 && sq_ok) { p.wide = p.sq = true; p.bm = QBM; p.bn = QBN; return p; }
    if (g_force == 5 && wide_ok) { p.wide = true; p.bm = WBM; p.bn = WBN; return p; }
    if (g_force >= 1 && g_force <= 4) {
      p.bm = (g_force == 1 || g_force == 3) ? 128 : 64;
      p.bn = (g_force == 1 || g_force == 2) ? 128 : 64;
      return p;
    }
  }
  // ping-pong square tile: same legality as the persistent form below
  const bool sq_ps_ok = is16(dtype) && a.tickets == nullptr && a.Nout % QBN == 0 &&
                        a.Ktot >= 64 && (long long)cdiv(a.M, QBM) * (a.Nout / QBN) >= g_min_tiles &&
                        (long long)a.M * a.ldy * 2 < (1LL << 31);
  // (the token-residual epilogue exists on the persistent 1x1 form only)
  if (sq_ps_ok && !a.tok_res &&
      (g_pp_mode >= 2 || (g_pp_mode == 1 && !(g_ps_enable && a.Ktot < 1024 && a.KH * a.KW == 1)))) {
    p.wide = p.sq = p.pp = true;
    p.bm = QBM;
    p.bn = QBN;
    return p;
  }
  // persistent square LDS-DMA tile: whole 256-column tiles, >= one tile per CU, no fused-finalize
  // tickets, output addressable by a 32-bit buffer offset
  if (is16(dtype) && g_ps_enable && a.tickets == nullptr && a.Nout % QBN == 0 &&
      a.Ktot >= 64 && (long long)cdiv(a.M, QBM) * (a.Nout / QBN) >= g_min_tiles &&
      (long long)a.M * a.ldy * 2 < (1LL << 31)) {
    p.wide = p.sq = p.ps = true;
    p.bm = QBM;
    p.bn = QBN;
    return p;
  }
  // square LDS-DMA tile: whole 256-column tiles and >= one block per CU
  // (measured: +15 % on the dilated 3x3s; a short-K 1x1 (K <= 1024) is epilogue-
  // bound at one 256x256 block per CU and stays on the 256x128 form)
  if (is16(dtype) && g_sq_enable && a.Nout % QBN == 0 &&
      (a.KH * a.KW > 1 ? a.Ktot >= 512 : a.Ktot >= 2048) && (long long)cdiv(a.M, QBM) * (a.Nout / QBN) >= g_min_tiles) {
    p.wide = p.sq = true;
    p.bm = QBM;
    p.bn = QBN;
    return p;
  }
  // wide LDS-DMA tile: bf16, whole 128-column tiles, long enough K, >= one block per CU
  if (is16(dtype) && a.Nout % WBN == 0 && a.Ktot >= 512 &&
      (long long)cdiv(a.M, WBM) * (a.Nout / WBN) >= g_wide_min_tiles) {
    p.wide = true;
    p.bm = WBM;
    p.bn = WBN;
    return p;
  }
  p.bn = a.Nout <= 64 ? 64 : 128;
  const long long blocks128 = (long long)cdiv(a.M, 128) * cdiv(a.Nout, p.bn);
  p.bm = blocks128 < 512 ? 64 : 128;
  return p;
}

// the body the most recent forward / dgrad launch on this host thread ran (dmf_conv_last_form: tests
// assert which forms a model-level parity run exercised)
static thread_local int g_last_form = -1;

// the forward / dgrad body of a plan for one storage type T (bf16, f16 or f32; the LDS-DMA forms exist for
// the 16-bit types only -- conv_plan never picks them for f32)
template <typename T>
static void launch_conv_t(const ConvPlan& plan, bool dgrad, ConvArgs& a, long long nblk, size_t lds_total,
                          hipStream_t st) {
  const dim3 g((unsigned)nblk), b(CTHREADS);
  const int bk = sizeof(T) == 2 ? 64 : 32;
  const bool fastc = a.C % bk == 0 && (a.x2 == nullptr || a.C1 % bk == 0);
  const bool plain = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0;
  const bool dual = a.x2 != nullptr;
#define DMF_CONV_LAUNCH(DG, INA)                                                                \
  do {                                                                                          \
    if (fastc) hipLaunchKernelGGL((k_conv_igemm<T, DG, INA, true>), g, b, lds_total, st, a);   \
    else hipLaunchKernelGGL((k_conv_igemm<T, DG, INA, false>), g, b, lds_total, st, a);        \
  } while (0)
#define DMF_BUF_LAUNCH(BM, BN)                                                                              \
  do {                                                                                                      \
    if (dual) hipLaunchKernelGGL((k_conv_fwd_buf<T, true, true, BM, BN>), g, b, lds_total, st, a);          \
    else if (plain) hipLaunchKernelGGL((k_conv_fwd_buf<T, false, false, BM, BN>), g, b, lds_total, st, a);  \
    else hipLaunchKernelGGL((k_conv_fwd_buf<T, true, false, BM, BN>), g, b, lds_total, st, a);              \
  } while (0)
  if (dgrad) {
    DMF_CONV_LAUNCH(true, -1);
    return;
  }
  if constexpr (sizeof(T) == 2) {
    if (plan.ps) {
      const dim3 gp((unsigned)std::min<long long>(nblk, cu_count())), bq(QTHREADS);
      // statistics without bias over whole tiles: the fast epilogue (EPI 5); a known BatchNorm: the
      // affine epilogue (EPI 8, plain shortcut / 11, BN'd shortcut)
      const int epi = a.tok_res ? 15
                      : (a.out_ss != nullptr || a.aff_acc) ? (a.res_ss != nullptr ? 11 : 8)
                      : a.y == nullptr ? 12
                      : a.partials != nullptr ? ((g_fast_epi && a.bias == nullptr && a.M % 256 == 0) ? 5 : 0)
                      : a.dp > 0.f ? 14
                                              : 1 + a.act;
      a.dbg = g_ps_dbg;
      if (g_ps_nt_mb > 0 && a.y && (long long)a.M * a.Nout * 2 >= ((long long)g_ps_nt_mb << 20)) a.dbg |= 32;
#define DMF_PS(E)                                                                                                \
  do {                                                                                                           \
    if (dual) hipLaunchKernelGGL((k_conv_fwd_ps<true, true, E, QBM, QBN, QWN, T>), gp, bq, lds_total, st, a);    \
    else if (plain) hipLaunchKernelGGL((k_conv_fwd_ps<false, false, E, QBM, QBN, QWN, T>), gp, bq, lds_total, st, a); \
    else hipLaunchKernelGGL((k_conv_fwd_ps<true, false, E, QBM, QBN, QWN, T>), gp, bq, lds_total, st, a);        \
  } while (0)
#define DMF_PS_AFF(E)                                                                                            \
  do {                                                                                                           \
    if (plain) hipLaunchKernelGGL((k_conv_fwd_ps<false, false, E, QBM, QBN, QWN, T>), gp, bq, lds_total, st, a); \
    else hipLaunchKernelGGL((k_conv_fwd_ps<true, false, E, QBM, QBN, QWN, T>), gp, bq, lds_total, st, a);        \
  } while (0)
      switch (epi) {
        case 12: DMF_PS_AFF(12); break;
        case 8: DMF_PS_AFF(8); break;
        case 11: DMF_PS_AFF(11); break;
        case 0: DMF_PS(0); break;
        case 1: DMF_PS(1); break;
        case 2: DMF_PS(2); break;
        case 3: DMF_PS(3); break;
        case 5: DMF_PS(5); break;
        case 14: DMF_PS_AFF(14); break;
        case 15: DMF_PS_AFF(15); break;
        default: DMF_PS(4); break;
      }
#undef DMF_PS
#undef DMF_PS_AFF
      return;
    }
    if (plan.sq) {
      const dim3 bq(QTHREADS);
#define DMF_SQ(V)                                                                                         \
  do {                                                                                                    \
    if (dual) hipLaunchKernelGGL((k_conv_fwd_sq<true, true, V, T>), g, bq, lds_total, st, a);             \
    else if (plain) hipLaunchKernelGGL((k_conv_fwd_sq<false, false, V, T>), g, bq, lds_total, st, a);     \
    else hipLaunchKernelGGL((k_conv_fwd_sq<true, false, V, T>), g, bq, lds_total, st, a);                 \
  } while (0)
      switch (g_sq_var) {
        case 1: DMF_SQ(1); break;
        case 2: DMF_SQ(2); break;
        case 3: DMF_SQ(3); break;
        default: DMF_SQ(0); break;
      }
#undef DMF_SQ
      return;
    }
    if (plan.wide) {
      const dim3 bw(WTHREADS);
      if (dual) hipLaunchKernelGGL((k_conv_fwd_wide<true, true, T>), g, bw, lds_total, st, a);
      else if (plain) hipLaunchKernelGGL((k_conv_fwd_wide<false, false, T>), g, bw, lds_total, st, a);
      else hipLaunchKernelGGL((k_conv_fwd_wide<true, false, T>), g, bw, lds_total, st, a);
      return;
    }
  }
  if (plan.buf && a.in_ss != nullptr) {
    const size_t lds_ina = lds_total + (size_t)a.C * 8;
    const int cfg = (plan.bm == 128 ? 2 : 0) + (plan.bn == 128 ? 1 : 0);
#define DMF_INA_BUF(IA)                                                                                   \
  do {                                                                                                    \
    switch (cfg) {                                                                                        \
      case 3: hipLaunchKernelGGL((k_conv_fwd_buf<T, false, false, 128, 128, IA>), g, b, lds_ina, st, a); break; \
      case 2: hipLaunchKernelGGL((k_conv_fwd_buf<T, false, false, 128, 64, IA>), g, b, lds_ina, st, a); break;  \
      case 1: hipLaunchKernelGGL((k_conv_fwd_buf<T, false, false, 64, 128, IA>), g, b, lds_ina, st, a); break;  \
      default: hipLaunchKernelGGL((k_conv_fwd_buf<T, false, false, 64, 64, IA>), g, b, lds_ina, st, a);         \
    }                                                                                                     \
  } while (0)
    switch (a.act_in) {
      case DMF_ACT_NONE: DMF_INA_BUF(DMF_ACT_NONE); break;
      case DMF_ACT_RELU: DMF_INA_BUF(DMF_ACT_RELU); break;
      default: DMF_INA_BUF(DMF_ACT_GELU); break;
    }
#undef DMF_INA_BUF
  } else if (plan.buf) {
    const int cfg = (plan.bm == 128 ? 2 : 0) + (plan.bn == 128 ? 1 : 0);
    switch (cfg) {
      case 3: DMF_BUF_LAUNCH(128, 128); break;
      case 2: DMF_BUF_LAUNCH(128, 64); break;
      case 1: DMF_BUF_LAUNCH(64, 128); break;
      default: DMF_BUF_LAUNCH(64, 64); break;
    }
  } else if (a.in_ss == nullptr) {
    DMF_CONV_LAUNCH(false, -1);
  } else {
    switch (a.act_in) {
      case DMF_ACT_NONE: DMF_CONV_LAUNCH(false, DMF_ACT_NONE); break;
      case DMF_ACT_RELU: DMF_CONV_LAUNCH(false, DMF_ACT_RELU); break;
      default: DMF_CONV_LAUNCH(false, DMF_ACT_GELU); break;
    }
  }
#undef DMF_BUF_LAUNCH
#undef DMF_CONV_LAUNCH
}

// In-kernel timing stamps (tools/stream_stamps.py): while armed, every forward-conv launch made from this
// process takes the next [start, end] pair of the armed device buffer (StampScope in the kernel) and its
// stream, form and GEMM shape are recorded here -- so the concurrency of a captured two-stream step can be
// read without a profiler (rocprofv3's kernel trace serialises a graph's branches).
struct StampRec { void* stream; int form, m, n, k; };
static unsigned long long* g_stamp_buf = nullptr;
static int g_stamp_cap = 0;
static std::vector<StampRec> g_stamp_rec;

extern "C" int dmf_stamp_arm(unsigned long long* buf, int capacity) {
  DMF_CHECK_ARG(buf == nullptr || (capacity > 0 && ((uintptr_t)buf % 8) == 0), "dmf_stamp_arm: bad buffer");
  g_stamp_buf = buf;
  g_stamp_cap = buf ? capacity : 0;
  g_stamp_rec.clear();
  return 0;
}
extern "C" int dmf_stamp_count(void) { return (int)g_stamp_rec.size(); }
extern "C" int dmf_stamp_info(int i, void** stream, int* form, int* m, int* n, int* k) {
  DMF_CHECK_ARG(i >= 0 && i < (int)g_stamp_rec.size() && stream && form && m && n && k, "dmf_stamp_info: %d", i);
  const StampRec& r = g_stamp_rec[i];
  *stream = r.stream; *form = r.form; *m = r.m; *n = r.n; *k = r.k;
  return 0;
}

static int launch_conv(int dtype, bool dgrad, ConvArgs& a, hipStream_t st, const char* what) {
  DMF_CHECK_ARG(dtype == DMF_F32 || is16(dtype), "%s: bad dtype %d", what, dtype);
  const int epc = is16(dtype) ? 8 : 4;
  DMF_CHECK_ARG(a.C % epc == 0 && a.ldx % epc == 0, "%s: input channels (%d) and stride (%d) must be multiples of %d",
                what, a.C, a.ldx, epc);
  DMF_CHECK_ARG(a.Nout % epc == 0 && a.ldy % epc == 0,
                "%s: output channels (%d) and stride (%d) must be multiples of %d", what, a.Nout, a.ldy, epc);
  DMF_CHECK_ARG(((uintptr_t)a.x % 16) == 0 && ((uintptr_t)a.y % 16) == 0 && ((uintptr_t)a.w % 16) == 0,
                "%s: pointers must be 16-byte aligned", what);
  DMF_CHECK_ARG(a.M > 0 && a.Nout > 0 && a.Ktot > 0, "%s: empty problem (M=%d N=%d K=%d)", what, a.M, a.Nout,
                a.Ktot);
  const ConvPlan plan = conv_plan(dtype, dgrad, a);
  g_last_form = plan.stem ? DMF_FORM_STEM : dgrad ? DMF_FORM_IGEMM : plan.pp ? DMF_FORM_PP : plan.ps ? DMF_FORM_PS
              : plan.sq ? DMF_FORM_SQ : plan.wide ? DMF_FORM_WIDE
              : plan.buf ? (a.in_ss != nullptr ? DMF_FORM_BUF_INA : DMF_FORM_BUF) : DMF_FORM_IGEMM;
  a.mtiles = cdiv(a.M, plan.bm);
  a.ntiles = cdiv(a.Nout, plan.bn);
  if (g_stamp_buf && !dgrad && (int)g_stamp_rec.size() < g_stamp_cap) {
    a.stamp = g_stamp_buf + g_stamp_rec.size() * (size_t)STAMP_MAX_BLOCKS * 16;
    g_stamp_rec.push_back(StampRec{(void*)st, g_last_form, a.M, a.Nout, a.Ktot});
  }
  const long long nblk = (long long)a.mtiles * a.ntiles;
  DMF_CHECK_ARG(nblk < (1LL << 31), "%s: grid too large", what);
  const int es = is16(dtype) ? 2 : 4;
  const size_t lds_total = plan.ps ? (size_t)PS_LDS + ((a.out_ss || a.aff_acc || a.tok_res) ? (a.res_ss ? 3 : 2) * (size_t)a.Nout * 4
                                                     : a.bias ? (size_t)a.Nout * 4 : 0)
                          : plan.sq ? (size_t)QLDS
                          : plan.wide ? (size_t)WLDS : conv_lds_main(es, plan.bm, plan.bn) + CONV_LDS_EXTRA;
  if (plan.stem) return launch_conv_stem(a, st, dtype);
  if (!dgrad && plan.pp) {
    // statistics without bias over whole tiles: the fast epilogue (EPI 5)
    const int epi = a.partials != nullptr ? ((g_fast_epi && a.bias == nullptr && a.M % 256 == 0) ? 5 : 0)
                                          : 1 + a.act;
    DMF_CHECK_ARG(epi >= 0 && epi <= 5 && a.act >= 0 && a.act <= 3, "%s: activation %d", what, a.act);
    const bool plain = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0;
    return launch_conv_pp(a, epi, plain, a.bias ? (size_t)a.Nout * 4 : 0, st, dtype);
  }
  DMF_CHECK_ARG(a.dp == 0.f || (!dgrad && plan.ps && a.x2 == nullptr && (a.act == DMF_ACT_GELU || a.tok_res) &&
                                 a.rng && a.partials == nullptr && a.y != nullptr),
                "%s: dropout needs the persistent 1x1 form with the GELU epilogue (one source, rng state)", what);
  DMF_CHECK_ARG((a.out_ss == nullptr && !a.aff_acc) || (!dgrad && plan.ps && a.bias == nullptr && a.x2 == nullptr && a.res),
                "%s: the affine epilogue needs the persistent 1x1 form (no bias, one source, a shortcut)", what);
  DMF_CHECK_ARG(a.y != nullptr || (!dgrad && plan.ps && a.bias == nullptr && a.x2 == nullptr && a.M % QBM == 0 &&
                                   a.stat_acc >= 1),
                "%s: a statistics-only pass needs the persistent 1x1 form, whole 256-row tiles, no bias and an arena",
                what);
  if (!dgrad && plan.ps) {
    DMF_CHECK_ARG(lds_total <= 160 * 1024, "%s: %d output channels of bias exceed the LDS staging", what, a.Nout);
    DMF_CHECK_ARG(a.act >= 0 && a.act <= 3, "%s: activation %d", what, a.act);
  }
  if (!dgrad && plan.buf && a.in_ss != nullptr) {
    DMF_CHECK_ARG(((uintptr_t)a.in_ss % 16) == 0, "%s: input scale/shift must be 16-byte aligned", what);
    DMF_CHECK_ARG(a.C <= 4096, "%s: input-affine conv over %d channels exceeds the LDS staging", what, a.C);
  }
  if (!dgrad && a.in_ss != nullptr) {
    DMF_CHECK_ARG(plan.buf || a.x2 == nullptr, "%s: input affine needs a single source", what);
    DMF_CHECK_ARG(((uintptr_t)a.in_ss % 16) == 0, "%s: input scale/shift must be 16-byte aligned", what);
    DMF_CHECK_ARG(a.act_in == DMF_ACT_NONE || a.act_in == DMF_ACT_RELU || a.act_in == DMF_ACT_GELU,
                  "%s: unsupported input activation %d", what, a.act_in);
  }
  DMF_DISPATCH_DTYPE(dtype, T, launch_conv_t<T>(plan, dgrad, a, nblk, lds_total, st));
  DMF_LAUNCH_CHECK(what);
  return 0;
}

// ------------------------------------------------------- weight re-layout
// torch Conv2d weight [Cout][Cin][KH][KW] (fp32 master) ->
//   mode 0: [Cout][KH][KW][CinP]   (forward B operand, zero-padded channels)
//   mode 1: [CinP][KH][KW][Cout]   (dgrad B operand)
//   mode 2: [CinP][KH][KW][Cout] with the taps flipped (r -> KH-1-r, s -> KW-1-s):
//           a stride-1 dgrad is then a forward conv of dY (pad' = dil*(K-1) - pad)
// element i of the re-laid-out weight (see k_weight_prep's modes)
__device__ __forceinline__ float weight_prep_elem(const float* __restrict__ w, long long i, int Cout, int Cin,
                                                  int CinP, int KH, int KW, int mode) {
  int co, ci, r, s;
  if (mode == 0) {
    ci = (int)(i % CinP);
    long long t = i / CinP;
    s = (int)(t % KW); t /= KW;
    r = (int)(t % KH);
    co = (int)(t / KH);
  } else {
    co = (int)(i % Cout);
    long long t = i / Cout;
    s = (int)(t % KW); t /= KW;
    r = (int)(t % KH);
    ci = (int)(t / KH);
  }
  if (mode == 2) {
    r = KH - 1 - r;
    s = KW - 1 - s;
  }
  return ci < Cin ? w[(((long long)co * Cin + ci) * KH + r) * KW + s] : 0.f;
}

// Every re-layout of a training step in ONE launch (dmf_conv_weight_prep_multi).
// Block code = (job << 40) | unit. Mode 0 ([Cout][KH][KW][CinP], rows of CinP
// channels): unit = first output element of a WPM_SPAN run, 32-bit index math,
// stores coalesced, the reads a KH*KW-strided walk over one torch row (L1/L2
// hits). Modes 1/2 ([CinP][KH][KW][Cout]) are a transpose of the torch
// [Cout][Cin*KH*KW] matrix (taps flipped for mode 2): unit = one 64x64 tile
// staged through LDS, both the reads (along K) and the writes (along Cout)
// coalesced -- a per-element gather there strides Cin*KH*KW floats per lane.
constexpr int WPM_SPAN = 4096;
__device__ __forceinline__ void wprep_store(const dmf_wprep_job& J, long long i, float v) {
  if (J.dtype == DMF_BF16) ((bf16_t*)J.out)[i] = f2bf(v);
  else if (J.dtype == DMF_F16) ((f16_t*)J.out)[i] = (f16_t)v;
  else ((float*)J.out)[i] = v;
}
__global__ void __launch_bounds__(256) k_weight_prep_multi(const dmf_wprep_job* __restrict__ jobs,
                                                           const long long* __restrict__ blk) {
  __shared__ float tile[64][65];
  const long long code = blk[blockIdx.x];
  const dmf_wprep_job J = jobs[(int)(code >> 40)];
  const int unit = (int)(code & ((1LL << 40) - 1));
  const int taps = J.KH * J.KW;
  const int tid = threadIdx.x;
  if (J.mode == 0) {
    const int total = J.Cout * taps * J.CinP;
    const int end = min(total, unit + WPM_SPAN);
    // all of a thread's loads issued before the first store: a rolled loop waits out one
    // global-load latency per element
    constexpr int PER = WPM_SPAN / 256;
    float v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = unit + tid + k * 256;
      const int row = i / J.CinP, ci = i - row * J.CinP;  // row = co * taps + (r, s)
      const int co = row / taps, rs = row - co * taps;
      v[k] = (i < end && ci < J.Cin) ? J.w[((size_t)co * J.Cin + ci) * taps + rs] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = unit + tid + k * 256;
      if (i < end) wprep_store(J, i, v[k]);
    }
    return;
  }
  const int K = J.CinP * taps;  // output rows
  const int ctiles = (J.Cout + 63) / 64;
  const int k0 = (unit / ctiles) * 64, co0 = (unit % ctiles) * 64;
  const int tx = tid & 63, ty = tid >> 6;
  // load: tile[kk][c] = W[co0 + c][src(k0 + kk)], lanes along kk (source columns nearly consecutive)
  {
    const int kk = k0 + tx;
    int src = -1;
    if (kk < K) {
      const int ci = kk / taps, rs = kk - ci * taps;
      const int r = rs / J.KW, s = rs - r * J.KW;
      const int rr = J.mode == 2 ? J.KH - 1 - r : r, ss = J.mode == 2 ? J.KW - 1 - s : s;
      if (ci < J.Cin) src = (ci * J.KH + rr) * J.KW + ss;
    }
    // constant trip counts, unrolled: the 16 loads (and stores) of a thread in flight together
    const size_t rowlen = (size_t)J.Cin * taps;
    float v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int co = co0 + ty + 4 * q;
      v[q] = (src >= 0 && co < J.Cout) ? J.w[(size_t)co * rowlen + src] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) tile[tx][ty + 4 * q] = v[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int kk = ty + 4 * q;
    const int k = k0 + kk, co = co0 + tx;
    if (k < K && co < J.Cout) wprep_store(J, (size_t)k * J.Cout + co, tile[kk][tx]);
  }
}

template <typename T>
__global__ void k_weight_prep(const float* __restrict__ w, T* __restrict__ out, int Cout, int Cin, int CinP, int KH,
                              int KW, int mode) {
  const long long total = (long long)Cout * CinP * KH * KW;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    out[i] = Cvt<T>::store(weight_prep_elem(w, i, Cout, Cin, CinP, KH, KW, mode));
  }
}

}  // namespace dmf

using namespace dmf;

extern "C" int dmf_conv_m_tile(void) { return CBM; }

extern "C" int dmf_conv_last_form(void) { return g_last_form; }


extern "C" int dmf_conv_tune(int key, int value) {
  switch (key) {
    case 0: g_sq_enable = value != 0; return 0;
    case 1: DMF_CHECK_ARG(value >= 0 && value < 4, "dmf_conv_tune: square-tile variant %d", value); g_sq_var = value; return 0;
    case 2: DMF_CHECK_ARG(value >= 0 && value <= 6, "dmf_conv_tune: forced tile %d", value); g_force = value; return 0;
    case 3: DMF_CHECK_ARG(value >= -2 && value <= 64, "dmf_conv_tune: stat mode %d", value); g_stat_mode = value; return 0;
    case 4: g_ps_enable = value != 0; return 0;
    case 6: g_ps_dbg = value; return 0;
    case 16: DMF_CHECK_ARG(value >= 0, "dmf_conv_tune: nontemporal threshold %d", value); g_ps_nt_mb = value; return 0;
    case 7: DMF_CHECK_ARG(value >= 0 && value <= 2, "dmf_conv_tune: ping-pong mode %d", value); g_pp_mode = value; return 0;
    case 8: return conv_pp_tune(value != 0);
    case 10: g_stem_enable = value != 0; return 0;
    case 11: g_fast_epi = value != 0; return 0;
    case 14: DMF_CHECK_ARG(value >= 1, "dmf_conv_tune: wide min tiles %d", value); g_wide_min_tiles = value; return 0;
    case 15: DMF_CHECK_ARG(value >= 1, "dmf_conv_tune: square min tiles %d", value); g_min_tiles = value; return 0;
    default: DMF_CHECK_ARG(false, "dmf_conv_tune: unknown key %d", key);
  }
}

// rows of the BN partial-statistics slab a forward launch of this shape writes
extern "C" int dmf_conv2d_fwd_stat_tiles(int dtype, int N, int H, int W, int Cin, int ldx, int Cin2, int ldx2,
                                         int Cout, int KH, int KW, int stride, int pad, int Ho, int Wo,
                                         int has_in_affine) {
  ConvArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = Cin + Cin2; a.ldx = ldx; a.C1 = Cin; a.ldx2 = ldx2;
  a.stride = stride; a.pad = pad;
  a.x2 = Cin2 > 0 ? (const void*)16 : nullptr;
  a.in_ss = has_in_affine ? (const float*)16 : nullptr;
  a.Nout = Cout; a.KH = KH; a.KW = KW; a.Ktot = KH * KW * a.C; a.M = N * Ho * Wo;
  a.Ho = Ho; a.Wo = Wo; a.ldy = Cout;
  // the dilation the output size implies (conv_plan's tile choice depends on it)
  a.dil = 1;
  for (int d = 1; KH > 1 && d <= 16; ++d)
    if ((H + 2 * pad - d * (KH - 1) - 1) / stride + 1 == Ho) { a.dil = d; break; }
  return cdiv(a.M, conv_plan(dtype, false, a).bm);
}

// 1 when a plain 1x1 conv of this shape that takes its producer's BN apply +
// activation in its operand loads (in_scale_shift) runs on the same
// buffer-load tile as without it -- i.e. the unfused launch would not pick
// the 256-wide LDS-DMA tiles, which have no input-affine form
extern "C" int dmf_conv2d_fwd_input_affine_fusable(int dtype, int N, int H, int W, int Cin, int Cout) {
  ConvArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = Cin; a.ldx = Cin; a.C1 = Cin;
  a.Nout = Cout; a.KH = 1; a.KW = 1; a.stride = 1; a.pad = 0; a.Ktot = Cin; a.M = N * H * W;
  const ConvPlan p = conv_plan(dtype, false, a);
  return p.buf && !p.wide ? 1 : 0;
}

static int conv_fwd_common(ConvArgs& a, int dtype, const void* x, int N, int H, int W, int Cin, int ldx,
                           const void* x2, int Cin2, int ldx2, const void* w, int Cout, int KH, int KW, int stride,
                           int pad, int dil, const float* bias, void* y, int Ho, int Wo, int ldy, int act,
                           const float* in_ss, int in_act, const char* what) {
  DMF_CHECK_ARG(dtype == DMF_F32 || is16(dtype), "%s: bad dtype %d", what, dtype);
  DMF_CHECK_ARG(stride >= 1 && dil >= 1 && KH >= 1 && KW >= 1, "%s: bad geometry", what);
  DMF_CHECK_ARG(Ho == (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1 && Wo == (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1,
                "%s: output size %dx%d inconsistent with input %dx%d k%d s%d p%d d%d", what, Ho, Wo, H, W, KH,
                stride, pad, dil);
  a.x = x; a.w = w; a.bias = bias; a.y = y;
  const int epc = is16(dtype) ? 8 : 4;
  DMF_CHECK_ARG(!x2 || (Cin2 > 0 && Cin2 % epc == 0 && ldx2 % epc == 0 && ((uintptr_t)x2 % 16) == 0),
                "%s: bad second source (C2=%d ld2=%d)", what, Cin2, ldx2);
  a.N = N; a.H = H; a.W = W; a.C = Cin + (x2 ? Cin2 : 0); a.ldx = ldx;
  a.x2 = x2; a.C1 = Cin; a.ldx2 = ldx2;
  a.Ho = Ho; a.Wo = Wo; a.ldy = ldy; a.Nout = Cout;
  a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad; a.dil = dil;
  a.Ktot = KH * KW * a.C;
  a.M = N * Ho * Wo;
  a.act = act;
  a.in_ss = in_ss;
  a.act_in = in_act;
  return 0;
}

extern "C" int dmf_conv2d_fwd(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* x2,
                              int Cin2, int ldx2, const void* w, int Cout, int KH, int KW, int stride, int pad, int dil,
                              const float* bias, void* y, int Ho, int Wo, int ldy, float* bn_partials, int act,
                              const float* in_scale_shift, int in_act, void* stream) {
  ConvArgs a{};
  int rc = conv_fwd_common(a, dtype, x, N, H, W, Cin, ldx, x2, Cin2, ldx2, w, Cout, KH, KW, stride, pad, dil, bias, y,
                           Ho, Wo, ldy, act, in_scale_shift, in_act, "dmf_conv2d_fwd");
  if (rc) return rc;
  a.partials = bn_partials;
  return launch_conv(dtype, false, a, (hipStream_t)stream, "dmf_conv2d_fwd");
}

static ConvArgs affine_args(int dtype, int N, int H, int W, int Cin, int ldx, int Cout, int stride);

// conv (+ bias) -> + residual -> act on the forms whose epilogue stages the C tile (buf / wide / sq / igemm):
// an eval-mode Bottleneck conv3 with its BatchNorm folded into w / bias where the persistent affine form
// (dmf_conv2d_fwd_affine) does not apply. Refuses shapes the planner would give the persistent forms.
extern "C" int dmf_conv2d_fwd_res(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* w,
                                  int Cout, int KH, int KW, int stride, int pad, int dil, const float* bias,
                                  const void* res, int ldr, int act, void* y, int Ho, int Wo, int ldy, void* stream) {
  ConvArgs a{};
  int rc = conv_fwd_common(a, dtype, x, N, H, W, Cin, ldx, nullptr, 0, 0, w, Cout, KH, KW, stride, pad, dil, bias, y,
                           Ho, Wo, ldy, act, nullptr, DMF_ACT_NONE, "dmf_conv2d_fwd_res");
  if (rc) return rc;
  const int epc = is16(dtype) ? 8 : 4;
  DMF_CHECK_ARG(res != nullptr && ldr >= Cout && ldr % epc == 0 && ((uintptr_t)res % 16) == 0 && Cout % epc == 0 &&
                    ldy % epc == 0,
                "dmf_conv2d_fwd_res: residual / output need 16-B aligned rows and whole 16-B channel chunks");
  const ConvPlan p = conv_plan(dtype, false, a);
  DMF_CHECK_ARG(!p.ps && !p.pp && !p.stem,
                "dmf_conv2d_fwd_res: this shape runs on a persistent form (use dmf_conv2d_fwd_affine)");
  a.res = res;
  a.ldr = ldr;
  a.res_add = 1;
  return launch_conv(dtype, false, a, (hipStream_t)stream, "dmf_conv2d_fwd_res");
}

extern "C" int dmf_conv2d_fwd_res_ok(int dtype, int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                     int pad, int dil) {
  ConvArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = Cin; a.ldx = Cin; a.C1 = Cin;
  a.Nout = Cout; a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad; a.dil = dil; a.Ktot = KH * KW * Cin;
  a.Ho = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
  a.Wo = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
  a.M = N * a.Ho * a.Wo; a.ldy = Cout;
  const ConvPlan p = conv_plan(dtype, false, a);
  return (!p.ps && !p.pp && !p.stem && Cout % (is16(dtype) ? 8 : 4) == 0) ? 1 : 0;
}

// token linear (1x1 conv over the rows' NHWC view) -> bias -> GELU -> dropout in one launch (forward-only
// transformer blocks' fc1 under MLP dropout, transformer_model.py:128-134)
extern "C" int dmf_conv2d_fwd_drop_ok(int dtype, int N, int H, int W, int Cin, int Cout) {
  if (!is16(dtype)) return 0;
  ConvArgs a = affine_args(dtype, N, H, W, Cin, Cin, Cout, 1);
  return conv_plan(dtype, false, a).ps && (size_t)PS_LDS + (size_t)Cout * 4 <= 160 * 1024 ? 1 : 0;
}

extern "C" int dmf_conv2d_fwd_drop(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* w,
                                   int Cout, const float* bias, void* y, int ldy, int act, float dropout_p,
                                   const unsigned long long* rng, int site, void* stream) {
  ConvArgs a{};
  int rc = conv_fwd_common(a, dtype, x, N, H, W, Cin, ldx, nullptr, 0, 0, w, Cout, 1, 1, 1, 0, 1, bias, y, H, W, ldy,
                           act, nullptr, DMF_ACT_NONE, "dmf_conv2d_fwd_drop");
  if (rc) return rc;
  DMF_CHECK_ARG(is16(dtype) && act == DMF_ACT_GELU && dropout_p > 0.f && dropout_p < 1.f && rng,
                "dmf_conv2d_fwd_drop: a 16-bit dtype, GELU, 0 < p < 1 and rng state");
  a.dp = dropout_p;
  a.rng = rng;
  a.site = site;
  return launch_conv(dtype, false, a, (hipStream_t)stream, "dmf_conv2d_fwd_drop");
}

extern "C" int dmf_conv2d_fwd_acc(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* x2,
                                  int Cin2, int ldx2, const void* w, int Cout, int KH, int KW, int stride, int pad,
                                  int dil, const float* bias, void* y, int Ho, int Wo, int ldy, double* bn_acc,
                                  int replicas, const float* in_scale_shift, int in_act, void* stream) {
  ConvArgs a{};
  int rc = conv_fwd_common(a, dtype, x, N, H, W, Cin, ldx, x2, Cin2, ldx2, w, Cout, KH, KW, stride, pad, dil, bias, y,
                           Ho, Wo, ldy, DMF_ACT_NONE, in_scale_shift, in_act, "dmf_conv2d_fwd_acc");
  if (rc) return rc;
  DMF_CHECK_ARG(bn_acc != nullptr && ((uintptr_t)bn_acc % 8) == 0, "dmf_conv2d_fwd_acc: bn_acc must be 8-byte aligned");
  DMF_CHECK_ARG(replicas >= 1 && replicas <= 64, "dmf_conv2d_fwd_acc: replicas %d out of [1, 64]", replicas);
  a.partials = (float*)bn_acc;
  a.stat_acc = g_stat_mode != 0 ? g_stat_mode : replicas;
  return launch_conv(dtype, false, a, (hipStream_t)stream, "dmf_conv2d_fwd_acc");
}

extern "C" int dmf_conv2d_fwd_bn(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* x2,
                                 int Cin2, int ldx2, const void* w, int Cout, int KH, int KW, int stride, int pad,
                                 int dil, const float* bias, void* y, int Ho, int Wo, int ldy,
                                 const float* in_scale_shift, int in_act, float* bn_partials, unsigned* bn_tickets,
                                 double count, double unbias_count, const float* gamma, const float* beta,
                                 float* running_mean, float* running_var, long long* num_batches_tracked,
                                 float momentum, float eps, float* scale_shift, float* save_mean_invstd,
                                 void* stream) {
  ConvArgs a{};
  int rc = conv_fwd_common(a, dtype, x, N, H, W, Cin, ldx, x2, Cin2, ldx2, w, Cout, KH, KW, stride, pad, dil, bias, y,
                           Ho, Wo, ldy, DMF_ACT_NONE, in_scale_shift, in_act, "dmf_conv2d_fwd_bn");
  if (rc) return rc;
  DMF_CHECK_ARG(bn_partials && bn_tickets && scale_shift && count > 0, "dmf_conv2d_fwd_bn: bad batch-norm args");
  a.partials = bn_partials;
  a.tickets = bn_tickets;
  a.fin = BnFin{gamma, beta, running_mean, running_var, num_batches_tracked, momentum, eps, count, unbias_count, 1,
                scale_shift, save_mean_invstd};
  return launch_conv(dtype, false, a, (hipStream_t)stream, "dmf_conv2d_fwd_bn");
}

// the ps plan (and so the affine epilogue) for a 1x1 conv of this shape
static ConvArgs affine_args(int dtype, int N, int H, int W, int Cin, int ldx, int Cout, int stride) {
  ConvArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = Cin; a.ldx = ldx; a.C1 = Cin;
  a.Nout = Cout; a.KH = 1; a.KW = 1; a.stride = stride; a.pad = 0; a.dil = 1; a.Ktot = Cin;
  a.Ho = (H - 1) / stride + 1; a.Wo = (W - 1) / stride + 1; a.M = N * a.Ho * a.Wo; a.ldy = Cout;
  (void)dtype;
  return a;
}

// token linear -> + bias -> dropout -> x colscale -> + f32 residual, f32 out, on the persistent 1x1 form
// (forward-only transformer blocks' proj / fc2, transformer_model.py:83-134; the k_gemm_bf16 epilogue of
// those linears with the same Philox masks)
extern "C" int dmf_conv2d_fwd_tokres_ok(int dtype, int N, int H, int W, int Cin, int Cout) {
  if (!is16(dtype)) return 0;
  ConvArgs a = affine_args(dtype, N, H, W, Cin, Cin, Cout, 1);
  a.tok_res = 1;
  return conv_plan(dtype, false, a).ps && (size_t)PS_LDS + (size_t)2 * Cout * 4 <= 160 * 1024 ? 1 : 0;
}

extern "C" int dmf_conv2d_fwd_tokres(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* w,
                                     int Cout, const float* bias, const float* colscale, const float* res, int ldr,
                                     float dropout_p, const unsigned long long* rng, int site, float* y, int ldy,
                                     void* stream) {
  ConvArgs a{};
  int rc = conv_fwd_common(a, dtype, x, N, H, W, Cin, ldx, nullptr, 0, 0, w, Cout, 1, 1, 1, 0, 1, bias, y, H, W, ldy,
                           DMF_ACT_NONE, nullptr, DMF_ACT_NONE, "dmf_conv2d_fwd_tokres");
  if (rc) return rc;
  DMF_CHECK_ARG(is16(dtype) && res && ldr >= Cout && ldr % 4 == 0 && ((uintptr_t)res % 16) == 0 &&
                    ldy % 4 == 0 && (dropout_p <= 0.f || (rng && dropout_p < 1.f)),
                "dmf_conv2d_fwd_tokres: a 16-bit dtype, a 16-B aligned f32 residual / output and rng for dropout");
  DMF_CHECK_ARG((long long)a.M * ldr * 4 < (1LL << 31) && (long long)a.M * ldy * 4 < (1LL << 31),
                "dmf_conv2d_fwd_tokres: residual / output exceed a 32-bit buffer offset");
  a.tok_res = 1;
  a.colscale = colscale;
  a.res = res;
  a.ldr = ldr;
  a.dp = dropout_p > 0.f ? dropout_p : 0.f;
  a.rng = rng;
  a.site = site;
  DMF_CHECK_ARG(conv_plan(dtype, false, a).ps, "dmf_conv2d_fwd_tokres: the shape does not take the persistent 1x1 "
                "form (dmf_conv2d_fwd_tokres_ok)");
  return launch_conv(dtype, false, a, (hipStream_t)stream, "dmf_conv2d_fwd_tokres");
}

extern "C" int dmf_conv2d_fwd_affine_ok(int dtype, int N, int H, int W, int Cin, int Cout, int stride) {
  if (!is16(dtype) || stride < 1) return 0;
  ConvArgs a = affine_args(dtype, N, H, W, Cin, Cin, Cout, stride);
  // (staged scale, shift and the shortcut's scale: 3 x Cout floats beside the ring; whole 256-row tiles for
  // the statistics-only first pass)
  return conv_plan(dtype, false, a).ps && a.M % QBM == 0 && (size_t)PS_LDS + (size_t)3 * Cout * 4 <= 160 * 1024
             ? 1 : 0;
}

extern "C" int dmf_conv2d_fwd_stats(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* w,
                                    int Cout, int stride, int Ho, int Wo, double* bn_acc, int replicas, void* stream) {
  ConvArgs a{};
  int rc = conv_fwd_common(a, dtype, x, N, H, W, Cin, ldx, nullptr, 0, 0, w, Cout, 1, 1, stride, 0, 1, nullptr, nullptr,
                           Ho, Wo, Cout, DMF_ACT_NONE, nullptr, DMF_ACT_NONE, "dmf_conv2d_fwd_stats");
  if (rc) return rc;
  DMF_CHECK_ARG(is16(dtype) && bn_acc && ((uintptr_t)bn_acc % 8) == 0 && replicas >= 1 && replicas <= 64,
                "dmf_conv2d_fwd_stats: needs a 16-bit dtype and a float64 arena slice");
  a.partials = (float*)bn_acc;
  a.stat_acc = replicas;
  return launch_conv(dtype, false, a, (hipStream_t)stream, "dmf_conv2d_fwd_stats");
}

extern "C" int dmf_conv2d_fwd_affine(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* w,
                                     int Cout, int stride, void* y, int Ho, int Wo, int ldy, const float* scale_shift,
                                     const void* res, int ldr, const float* res_scale_shift, void* stream) {
  ConvArgs a{};
  int rc = conv_fwd_common(a, dtype, x, N, H, W, Cin, ldx, nullptr, 0, 0, w, Cout, 1, 1, stride, 0, 1, nullptr, y, Ho,
                           Wo, ldy, DMF_ACT_RELU, nullptr, DMF_ACT_NONE, "dmf_conv2d_fwd_affine");
  if (rc) return rc;
  DMF_CHECK_ARG(is16(dtype) && scale_shift && res && ldr % 8 == 0 && ((uintptr_t)res % 16) == 0 &&
                    ((long long)a.M * ldr * 2 < (1LL << 31)),
                "dmf_conv2d_fwd_affine: needs a 16-bit dtype, scale_shift and an aligned shortcut");
  a.out_ss = scale_shift;
  a.res = res;
  a.ldr = ldr;
  a.res_ss = res_scale_shift;
  return launch_conv(dtype, false, a, (hipStream_t)stream, "dmf_conv2d_fwd_affine");
}

extern "C" int dmf_conv2d_fwd_affine_acc(int dtype, const void* x, int N, int H, int W, int Cin, int ldx,
                                         const void* w, int Cout, int stride, void* y, int Ho, int Wo, int ldy,
                                         const dmf_bn_desc* bn, const void* res, int ldr,
                                         const float* res_scale_shift, void* stream) {
  ConvArgs a{};
  int rc = conv_fwd_common(a, dtype, x, N, H, W, Cin, ldx, nullptr, 0, 0, w, Cout, 1, 1, stride, 0, 1, nullptr, y, Ho,
                           Wo, ldy, DMF_ACT_RELU, nullptr, DMF_ACT_NONE, "dmf_conv2d_fwd_affine_acc");
  if (rc) return rc;
  DMF_CHECK_ARG(is16(dtype) && bn && bn->acc && ((uintptr_t)bn->acc % 16) == 0 && bn->replicas >= 1 &&
                    bn->replicas <= ARENA_MAX_REPLICAS && bn->count > 0.0 && res && ldr % 8 == 0 &&
                    ((uintptr_t)res % 16) == 0 && ((long long)a.M * ldr * 2 < (1LL << 31)),
                "dmf_conv2d_fwd_affine_acc: needs a 16-bit dtype, a float64 arena of <= %d replicas and an aligned "
                "shortcut", ARENA_MAX_REPLICAS);
  a.aff_acc = 1;
  a.partials = (float*)const_cast<double*>(bn->acc);
  a.stat_acc = bn->replicas;
  a.fin = BnFin{bn->gamma, bn->beta, bn->running_mean, bn->running_var, bn->num_batches_tracked, bn->momentum,
                bn->eps, bn->count, bn->unbias_count, 1, nullptr, nullptr};
  a.res = res;
  a.ldr = ldr;
  a.res_ss = res_scale_shift;
  return launch_conv(dtype, false, a, (hipStream_t)stream, "dmf_conv2d_fwd_affine_acc");
}

extern "C" int dmf_conv2d_dgrad(int dtype, const void* dy, int N, int Ho, int Wo, int Cout, int lddy, const void* wt,
                                int Cin, int KH, int KW, int stride, int pad, int dil, void* dx, int H, int W, int lddx,
                                void* stream) {
  DMF_CHECK_ARG(dtype == DMF_F32 || is16(dtype), "dmf_conv2d_dgrad: bad dtype %d", dtype);
  DMF_CHECK_ARG(Ho == (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1 && Wo == (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1,
                "dmf_conv2d_dgrad: geometry mismatch");
  ConvArgs a{};
  a.x = dy; a.w = wt; a.bias = nullptr; a.y = dx; a.partials = nullptr;
  a.N = N; a.H = Ho; a.W = Wo; a.C = Cout; a.ldx = lddy;
  a.x2 = nullptr; a.C1 = Cout; a.ldx2 = 0;
  a.Ho = H; a.Wo = W; a.ldy = lddx; a.Nout = Cin;
  a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad; a.dil = dil;
  a.Ktot = KH * KW * Cout;
  a.M = N * H * W;
  a.act = DMF_ACT_NONE;
  return launch_conv(dtype, true, a, (hipStream_t)stream, "dmf_conv2d_dgrad");
}

extern "C" int dmf_conv_weight_prep_multi(const dmf_wprep_job* jobs, const long long* blk, long long nblocks,
                                          void* stream) {
  DMF_CHECK_ARG(jobs && blk && nblocks > 0 && nblocks < (1LL << 31), "dmf_conv_weight_prep_multi: bad tables");
  hipLaunchKernelGGL(k_weight_prep_multi, dim3((unsigned)nblocks), dim3(256), 0, (hipStream_t)stream, jobs, blk);
  DMF_LAUNCH_CHECK("dmf_conv_weight_prep_multi");
  return 0;
}

extern "C" int dmf_conv_weight_prep(int dtype, const float* w, void* out, int Cout, int Cin, int CinP, int KH, int KW,
                                    int mode, void* stream) {
  DMF_CHECK_ARG(CinP >= Cin && mode >= 0 && mode <= 2, "dmf_conv_weight_prep: bad args");
  const long long total = (long long)Cout * CinP * KH * KW;
  const int grid = (int)(total < 65536 * 256LL ? cdiv(total, 256) : 65536);
  DMF_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_weight_prep<T>, dim3(grid), dim3(256), 0, (hipStream_t)stream, w,
                                                   (T*)out, Cout, Cin, CinP, KH, KW, mode));
  DMF_LAUNCH_CHECK("dmf_conv_weight_prep");
  return 0;
}
